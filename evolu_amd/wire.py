"""SyncRequest / SyncResponse wire codec (protobuf.ts:60-171) over libevm's
host codec (evm_pb_*).  Mirrors protobuf-ts' fromBinary / toBinary for the
two sync messages; the timestamps come out as the engine's 48-byte arena.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check
from .engine import TS_LEN, TS_STRIDE, encode_timestamps

REQUEST = _lib.PB_SYNC_REQUEST
RESPONSE = _lib.PB_SYNC_RESPONSE


class _Sync(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("n_messages", "content_bytes", "user_off", "user_len", "node_off",
                                          "node_len", "tree_off", "tree_len", "nonstd_ts")]


@dataclass
class Sync:
    """A decoded SyncRequest (user/node set) or SyncResponse."""
    ts: np.ndarray           # (n, stride) uint8 timestamp arena (0xFF rows: not 46 bytes)
    ts_len: np.ndarray       # (n,) uint32 original timestamp lengths
    content_off: np.ndarray  # (n + 1,) uint64
    content: bytes
    tree: str
    raw: Optional[List[str]] = None  # the timestamp strings as sent (any length)
    user: Optional[str] = None
    node: Optional[str] = None

    def timestamps(self) -> List[str]:
        """The 46-byte timestamps (rows of other lengths read as 0xFF bytes)."""
        return [bytes(self.ts[i, :TS_LEN]).decode("latin-1") for i in range(len(self.ts_len))]

    def contents(self) -> List[bytes]:
        o = self.content_off
        return [self.content[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def decode(kind: int, body: bytes, stride: int = TS_STRIDE) -> Sync:
    lib = _lib.load()
    buf = (C.c_uint8 * max(len(body), 1)).from_buffer_copy(body or b"\0")
    info = _Sync()
    check(lib.evm_pb_scan(kind, buf, len(body), C.byref(info)), "evm_pb_scan")
    n = info.n_messages
    ts = np.zeros((n, stride), dtype=np.uint8)
    ts_len = np.zeros(n, dtype=np.uint32)
    off = np.zeros(n + 1, dtype=np.uint64)
    content = np.zeros(max(info.content_bytes, 1), dtype=np.uint8)
    ts_off = np.zeros(n, dtype=np.uint64)
    check(lib.evm_pb_split(kind, buf, len(body), ts.ctypes.data_as(C.c_void_p), stride,
                           ts_len.ctypes.data_as(C.c_void_p), ts_off.ctypes.data_as(C.c_void_p),
                           off.ctypes.data_as(C.c_void_p),
                           content.ctypes.data_as(C.c_void_p)), "evm_pb_split")
    s = lambda o, k: body[o:o + k].decode("utf-8", "replace")  # noqa: E731
    out = Sync(ts, ts_len, off, content[: info.content_bytes].tobytes(), s(info.tree_off, info.tree_len),
               raw=[body[int(o):int(o) + int(k)].decode("utf-8", "replace") for o, k in zip(ts_off, ts_len)])
    if kind == REQUEST:
        out.user = s(info.user_off, info.user_len)
        out.node = s(info.node_off, info.node_len)
    return out


def encode(kind: int, timestamps: Sequence[str], contents: Sequence[bytes], tree: str = "",
           user: str = "", node: str = "") -> bytes:
    """protobuf-ts toBinary of a SyncRequest (user/node) or SyncResponse."""
    lib = _lib.load()
    n = len(timestamps)
    raw = [t.encode("utf-8") for t in timestamps]
    stride = max([TS_STRIDE] + [len(r) for r in raw])
    ts = np.zeros((n, stride), dtype=np.uint8)
    ts_len = np.zeros(n, dtype=np.uint32)
    for i, r in enumerate(raw):
        ts[i, :len(r)] = np.frombuffer(r, dtype=np.uint8)
        ts_len[i] = len(r)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(c) for c in contents]) if n else []
    cat = np.frombuffer(b"".join(contents) or b"\0", dtype=np.uint8).copy()
    ub, nb, tb = user.encode(), node.encode(), tree.encode()
    need = C.c_size_t()
    args = [kind, ts.ctypes.data_as(C.c_void_p), stride, ts_len.ctypes.data_as(C.c_void_p), n,
            off.ctypes.data_as(C.c_void_p), cat.ctypes.data_as(C.c_void_p), ub, len(ub), nb, len(nb), tb, len(tb)]
    check(lib.evm_pb_encode(*args, None, 0, C.byref(need)), "evm_pb_encode")
    out = (C.c_uint8 * max(need.value, 1))()
    check(lib.evm_pb_encode(*args, out, need.value, C.byref(need)), "evm_pb_encode")
    return bytes(out)[: need.value]


__all__ = ["REQUEST", "RESPONSE", "Sync", "decode", "encode", "encode_timestamps"]
