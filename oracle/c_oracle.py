"""ctypes binding of oracle/c/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The C restatement (oracle/c/evolu_oracle.c) is the large-N checker and the
timed CPU baseline; it is pinned against the Python oracle by
tests/test_oracle_c.py.  Build: make -C oracle/c (done by __graft_entry__.build()).
"""
import ctypes as C
import os

import numpy as np

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "liboracle.so")
_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            import subprocess

            subprocess.run(["make", "-s", "-C", os.path.dirname(LIB)], check=True)
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.evo_murmur3.restype = C.c_uint32
        L.evo_murmur3.argtypes = [C.c_char_p, C.c_size_t]
        L.evo_apply.restype = C.c_int
        L.evo_apply.argtypes = [vp, C.c_size_t, C.c_size_t, vp, C.c_uint32, vp, C.c_size_t, vp, vp, vp,
                                C.POINTER(C.c_void_p)]
        L.evo_server_new.restype = vp
        L.evo_server_new.argtypes = [C.c_uint32, C.c_size_t]
        L.evo_server_free.argtypes = [vp]
        L.evo_server_ingest.restype = C.c_int
        L.evo_server_ingest.argtypes = [vp, vp, C.c_size_t, C.c_size_t, vp, vp]
        L.evo_server_tree_json.restype = C.c_void_p
        L.evo_server_tree_json.argtypes = [vp, C.c_uint32]
        L.evo_server_diff.restype = C.c_int
        L.evo_server_diff.argtypes = [vp, vp, C.c_uint32, C.POINTER(C.c_int64)]
        L.evo_tree_json.restype = C.c_void_p
        L.evo_tree_json.argtypes = [vp, C.c_size_t, C.c_size_t]
        L.evo_free.argtypes = [vp]
        _L = L
    return _L


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _take_str(p):
    s = C.string_at(p).decode()
    lib().evo_free(p)
    return s


def apply(ts: np.ndarray, cell: np.ndarray, n_cells: int, prior: np.ndarray = None, prior_present: np.ndarray = None):
    """-> (status, flags u8[n], winner i32[n_cells], tree JSON or None)"""
    ts = np.ascontiguousarray(ts)
    cell = np.ascontiguousarray(cell, dtype=np.uint32)
    n, stride = ts.shape
    flags = np.zeros(max(n, 1), dtype=np.uint8)
    winner = np.zeros(max(n_cells, 1), dtype=np.int32)
    js = C.c_void_p()
    pstride = prior.shape[1] if prior is not None else 48
    st = lib().evo_apply(_ptr(ts), stride, n, _ptr(cell), n_cells, _ptr(prior), pstride,
                         _ptr(None if prior_present is None else np.ascontiguousarray(prior_present, dtype=np.uint8)),
                         _ptr(flags), _ptr(winner), C.byref(js))
    return st, flags[:n], winner[:n_cells], (_take_str(js.value) if st == 0 else None)


class Server:
    def __init__(self, n_owners: int, cap: int):
        self.h = lib().evo_server_new(n_owners, cap)

    def ingest(self, ts: np.ndarray, owner: np.ndarray):
        ts = np.ascontiguousarray(ts)
        owner = np.ascontiguousarray(owner, dtype=np.uint32)
        flags = np.zeros(max(len(ts), 1), dtype=np.uint8)
        st = lib().evo_server_ingest(self.h, _ptr(ts), ts.shape[1], len(ts), _ptr(owner), _ptr(flags))
        return st, flags[: len(ts)]

    def tree_json(self, owner: int) -> str:
        return _take_str(lib().evo_server_tree_json(self.h, owner))

    def diff(self, other: "Server", owner: int):
        m = C.c_int64()
        st = lib().evo_server_diff(self.h, other.h, owner, C.byref(m))
        return {0: -1, 1: m.value, 2: -2}[st]

    def __del__(self):
        if getattr(self, "h", None):
            lib().evo_server_free(self.h)
            self.h = None


def tree_json(ts: np.ndarray) -> str:
    ts = np.ascontiguousarray(ts)
    return _take_str(lib().evo_tree_json(_ptr(ts), ts.shape[1], len(ts)))
