"""Device-level host wrapper of libevm (torch tensors as device buffers).

torch is plumbing here (device memory, streams, torch.distributed); every
computation runs in libevm's HIP kernels.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check

TS_LEN = 46
TS_STRIDE = 48  # native coalesced layout: 46 bytes + 2 pad


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def encode_timestamps(strings: Sequence[str], stride: int = TS_STRIDE) -> np.ndarray:
    """Packs timestamp strings into a (n, stride) uint8 arena.

    Strings that are not exactly 46 ASCII bytes cannot be canonical: their
    slot is filled with 0xFF bytes so the engine flags them (EVM_META_NONCANON).
    """
    n = len(strings)
    arena = np.zeros((n, stride), dtype=np.uint8)
    if n == 0:
        return arena
    try:
        raw = "".join(strings).encode("ascii")
        ok = len(raw) == TS_LEN * n and all(len(s) == TS_LEN for s in strings)
    except UnicodeEncodeError:
        ok = False
    if ok:
        arena[:, :TS_LEN] = np.frombuffer(raw, dtype=np.uint8).reshape(n, TS_LEN)
        return arena
    for i, s in enumerate(strings):
        b = s.encode("utf-8", "replace")
        if len(b) == TS_LEN and len(s) == TS_LEN:
            arena[i, :TS_LEN] = np.frombuffer(b, dtype=np.uint8)
        else:
            arena[i, :TS_LEN] = 0xFF
    return arena


class Engine:
    """One libevm context bound to one GPU (one per thread)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        self.device = device
        torch.cuda.set_device(device)
        h = C.c_void_p()
        check(self.lib.evm_create(device, C.byref(h)), "evm_create")
        self.h = h
        self.bind_stream(torch.cuda.current_stream(device))

    def bind_stream(self, stream: torch.cuda.Stream):
        check(self.lib.evm_set_stream(self.h, C.c_void_p(stream.cuda_stream)), "evm_set_stream")

    def close(self):
        if getattr(self, "h", None):
            self.lib.evm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, option: int, value: int):
        check(self.lib.evm_set_option(self.h, option, value), "evm_set_option")

    STATS_FIELDS = ("workspace_regrows", "workspace_bytes", "scratch_pool_allocs", "scratch_pool_bytes",
                    "block_allocs", "block_bytes", "tc_batches", "tc_redos", "small_batches", "small_fallbacks")

    def stats(self) -> dict:
        """Allocation counters (evm_get_stats)."""
        buf = (C.c_uint64 * len(self.STATS_FIELDS))()
        check(self.lib.evm_get_stats(self.h, C.byref(buf)), "evm_get_stats")
        return dict(zip(self.STATS_FIELDS, [int(x) for x in buf]))

    # ------------------------------------------------------------- profiling
    def prof_enable(self, on: bool = True):
        check(self.lib.evm_prof_enable(self.h, 1 if on else 0), "evm_prof_enable")

    def prof_only(self, kernel: Optional[str] = None):
        """Time only `kernel`'s launches (its report name); None = every kernel."""
        check(self.lib.evm_prof_only(self.h, (kernel or "").encode()), "evm_prof_only")

    def prof_reset(self):
        check(self.lib.evm_prof_reset(self.h), "evm_prof_reset")

    def prof_report(self) -> dict:
        """{kernel name: (total ms, launches)} from HIP events on the engine stream."""
        import json

        ln = C.c_size_t()
        check(self.lib.evm_prof_report(self.h, None, 0, C.byref(ln)), "evm_prof_report")
        buf = C.create_string_buffer(ln.value + 64)
        check(self.lib.evm_prof_report(self.h, buf, ln.value + 64, C.byref(ln)), "evm_prof_report")
        return {k: (v[0], int(v[1])) for k, v in json.loads(buf.raw[: ln.value].decode()).items()}

    # --------------------------------------------------------------- buffers
    def dev(self, a: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(a)).to(f"cuda:{self.device}")

    def timestamps(self, strings: Sequence[str], stride: int = TS_STRIDE) -> torch.Tensor:
        return self.dev(encode_timestamps(strings, stride))

    # ------------------------------------------------------------------- K1
    def pack(self, ts: torch.Tensor, aux: Optional[torch.Tensor] = None):
        """-> (records int64 tensor view [n,4], status)."""
        n, stride = ts.shape
        out = torch.empty((n, 4), dtype=torch.int64, device=ts.device)
        st = self.lib.evm_pack(self.h, _ptr(ts), stride, n, _ptr(aux), _ptr(out))
        if st not in (_lib.EVM_OK, _lib.EVM_ENONCANON):
            check(st, "evm_pack")
        return out, st

    # ----------------------------------------------------------------- trees
    def tree_new(self, n_owners: int = 1) -> "Trees":
        h = C.c_void_p()
        check(self.lib.evm_tree_new(self.h, n_owners, C.byref(h)), "evm_tree_new")
        return Trees(self, h)

    def tree_from_json(self, texts: Sequence[str]) -> "Trees":
        bs = [t.encode() for t in texts]
        arr = (C.c_char_p * len(bs))(*bs)
        lens = (C.c_size_t * len(bs))(*[len(b) for b in bs])
        h = C.c_void_p()
        check(self.lib.evm_tree_from_json(self.h, len(bs), arr, lens, C.byref(h)), "evm_tree_from_json")
        return Trees(self, h)

    def receive_fold(self, ts: torch.Tensor, local: tuple, now: int, max_drift: int = 60000):
        """receive.ts:45-66 -> ("ok", (millis, counter, node)) or (error kind, info dict)."""
        class Res(C.Structure):
            _fields_ = [("error", C.c_int32), ("counter", C.c_uint32), ("millis", C.c_int64),
                        ("error_index", C.c_int64), ("next", C.c_int64)]

        n, stride = ts.shape
        r = Res()
        check(self.lib.evm_receive_fold(self.h, _ptr(ts), stride, n, local[0], local[1], local[2].encode(), now,
                                        max_drift, C.byref(r)), "evm_receive_fold")
        kinds = {1: "TimestampDriftError", 2: "TimestampDuplicateNodeError", 3: "TimestampCounterOverflowError"}
        if r.error == 0:
            return "ok", (r.millis, r.counter, local[2])
        return kinds[r.error], {"index": r.error_index, "next": r.next}

    def store_new(self, n_owners: int) -> "Store":
        return Store(self, n_owners)

    def tree_from_leaves(self, off: np.ndarray, code: np.ndarray, xr: np.ndarray) -> "Trees":
        off = np.ascontiguousarray(off, dtype=np.uint64)
        code = np.ascontiguousarray(code, dtype=np.uint64)
        xr = np.ascontiguousarray(xr, dtype=np.int32)
        h = C.c_void_p()
        check(
            self.lib.evm_tree_from_leaves(
                self.h, len(off) - 1, off.ctypes.data_as(C.c_void_p), code.ctypes.data_as(C.c_void_p),
                xr.ctypes.data_as(C.c_void_p), C.byref(h)),
            "evm_tree_from_leaves",
        )
        return Trees(self, h)

    def merkle_insert(self, trees: "Trees", ts: torch.Tensor, owner: Optional[torch.Tensor] = None) -> "Trees":
        n, stride = ts.shape
        h = C.c_void_p()
        check(self.lib.evm_merkle_insert(self.h, trees.h, _ptr(ts), stride, n, _ptr(owner), C.byref(h)),
              "evm_merkle_insert")
        return Trees(self, h)

    def tree_from_device_leaves(self, off: torch.Tensor, code: torch.Tensor, xr: torch.Tensor) -> "Trees":
        """Trees from device leaf lists (int64 off[n_owners+1], int64 code, int32 xr)."""
        off = off.to(torch.int64).contiguous()
        code = code.to(torch.int64).contiguous()
        xr = xr.to(torch.int32).contiguous()
        h = C.c_void_p()
        check(self.lib.evm_tree_from_device_leaves(self.h, off.numel() - 1, _ptr(off), _ptr(code), _ptr(xr),
                                                   C.byref(h)), "evm_tree_from_device_leaves")
        return Trees(self, h)

    def tree_merge(self, a: "Trees", b: "Trees") -> "Trees":
        """Union of two tree sets' inserts (equal leaves XOR-combine)."""
        h = C.c_void_p()
        check(self.lib.evm_tree_merge(self.h, a.h, b.h, C.byref(h)), "evm_tree_merge")
        return Trees(self, h)

    def merkle_diff(self, a: "Trees", b: "Trees") -> torch.Tensor:
        out = torch.empty(a.n_owners, dtype=torch.int64, device=f"cuda:{self.device}")
        check(self.lib.evm_merkle_diff(self.h, a.h, b.h, _ptr(out)), "evm_merkle_diff")
        return out

    # ---------------------------------------------------------------- client
    def apply_batch(self, trees: "Trees", ts: torch.Tensor, cell: torch.Tensor, n_cells: int,
                    cell_owner: Optional[torch.Tensor] = None, prior_ts: Optional[torch.Tensor] = None,
                    prior_present: Optional[torch.Tensor] = None, flags: Optional[torch.Tensor] = None,
                    winner: Optional[torch.Tensor] = None, raise_on_error: bool = True,
                    stored_ts: Optional[torch.Tensor] = None, stored_cell: Optional[torch.Tensor] = None):
        """applyMessages for one batch -> (flags u8[n], winner i32[n_cells], Trees, status).

        stored_ts / stored_cell: the rows already in __message whose timestamp
        is in the batch (evm_apply_batch_ex; a cell id >= n_cells = a cell the
        batch does not touch)."""
        n, stride = ts.shape
        dev = ts.device
        if flags is None:
            flags = torch.empty(n, dtype=torch.uint8, device=dev)
        if winner is None:
            winner = torch.empty(max(n_cells, 1), dtype=torch.int32, device=dev)
        pstride = prior_ts.shape[1] if prior_ts is not None else 48
        h = C.c_void_p()
        if stored_ts is not None and stored_ts.shape[0]:
            st = self.lib.evm_apply_batch_ex(self.h, trees.h, _ptr(ts), stride, n, _ptr(cell), n_cells,
                                             _ptr(cell_owner), _ptr(prior_ts), pstride, _ptr(prior_present),
                                             _ptr(stored_ts), stored_ts.shape[1], stored_ts.shape[0],
                                             _ptr(stored_cell), _ptr(flags), _ptr(winner), C.byref(h))
        else:
            st = self.lib.evm_apply_batch(self.h, trees.h, _ptr(ts), stride, n, _ptr(cell), n_cells,
                                          _ptr(cell_owner), _ptr(prior_ts), pstride, _ptr(prior_present),
                                          _ptr(flags), _ptr(winner), C.byref(h))
        if raise_on_error:
            check(st, "evm_apply_batch")
        return flags, winner[:n_cells], (Trees(self, h) if st == _lib.EVM_OK else None), st


    def apply_batch_async(self, trees: "Trees", ts: torch.Tensor, cell: torch.Tensor, n_cells: int,
                          flags: torch.Tensor, winner: torch.Tensor, prior_ts: Optional[torch.Tensor] = None,
                          prior_present: Optional[torch.Tensor] = None, stored_ts: Optional[torch.Tensor] = None,
                          stored_cell: Optional[torch.Tensor] = None) -> "Pending":
        """evm_apply_batch_async: enqueue; .wait() -> (flags, winner, Trees or None, status).
        Every tensor passed must stay alive and untouched until the wait."""
        n, stride = ts.shape
        pstride = prior_ts.shape[1] if prior_ts is not None else 48
        sn = 0 if stored_ts is None else stored_ts.shape[0]
        sstride = 48 if stored_ts is None else stored_ts.shape[1]
        h = C.c_void_p()
        check(self.lib.evm_apply_batch_async(self.h, trees.h, _ptr(ts), stride, n, _ptr(cell), n_cells, None,
                                             _ptr(prior_ts), pstride, _ptr(prior_present), _ptr(stored_ts), sstride,
                                             sn, _ptr(stored_cell), _ptr(flags), _ptr(winner), C.byref(h)),
              "evm_apply_batch_async")
        return Pending(self, h, (trees, ts, cell, flags, winner, prior_ts, prior_present, stored_ts, stored_cell),
                       n_cells)

    def cross_cell_check(self, ts: torch.Tensor, cell: torch.Tensor, n_cells: int) -> bool:
        """True iff some timestamp of the batch occurs with two different cells
        (the global __message PK case evm_apply_batch reports as EVM_ECOLLISION)."""
        n, stride = ts.shape
        found = C.c_int32(0)
        check(self.lib.evm_cross_cell_check(self.h, _ptr(ts), stride, n, _ptr(cell), n_cells, C.byref(found)),
              "evm_cross_cell_check")
        return bool(found.value)


class Pending:
    """An enqueued applyMessages batch (evm_apply_batch_async); keeps its
    tensors alive until wait()."""

    def __init__(self, eng: "Engine", h, keep, n_cells: int):
        self.eng = eng
        self.h = h
        self.keep = keep
        self.n_cells = n_cells

    def __del__(self):
        # dropped without a wait (e.g. an exception between enqueue and wait):
        # wait anyway, so the handle is released and no tensor the batch still
        # reads or writes goes back to the caching allocator early
        try:
            if self.h is not None and self.eng.h:
                t = C.c_void_p()
                if self.eng.lib.evm_apply_wait(self.eng.h, self.h, C.byref(t)) == _lib.EVM_OK and t.value:
                    self.eng.lib.evm_tree_free(self.eng.h, t)
                self.h = None
        except Exception:
            pass

    def wait(self, raise_on_error: bool = True):
        if self.h is None:
            raise RuntimeError("evm_apply_wait: this batch was already waited")
        t = C.c_void_p()
        st = self.eng.lib.evm_apply_wait(self.eng.h, self.h, C.byref(t))
        self.h = None
        flags, winner = self.keep[3], self.keep[4]
        self.keep = None
        if raise_on_error:
            check(st, "evm_apply_wait")
        return flags, winner[: self.n_cells], (Trees(self.eng, t) if st == _lib.EVM_OK else None), st


class Store:
    """Server state: per-owner stored messages + MerkleTrees (index.ts tables)."""

    def __init__(self, eng: "Engine", n_owners: int):
        self.eng = eng
        h = C.c_void_p()
        check(eng.lib.evm_store_new(eng.h, n_owners, C.byref(h)), "evm_store_new")
        self.h = h
        self.n_owners = n_owners

    def free(self):
        if self.h:
            self.eng.lib.evm_store_free(self.eng.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    @property
    def n_messages(self) -> int:
        no = C.c_uint32()
        nm = C.c_uint64()
        check(self.eng.lib.evm_store_info(self.h, C.byref(no), C.byref(nm)), "evm_store_info")
        return nm.value

    def tree(self) -> "Trees":
        """The store's trees (borrowed: valid until the next ingest)."""
        return Trees(self.eng, C.c_void_p(self.eng.lib.evm_store_tree(self.h)), owned=False)

    def messages(self):
        off = np.zeros(self.n_owners + 1, dtype=np.uint64)
        ids = np.zeros(max(self.n_messages, 1), dtype=np.uint64)
        check(self.eng.lib.evm_store_messages(self.eng.h, self.h, off.ctypes.data_as(C.c_void_p),
                                              ids.ctypes.data_as(C.c_void_p)), "evm_store_messages")
        return off, ids[: self.n_messages]

    def ingest(self, ts: torch.Tensor, owner: torch.Tensor, id_base: int = 0, flags: Optional[torch.Tensor] = None,
               raise_on_error: bool = True):
        n, stride = ts.shape
        if flags is None:
            flags = torch.empty(max(n, 1), dtype=torch.uint8, device=ts.device)
        st = self.eng.lib.evm_server_ingest(self.eng.h, self.h, _ptr(ts), stride, n, _ptr(owner), id_base, _ptr(flags))
        if raise_on_error:
            check(st, "evm_server_ingest")
        return flags[:n], st

    def ingest_ex(self, ts: torch.Tensor, owner: torch.Tensor, id_base: int = 0, flags: Optional[torch.Tensor] = None):
        """evm_server_ingest_ex: per-owner transactions -> (flags, owner_status
        uint8[n_owners] (1: that owner committed nothing), status)."""
        n, stride = ts.shape
        if flags is None:
            flags = torch.empty(max(n, 1), dtype=torch.uint8, device=ts.device)
        ost = torch.empty(max(self.n_owners, 1), dtype=torch.uint8, device=ts.device)
        st = self.eng.lib.evm_server_ingest_ex(self.eng.h, self.h, _ptr(ts), stride, n, _ptr(owner), id_base,
                                               _ptr(flags), _ptr(ost))
        if st not in (_lib.EVM_OK, _lib.EVM_ENONCANON):
            check(st, "evm_server_ingest_ex")
        return flags[:n], ost[: self.n_owners], st

    def select(self, client: "Trees", node: torch.Tensor, active: Optional[torch.Tensor] = None, cap: int = None):
        """-> (diff int64[n_owners], sel_off uint64[n_owners+1], sel_id uint64[n_sel])."""
        dev = node.device
        O = self.n_owners
        diff = torch.empty(max(O, 1), dtype=torch.int64, device=dev)
        off = torch.empty(O + 1, dtype=torch.int64, device=dev)
        cap = self.n_messages if cap is None else cap
        ids = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        nsel = C.c_uint64()
        check(self.eng.lib.evm_server_select(self.eng.h, self.h, client.h, _ptr(node), _ptr(active), _ptr(diff),
                                             _ptr(off), _ptr(ids), cap, C.byref(nsel)), "evm_server_select")
        return diff[:O], off, ids[: nsel.value]

    def select_after(self, bound: torch.Tensor, node: Optional[torch.Tensor] = None,
                     active: Optional[torch.Tensor] = None, cap: int = None, keys: bool = False):
        """Selection with given per-owner bounds (evm_store_select_after):
        -> (sel_off int64[n_owners+1], sel_id int64[n_sel], sel_key int64[n_sel, 3] or None)."""
        dev = bound.device
        O = self.n_owners
        bound = bound.to(torch.int64).contiguous()
        off = torch.empty(O + 1, dtype=torch.int64, device=dev)
        cap = self.n_messages if cap is None else cap
        ids = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        key = torch.empty((max(cap, 1), 3), dtype=torch.int64, device=dev) if keys else None
        nsel = C.c_uint64()
        check(self.eng.lib.evm_store_select_after(self.eng.h, self.h, _ptr(bound), _ptr(node), _ptr(active),
                                                  _ptr(off), _ptr(ids), _ptr(key), cap, C.byref(nsel)),
              "evm_store_select_after")
        return off, ids[: nsel.value], (key[: nsel.value] if keys else None)

    def since(self, since: torch.Tensor, cap: int = None):
        """receive.ts:118-124 resend range, batched over owners: for since[o] >= 0
        the owner's ids with timestamp > syncTs(since[o]), in timestamp order.
        -> (sel_off uint64[n_owners+1], sel_id uint64[n_sel])."""
        dev = since.device
        O = self.n_owners
        since = since.to(torch.int64).contiguous()
        off = torch.empty(O + 1, dtype=torch.int64, device=dev)
        cap = self.n_messages if cap is None else cap
        ids = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        nsel = C.c_uint64()
        check(self.eng.lib.evm_store_since(self.eng.h, self.h, _ptr(since), _ptr(off), _ptr(ids), cap,
                                           C.byref(nsel)), "evm_store_since")
        return off, ids[: nsel.value]


class Trees:
    """A device-resident set of per-owner MerkleTrees (owns its evm_tree)."""

    def __init__(self, eng: Engine, h, owned: bool = True):
        self.eng = eng
        self.h = h
        self.owned = owned
        no = C.c_uint32()
        nl = C.c_uint64()
        check(eng.lib.evm_tree_info(h, C.byref(no), C.byref(nl)), "evm_tree_info")
        self.n_owners = no.value
        self.n_leaves = nl.value

    def free(self):
        if self.h and self.owned:
            self.eng.lib.evm_tree_free(self.eng.h, self.h)
        self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def leaves(self):
        off = np.zeros(self.n_owners + 1, dtype=np.uint64)
        code = np.zeros(max(self.n_leaves, 1), dtype=np.uint64)
        xr = np.zeros(max(self.n_leaves, 1), dtype=np.int32)
        check(self.eng.lib.evm_tree_leaves(self.eng.h, self.h, off.ctypes.data_as(C.c_void_p),
                                           code.ctypes.data_as(C.c_void_p), xr.ctypes.data_as(C.c_void_p)),
              "evm_tree_leaves")
        return off, code[: self.n_leaves], xr[: self.n_leaves]

    def slice_device(self, owner_lo: int, count: int):
        """Device copy of owners [owner_lo, owner_lo+count)'s leaves ->
        (off int64[count+1] from 0, code int64[L], xr int32[L])."""
        dev = torch.device("cuda", self.eng.device)
        nl = C.c_uint64()
        off = torch.empty(count + 1, dtype=torch.int64, device=dev)
        st = self.eng.lib.evm_tree_slice(self.eng.h, self.h, owner_lo, count, _ptr(off), None, None, 0, C.byref(nl))
        if st not in (_lib.EVM_OK, _lib.EVM_ECAPACITY):
            check(st, "evm_tree_slice")
        L = nl.value
        code = torch.empty(max(L, 1), dtype=torch.int64, device=dev)
        xr = torch.empty(max(L, 1), dtype=torch.int32, device=dev)
        check(self.eng.lib.evm_tree_slice(self.eng.h, self.h, owner_lo, count, _ptr(off), _ptr(code), _ptr(xr), L,
                                          C.byref(nl)), "evm_tree_slice")
        return off, code[:L], xr[:L]

    def roots(self):
        r = np.zeros(max(self.n_owners, 1), dtype=np.int32)
        p = np.zeros(max(self.n_owners, 1), dtype=np.uint8)
        check(self.eng.lib.evm_tree_roots(self.eng.h, self.h, r.ctypes.data_as(C.c_void_p),
                                          p.ctypes.data_as(C.c_void_p)), "evm_tree_roots")
        return r[: self.n_owners], p[: self.n_owners].astype(bool)

    def to_json_batch(self, owners: Optional[torch.Tensor] = None, count: Optional[int] = None):
        """Many owners' JSON in one device call (evm_tree_to_json_batch):
        owners (device int32/uint32, or None = 0..count-1) -> (bytes uint8
        device tensor, offsets int64 device tensor [n + 1])."""
        dev = torch.device("cuda", self.eng.device)
        n = int(owners.numel()) if owners is not None else (self.n_owners if count is None else count)
        off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        tot = C.c_uint64()
        check(self.eng.lib.evm_tree_to_json_batch(self.eng.h, self.h, _ptr(owners), n, None, 0, _ptr(off),
                                                  C.byref(tot)), "evm_tree_to_json_batch")
        out = torch.empty(max(tot.value, 1), dtype=torch.uint8, device=dev)
        check(self.eng.lib.evm_tree_to_json_batch(self.eng.h, self.h, _ptr(owners), n, _ptr(out), out.numel(),
                                                  _ptr(off), C.byref(tot)), "evm_tree_to_json_batch")
        return out[: tot.value], off

    def to_json(self, owner: int = 0) -> str:
        ln = C.c_size_t()
        check(self.eng.lib.evm_tree_to_json(self.eng.h, self.h, owner, None, 0, C.byref(ln)), "evm_tree_to_json")
        buf = C.create_string_buffer(ln.value)
        check(self.eng.lib.evm_tree_to_json(self.eng.h, self.h, owner, buf, ln.value, C.byref(ln)),
              "evm_tree_to_json")
        return buf.raw[: ln.value].decode()


def key_string(code: int) -> str:
    """Leaf code -> base-3 key string (inverse of the engine's path code)."""
    out = []
    for i in range(20):
        d = (code >> (2 * (19 - i))) & 3
        if d == 0:
            break
        out.append(str(d - 1))
    return "".join(out)


def key_code(key: str) -> int:
    code = 0
    for i, ch in enumerate(key):
        code |= (int(ch) + 1) << (2 * (19 - i))
    return code


def dist_unique_id() -> bytes:
    """A new RCCL communicator id (evm_dist_unique_id); rank 0 makes it."""
    lib = _lib.load()
    buf = (C.c_uint8 * _lib.DIST_ID_BYTES)()
    check(lib.evm_dist_unique_id(buf), "evm_dist_unique_id")
    return bytes(buf)


class DistHub:
    """In-process rendezvous of `world` loopback ranks (evm_dist_hub): one
    Engine + Dist per rank, each driven by its own host thread."""

    def __init__(self, world: int):
        self.lib = _lib.load()
        self.world = world
        h = C.c_void_p()
        check(self.lib.evm_dist_hub_new(world, C.byref(h)), "evm_dist_hub_new")
        self.h = h

    def abort(self):
        """A rank failed: its peers' pending and later collectives return EVM_EDIST."""
        if getattr(self, "h", None):
            self.lib.evm_dist_hub_abort(self.h)

    def free(self):
        if getattr(self, "h", None):
            self.lib.evm_dist_hub_free(self.h)
            self.h = None


def run_loopback(world: int, fn, device: int = 0):
    """fn(rank, eng, dist) on `world` loopback ranks: one thread, Engine (on its
    own HIP stream) and Dist per rank over one DistHub on `device`.  Returns
    the ranks' results; raises if any rank raised (the others' collectives
    are aborted rather than left waiting)."""
    import threading

    hub = DistHub(world)
    results, errors = [None] * world, []

    def run(r):
        eng = dd = None
        try:
            torch.cuda.set_device(device)
            s = torch.cuda.Stream(device)
            with torch.cuda.stream(s):
                eng = Engine(device)
                dd = Dist(eng, None, r, world, hub=hub)
                dd.transport = "loopback hub (%d threads, 1 GPU)" % world
                results[r] = fn(r, eng, dd)
                torch.cuda.synchronize(device)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errors.append((r, e))
            hub.abort()
        finally:
            if dd is not None:
                dd.free()
            if eng is not None:
                eng.close()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    hub.free()
    if errors:
        r, e = sorted(errors, key=lambda x: x[0])[0]
        raise RuntimeError("loopback rank %d failed: %r" % (r, e)) from e
    return results


class Dist:
    """Owner sharding (evm_dist_*): one per Engine, collective calls in the
    same order on every rank.  Over RCCL (uid from dist_unique_id), or over a
    DistHub (loopback ranks in one process)."""

    def __init__(self, eng: Engine, uid: Optional[bytes], rank: int, world: int, hub: Optional[DistHub] = None):
        self.eng = eng
        self.rank, self.world = rank, world
        h = C.c_void_p()
        if hub is not None:
            if hub.world != world:
                raise ValueError("hub world %d != %d" % (hub.world, world))
            check(eng.lib.evm_dist_init_loopback(eng.h, hub.h, rank, C.byref(h)), "evm_dist_init_loopback")
        else:
            if len(uid) != _lib.DIST_ID_BYTES:
                raise ValueError("unique id must be %d bytes" % _lib.DIST_ID_BYTES)
            buf = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
            check(eng.lib.evm_dist_init(eng.h, buf, rank, world, C.byref(h)), "evm_dist_init")
        self.h = h
        self.transport = "loopback hub" if hub is not None else "RCCL"
        self.n_recv = 0
        self.stride = TS_STRIDE
        self.n_local = None  # owners this rank serves (after directory())
        self.n_dir = 0

    def free(self):
        if getattr(self, "h", None):
            self.eng.lib.evm_dist_free(self.eng.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def directory(self, ids: torch.Tensor):
        """Owner directory from userId strings (uint8 [n_owners, stride] device
        rows, every id id_len = stride bytes unless given as (rows, id_len)):
        owner g -> rank murmur3(userId_g) % world, dense local ids.  Returns
        (dest uint8[n], local int32[n]) on the device; sets self.n_local."""
        if isinstance(ids, tuple):
            ids, id_len = ids
        else:
            id_len = ids.shape[1]
        n, stride = ids.shape
        dest = torch.empty(max(n, 1), dtype=torch.uint8, device=ids.device)
        local = torch.empty(max(n, 1), dtype=torch.int32, device=ids.device)
        nl = C.c_uint32()
        check(self.eng.lib.evm_dist_directory(self.eng.h, self.h, _ptr(ids), stride, id_len, n, _ptr(dest),
                                              _ptr(local), C.byref(nl)), "evm_dist_directory")
        self.n_local = nl.value
        self.n_dir = n
        return dest[:n], local[:n]

    def route(self, ts: torch.Tensor, owner: torch.Tensor, aux: Optional[torch.Tensor] = None,
              dest: Optional[torch.Tensor] = None, need_src: bool = True, keep_input: bool = False) -> int:
        """Collective: rows to rank dest (default owner % world) -> rows received.
        need_src=False (every rank alike): take() will not return sources and no
        send_back / split_winners follows -- without aux the rows travel as
        24-B records (evm_dist_route_ex, EVM_ROUTE_NO_SRC).  keep_input=True
        (with need_src=False): `ts` stays valid and unchanged until the last
        take() / ingest() of this route, which read this rank's own rows there
        (EVM_ROUTE_KEEP_INPUT: the route neither parses nor copies them)."""
        n, stride = ts.shape
        nr = C.c_uint64()
        flags = 0 if need_src else _lib.ROUTE_NO_SRC
        if keep_input and not need_src:
            flags |= _lib.ROUTE_KEEP_INPUT
            self._kept = (ts, owner)  # (alive until the next route: take / ingest read them)
        check(self.eng.lib.evm_dist_route_ex(self.eng.h, self.h, _ptr(ts), stride, n, _ptr(owner), _ptr(aux),
                                             _ptr(dest), flags, C.byref(nr)), "evm_dist_route")
        self.n_recv = nr.value
        self.stride = stride
        return self.n_recv

    def take(self, group: int = 0, aux: bool = True, src: bool = True, out=None):
        """The last route's rows -> (ts, owner, aux or None, src or None, group_off or None);
        out: optional preallocated (ts, owner, aux, src) tensors with >= n_recv rows."""
        n = self.n_recv
        dev = torch.device("cuda", self.eng.device)
        if out is None:
            out = (torch.empty((max(n, 1), self.stride), dtype=torch.uint8, device=dev),
                   torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                   torch.empty(max(n, 1), dtype=torch.int32, device=dev) if aux else None,
                   torch.empty(max(n, 1), dtype=torch.int64, device=dev) if src else None)
        ts, ow, ax, sr = out
        cap = ts.shape[0]
        goff = (C.c_uint64 * (group + 1))() if group else None
        check(self.eng.lib.evm_dist_take(self.eng.h, self.h, group, _ptr(ts), ts.shape[1], _ptr(ow), _ptr(ax), _ptr(sr),
                                         cap, goff), "evm_dist_take")
        g = [int(x) for x in goff] if group else None
        return ts[:n], ow[:n], (ax[:n] if ax is not None else None), (sr[:n] if sr is not None else None), g

    def ingest(self, store: "Store", id_base: int = 0, flags: Optional[torch.Tensor] = None) -> torch.Tensor:
        """addMessages of the last route's rows into `store` (evm_dist_ingest:
        the packed records read where they arrived; row i of the receive
        order has id id_base + i) -> flags uint8[n_recv]."""
        n = self.n_recv
        if flags is None:
            flags = torch.empty(max(n, 1), dtype=torch.uint8, device=torch.device("cuda", self.eng.device))
        if flags.numel() < n:
            raise ValueError("flags holds %d < %d rows" % (flags.numel(), n))
        check(self.eng.lib.evm_dist_ingest(self.eng.h, self.h, store.h, id_base, _ptr(flags)), "evm_dist_ingest")
        return flags[:n]

    def gather_roots(self, trees, n_owners_global: int):
        """Collective: every global owner's (root int32, present bool) on the device.
        trees: one Trees (its owners = this rank's local owners) or a list of them."""
        dev = torch.device("cuda", self.eng.device)
        ts = list(trees) if isinstance(trees, (list, tuple)) else [trees]
        arr = (C.c_void_p * max(len(ts), 1))(*[t.h.value if isinstance(t.h, C.c_void_p) else t.h for t in ts])
        root = torch.empty(max(n_owners_global, 1), dtype=torch.int32, device=dev)
        present = torch.empty(max(n_owners_global, 1), dtype=torch.uint8, device=dev)
        check(self.eng.lib.evm_dist_gather_roots(self.eng.h, self.h, arr, len(ts), n_owners_global, _ptr(root),
                                                 _ptr(present)), "evm_dist_gather_roots")
        return root[:n_owners_global], present[:n_owners_global].bool()

    # ------------------------------------------------ hot-owner / cell split
    def hot_owners(self, owner: torch.Tensor, n_owners_global: int, share: float = 0.25, cap: int = 4096) -> np.ndarray:
        """Collective: global owners holding more than `share` of one rank's
        fair share of all rows (evm_dist_hot_owners) -> sorted uint32 array."""
        buf = np.zeros(max(cap, 1), dtype=np.uint32)
        nh = C.c_uint32()
        check(self.eng.lib.evm_dist_hot_owners(self.eng.h, self.h, _ptr(owner), owner.numel(), n_owners_global,
                                               share, buf.ctypes.data_as(C.c_void_p), cap, C.byref(nh)),
              "evm_dist_hot_owners")
        return buf[: nh.value].copy()

    def split(self, hot, n_owners_global: int) -> int:
        """Split the listed global owners over every rank (evm_dist_split);
        returns hot_base (hot owner h is local owner hot_base + h)."""
        hot = np.ascontiguousarray(np.asarray(hot, dtype=np.uint32))
        base = C.c_uint32()
        check(self.eng.lib.evm_dist_split(self.eng.h, self.h, hot.ctypes.data_as(C.c_void_p), hot.size,
                                          n_owners_global, C.byref(base)), "evm_dist_split")
        self.hot = hot
        self.n_hot = int(hot.size)
        self.hot_base = base.value
        return self.hot_base

    def merge_trees(self, trees: "Trees", owner_lo: int, count: int) -> "Trees":
        """Collective: the XOR merge over ranks of owners [owner_lo, +count) of
        every rank's trees (evm_dist_merge_trees) -- the same on every rank."""
        h = C.c_void_p()
        check(self.eng.lib.evm_dist_merge_trees(self.eng.h, self.h, trees.h, owner_lo, count, C.byref(h)),
              "evm_dist_merge_trees")
        return Trees(self.eng, h)

    def merge_select(self, off: torch.Tensor, ids: torch.Tensor, keys: torch.Tensor, cap: Optional[int] = None):
        """Collective: per-group selections split over ranks (off: n_groups+1
        bounds, may start past 0) -> (off int64[n_groups+1], ids int64[m]) in
        timestamp order, the same on every rank (evm_dist_merge_select)."""
        dev = off.device
        ng = off.numel() - 1
        out_off = torch.empty(ng + 1, dtype=torch.int64, device=dev)
        nout = C.c_uint64()
        if cap is None:  # size first (the same total on every rank: both calls stay collective)
            st = self.eng.lib.evm_dist_merge_select(self.eng.h, self.h, ng, _ptr(off), _ptr(ids), _ptr(keys),
                                                    _ptr(out_off), None, 0, C.byref(nout))
            if st not in (_lib.EVM_OK, _lib.EVM_ECAPACITY):
                check(st, "evm_dist_merge_select")
            if st == _lib.EVM_OK:
                return out_off, torch.empty(0, dtype=torch.int64, device=dev)
            cap = nout.value
        out_id = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        check(self.eng.lib.evm_dist_merge_select(self.eng.h, self.h, ng, _ptr(off), _ptr(ids), _ptr(keys),
                                                 _ptr(out_off), _ptr(out_id), cap, C.byref(nout)),
              "evm_dist_merge_select")
        return out_off, out_id[: nout.value]

    def ts_dest(self, ts: torch.Tensor) -> torch.Tensor:
        """Rank of every row by timestamp hash (evm_dist_ts_dest)."""
        n, stride = ts.shape
        dest = torch.empty(max(n, 1), dtype=torch.uint8, device=ts.device)
        check(self.eng.lib.evm_dist_ts_dest(self.eng.h, self.h, _ptr(ts), stride, n, _ptr(dest)), "evm_dist_ts_dest")
        return dest[:n]

    def cell_dest(self, cell: torch.Tensor) -> torch.Tensor:
        """Rank of every row's cell (evm_dist_cell_dest)."""
        n = cell.numel()
        dest = torch.empty(max(n, 1), dtype=torch.uint8, device=cell.device)
        check(self.eng.lib.evm_dist_cell_dest(self.eng.h, self.h, _ptr(cell), n, _ptr(dest)), "evm_dist_cell_dest")
        return dest[:n]

    def send_back(self, val: torch.Tensor, n_out: int) -> torch.Tensor:
        """Collective: per received row values (receive order) back to their
        source positions (evm_dist_return) -> tensor [n_out] of val's dtype."""
        val = val.contiguous()
        elem = val.element_size()
        out = torch.zeros(max(n_out, 1), dtype=val.dtype, device=val.device)
        check(self.eng.lib.evm_dist_return(self.eng.h, self.h, _ptr(val), elem, _ptr(out), n_out), "evm_dist_return")
        return out[:n_out]

    def split_winners(self, win: torch.Tensor, n_cells: int) -> torch.Tensor:
        """Collective: winners (index into the last route's receive order or -1)
        -> global batch indexes int64[n_cells] (evm_dist_split_winners)."""
        out = torch.empty(max(n_cells, 1), dtype=torch.int64, device=win.device)
        w = win.to(torch.int32).contiguous()  # (kept alive across the call)
        check(self.eng.lib.evm_dist_split_winners(self.eng.h, self.h, _ptr(w), n_cells, _ptr(out)),
              "evm_dist_split_winners")
        return out[:n_cells]

    def agree_status(self, local: int) -> int:
        """Collective: the largest status over the ranks."""
        m = C.c_int32()
        check(self.eng.lib.evm_dist_agree_status(self.eng.h, self.h, int(local), C.byref(m)), "evm_dist_agree_status")
        return m.value
