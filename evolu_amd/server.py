"""The sync server's request path over a device store: SyncRequest bodies in,
SyncResponse bodies out (apps/server/src/index.ts:204-251).

Per request the reference runs parseBody (:108-116, SyncRequest.fromBinary),
getMerkleTree (:118-134), addMessages (:136-171), getMessages (:173-202) and
answers SyncResponse.toBinary({merkleTree: merkleTreeToString(tree),
messages}) (:233-241); any throw answers 500 and rolls back THAT request
(:147-169, :224-233).  Here a list of bodies is one call: the bodies are
decoded on the host (evm_pb_*), the requests are cut into rounds in which
every owner (userId) appears at most once -- a later request of the same
owner must see the earlier one's inserts and must not see its own later
ones, exactly the reference's one-request-at-a-time order -- and each round
is one evm_server_ingest_ex + one evm_server_select over all its owners.

Per-request failure, as the reference: evm_server_ingest_ex commits every
owner but the ones with a timestamp outside the engine's canonical domain.
Those requests go through the host's restatement of timestampFromString
(evolu_amd/lenient.py, pinned by node): an invalid date fails the request
(RangeError -> the reference's 500; nothing of it is stored), a lenient but
valid one (V8 rolls "02-30" into March, a lower-case counter parses) is
re-ingested in the same round in the form the reference's tree sees
(timestampToString(timestampFromString(raw))) while the response keeps the raw
string, which is what the reference stores.  Rows stored under a lenient
spelling are tracked per user, so getMessages still orders and bounds them
by their raw strings.

The common case runs as whole-call arrays (`_sync_fast`): every body
decoded on host threads in one call (evm_pb_scan_batch / split_batch), each
round's requests ingested together, their client trees parsed on host
threads in one call (evm_tree_from_json), one selection, every touched
owner's tree JSON emitted on the device in one launch
(evm_tree_to_json_batch) and every response encoded on host threads in one
call (evm_pb_encode_responses).  Requests of users with rows stored under a
lenient spelling, and requests whose owner the ingest rejected, take the
per-request path below (`_round`) -- the same results either way.

Results per body: the SyncResponse bytes, an exception object standing for
the reference's 500 answer (ParseBodyError, RangeError), or None where the
engine does not model the request (a nodeId that is not 16 hex chars, a
timestamp shape timestampFromString would read in a way lenient.py does not
restate, one timestamp stored under two spellings).  The user is then handed
to the caller for good: every later request of that user also answers None,
so the caller runs them, in order, on the reference path.  None always means
unapplied.  A spelling conflict found only after `evm_server_ingest_ex`
committed the request (pass 1, or the canonical re-ingest) answers
`HandedOver(applied=True)` instead: its rows are in this server's store and
tree, the user is handed over all the same, and the caller must serve that
user from its own reference state from then on and treat this server's rows
and tree of that user as stale.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Sequence, Set, Union

import numpy as np

from . import _lib
from ._lib import check
from . import lenient as LN
from . import wire
from .engine import TS_LEN, Engine

class HandedOver:
    """A request whose user was handed to the caller after this server had
    already committed it (applied=True): unlike None, its rows are in the store."""

    def __init__(self, applied: bool):
        self.applied = applied

    def __repr__(self):
        return "HandedOver(applied=%r)" % self.applied


Result = Union[bytes, Exception, HandedOver, None]
REQUEST_KIND = _lib.PB_SYNC_REQUEST
_EMPTY = C.create_string_buffer(b"{}")  # the client tree of an owner not in the round
_EMPTY_PTR = C.addressof(_EMPTY)


def _np_ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)
_HEX = set(b"0123456789abcdefABCDEF")


class _Seg:
    """A message-log segment (SyncServer._log): the timestamp rows (N, 48),
    content offsets (N + 1), contents and an optional row map, held where the
    call that logged them had them (numpy arrays: the host path; device
    tensors: sync_device) and copied to the other side on first use there."""

    def __init__(self, ts, coff, content, rowmap=None):
        self.h = self.d = None
        if isinstance(ts, np.ndarray):
            self.h = (ts, np.ascontiguousarray(coff, dtype=np.uint64), content,
                      None if rowmap is None else np.ascontiguousarray(rowmap, dtype=np.uint64))
        else:
            self.d = (ts, coff, content, rowmap)

    def host(self):
        if self.h is None:
            ts, coff, content, rowmap = self.d
            self.h = (ts.cpu().numpy(), coff.cpu().numpy().view(np.uint64), content.cpu().numpy(),
                      None if rowmap is None else rowmap.cpu().numpy().view(np.uint64))
        return self.h

    def dev(self, device):
        if self.d is None:
            import torch

            ts, coff, content, rowmap = self.h
            up = lambda a: torch.from_numpy(a if a.flags.c_contiguous and a.flags.writeable else a.copy()).to(device)  # noqa: E731
            self.d = (up(ts), up(coff.view(np.int64)), up(content), None if rowmap is None else up(rowmap.view(np.int64)))
        return self.d


def _decode_spans(pk: np.ndarray, off: np.ndarray, ln: np.ndarray) -> List[str]:
    """The byte spans pk[off[k] .. off[k + 1]) as str (UTF-8, errors replaced),
    as the host path decodes userIds; equal-length spans without NUL bytes in
    one numpy call."""
    n = len(off) - 1
    if n and (ln == ln[0]).all() and int(ln[0]) > 0 and (pk < 0x80).all():  # (ASCII: bytes = chars)
        L = int(ln[0])
        big = pk.tobytes().decode("ascii")
        return [big[i:i + L] for i in range(0, n * L, L)]
    b = pk.tobytes()
    o = off.astype(np.int64)
    return [b[o[k]:o[k + 1]].decode("utf-8", "replace") for k in range(n)]


class DeviceResponses:
    """sync_device's answer: result[i] is True where response i is the bytes
    buf[off[i] .. off[i + 1]) of the device buffer `buf`, else what sync()
    would return for it (bytes from the host path, an exception object, a
    HandedOver, or None)."""

    def __init__(self, buf, off: np.ndarray, result: List):
        self.buf, self.off, self.result = buf, off, result

    def __len__(self):
        return len(self.result)

    def to_host(self) -> List[Result]:
        """Every result as sync() returns it (the device bytes copied back)."""
        hb = self.buf.cpu().numpy() if self.buf is not None else None
        return [hb[int(self.off[i]):int(self.off[i + 1])].tobytes() if r is True else r
                for i, r in enumerate(self.result)]


class ParseBodyError(Exception):
    """index.ts:108-116: SyncRequest.fromBinary threw."""


class RangeError(Exception):
    """A JS RangeError -> 500: diffMerkleTrees' keyToTimestamp (merkleTree.ts:55-61)
    or addMessages' toISOString of an invalid date (timestamp.ts:45)."""


class SyncServer:
    """One device store for up to ``capacity`` users (owner slots)."""

    def __init__(self, eng: Engine, capacity: int):
        self.eng = eng
        self.store = eng.store_new(capacity)
        self.capacity = capacity
        self._slot_d: Dict[str, int] = {}
        # the device rounds' userIds (sync_device): equal-length ASCII ids as
        # 24-B keys by slot on the device, their 64-bit hashes sorted for the
        # lookups; slots >= _host_upto are not in the host dict yet (`slot`
        # adds them when a host path asks).  None: the device keys do not
        # cover every slot -- the rounds map userIds through the host dict.
        self._dkeys = None
        self._dlen = 0
        self._dhash = None
        self._dslot = None
        self._host_upto = 0
        self.next_id = 0
        # the message log, by id: segments of ids [base, base + n) -- the
        # timestamp rows (N, 48), content offsets (N + 1) and contents of a
        # decode, and a row map (id - base -> row) when a segment covers part
        # of them (None: row = id - base)
        self._base: List[int] = []
        self._segs: List[tuple] = []
        self.timing: Dict[str, float] = {}  # seconds of the last sync() by part (host / device)
        self._raw: Dict[int, str] = {}      # message id -> the raw timestamp, for rows stored under a lenient spelling
        # user -> canonical timestamp -> (raw spelling, message id) of rows stored under a lenient spelling
        self.lenient: Dict[str, Dict[str, tuple]] = {}
        self.detached: Set[str] = set()    # users whose requests the caller runs (see the module docstring)

    def close(self):
        self.store.free()

    @property
    def slot(self) -> Dict[str, int]:
        """userId -> owner slot (every user seen so far)."""
        if self._dkeys is not None and self._host_upto < self._dkeys.shape[0]:
            S, L = self._dkeys.shape[0], self._dlen
            b = self._dkeys[self._host_upto:, :L].cpu().numpy()
            big = b.tobytes().decode("ascii")
            self._slot_d.update(zip((big[i:i + L] for i in range(0, len(big), L)), range(self._host_upto, S)))
            self._host_upto = S
        return self._slot_d

    @slot.setter
    def slot(self, d: Dict[str, int]):
        self._slot_d = d
        self._dkeys = self._dhash = self._dslot = None
        self._host_upto = len(d)

    def _slot(self, user: str) -> int:
        d = self.slot
        s = d.get(user)
        if s is None:
            if len(d) >= self.capacity:
                raise _lib.EngineError(_lib.EVM_ECAPACITY, "SyncServer: more users than owner slots")
            s = d[user] = len(d)
            self._dkeys = self._dhash = self._dslot = None  # (a slot the device keys do not hold)
            self._host_upto = len(d)
        return s

    def _device_slots(self, packed, ulen: np.ndarray, n: int):
        """The slots of a device round's users from the device keys: packed
        (device uint8) holds the n userIds back to back.  -> int64 numpy
        slots, or None when the host dict must decide (ids of several lengths,
        longer than 24 bytes or not ASCII; a user twice; a hash shared by two
        keys; the device keys not covering every slot)."""
        import torch

        L = int(ulen[0]) if n else 0
        if not n or not 0 < L <= 24 or not (ulen == L).all():
            return None
        fresh = not self._slot_d and self._dkeys is None
        if not fresh and (self._dkeys is None or self._dlen != L):
            return None
        dev = packed.device
        k = packed[:n * L].view(n, L)
        if bool((k >= 0x80).any()):
            return None
        keys = torch.zeros((n, 24), dtype=torch.uint8, device=dev)
        keys[:, :L] = k
        w = keys.view(torch.int64)  # (n, 3)
        h = (w[:, 0] * -7046029254386353131) ^ (w[:, 1] * -4658895280553007687) ^ (w[:, 2] * 7640891576956012809)
        if torch.unique(h).numel() != n:
            return None  # (a user twice, or two of them sharing a hash: the host dict decides)
        S = 0 if fresh else self._dkeys.shape[0]
        if fresh:
            found = torch.zeros(n, dtype=torch.bool, device=dev)
            old = torch.zeros(n, dtype=torch.int64, device=dev)
        else:
            i = torch.searchsorted(self._dhash, h).clamp_(max=max(S - 1, 0))
            hit = self._dhash[i] == h
            old = self._dslot[i]
            found = hit & (self._dkeys[old] == keys).all(1)
            if bool((hit & ~found).any()):
                return None  # (a hash shared by two keys)
        new = ~found
        n_new = int(new.sum())
        if S + n_new > self.capacity:
            raise _lib.EngineError(_lib.EVM_ECAPACITY, "SyncServer: more users than owner slots")
        rank = torch.cumsum(new.to(torch.int64), 0) - 1 + S  # (new users: slots in request order)
        slots = torch.where(found, old, rank)
        if n_new:
            nk = keys[new]
            self._dkeys = nk if fresh else torch.cat([self._dkeys, nk])
            hh = h[new] if fresh else torch.cat([self._dhash, h[new]])
            ss = slots[new] if fresh else torch.cat([self._dslot, slots[new]])
            order = torch.argsort(hh)
            self._dhash, self._dslot, self._dlen = hh[order], ss[order], L
        return slots.cpu().numpy()

    def _log(self, base: int, ts, coff, content, rowmap=None):
        self._base.append(base)
        self._segs.append(_Seg(ts, coff, content, rowmap))

    def _message(self, mid: int):
        r = int(np.searchsorted(np.asarray(self._base), mid, side="right")) - 1
        ts_a, o, content, rowmap = self._segs[r].host()
        k = mid - self._base[r]
        if rowmap is not None:
            k = int(rowmap[k])
        ts = self._raw.get(mid)
        if ts is None:
            ts = bytes(ts_a[k, :TS_LEN]).decode("latin-1")
        return ts, content[int(o[k]):int(o[k + 1])].tobytes()

    def sync(self, bodies: Sequence[bytes]) -> List[Result]:
        n = len(bodies)
        boff = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.fromiter((len(b) for b in bodies), dtype=np.uint64, count=n), out=boff[1:])
        return self._sync_fast(np.frombuffer(b"".join(bodies) or b"\0", dtype=np.uint8), boff)

    def sync_arena(self, arena: np.ndarray, off: np.ndarray, views: bool = True) -> List[Result]:
        """sync() of the bodies arena[off[k] .. off[k + 1]) (uint8 / uint64 arrays);
        views=True: the responses are memoryviews into one response arena
        (no per-response copy), equal to the bytes sync() would return."""
        return self._sync_fast(np.ascontiguousarray(arena, dtype=np.uint8),
                               np.ascontiguousarray(off, dtype=np.uint64), views)

    def sync_per_request(self, bodies: Sequence[bytes]) -> List[Result]:
        """The same, every request through the per-request path (A/B, tests)."""
        out: List[Result] = [None] * len(bodies)
        reqs = []
        for i, b in enumerate(bodies):
            try:
                d = wire.decode(wire.REQUEST, b)
            except _lib.EngineError as e:
                out[i] = ParseBodyError(str(e))
                continue
            reqs.append((i, d))
        # rounds: the k-th request of an owner goes to round k
        seen: Dict[str, int] = {}
        rounds: List[list] = []
        for i, d in reqs:
            k = seen.get(d.user, 0)
            seen[d.user] = k + 1
            if k == len(rounds):
                rounds.append([])
            rounds[k].append((i, d))
        for rnd in rounds:
            self._round(rnd, out)
        return out

    # ---------------------------------------------------------- device path
    def sync_device(self, arena, off) -> "DeviceResponses":
        """sync() of bodies resident in device memory: arena (uint8 tensor on
        the engine's GPU), off (host uint64 [n + 1]).  The round runs on the
        device end to end -- bodies decoded where they lie (evm_pb_scan_index_dev /
        split_index_dev), one evm_server_ingest_ex, the client trees parsed there
        (evm_tree_from_json_dev), one selection, the responses built in device
        memory (evm_pb_encode_responses_dev, each tree's JSON emitted straight
        into its response) -- and answers a DeviceResponses.  Only the round's
        bookkeeping comes to the host: per body its sizes, userId and nodeId.

        The same results as sync() on the same bodies: a call the device path
        does not model as a whole -- an unparsable body, a timestamp that is
        not 46 bytes, a nodeId that is not 16 hex chars, a userId twice, users
        with rows under lenient spellings or handed over -- runs sync() on a
        host copy of the bodies; requests whose owner the ingest rejects, or
        whose merkleTree the device does not read (EVM_ETREE, or keys out of
        order), take the per-request path as in sync()."""
        import time

        import torch

        lib, eng = _lib.load(), self.eng
        T = self.timing = dict.fromkeys(("decode", "ingest", "trees", "select", "encode", "per_request"), 0.0)
        t_call = time.perf_counter()
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        dev = arena.device
        P = lambda x: C.c_void_p(x.data_ptr())  # noqa: E731
        if n == 0:
            return DeviceResponses(None, np.zeros(1, dtype=np.uint64), [])
        t0 = time.perf_counter()
        off_d = torch.from_numpy(off.view(np.int64)).to(dev)
        info_d = torch.empty((n, 9), dtype=torch.int64, device=dev)
        st_d = torch.empty(n, dtype=torch.int32, device=dev)
        slots_d = torch.empty(int(off[-1]) // 50 + 1, dtype=torch.int64, device=dev)  # (each message's place: the split reads it)
        check(lib.evm_pb_scan_index_dev(eng.h, REQUEST_KIND, P(arena), P(off_d), n, P(info_d), P(st_d), P(slots_d)),
              "evm_pb_scan_index_dev")
        inf = info_d.cpu().numpy().view(np.uint64)
        st = st_d.cpu().numpy()
        if st.any() or inf[:, 8].any() or (inf[:, 5] != 16).any() or self.detached or self.lenient:
            return self._device_fallback(arena, off, T, t_call)
        # the userIds and nodeIds, packed, to the host
        ulen = inf[:, 3]
        lens = np.concatenate([ulen, np.full(n, 16, dtype=np.uint64)])
        src = np.concatenate([off[:-1] + inf[:, 2], off[:-1] + inf[:, 4]])
        dst = np.zeros(2 * n + 1, dtype=np.uint64)
        np.cumsum(lens, out=dst[1:])
        packed = torch.empty(max(int(dst[-1]), 1), dtype=torch.uint8, device=dev)
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)  # noqa: E731
        src_d, len_d, dst_d = up(src), up(lens), up(dst[:-1])
        check(lib.evm_gather_spans_dev(eng.h, P(arena), P(src_d), P(len_d), P(dst_d), 2 * n, P(packed)),
              "evm_gather_spans_dev")
        ub = int(dst[n])
        nodes_d = packed[ub:ub + 16 * n].view(n, 16)
        hexd = torch.zeros(256, dtype=torch.bool, device=dev)
        hexd[torch.frombuffer(bytearray(b"0123456789abcdefABCDEF"), dtype=torch.uint8).to(dev).long()] = True
        if not bool(hexd[nodes_d.long()].all()):
            return self._device_fallback(arena, off, T, t_call)
        t1 = time.perf_counter()
        slots = self._device_slots(packed, ulen, n)
        if slots is not None:
            pass  # (the device keys: no userId decoded on the host)
        elif not self.slot and n <= self.capacity:
            users = _decode_spans(packed[:ub].cpu().numpy(), dst[:n + 1], ulen)
            # a new server's first round: every user new, slots in request order
            self.slot = dict(zip(users, range(n)))
            if len(self.slot) != n:
                self.slot = {}
                return self._device_fallback(arena, off, T, t_call)  # (an owner twice: rounds)
            slots = np.arange(n, dtype=np.int64)
        else:
            users = _decode_spans(packed[:ub].cpu().numpy(), dst[:n + 1], ulen)
            get = self.slot.get
            new = [u for u in users if get(u) is None]  # (new users take slots in request order)
            if new:
                new = list(dict.fromkeys(new))
                if len(self.slot) + len(new) > self.capacity:
                    raise _lib.EngineError(_lib.EVM_ECAPACITY, "SyncServer: more users than owner slots")
                self.slot.update(zip(new, range(len(self.slot), len(self.slot) + len(new))))
                self.slot = self._slot_d  # (slots the device keys do not hold)
            slots = np.fromiter(map(get, users), dtype=np.int64, count=n)
            if np.unique(slots).size != n:
                return self._device_fallback(arena, off, T, t_call)  # (an owner twice: rounds)
        T["users"] = time.perf_counter() - t1
        nmsg, cbytes = inf[:, 0], inf[:, 1]
        msg_base = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(nmsg, out=msg_base[1:])
        con_base = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(cbytes, out=con_base[1:])
        N, CB = int(msg_base[n]), int(con_base[n])
        ts = torch.empty((max(N, 1), 48), dtype=torch.uint8, device=dev)  # (every row written by the split)
        coff = torch.empty(N + 1, dtype=torch.int64, device=dev)
        coff[N] = CB
        content = torch.empty(max(CB, 1), dtype=torch.uint8, device=dev)
        owner = torch.empty(max(N, 1), dtype=torch.int32, device=dev)
        slot_d = torch.from_numpy(slots.astype(np.int32)).to(dev)
        mb_d, cb_d = up(msg_base), up(con_base)  # (held: the kernels read them after P() returns)
        check(lib.evm_pb_split_index_dev(eng.h, REQUEST_KIND, P(arena), P(off_d), n, P(st_d), P(mb_d), P(cb_d),
                                         P(slot_d), P(ts), 48, P(coff), P(content), P(owner), P(slots_d)),
              "evm_pb_split_index_dev")
        del slots_d
        T["decode"] += time.perf_counter() - t0
        t0 = time.perf_counter()
        bad = np.zeros(n, dtype=bool)
        if N:
            _, ost, _ = self.store.ingest_ex(ts[:N], owner[:N], self.next_id)
            bad = ost.cpu().numpy()[slots] != 0
            self._log(self.next_id, ts[:N], coff, content)
            self.next_id += N
        T["ingest"] += time.perf_counter() - t0
        # the client trees (owners without a request this round: the empty tree)
        t0 = time.perf_counter()
        O = self.capacity
        at = np.zeros(O, dtype=np.uint64)
        ln = np.zeros(O, dtype=np.uint64)
        ok = ~bad
        at[slots[ok]] = off[:-1][ok] + inf[ok, 6]
        ln[slots[ok]] = inf[ok, 7]
        tst_d = torch.empty(max(O, 1), dtype=torch.int32, device=dev)
        h = C.c_void_p()
        at_d, ln_d = up(at), up(ln)
        check(lib.evm_tree_from_json_dev(eng.h, O, P(arena), P(at_d), P(ln_d), P(tst_d), C.byref(h)),
              "evm_tree_from_json_dev")
        from .engine import Trees

        client = Trees(eng, h)
        tbad = tst_d.cpu().numpy()[slots] != 0
        T["trees"] += time.perf_counter() - t0
        result: List = [None] * n
        late = np.flatnonzero(bad | (tbad & ok))  # the per-request path's requests
        ans = np.flatnonzero(ok & ~tbad)
        buf, roff = None, np.zeros(n + 1, dtype=np.uint64)
        if len(ans):
            t0 = time.perf_counter()
            sl = slots[ans]
            sl_d = torch.from_numpy(sl).to(dev)
            node = torch.full((O, 16), ord("0"), dtype=torch.uint8, device=dev)
            node[sl_d] = nodes_d[torch.from_numpy(ans).to(dev)]
            active = torch.zeros(O, dtype=torch.uint8, device=dev)
            active[sl_d] = 1
            diff, soff, sid = self.store.select(client, node, active)
            client.free()
            rng_err_d = (diff[sl_d] == _lib.DIFF_RANGE_ERROR).to(torch.uint8)
            T["select"] += time.perf_counter() - t0
            t0 = time.perf_counter()
            segs = [g.dev(dev) for g in self._segs]
            VP = C.c_void_p * max(len(segs), 1)
            seg_base = np.asarray(self._base, dtype=np.uint64)
            seg_row = VP(*[None if r is None else r.data_ptr() for _, _, _, r in segs])
            seg_ts = VP(*[t.data_ptr() for t, _, _, _ in segs])
            seg_coff = VP(*[o.data_ptr() for _, o, _, _ in segs])
            seg_con = VP(*[c.data_ptr() for _, _, c, _ in segs])
            owners_d = sl_d.to(torch.int32)
            rout = torch.empty(len(sl) + 1, dtype=torch.int64, device=dev)
            tot = C.c_uint64()
            tree = self.store.tree()
            args = [eng.h, len(sl), tree.h, P(owners_d), P(soff), P(sid), P(rng_err_d), len(segs), _np_ptr(seg_base),
                    seg_row, seg_ts, 48, seg_coff, seg_con]
            check(lib.evm_pb_encode_responses_dev(*args, None, 0, P(rout), C.byref(tot)), "evm_pb_encode_responses_dev")
            buf = torch.empty(max(tot.value, 1), dtype=torch.uint8, device=dev)
            check(lib.evm_pb_encode_responses_dev(*args, P(buf), tot.value, P(rout), C.byref(tot)),
                  "evm_pb_encode_responses_dev")
            ro = rout.cpu().numpy().view(np.uint64)
            rng_err = rng_err_d.cpu().numpy().astype(bool)
            # (the responses lie in buf in request order: per-request lengths -> offsets)
            rlen = np.zeros(n, dtype=np.uint64)
            rlen[ans] = np.diff(ro)
            np.cumsum(rlen, out=roff[1:])
            res = np.empty(n, dtype=object)
            res[ans] = True
            for i in ans[rng_err].tolist():
                res[i] = RangeError("Invalid count value")
            result = res.tolist()
            T["encode"] += time.perf_counter() - t0
        else:
            client.free()
        if len(late):
            # an owner the ingest rejected: the per-request path's round (nothing of
            # it was stored); a tree the device did not read: that request's select
            t0 = time.perf_counter()
            out: List[Result] = [None] * n
            hb = {int(i): arena[int(off[i]):int(off[i + 1])].cpu().numpy().tobytes() for i in late}
            rnd = [(int(i), wire.decode(wire.REQUEST, hb[int(i)])) for i in late if bad[i]]
            if rnd:
                self._round(rnd, out)
            sel_only = [(int(i), wire.decode(wire.REQUEST, hb[int(i)]), int(slots[i])) for i in late if not bad[i]]
            if sel_only:
                self._select(sel_only, out)
            for i in late:
                result[int(i)] = out[int(i)]
            T["per_request"] += time.perf_counter() - t0
        T["other"] = time.perf_counter() - t_call - sum(v for k, v in T.items() if k != "users")  # (users: part of decode)
        return DeviceResponses(buf, roff, result)

    def _device_fallback(self, arena, off, T, t_call):
        """sync_device's whole-call fallback: sync() on a host copy of the bodies."""
        import time

        t0 = time.perf_counter()
        host = arena.cpu().numpy()
        res = self._sync_fast(host, off)
        self.timing = dict(self.timing, device_fallback=time.perf_counter() - t0)
        return DeviceResponses(None, np.zeros(len(off), dtype=np.uint64), res)

    # ------------------------------------------------------------ fast path
    def _sync_fast(self, arena: np.ndarray, boff: np.ndarray, views: bool = False) -> List[Result]:
        """sync() over whole-call arrays (module docstring); timings by part in self.timing."""
        import time

        import torch

        lib, eng = _lib.load(), self.eng
        T = self.timing = dict.fromkeys(("decode", "ingest", "trees", "select", "json", "encode", "per_request"), 0.0)
        t_call = time.perf_counter()
        n = len(boff) - 1
        out: List[Result] = [None] * n
        if n == 0:
            return out
        t0 = time.perf_counter()
        info = (wire._Sync * n)()
        st = np.zeros(n, dtype=np.int32)
        check(lib.evm_pb_scan_batch(REQUEST_KIND, _np_ptr(arena), _np_ptr(boff), n, info, _np_ptr(st)),
              "evm_pb_scan_batch")
        inf = np.ctypeslib.as_array(info).view(np.uint64).reshape(n, 9).copy()
        ok = st == 0
        inf[~ok] = 0
        nmsg, cbytes = inf[:, 0], inf[:, 1]
        msg_base = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(nmsg, out=msg_base[1:])
        con_base = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(cbytes, out=con_base[1:])
        N, CB = int(msg_base[n]), int(con_base[n])
        ts = np.zeros((max(N, 1), 48), dtype=np.uint8)
        ts_len = np.zeros(max(N, 1), dtype=np.uint32)
        ts_off = np.zeros(max(N, 1), dtype=np.uint64)
        coff = np.zeros(N + 1, dtype=np.uint64)
        content = np.zeros(max(CB, 1), dtype=np.uint8)
        check(lib.evm_pb_split_batch(REQUEST_KIND, _np_ptr(arena), _np_ptr(boff), n, _np_ptr(st), _np_ptr(msg_base),
                                     _np_ptr(con_base), _np_ptr(ts), 48, _np_ptr(ts_len), _np_ptr(ts_off),
                                     _np_ptr(coff), _np_ptr(content)), "evm_pb_split_batch")
        for i in np.flatnonzero(~ok):
            out[i] = ParseBodyError(_lib.load().evm_strerror(int(st[i])).decode())
        span = lambda i, f: arena[int(boff[i] + inf[i, f]):int(boff[i] + inf[i, f] + inf[i, f + 1])]  # noqa: E731
        users = [span(i, 2).tobytes().decode("utf-8", "replace") if ok[i] else None for i in range(n)]
        # nodeId usable by NOT LIKE '%' || nodeId: 16 hex chars (else the user is handed over)
        node_ok = np.zeros(n, dtype=bool)
        nodes16 = np.full((n, 16), ord("0"), dtype=np.uint8)
        has16 = ok & (inf[:, 5] == 16)
        if has16.any():
            k16 = np.flatnonzero(has16)
            nodes16[k16] = arena[(boff[k16] + inf[k16, 4])[:, None].astype(np.int64) + np.arange(16)]
            hexok = np.isin(nodes16[k16], np.frombuffer(b"0123456789abcdefABCDEF", dtype=np.uint8)).all(1)
            node_ok[k16[hexok]] = True
        rnd_of = np.full(n, -1, dtype=np.int64)
        seen: Dict[str, int] = {}
        for i in np.flatnonzero(ok):
            k = seen.get(users[i], 0)
            seen[users[i]] = k + 1
            rnd_of[i] = k
        T["decode"] += time.perf_counter() - t0
        log = (ts, coff, content)
        ts_dev = None
        for k in range(int(rnd_of.max()) + 1 if n else 0):
            idx = np.flatnonzero(rnd_of == k)
            fast, slow = [], []
            if not self.detached and not self.lenient:  # (the common case, without a loop)
                for i in idx[~node_ok[idx]]:
                    self.detached.add(users[i])  # NOT LIKE '%' || nodeId with any nodeId is not modelled
                fast = idx[node_ok[idx]].tolist()
            else:
                for i in idx.tolist():
                    u = users[i]
                    if u in self.detached:
                        continue  # out[i] stays None
                    if not node_ok[i]:
                        self.detached.add(u)
                        continue
                    (slow if u in self.lenient else fast).append(i)
            rejected = []
            if fast:
                t0 = time.perf_counter()
                if ts_dev is None:
                    ts_dev = eng.dev(ts)
                F = np.asarray(fast, dtype=np.int64)
                slots = np.fromiter((self._slot(users[i]) for i in F), dtype=np.int64, count=len(F))
                cnt = nmsg[F].astype(np.int64)
                tot = int(cnt.sum())
                first = np.cumsum(cnt) - cnt
                rows = (np.repeat(msg_base[F].astype(np.int64) - first, cnt) + np.arange(tot)).astype(np.int64)
                owner = np.repeat(slots, cnt).astype(np.int32)
                if tot:
                    rows_dev = torch.from_numpy(rows).to(ts_dev.device)
                    flags, ost, _ = self.store.ingest_ex(ts_dev.index_select(0, rows_dev),
                                                         torch.from_numpy(owner).to(ts_dev.device), self.next_id)
                    ost = ost.cpu().numpy()
                    self._log(self.next_id, ts, coff, content, rowmap=rows)
                    self.next_id += tot
                    bad = ost[slots] != 0
                else:
                    bad = np.zeros(len(F), dtype=bool)
                rejected = [int(i) for i in F[bad]]
                answered = [(int(i), int(sl)) for i, sl in zip(F[~bad], slots[~bad])]
                T["ingest"] += time.perf_counter() - t0
            else:
                answered = []
            if slow or rejected:
                # rows stored under lenient spellings, or an owner the ingest rejected
                # (its requests committed nothing there): the per-request path
                t0 = time.perf_counter()
                self._round([(i, self._request_at(i, arena, boff, inf, users, log, ts_len, ts_off, msg_base))
                             for i in sorted(slow + rejected)], out)
                T["per_request"] += time.perf_counter() - t0
            if answered:
                self._respond_fast(answered, arena, boff, inf, nodes16, out, T,
                                   lambda i: self._request_at(i, arena, boff, inf, users, log, ts_len, ts_off,
                                                              msg_base), views)
        T["other"] = time.perf_counter() - t_call - sum(T.values())  # (the host's round bookkeeping)
        return out

    def _request_at(self, i, arena, boff, inf, users, log, ts_len, ts_off, msg_base):
        """Request i of a fast-path call as the per-request path's Sync."""
        ts, coff, content = log
        m0, k = int(msg_base[i]), int(inf[i, 0])
        c0, c1 = int(coff[m0]), int(coff[m0 + k])
        raw = [arena[int(o):int(o) + int(ln)].tobytes().decode("utf-8", "replace")
               for o, ln in zip(ts_off[m0:m0 + k], ts_len[m0:m0 + k])]
        span = lambda f: arena[int(boff[i] + inf[i, f]):int(boff[i] + inf[i, f] + inf[i, f + 1])]  # noqa: E731
        return wire.Sync(ts[m0:m0 + k].copy(), ts_len[m0:m0 + k].copy(), (coff[m0:m0 + k + 1] - c0).copy(),
                         content[c0:c1].tobytes(), span(6).tobytes().decode("utf-8", "replace"), raw=raw,
                         user=users[i], node=span(4).tobytes().decode("utf-8", "replace"))

    def _respond_fast(self, answered, arena, boff, inf, nodes16, out: List[Result], T, request_at, views=False):
        """getMessages + SyncResponse.toBinary for requests i at owner slots
        sl (no lenient rows): client trees parsed on host threads in one call,
        one selection, the trees' JSON in one device launch, the responses
        encoded on host threads in one call."""
        import time

        import torch

        lib, eng, O = _lib.load(), self.eng, self.capacity
        t0 = time.perf_counter()
        req = np.asarray([i for i, _ in answered], dtype=np.int64)
        sl = np.asarray([s_ for _, s_ in answered], dtype=np.int64)
        ptrs = np.full(O, _EMPTY_PTR, dtype=np.uint64)
        lens = np.full(O, 2, dtype=np.uint64)
        base = arena.ctypes.data
        ptrs[sl] = base + boff[req] + inf[req, 6]
        lens[sl] = inf[req, 7]
        h = C.c_void_p()
        stt = lib.evm_tree_from_json(eng.h, O, ptrs.ctypes.data_as(C.POINTER(C.c_char_p)),
                                     lens.ctypes.data_as(C.POINTER(C.c_size_t)), C.byref(h))
        T["trees"] += time.perf_counter() - t0
        if stt != _lib.EVM_OK:
            # some request's merkleTree does not parse (merkleTreeFromString throws -> 500 for that
            # request only): the per-request selection finds which
            t0 = time.perf_counter()
            self._select([(int(i), request_at(int(i)), int(s_)) for i, s_ in answered], out)
            T["per_request"] += time.perf_counter() - t0
            return
        from .engine import Trees

        client = Trees(eng, h)
        t0 = time.perf_counter()
        node = np.full((O, 16), ord("0"), dtype=np.uint8)
        node[sl] = nodes16[req]
        active = np.zeros(O, dtype=np.uint8)
        active[sl] = 1
        diff, soff, sid = self.store.select(client, eng.dev(node), eng.dev(active))
        client.free()
        diff, soff, sid = diff.cpu().numpy(), soff.cpu().numpy().astype(np.int64), sid.cpu().numpy()
        T["select"] += time.perf_counter() - t0
        t0 = time.perf_counter()
        jbuf, joff = self.store.tree().to_json_batch(torch.from_numpy(sl.astype(np.int32)).to(f"cuda:{eng.device}"))
        jbuf, joff = jbuf.cpu().numpy(), joff.cpu().numpy()
        T["json"] += time.perf_counter() - t0
        t0 = time.perf_counter()
        rng_err = diff[sl] == _lib.DIFF_RANGE_ERROR
        cnt = np.where(rng_err, 0, soff[sl + 1] - soff[sl])
        first = np.cumsum(cnt) - cnt
        tot = int(cnt.sum())
        pick = np.repeat(soff[sl] - first, cnt) + np.arange(tot)
        sel = np.ascontiguousarray(sid[pick], dtype=np.uint64)
        sel_off = np.zeros(len(sl) + 1, dtype=np.uint64)
        np.cumsum(cnt, out=sel_off[1:])
        segs = [g.host() for g in self._segs]
        seg_base = np.asarray(self._base, dtype=np.uint64)
        P = C.c_void_p
        seg_row = (P * len(segs))(*[None if r is None else r.ctypes.data for _, _, _, r in segs])
        seg_ts = (P * len(segs))(*[t.ctypes.data for t, _, _, _ in segs])
        seg_coff = (P * len(segs))(*[o.ctypes.data for _, o, _, _ in segs])
        seg_con = (P * len(segs))(*[c.ctypes.data for _, _, c, _ in segs])
        ooff = np.zeros(len(sl) + 1, dtype=np.uint64)
        args = [len(sl), _np_ptr(sel_off), _np_ptr(sel), len(segs), _np_ptr(seg_base), seg_row, seg_ts, 48, seg_coff,
                seg_con, _np_ptr(jbuf), _np_ptr(joff)]
        check(lib.evm_pb_encode_responses(*args, None, _np_ptr(ooff)), "evm_pb_encode_responses")
        resp = np.zeros(max(int(ooff[-1]), 1), dtype=np.uint8)
        check(lib.evm_pb_encode_responses(*args, _np_ptr(resp), _np_ptr(ooff)), "evm_pb_encode_responses")
        rb = memoryview(resp) if views else resp.tobytes()
        for k, i in enumerate(req):
            out[int(i)] = RangeError("Invalid count value") if rng_err[k] else rb[int(ooff[k]):int(ooff[k + 1])]
        T["encode"] += time.perf_counter() - t0

    # ------------------------------------------------------------------ ingest
    def _ingest(self, reqs, rows_of):
        """One evm_server_ingest_ex over the requests' rows -> (flags per
        request, set of request positions whose owner committed nothing)."""
        eng = self.eng
        parts = [rows_of(d) for _, d, _ in reqs]
        n = sum(len(p) for p in parts)
        ts = np.zeros((n, 48), dtype=np.uint8)
        owner = np.zeros(n, dtype=np.uint32)
        off = np.zeros(n + 1, dtype=np.uint64)
        content = []
        p = 0
        spans = []
        for (_, d, s), rows in zip(reqs, parts):
            m = len(rows)
            ts[p:p + m] = rows
            owner[p:p + m] = s
            off[p + 1:p + m + 1] = off[p] + d.content_off[1:]
            content.append(d.content)
            spans.append((p, p + m))
            p += m
        if n == 0:
            return [np.zeros(0, np.uint8)] * len(reqs), set(), [self.next_id] * len(reqs)
        flags, ost, _ = self.store.ingest_ex(eng.dev(ts), eng.dev(owner), self.next_id)
        flags, ost = flags.cpu().numpy(), ost.cpu().numpy()
        base = self.next_id
        self._log(base, ts, off, np.frombuffer(b"".join(content) or b"\0", dtype=np.uint8))
        self.next_id += n
        rejected = {k for k, (_, _, s) in enumerate(reqs) if ost[s]}
        return [flags[a:b] for a, b in spans], rejected, [base + a for a, _ in spans]

    def _check(self, user: str, spellings, flags, mids):
        """Walks a request's rows in order against the user's rows stored under
        lenient spellings.  Returns the tracking entries to add, or None when
        the device and the reference part ways: a row the device reports as
        already stored although the reference would insert it, because its
        timestamp is stored under another spelling."""
        known = self.lenient.get(user, {})
        added = {}
        for (raw, canon), f, mid in zip(spellings, flags, mids):
            have = added.get(canon) or known.get(canon)
            if f & _lib.MSG_INS:
                if raw != canon:
                    added[canon] = (raw, mid)
            elif have is not None:
                if have[0] != raw:
                    return None  # the key is stored under another (lenient) spelling
            elif raw != canon:
                return None  # the key is stored under its canonical spelling, this lenient one is not
        return added

    def _round(self, rnd, out: List[Result]):
        live = []
        for i, d in rnd:
            if d.user in self.detached:
                continue  # out[i] stays None
            nb = d.node.encode("latin-1", "replace")
            if len(nb) != 16 or not all(c in _HEX for c in nb):
                # NOT LIKE '%' || nodeId with any nodeId is not modelled: hand the user over, unapplied
                self.detached.add(d.user)
                continue
            live.append((i, d, self._slot(d.user)))
        if not live:
            return
        # pass 1: every request as sent (rows of other lengths arrive as 0xFF: rejected)
        flags, rejected, mids = self._ingest(live, lambda d: d.ts[:, :48])
        answered = []
        for k, (i, d, s) in enumerate(live):
            if k in rejected:
                continue
            if d.user in self.lenient:
                sp = [(t, t) for t in d.timestamps()]
                if self._check(d.user, sp, flags[k], range(mids[k], mids[k] + len(sp))) is None:
                    self.detached.add(d.user)
                    out[i] = HandedOver(applied=True)  # (committed by the ingest above)
                    continue
            answered.append((i, d, s))
        # the rejected owners' requests: invalid date -> 500; lenient -> their canonical form
        fix = []
        for k in sorted(rejected):
            i, d, s = live[k]
            kinds = [LN.classify(raw) for raw in d.raw]
            if any(kd == "range_error" for kd, _ in kinds):
                out[i] = RangeError("Invalid time value")  # toISOString of an invalid date: nothing stored
            elif any(kd != "ok" for kd, _ in kinds):
                self.detached.add(d.user)
            else:
                fix.append((i, d, s, [c for _, c in kinds]))
        if fix:
            canon_rows = {id(d): np.frombuffer("".join(c).encode(), dtype=np.uint8).reshape(-1, TS_LEN)
                          for _, d, _, c in fix}

            def rows_of(d):
                r = np.zeros((len(d.raw), 48), dtype=np.uint8)
                r[:, :TS_LEN] = canon_rows[id(d)]
                return r

            f2, rej2, mids2 = self._ingest([(i, d, s) for i, d, s, _ in fix], rows_of)
            for k, (i, d, s, canon) in enumerate(fix):
                sp = list(zip(d.raw, canon))
                added = None if k in rej2 else self._check(d.user, sp, f2[k], range(mids2[k], mids2[k] + len(sp)))
                if added is None:
                    self.detached.add(d.user)
                    if k not in rej2:
                        out[i] = HandedOver(applied=True)  # (committed by the re-ingest)
                    continue
                self.lenient.setdefault(d.user, {}).update(added)
                for raw, mid in added.values():
                    self._raw[mid] = raw
                answered.append((i, d, s))
        answered = [(i, d, s) for i, d, s in answered if d.user not in self.detached]
        if answered:
            self._select(answered, out)

    # ------------------------------------------------------------ getMessages
    def _select(self, reqs, out: List[Result]):
        eng, O = self.eng, self.capacity
        trees = ["{}"] * O
        node = np.full((O, 16), ord("0"), dtype=np.uint8)
        active = np.zeros(O, dtype=np.uint8)
        for i, d, s in reqs:
            trees[s] = d.tree
            node[s] = np.frombuffer(d.node.encode("latin-1"), dtype=np.uint8)
            active[s] = 1
        try:
            client = eng.tree_from_json(trees)
        except _lib.EngineError:
            # some request's merkleTree JSON does not parse: select owner by owner,
            # so only that request fails (merkleTreeFromString throws -> 500)
            for i, d, s in reqs:
                one = ["{}"] * O
                one[s] = d.tree
                mask = np.zeros(O, dtype=np.uint8)
                mask[s] = 1
                try:
                    c1 = eng.tree_from_json(one)
                except _lib.EngineError as e:
                    out[i] = e
                    continue
                self._respond([(i, d, s)], c1, node, mask, out)
            return
        self._respond(reqs, client, node, active, out)

    def _respond(self, reqs, client, node, active, out: List[Result]):
        """getMessages for the active owners, then SyncResponse.toBinary per request."""
        eng = self.eng
        diff, soff, sid = self.store.select(client, eng.dev(node), eng.dev(active))
        client.free()
        diff, soff, sid = diff.cpu().numpy(), soff.cpu().numpy(), sid.cpu().numpy()
        tree = self.store.tree()
        for i, d, s in reqs:
            if diff[s] == _lib.DIFF_RANGE_ERROR:
                out[i] = RangeError("Invalid count value")
                continue
            ids = [int(m) for m in sid[int(soff[s]):int(soff[s + 1])]]
            msgs = [self._message(m) for m in ids]
            if d.user in self.lenient and diff[s] >= 0:
                msgs = self._raw_order(d, int(diff[s]), ids, msgs)
            out[i] = wire.encode(wire.RESPONSE, [t for t, _ in msgs], [c for _, c in msgs], tree=tree.to_json(s))

    def _raw_order(self, d, diff: int, ids, msgs):
        """index.ts:98-102 compares and orders the STORED (raw) strings: rows
        kept under a lenient spelling join or leave the selection by their raw
        string against the bound, and everything sorts by raw string."""
        bound = LN.to_string(diff, 0, "0000000000000000")
        nl = d.node.lower()
        keep = [(t, c, m) for (t, c), m in zip(msgs, ids) if t > bound]
        have = set(m for _, _, m in keep)
        for raw, mid in self.lenient[d.user].values():
            if mid not in have and raw > bound and not raw.lower().endswith(nl):
                t, c = self._message(mid)
                keep.append((t, c, mid))
        keep.sort(key=lambda x: x[0].encode("latin-1"))
        return [(t, c) for t, c, _ in keep]


__all__ = ["SyncServer", "ParseBodyError", "RangeError", "HandedOver"]
