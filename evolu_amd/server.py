"""The sync server's request path over a device store: SyncRequest bodies in,
SyncResponse bodies out (apps/server/src/index.ts:204-251).

Per request the reference runs parseBody (:108-116, SyncRequest.fromBinary),
getMerkleTree (:118-134), addMessages (:136-171), getMessages (:173-202) and
answers SyncResponse.toBinary({merkleTree: merkleTreeToString(tree),
messages}) (:233-241); any throw answers 500 and rolls back THAT request
(:147-169, :224-233).

A call is one native round (include/evm.h evm_sync_round, evm_sync.hip): the
bodies decoded where they lie on the device, the userId -> owner slot
directory a device hash table, one evm_server_ingest_ex, the client trees
parsed, one selection and every response built on the device -- from host
bodies (sync / sync_arena: staged through pinned chunks both ways) or from
bodies resident in HBM (sync_device: the responses stay there).  A call in
which a user sends two requests is cut into rounds (the k-th request of each
user in round k): a later request must see the earlier one's inserts and not
its own later ones, exactly the reference's one-request-at-a-time order.

Per-request failure, as the reference: the round commits every request but
the ones with a timestamp outside the engine's canonical domain
(EVM_ENONCANON).  Those go through the host's restatement of
timestampFromString (evolu_amd/lenient.py, pinned by node): an invalid date
fails the request (RangeError -> the reference's 500; nothing of it is
stored), a lenient but valid one (V8 rolls "02-30" into March, a lower-case
counter parses) is re-ingested in the form the reference's tree sees
(timestampToString(timestampFromString(raw))) while the response keeps the raw
string, which is what the reference stores.  Rows stored under a lenient
spelling are tracked per user, so getMessages still orders and bounds them
by their raw strings; those users' later requests take the per-request path
(the round hands them back as EVM_EHANDOVER).

Results per body: the SyncResponse bytes, an exception object standing for
the reference's 500 answer (ParseBodyError, RangeError, EngineError of the
client tree's parse), or None where the engine does not model the request
(a nodeId that is not 16 hex chars, a timestamp shape timestampFromString
would read in a way lenient.py does not restate, one timestamp stored under
two spellings).  The user is then handed to the caller for good: every later
request of that user also answers None, so the caller runs them, in order, on
the reference path.  None always means unapplied.  A spelling conflict found
only after the request was committed answers `HandedOver(applied=True)`
instead: its rows are in this server's store and tree, the user is handed
over all the same, and the caller must serve that user from its own
reference state from then on and treat this server's rows and tree of that
user as stale.
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Sequence as _SequenceABC
from typing import Dict, List, Optional, Sequence, Set, Union

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
TIMING_PARTS = ("h2d", "decode", "users", "ingest", "trees", "select", "encode", "d2h")


def _np_ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


_HEX = set(b"0123456789abcdefABCDEF")


def rounds_of(users: Sequence[Optional[bytes]]) -> List[List[int]]:
    """Requests cut into rounds: the k-th request of a user goes to round k
    (request order kept inside a round); a request without a user (its body
    did not parse) goes to round 0."""
    seen: Dict[bytes, int] = {}
    rounds: List[List[int]] = []
    for i, u in enumerate(users):
        k = 0
        if u is not None:
            k = seen.get(u, 0)
            seen[u] = k + 1
        while k >= len(rounds):
            rounds.append([])
        rounds[k].append(i)
    return rounds


class _Results:
    """A round's per-request codes as results: True (answered), an exception
    object (the reference's 500), or None (the host's per-request path)."""

    def __init__(self, codes: np.ndarray):
        self.codes = codes

    def __len__(self):
        return len(self.codes)

    def __getitem__(self, k):
        code = int(self.codes[k])
        if code == _lib.EVM_OK:
            return True
        if code == _lib.EVM_EINVAL:
            return ParseBodyError(_lib.load().evm_strerror(code).decode())
        if code == _lib.EVM_ERANGE:
            return RangeError("Invalid count value")
        if code == _lib.EVM_ETREE:
            return _lib.EngineError(code, "merkleTreeFromString")
        return None  # EVM_ENONCANON, EVM_EHANDOVER: the per-request path decides

    def __iter__(self):
        return (self[k] for k in range(len(self.codes)))

    def late(self) -> List[int]:
        return np.flatnonzero((self.codes == _lib.EVM_ENONCANON) | (self.codes == _lib.EVM_EHANDOVER)).tolist()


def _body_users(arena: np.ndarray, off: np.ndarray) -> List[Optional[bytes]]:
    """Each body's userId bytes (None: the body does not parse), host codec."""
    lib = _lib.load()
    n = len(off) - 1
    info = (wire._Sync * max(n, 1))()
    st = np.zeros(max(n, 1), dtype=np.int32)
    check(lib.evm_pb_scan_batch(REQUEST_KIND, _np_ptr(arena), _np_ptr(off), n, info, _np_ptr(st)),
          "evm_pb_scan_batch")
    out: List[Optional[bytes]] = []
    for k in range(n):
        if st[k]:
            out.append(None)
            continue
        a = int(off[k]) + int(info[k].user_off)
        out.append(arena[a:a + int(info[k].user_len)].tobytes())
    return out


def _sub_arena(arena: np.ndarray, off: np.ndarray, idx: np.ndarray):
    """The bodies idx (in that order) as one arena and its offsets."""
    ln = (off[1:] - off[:-1])[idx]
    sub_o = np.zeros(len(idx) + 1, dtype=np.uint64)
    np.cumsum(ln, out=sub_o[1:])
    sub_a = np.concatenate([arena[int(off[i]):int(off[i + 1])] for i in idx.tolist()] or [np.zeros(0, np.uint8)])
    return np.ascontiguousarray(sub_a if len(sub_a) else np.zeros(1, np.uint8)), sub_o


class Responses(_SequenceABC):
    """sync_arena(views=True)'s answer: result k is response k's bytes as a
    memoryview into one host response arena (made when read), or what sync()
    returns for it (an exception object, a HandedOver, None)."""

    def __init__(self, n: int):
        self.n = n
        self.arena = None  # memoryview of the response arena, off: uint64 [n + 1] (every request answered)
        self.off = None
        self.items: Optional[List[Result]] = None  # (or each result on its own)

    def __len__(self):
        return self.n

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(self.n))]
        if k < 0:
            k += self.n
        if not 0 <= k < self.n:
            raise IndexError(k)
        if self.items is not None:
            return self.items[k]
        if self.arena is not None:
            return self.arena[int(self.off[k]):int(self.off[k + 1])]
        return None

    def __setitem__(self, k, v):
        if self.items is None:
            self.items = [self[i] for i in range(self.n)]
        self.items[k] = v


class DeviceResponses:
    """sync_device's answer: result[i] is True where response i is the bytes
    [off[i], off[i + 1]) of the round's response arena in device memory (the
    server's, valid until its next round), else what sync() would return for
    it (bytes, an exception object, a HandedOver, or None)."""

    def __init__(self, srv, off: np.ndarray, result: List, nbytes: int = 0):
        self.srv, self.off, self.result, self.nbytes = srv, off, result, nbytes
        self._round = srv._rounds if srv is not None else 0

    def __len__(self):
        return len(self.result)

    def _arena(self) -> np.ndarray:
        if self.srv is None or not self.nbytes:
            return np.zeros(1, dtype=np.uint8)
        if self.srv._rounds != self._round:
            raise RuntimeError("DeviceResponses: the server ran another round since (its response arena is reused)")
        return self.srv._fetch(self.nbytes)

    def get(self, i: int) -> Result:
        """Response i as sync() returns it (one range copied back)."""
        r = self.result[i]
        if r is not True:
            return r
        if self.srv._rounds != self._round:
            raise RuntimeError("DeviceResponses: the server ran another round since (its response arena is reused)")
        a, b = int(self.off[i]), int(self.off[i + 1])
        out = np.empty(max(b - a, 1), dtype=np.uint8)
        lib = _lib.load()
        if b > a:
            check(lib.evm_copy_d2h(self.srv.eng.h, _np_ptr(out),
                                   C.c_void_p(lib.evm_sync_responses_dev(self.srv.h) + a), b - a), "evm_copy_d2h")
        return out[: b - a].tobytes()

    def to_host(self) -> List[Result]:
        """Every result as sync() returns it (the device bytes copied back)."""
        hb = self._arena() if any(r is True for r in self.result) else None
        return [hb[int(self.off[i]):int(self.off[i + 1])].tobytes() if r is True else r
                for i, r in enumerate(self.result)]


class ParseBodyError(Exception):
    """index.ts:108-116: SyncRequest.fromBinary threw."""


class RangeError(Exception):
    """A JS RangeError -> 500: diffMerkleTrees' keyToTimestamp (merkleTree.ts:55-61)
    or addMessages' toISOString of an invalid date (timestamp.ts:45)."""


class SyncServer:
    """One device store for up to ``capacity`` users (owner slots), served by
    a native round (evm_sync_*) that owns the user directory and the message
    log."""

    def __init__(self, eng: Engine, capacity: int):
        self.eng = eng
        self.store = eng.store_new(capacity)
        self.capacity = capacity
        lib = _lib.load()
        h = C.c_void_p()
        check(lib.evm_sync_create(eng.h, self.store.h, C.byref(h)), "evm_sync_create")
        self.h = h
        self._rounds = 0  # native rounds run (a DeviceResponses is valid until the next)
        self._ok = None   # the last round's answered requests (bool array)
        self.timing: Dict[str, float] = {}  # seconds of the last call by part
        self._raw: Dict[int, str] = {}      # message id -> the raw timestamp, for rows stored under a lenient spelling
        # user -> canonical timestamp -> (raw spelling, message id) of rows stored under a lenient spelling
        self.lenient: Dict[str, Dict[str, tuple]] = {}
        self.detached: Set[str] = set()    # users whose requests the caller runs (see the module docstring)

    def close(self):
        if self.h:
            _lib.load().evm_sync_destroy(self.h)
            self.h = None
        self.store.free()

    @property
    def next_id(self) -> int:
        """The id the next stored message gets (ids are consecutive over rounds and per-request ingests)."""
        return int(_lib.load().evm_sync_next_id(self.h))

    @property
    def slot(self) -> Dict[str, int]:
        """userId -> owner slot (every user the directory holds)."""
        lib = _lib.load()
        n, kb = C.c_uint32(), C.c_uint64()
        check(lib.evm_sync_user_count(self.h, C.byref(n), C.byref(kb)), "evm_sync_user_count")
        keys = np.zeros(max(kb.value, 1), dtype=np.uint8)
        off = np.zeros(n.value + 1, dtype=np.uint64)
        check(lib.evm_sync_user_keys(self.h, _np_ptr(keys), _np_ptr(off)), "evm_sync_user_keys")
        return {keys[int(off[i]):int(off[i + 1])].tobytes().decode("utf-8", "replace"): i for i in range(n.value)}

    def _users(self, users: Sequence[str], insert: bool) -> List[Optional[int]]:
        """The directory's slots of distinct users (insert: new ones added in order)."""
        if not users:
            return []
        lib = _lib.load()
        b = [u.encode("utf-8") for u in users]
        ids = np.frombuffer(b"".join(b) or b"\0", dtype=np.uint8)
        off = np.zeros(len(b) + 1, dtype=np.uint64)
        np.cumsum([len(x) for x in b], out=off[1:])
        slots = np.zeros(len(b), dtype=np.uint32)
        st = lib.evm_sync_users(self.h, _np_ptr(ids), _np_ptr(off), len(b), 1 if insert else 0, _np_ptr(slots))
        if st == _lib.EVM_ECAPACITY:
            raise _lib.EngineError(st, "SyncServer: more users than owner slots")
        check(st, "evm_sync_users")
        return [None if s == 0xFFFFFFFF else int(s) for s in slots]

    def _slot(self, user: str) -> int:
        return self._users([user], True)[0]

    def _hand(self, user: str, lenient: bool = False):
        """The user's later requests are the host's (handed over, or rows under
        lenient spellings): the round answers them EVM_EHANDOVER.  (The user
        takes a slot if it has none, so the directory knows it.)"""
        if not lenient:
            self.detached.add(user)
        (s,) = self._users([user], True)
        check(_lib.load().evm_sync_user_flag(self.h, s, 1), "evm_sync_user_flag")

    def _messages(self, ids: Sequence[int]):
        """[(timestamp, content)] of message ids (the log; raw spellings where kept)."""
        n = len(ids)
        if not n:
            return []
        lib = _lib.load()
        idv = np.ascontiguousarray(ids, dtype=np.uint64)
        ts = np.zeros((n, TS_LEN), dtype=np.uint8)
        co = np.zeros(n + 1, dtype=np.uint64)
        check(lib.evm_sync_log_read(self.h, _np_ptr(idv), n, _np_ptr(ts), _np_ptr(co), None), "evm_sync_log_read")
        content = np.zeros(max(int(co[-1]), 1), dtype=np.uint8)
        check(lib.evm_sync_log_read(self.h, _np_ptr(idv), n, _np_ptr(ts), _np_ptr(co), _np_ptr(content)),
              "evm_sync_log_read")
        out = []
        for k, m in enumerate(idv.tolist()):
            t = self._raw.get(m)
            if t is None:
                t = ts[k].tobytes().decode("latin-1")
            out.append((t, content[int(co[k]):int(co[k + 1])].tobytes()))
        return out

    def _fetch(self, nbytes: int) -> np.ndarray:
        out = np.empty(max(nbytes, 1), dtype=np.uint8)
        check(_lib.load().evm_sync_fetch(self.h, _np_ptr(out)), "evm_sync_fetch")
        return out

    # ------------------------------------------------------------ the rounds
    def sync(self, bodies: Sequence[bytes]) -> List[Result]:
        n = len(bodies)
        boff = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.fromiter((len(b) for b in bodies), dtype=np.uint64, count=n), out=boff[1:])
        return self.sync_arena(np.frombuffer(b"".join(bodies) or b"\0", dtype=np.uint8), boff, views=False)

    def sync_arena(self, arena: np.ndarray, off: np.ndarray, views: bool = True) -> List[Result]:
        """sync() of the bodies arena[off[k] .. off[k + 1]) (uint8 / uint64 host
        arrays) through the native round (pinned H2D -> the round on the
        device -> pinned D2H); views=True: the responses are memoryviews into
        one response arena (no per-response copy), equal to the bytes sync()
        would return."""
        import time

        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        t_call = time.perf_counter()
        T = self.timing = dict.fromkeys(TIMING_PARTS + ("per_request", "other"), 0.0)
        n = len(off) - 1
        out = Responses(n) if views else [None] * n
        if n == 0:
            return out
        if not self._host_round(arena, off, np.arange(n), out, views, T):
            # a user with two requests: the k-th request of every user in round k
            for rnd in rounds_of(_body_users(arena, off)):
                idx = np.asarray(rnd, dtype=np.int64)
                sub_a, sub_o = _sub_arena(arena, off, idx)
                done = self._host_round(sub_a, sub_o, idx, out, views, T)
                assert done, "a round with one request per user"
        T["other"] = time.perf_counter() - t_call - sum(v for k, v in T.items() if not k.endswith("_call"))
        return out

    def _host_round(self, arena, off, idx, out, views, T) -> bool:
        """One native round over host bodies, results into out[idx[k]];
        False (nothing applied) when a user sends two of the requests."""
        import time

        t0 = time.perf_counter()
        res, roff, total = self._round_native(arena, off, _lib.SYNC_HOST)
        if res is None:
            return False
        T["round_call"] = T.get("round_call", 0.0) + time.perf_counter() - t0
        self._add_timing(T)
        t0 = time.perf_counter()
        resp = self._fetch(total) if total else None
        T["fetch_call"] = T.get("fetch_call", 0.0) + time.perf_counter() - t0
        T["d2h"] += self._part_ms(7) / 1e3
        rb = memoryview(resp) if views and resp is not None else resp
        ok = self._ok
        if views and isinstance(out, Responses) and ok is not None and len(idx) == len(out) and ok.all():
            out.arena, out.off = rb, roff  # (the common case: every request answered, views made on access)
            return True
        ro = roff.tolist()
        for k, i in enumerate(idx.tolist()):
            r = res[k]
            if r is True:
                out[i] = rb[ro[k]:ro[k + 1]] if views else rb[ro[k]:ro[k + 1]].tobytes()
            else:
                out[i] = r
        self._late(res, arena, off, idx, out, T)
        return True

    def _part_ms(self, k: int) -> float:
        ms = (C.c_double * 8)()
        check(_lib.load().evm_sync_timing(self.h, ms), "evm_sync_timing")
        return ms[k]

    def sync_device(self, arena, off) -> DeviceResponses:
        """sync() of bodies resident in device memory: arena (uint8 tensor on
        the engine's GPU), off (host uint64 [n + 1]).  The round runs on the
        device end to end (evm_sync_round, EVM_SYNC_DEVICE) and the responses
        stay in device memory (DeviceResponses).  A call the round cannot take
        as one (a user with two requests) is cut into rounds on a host copy of
        the bodies."""
        import time

        off = np.ascontiguousarray(off, dtype=np.uint64)
        t_call = time.perf_counter()
        T = self.timing = dict.fromkeys(TIMING_PARTS + ("per_request", "other"), 0.0)
        n = len(off) - 1
        if n == 0:
            return DeviceResponses(None, np.zeros(1, dtype=np.uint64), [])
        res, roff, total = self._round_native(arena, off, _lib.SYNC_DEVICE)
        if res is None:  # (a user with two requests: rounds, on a host copy)
            host = arena.cpu().numpy()
            out = self.sync_arena(host, off, views=False)
            self.timing = dict(self.timing, device_fallback=time.perf_counter() - t_call)
            return DeviceResponses(None, np.zeros(n + 1, dtype=np.uint64), out)
        self._add_timing(T)
        result: List = [True] * n
        for k in np.flatnonzero(res.codes != _lib.EVM_OK).tolist():
            result[k] = res[k]
        if res.late():
            host_of = lambda i: arena[int(off[i]):int(off[i + 1])].cpu().numpy()  # noqa: E731
            self._late(res, None, off, np.arange(n), result, T, body_of=host_of)
        T["other"] = time.perf_counter() - t_call - sum(v for v in T.values())
        return DeviceResponses(self, roff, result, total)

    def _add_timing(self, T):
        ms = (C.c_double * 8)()
        check(_lib.load().evm_sync_timing(self.h, ms), "evm_sync_timing")
        for k, name in enumerate(TIMING_PARTS[:-1]):  # (the fetch's part: after it)
            T[name] += ms[k] / 1e3

    def _round_native(self, arena, off, where):
        """One evm_sync_round -> (per request: True (response bytes at
        [roff[k], roff[k + 1])), an exception object, or None = the host's
        per-request path decides; roff; response bytes), or (None, None, 0)
        when a user sends two of the requests (nothing applied)."""
        lib = _lib.load()
        n = len(off) - 1
        result = np.zeros(n, dtype=np.int32)
        roff = np.zeros(n + 1, dtype=np.uint64)
        total = C.c_uint64()
        ptr = C.c_void_p(arena.data_ptr()) if where == _lib.SYNC_DEVICE else _np_ptr(arena)
        st = lib.evm_sync_round(self.h, ptr, _np_ptr(off), n, where, _np_ptr(result), _np_ptr(roff), C.byref(total))
        self._rounds += 1
        if st == _lib.EVM_EROUNDS:
            return None, None, 0
        if st == _lib.EVM_ECAPACITY:
            raise _lib.EngineError(st, "SyncServer: more users than owner slots")
        check(st, "evm_sync_round")
        self._ok = result == _lib.EVM_OK
        res = _Results(result)
        return res, roff, total.value

    def _late(self, res, arena, off, idx, out, T, body_of=None):
        """The requests a round handed back (None): rejected by the ingest
        (a timestamp outside the native domain: nothing of it stored), a
        nodeId that is not 16 hex chars, a non-ASCII userId, or a user handed
        over / with rows under lenient spellings -- each the host's, in
        request order (rounds when a user sends several)."""
        import time

        late = res.late() if isinstance(res, _Results) else [k for k, r in enumerate(res) if r is None]
        if not late:
            return
        t0 = time.perf_counter()
        if body_of is None:
            body_of = lambda k: arena[int(off[k]):int(off[k + 1])]  # noqa: E731
        reqs = []
        for k in late:
            d = wire.decode(wire.REQUEST, body_of(k).tobytes())
            i = int(idx[k])
            out[i] = None
            if d.user in self.detached:
                continue  # stays None
            nb = d.node.encode("latin-1", "replace")
            if len(nb) != 16 or not all(c in _HEX for c in nb):
                self._hand(d.user)  # NOT LIKE '%' || nodeId with any nodeId is not modelled
                continue
            reqs.append((i, d))
        seen: Dict[str, int] = {}
        rounds: List[list] = []
        for i, d in reqs:
            k = seen.get(d.user, 0)
            seen[d.user] = k + 1
            while k >= len(rounds):
                rounds.append([])
            rounds[k].append((i, d))
        for rnd in rounds:
            self._round(rnd, out)
        T["per_request"] += time.perf_counter() - t0

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
        # (the rows into the native round's message log first: their ids)
        cont = np.frombuffer(b"".join(content) or b"\0", dtype=np.uint8)
        first = C.c_uint64()
        check(_lib.load().evm_sync_log_add(self.h, _np_ptr(ts), 48, n, _np_ptr(off), _np_ptr(cont), C.byref(first)),
              "evm_sync_log_add")
        base = first.value
        flags, ost, _ = self.store.ingest_ex(eng.dev(ts), eng.dev(owner), base)
        flags, ost = flags.cpu().numpy(), ost.cpu().numpy()
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
                self._hand(d.user)
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
                    self._hand(d.user)
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
                self._hand(d.user)
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
                    self._hand(d.user)
                    if k not in rej2:
                        out[i] = HandedOver(applied=True)  # (committed by the re-ingest)
                    continue
                if added and d.user not in self.lenient:
                    self._hand(d.user, lenient=True)  # (its later requests: the per-request path)
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
            msgs = self._messages(ids)
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
                ((t, c),) = self._messages([mid])
                keep.append((t, c, mid))
        keep.sort(key=lambda x: x[0].encode("latin-1"))
        return [(t, c) for t, c, _ in keep]


__all__ = ["SyncServer", "ParseBodyError", "RangeError", "HandedOver"]
