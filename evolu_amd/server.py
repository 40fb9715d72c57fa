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

from typing import Dict, List, Sequence, Set, Union

import numpy as np

from . import _lib
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
_HEX = set(b"0123456789abcdefABCDEF")


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
        self.slot: Dict[str, int] = {}
        self.next_id = 0
        self._base: List[int] = []          # first message id of each ingested batch
        self._ts: List[np.ndarray] = []     # that batch's (n, stride) timestamp rows
        self._off: List[np.ndarray] = []    # its content offsets (n + 1)
        self._content: List[bytes] = []     # its concatenated contents
        self._raw: Dict[int, str] = {}      # message id -> the raw timestamp, for rows stored under a lenient spelling
        # user -> canonical timestamp -> (raw spelling, message id) of rows stored under a lenient spelling
        self.lenient: Dict[str, Dict[str, tuple]] = {}
        self.detached: Set[str] = set()    # users whose requests the caller runs (see the module docstring)

    def close(self):
        self.store.free()

    def _slot(self, user: str) -> int:
        s = self.slot.get(user)
        if s is None:
            if len(self.slot) >= self.capacity:
                raise _lib.EngineError(_lib.EVM_ECAPACITY, "SyncServer: more users than owner slots")
            s = self.slot[user] = len(self.slot)
        return s

    def _message(self, mid: int):
        r = int(np.searchsorted(np.asarray(self._base), mid, side="right")) - 1
        k = mid - self._base[r]
        o = self._off[r]
        ts = self._raw.get(mid)
        if ts is None:
            ts = bytes(self._ts[r][k, :TS_LEN]).decode("latin-1")
        return ts, self._content[r][int(o[k]):int(o[k + 1])]

    def sync(self, bodies: Sequence[bytes]) -> List[Result]:
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
        flags, ost, _ = self.store.ingest_ex(eng.dev(ts), eng.dev(owner), self.next_id)
        flags, ost = flags.cpu().numpy(), ost.cpu().numpy()
        base = self.next_id
        self._base.append(base)
        self._ts.append(ts)
        self._off.append(off)
        self._content.append(b"".join(content))
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
