"""The sync server's request path over a device store: SyncRequest bodies in,
SyncResponse bodies out (apps/server/src/index.ts:204-251).

Per request the reference runs parseBody (:108-116, SyncRequest.fromBinary),
getMerkleTree (:118-134), addMessages (:136-171), getMessages (:173-202) and
answers SyncResponse.toBinary({merkleTree: merkleTreeToString(tree),
messages}) (:233-241).  Here a list of bodies is one call: the bodies are
decoded on the host (evm_pb_*), the requests are cut into rounds in which
every owner (userId) appears at most once -- a later request of the same
owner must see the earlier one's inserts and must not see its own later
ones, exactly the reference's one-request-at-a-time order -- and each round
is one evm_server_ingest + one evm_server_select over all its owners.

What stays on the host: the userId -> owner-slot map, the message contents
(keyed by the message id the store reports; the store keeps the first
inserted row of a (timestamp, userId) pair, INSERT OR IGNORE, so the id's
content is the stored content), and the protobuf framing.

Results per body: the SyncResponse bytes, or an exception object standing
for the reference's 500 answer (ParseBodyError, a RangeError from
diffMerkleTrees), or None where the engine does not model the input (a
non-canonical timestamp in the round, a nodeId that is not 16 hex chars):
the caller runs the reference code for those requests.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Union

import numpy as np

from . import _lib
from . import wire
from .engine import TS_LEN, Engine

Result = Union[bytes, Exception, None]


class ParseBodyError(Exception):
    """index.ts:108-116: SyncRequest.fromBinary threw."""


class SyncServer:
    """One device store for up to ``capacity`` users (owner slots)."""

    def __init__(self, eng: Engine, capacity: int):
        self.eng = eng
        self.store = eng.store_new(capacity)
        self.capacity = capacity
        self.slot: Dict[str, int] = {}
        self.next_id = 0
        self._base: List[int] = []          # first message id of each ingested round
        self._ts: List[np.ndarray] = []     # that round's (n, stride) timestamp rows
        self._off: List[np.ndarray] = []    # its content offsets (n + 1)
        self._content: List[bytes] = []     # its concatenated contents

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
        return bytes(self._ts[r][k, :TS_LEN]).decode("latin-1"), self._content[r][int(o[k]):int(o[k + 1])]

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

    def _round(self, rnd, out: List[Result]):
        eng, O = self.eng, self.capacity
        slots = [self._slot(d.user) for _, d in rnd]
        n = sum(len(d.ts_len) for _, d in rnd)
        stride = 48
        ts = np.zeros((n, stride), dtype=np.uint8)
        owner = np.zeros(n, dtype=np.uint32)
        off = np.zeros(n + 1, dtype=np.uint64)
        content = []
        p = 0
        for (_, d), s in zip(rnd, slots):
            m = len(d.ts_len)
            ts[p:p + m] = d.ts[:, :stride]
            owner[p:p + m] = s
            off[p + 1:p + m + 1] = off[p] + d.content_off[1:]
            content.append(d.content)
            p += m
        if n:
            # index.ts:136-171 for every request of the round at once
            _, st = self.store.ingest(eng.dev(ts), eng.dev(owner), self.next_id, raise_on_error=False)
            if st == _lib.EVM_ENONCANON:
                return  # nothing applied; every request of the round -> None (reference path)
            _lib.check(st, "evm_server_ingest")
            self._base.append(self.next_id)
            self._ts.append(ts)
            self._off.append(off)
            self._content.append(b"".join(content))
            self.next_id += n
        # index.ts:173-202: the client trees and nodeIds of the round's owners
        trees = ["{}"] * O
        node = np.full((O, 16), ord("0"), dtype=np.uint8)
        active = np.zeros(O, dtype=np.uint8)
        for (i, d), s in zip(rnd, slots):
            nb = d.node.encode("latin-1", "replace")
            if len(nb) != 16 or not all(c in b"0123456789abcdefABCDEF" for c in nb):
                continue  # out[i] stays None
            trees[s] = d.tree
            node[s] = np.frombuffer(nb, dtype=np.uint8)
            active[s] = 1
        if not active.any():
            return
        try:
            client = eng.tree_from_json(trees)
        except _lib.EngineError:
            # some request's merkleTree JSON does not parse: select owner by owner,
            # so only that request fails (merkleTreeFromString throws -> 500)
            for (i, d), s in zip(rnd, slots):
                if active[s]:
                    one = ["{}"] * O
                    one[s] = d.tree
                    mask = np.zeros(O, dtype=np.uint8)
                    mask[s] = 1
                    try:
                        c1 = eng.tree_from_json(one)
                    except _lib.EngineError as e:
                        out[i] = e
                        continue
                    self._respond([(i, s)], c1, node, mask, out)
            return
        self._respond([(i, s) for (i, _), s in zip(rnd, slots) if active[s]], client, node, active, out)

    def _respond(self, reqs, client, node, active, out: List[Result]):
        """getMessages for the active owners, then SyncResponse.toBinary per request."""
        eng = self.eng
        diff, soff, sid = self.store.select(client, eng.dev(node), eng.dev(active))
        client.free()
        diff, soff, sid = diff.cpu().numpy(), soff.cpu().numpy(), sid.cpu().numpy()
        tree = self.store.tree()
        for i, s in reqs:
            if diff[s] == _lib.DIFF_RANGE_ERROR:
                out[i] = RangeError("Invalid count value")
                continue
            msgs = [self._message(int(m)) for m in sid[int(soff[s]):int(soff[s + 1])]]
            out[i] = wire.encode(wire.RESPONSE, [t for t, _ in msgs], [c for _, c in msgs], tree=tree.to_json(s))


class RangeError(Exception):
    """diffMerkleTrees' keyToTimestamp RangeError (merkleTree.ts:55-61) -> 500."""


__all__ = ["SyncServer", "ParseBodyError", "RangeError"]
