"""The sync server's addMessages + getMessages over owners sharded across GPUs
(apps/server/src/index.ts:138-202 per owner).

One process (or loopback thread) per GPU.  Every owner lives on the rank
murmur3(userId) mod G picks (evm_dist_directory, computed on the device from
the userId strings), as a dense local id.  A round of requests arrives on any
rank; `ingest` routes every message to its owner's rank (one all-to-all of
counts, one exchange of 32-B packed records, evm_dist_route), takes the rows
out with local owner ids (evm_dist_take) and runs addMessages on the local
store (evm_server_ingest); `select` is getMessages against the owners'
client trees (evm_server_select); `roots` all-gathers every owner's root
(evm_dist_gather_roots) so any rank can answer for any owner's tree hash.
No step needs a host copy of message data.
"""
from __future__ import annotations

from typing import Optional

import torch

from .engine import Dist, Engine


class ShardedServer:
    """Owners 0..n_owners-1 (their userId strings on the device) over the
    ranks of `dd`; a store for this rank's owners."""

    def __init__(self, eng: Engine, dd: Dist, user_ids: torch.Tensor, id_len: int = 21):
        self.eng, self.dd = eng, dd
        self.n_owners = int(user_ids.shape[0])
        self.dest, self.local = dd.directory((user_ids, id_len))
        self.n_local = dd.n_local
        # global ids of this rank's owners in local-id order
        self.owners_here = torch.nonzero(self.dest == dd.rank).flatten().to(torch.int32)
        assert self.owners_here.numel() == self.n_local
        self.store = None

    def new_store(self):
        if self.store is not None:
            self.store.free()
        self.store = self.eng.store_new(self.n_local)
        return self.store

    def route(self, ts: torch.Tensor, owner: torch.Tensor, out=None):
        """Rows (global owner ids) of this rank's slice -> the rows of this
        rank's owners from every rank: (ts, local owner int32), batch order."""
        n = self.dd.route(ts, owner)
        t, o, _, _, _ = self.dd.take(aux=False, src=False, out=out)
        return t[:n], o[:n]

    def ingest(self, ts: torch.Tensor, owner: torch.Tensor, id_base: int = 0, flags: Optional[torch.Tensor] = None,
               out=None):
        """addMessages for a round: route + take + evm_server_ingest into this
        rank's store.  Returns (received ts, local owners, flags)."""
        t, o = self.route(ts, owner, out=out)
        if self.store is None:
            self.new_store()
        f, _ = self.store.ingest(t, o, id_base, flags=flags)
        return t, o, f

    def select(self, client, node: torch.Tensor, active: Optional[torch.Tensor] = None):
        """getMessages for this rank's owners (client: Trees over the local
        owners; node: uint8 [n_local * 16] requester nodeIds)."""
        return self.store.select(client, node, active)

    def roots(self):
        """Every owner's (root int32, present bool), on the device."""
        return self.dd.gather_roots(self.store.tree(), self.n_owners)

    def close(self):
        if self.store is not None:
            self.store.free()
            self.store = None
