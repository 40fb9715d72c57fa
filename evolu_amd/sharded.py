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

Hot owners (BASELINE config 5: Zipf 1.2, the top owner ~18 % of all rows)
would pin one rank: `split_hot` finds them from a round's rows
(evm_dist_hot_owners) and splits them over every rank (evm_dist_split):
each of their rows goes to the rank its timestamp hash picks, their trees are
XOR merges of the per-rank partial trees (evm_dist_merge_trees), and their
getMessages rows are each rank's share after the full-tree bound, merged in
timestamp order (evm_dist_merge_select).  `split_apply` is the client side:
one owner's applyMessages batch split over the ranks by cell.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
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
        self.hot = np.zeros(0, dtype=np.uint32)  # split owners (global ids), local hot_base + h
        self.hot_base = self.n_local

    def split_hot(self, owner: torch.Tensor, share: float = 0.25, cap: int = 4096) -> np.ndarray:
        """Collective: the owners holding more than `share` of one rank's fair
        share of this round's rows (owner: this rank's rows, global ids) are
        split over every rank.  Local ids: [0, n_cold) this rank's own owners,
        then hot_base + h for split owner h.  Start a new store afterwards."""
        return self.set_hot(self.dd.hot_owners(owner, self.n_owners, share, cap))

    def set_hot(self, hot) -> np.ndarray:
        self.hot = np.asarray(hot, dtype=np.uint32)
        self.hot_base = self.dd.split(self.hot, self.n_owners)
        self.n_local = self.hot_base + int(self.hot.size)
        return self.hot

    def local_owners(self) -> torch.Tensor:
        """Global owner of every local id (-1: an unused slot) on the device."""
        g = torch.full((self.n_local,), -1, dtype=torch.int64, device=self.owners_here.device)
        n_cold = self.owners_here.numel()
        g[:n_cold] = self.owners_here.to(torch.int64)
        if self.hot.size:
            hot = torch.from_numpy(self.hot.astype(np.int64)).to(g.device)
            g[self.hot_base:] = hot
            # a split owner's own cold slot stays empty
            g[:n_cold] = torch.where(torch.isin(g[:n_cold], hot), torch.full_like(g[:n_cold], -1), g[:n_cold])
        return g

    def client_trees(self, partial):
        """Collective: client trees over the local ids from this rank's
        partial ones (each owner's known messages that were routed here):
        a cold owner's partial tree is its whole tree; a split owner's
        slot gets the XOR merge of every rank's part (evm_dist_merge_trees),
        the same on every rank -- what select_split expects.  Without split
        owners that is `partial` itself."""
        nh, base = int(self.hot.size), self.hot_base
        if not nh:
            return partial
        full = self.dd.merge_trees(partial, base, nh)
        off_c, code_c, xr_c = partial.slice_device(0, base)
        off_h, code_h, xr_h = full.slice_device(0, nh)
        full.free()
        off = torch.cat([off_c, off_h[1:] + off_c[-1]])
        return self.eng.tree_from_device_leaves(off, torch.cat([code_c, code_h]), torch.cat([xr_c, xr_h]))

    def new_store(self):
        if self.store is not None:
            self.store.free()
        self.store = self.eng.store_new(self.n_local)
        return self.store

    def route(self, ts: torch.Tensor, owner: torch.Tensor, out=None):
        """Rows (global owner ids) of this rank's slice -> the rows of this
        rank's owners from every rank: (ts, local owner int32), batch order."""
        # (24-B records: no aux, no sources; this rank's own rows read from ts by the take)
        n = self.dd.route(ts, owner, need_src=False, keep_input=True)
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

    def route_ingest(self, ts: torch.Tensor, owner: torch.Tensor, id_base: int = 0,
                     flags: Optional[torch.Tensor] = None) -> torch.Tensor:
        """addMessages for a round without rebuilding the received rows:
        route (24-B records) + evm_dist_ingest into this rank's store.
        Returns the flags in receive order (ids id_base + receive index);
        `take_routed` gives the rows themselves when a caller needs them
        (this rank's own rows are read from `ts` by the ingest and by
        take_routed: the caller keeps it until then)."""
        self.dd.route(ts, owner, need_src=False, keep_input=True)
        if self.store is None:
            self.new_store()
        return self.dd.ingest(self.store, id_base, flags)

    def take_routed(self, out=None):
        """The last route's rows (ts, local owner int32) in receive order."""
        t, o, _, _, _ = self.dd.take(aux=False, src=False, out=out)
        return t, o

    def select(self, client, node: torch.Tensor, active: Optional[torch.Tensor] = None):
        """getMessages for this rank's owners (client: Trees over the local
        owners; node: uint8 [n_local * 16] requester nodeIds).  Without split
        owners -> (diff, sel_off, sel_id); with them see select_split."""
        if self.hot.size:
            return self.select_split(client, node)
        return self.store.select(client, node, active)

    def select_split(self, client, node: torch.Tensor):
        """getMessages when owners are split (index.ts:173-202): a split
        owner's diff is that of its FULL server tree (the per-rank partial
        trees merged) against its client tree, each rank selects its share
        after that bound, and the shares merge in timestamp order.  client:
        Trees over the local ids (the hot slots: each split owner's full
        client tree, the same on every rank).  Returns (diff int64[n_local],
        (off, ids) over the local ids with the hot slots' rows this rank's
        share, (hot_off, hot_ids) every rank's rows of the split owners in
        timestamp order -- the same on every rank)."""
        eng, nh, base = self.eng, int(self.hot.size), self.hot_base
        tree = self.store.tree()
        diff = eng.merkle_diff(tree, client)
        full = self.dd.merge_trees(tree, base, nh)
        # the client's trees of the split owners sit in the hot slots of `client`
        sub = eng.tree_from_device_leaves(*client.slice_device(base, nh))
        diff[base:base + nh] = eng.merkle_diff(full, sub)
        sub.free()
        full.free()
        off, ids, keys = self.store.select_after(diff, node, keys=True)
        hot = self.dd.merge_select(off[base:base + nh + 1].contiguous(), ids, keys)
        return diff, (off, ids), hot

    def roots(self):
        """Every owner's (root int32, present bool), on the device."""
        return self.dd.gather_roots(self.store.tree(), self.n_owners)

    def close(self):
        if self.store is not None:
            self.store.free()
            self.store = None


def split_apply(eng: Engine, dd: Dist, ts: torch.Tensor, cell: torch.Tensor, n_cells: int, tree_in=None,
                prior_ts: Optional[torch.Tensor] = None, prior_present: Optional[torch.Tensor] = None,
                stored_ts: Optional[torch.Tensor] = None, stored_cell: Optional[torch.Tensor] = None):
    """applyMessages (applyMessages.ts:26-131) of ONE owner's batch split over
    the ranks by cell, through the evm_dist C ABI.

    ts (n, 48) uint8 / cell (n,) int32 on the device: this rank's slice of the
    batch (the batch = the ranks' slices in rank order).  The LWW decisions are
    per cell, so every row goes to its cell's rank in global batch order
    (evm_dist_cell_dest + route); the global __message PK check (one timestamp
    in two cells) runs on the rank the timestamp hash picks; statuses combine
    over ranks.  The owner's DB state is that of a single-rank apply: every
    cell's current max (prior_ts [n_cells, 48] + prior_present,
    applyMessages.ts:34-40) and the __message rows holding a batch timestamp
    (stored_ts / stored_cell, :42-45) -- the SAME tensors on every rank; each
    rank decides its own cells against them (evm_apply_batch_ex), so a stored
    row of another cell is the global-PK case wherever it lands.  Returns
    (flags u8[n] of this rank's slice, winner int64 [n_cells] global batch
    index or -1, tree = tree_in + every rank's partial tree, status) -- the
    same winner, tree and status on every rank."""
    from . import _lib

    n = ts.shape[0]
    zero = torch.zeros(max(n, 1), dtype=torch.int32, device=ts.device)[:n]
    cell = cell.to(torch.int32).contiguous()
    # the PK check: every copy of one timestamp meets on one rank
    dd.route(ts, zero, aux=cell, dest=dd.ts_dest(ts))
    t_t, _, c_t, _, _ = dd.take(src=False)
    collide = eng.cross_cell_check(t_t.contiguous(), c_t.contiguous(), n_cells) if t_t.shape[0] else False
    # the LWW decisions: every row of a cell on the cell's rank, in batch order
    dd.route(ts, zero, aux=cell, dest=dd.cell_dest(cell))
    t_c, _, c_c, _, _ = dd.take(src=False)
    empty = eng.tree_new(1)
    if t_c.shape[0]:
        flags_c, win_c, part, st = eng.apply_batch(empty, t_c.contiguous(), c_c.contiguous(), n_cells,
                                                   prior_ts=prior_ts, prior_present=prior_present,
                                                   raise_on_error=False, stored_ts=stored_ts, stored_cell=stored_cell)
    else:
        flags_c = torch.zeros(0, dtype=torch.uint8, device=ts.device)
        win_c = torch.full((n_cells,), -1, dtype=torch.int32, device=ts.device)
        part, st = empty, _lib.EVM_OK
    local = max(int(st), _lib.EVM_ECOLLISION if collide else _lib.EVM_OK)
    status = dd.agree_status(local)
    if status != _lib.EVM_OK:
        return torch.zeros(n, dtype=torch.uint8, device=ts.device), None, None, status
    flags = dd.send_back(flags_c, n)
    winner = dd.split_winners(win_c, n_cells)
    tree = dd.merge_trees(part, 0, 1)
    if tree_in is not None:
        merged = eng.tree_merge(tree_in, tree)
        tree.free()
        tree = merged
    return flags, winner, tree, status
