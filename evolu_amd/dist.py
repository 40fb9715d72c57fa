"""The owner-sharding plan of evm_dist_* restated over torch.distributed.

This is NOT a second product path.  The shipped multi-GPU path is the C ABI
(include/evm.h evm_dist_*, driven by evolu_amd/sharded.py and the N-API
addon); bench.py never imports this module.  This file restates the SAME
partition -- bit for bit the same destination rank and local id of every
row -- with torch collectives, so that:

* the multi-process CPU tests (gloo, world_size 2) can check the plan's
  exactness against the unsharded oracle without a GPU, and
* a -m gpu test pins this restatement to evm_dist_directory / hot_owners /
  split / ts_dest / cell_dest (tests/test_gpu_dist_abi.py), so the plan the
  gloo tests prove is the plan the C ABI runs.

The plan (evm_dist.hip):

* owner g lives on rank murmur3(userId_g) mod world (MurmurHash3_x86_32,
  seed 0 -- murmurhash@2.0.1, the hash of timestamp.ts:87-88) as local id
  = its rank among that rank's owners in global order (evm_dist_directory);
* an owner with more than `share` x (all rows / world) rows is hot
  (evm_dist_hot_owners) and lives on EVERY rank as local id hot_base + h,
  hot_base = the largest per-rank owner count (evm_dist_split); each of its
  rows goes to rank murmur3(the 46 timestamp bytes) mod world, so every copy
  of one (owner, timestamp) meets on one rank and INSERT OR IGNORE
  (index.ts:154) and the Merkle XOR stay exact per rank;
* routing keeps (source rank, source order) = the global batch order;
* roots are all-gathered; a split owner's root is the XOR of its partial
  roots (insertIntoMerkleTree is order-independent, merkleTree.test.ts:30-42);
* one owner's client batch splits by cell: rank ((cell * 0x9E3779B1) mod
  2^32 >> 8) mod world (evm_dist_cell_dest), the global PK check by
  timestamp hash (evm_dist_ts_dest).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

_C1, _C2 = np.uint32(0xCC9E2D51), np.uint32(0x1B873593)


def _rotl(x: np.ndarray, r: int) -> np.ndarray:
    return (x << np.uint32(r)) | (x >> np.uint32(32 - r))


def murmur3_rows(rows: np.ndarray) -> np.ndarray:
    """MurmurHash3_x86_32, seed 0, of every row of a uint8 [n, L] array (all
    rows L bytes) -> uint32 [n].  The function of murmurhash@2.0.1 over ASCII
    input (evm_device.hpp murmur3_46, evm_dist.hip murmur3_bytes)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, L = rows.shape
    h = np.zeros(n, dtype=np.uint32)
    nb = L // 4
    with np.errstate(over="ignore"):
        if nb:
            blocks = rows[:, :4 * nb].copy().view("<u4")
            for i in range(nb):
                k = blocks[:, i] * _C1
                k = _rotl(k, 15) * _C2
                h ^= k
                h = _rotl(h, 13) * np.uint32(5) + np.uint32(0xE6546B64)
        rem = L & 3
        if rem:
            tail = rows[:, 4 * nb:].astype(np.uint32)
            k = np.zeros(n, dtype=np.uint32)
            for j in range(rem - 1, -1, -1):
                k ^= tail[:, j] << np.uint32(8 * j)
            k = _rotl(k * _C1, 15) * _C2
            h ^= k
        h ^= np.uint32(L)
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return h


def ts_dest(ts: torch.Tensor, world: int) -> torch.Tensor:
    """Rank of every row by timestamp hash (evm_dist_ts_dest): murmur3 of the
    46 timestamp bytes mod world -> int64 [n]."""
    h = murmur3_rows(ts[:, :46].cpu().numpy())
    return torch.from_numpy((h % np.uint32(world)).astype(np.int64)).to(ts.device)


def cell_dest(cell: torch.Tensor, world: int) -> torch.Tensor:
    """Rank of each cell of a split owner (evm_dist_cell_dest)."""
    c = cell.to(torch.int64) & 0xFFFFFFFF
    return (((c * 0x9E3779B1) & 0xFFFFFFFF) >> 8) % world


class Directory:
    """evm_dist_directory: owner g -> rank murmur3(userId_g) mod world, local
    id = its rank among that rank's owners in global order.  user_ids: uint8
    [n_owners, id_len] (every id id_len bytes); the same on every rank."""

    def __init__(self, user_ids: np.ndarray, world: int):
        self.world = world
        self.n_owners = int(user_ids.shape[0])
        self.dest = (murmur3_rows(user_ids) % np.uint32(world)).astype(np.int64)
        self.local = np.zeros(self.n_owners, dtype=np.int64)
        self.count = np.zeros(world, dtype=np.int64)
        for r in range(world):
            m = self.dest == r
            self.local[m] = np.arange(int(m.sum()))
            self.count[r] = int(m.sum())
        self.per = int(self.count.max()) if world else 0  # evm_dist.hip dir_per


class OwnerMap:
    """Global owner id -> (rank, local owner id), as the C ABI assigns them
    after evm_dist_directory (+ evm_dist_split of the hot owners)."""

    def __init__(self, directory: Directory, rank: int, hot: Optional[np.ndarray] = None):
        self.dir = directory
        self.world, self.rank = directory.world, rank
        self.n_owners = directory.n_owners
        self.hot = np.sort(np.asarray(hot if hot is not None else [], dtype=np.int64))
        self.hot_base = directory.per  # evm_dist_split: the cold slots per rank
        n_hot = int(self.hot.size)
        self.n_local = self.hot_base + n_hot if n_hot else int(directory.count[rank])
        self._hot_ix = np.full(self.n_owners, -1, dtype=np.int64)
        self._hot_ix[self.hot] = np.arange(n_hot)

    def hot_index(self, owner: torch.Tensor) -> torch.Tensor:
        return torch.from_numpy(self._hot_ix[owner.cpu().numpy().astype(np.int64)]).to(owner.device)

    def dest(self, owner: torch.Tensor, ts: torch.Tensor) -> torch.Tensor:
        """Rank of every row (evm_dist.hip bucket_of<SEND>)."""
        o = owner.cpu().numpy().astype(np.int64)
        d = torch.from_numpy(self.dir.dest[o]).to(owner.device)
        hot = self.hot_index(owner) >= 0
        if bool(hot.any()):
            d = torch.where(hot, ts_dest(ts, self.world), d)
        return d

    def local(self, owner: torch.Tensor) -> torch.Tensor:
        """Local owner ids of the rows this rank received (evm_dist.hip local_of)."""
        o = owner.cpu().numpy().astype(np.int64)
        loc = torch.from_numpy(self.dir.local[o]).to(owner.device)
        h = self.hot_index(owner)
        return torch.where(h >= 0, self.hot_base + h, loc).to(torch.int32)

    def owners_here(self) -> np.ndarray:
        """Global owner of every local id (-1: an unused slot; a split owner's own cold slot stays empty)."""
        g = np.full(self.n_local, -1, dtype=np.int64)
        mine = np.flatnonzero(self.dir.dest == self.rank)
        g[self.dir.local[mine]] = mine
        if self.hot.size:
            g[np.isin(g, self.hot) & (np.arange(self.n_local) < self.hot_base)] = -1
            g[self.hot_base:] = self.hot
        return g


def owner_counts(owner: torch.Tensor, n_owners: int, group=None) -> torch.Tensor:
    """Rows per global owner over all ranks (all_reduce of local counts)."""
    c = torch.bincount(owner.to(torch.int64), minlength=n_owners)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(c, group=group)
    return c


def hot_owners(counts: torch.Tensor, world: int, share: float = 0.25) -> np.ndarray:
    """evm_dist_hot_owners: the owners holding more than `share` of one rank's
    fair share of all rows (threshold truncated to an integer), sorted."""
    if world <= 1:
        return np.zeros(0, dtype=np.int64)
    c = counts.cpu().numpy().astype(np.int64)
    thr = int(share * (float(c.sum()) / world))
    return np.flatnonzero(c > thr).astype(np.int64)


def route_by_owner(ts: torch.Tensor, owner: torch.Tensor, dest: torch.Tensor, group=None
                   ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """All-to-all of rows to rank dest[i] (OwnerMap.dest, or a cell / timestamp
    rank).  Returns (ts_recv, owner_recv, src_rank, src_index) in (source
    rank, source order) = the global batch order when each rank's input is
    its slice of the batch in rank order (evm_dist_route + evm_dist_take)."""
    world = dist.get_world_size(group)
    dev = ts.device
    n, stride = ts.shape
    dest = dest.to(torch.int64)
    order = torch.argsort(dest, stable=True)
    send_counts = torch.bincount(dest, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc = send_counts.tolist()
    rc = recv_counts.tolist()
    m = sum(rc)
    ts_send = ts.index_select(0, order).contiguous()
    ts_recv = torch.empty((m, stride), dtype=ts.dtype, device=dev)
    dist.all_to_all_single(ts_recv.view(-1), ts_send.view(-1), [c * stride for c in rc], [c * stride for c in sc],
                           group=group)
    meta_send = torch.stack([owner.index_select(0, order).to(torch.int64), order.to(torch.int64)], 1).contiguous()
    meta_recv = torch.empty((m, 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(meta_recv.view(-1), meta_send.view(-1), [2 * c for c in rc], [2 * c for c in sc],
                           group=group)
    src_rank = torch.repeat_interleave(torch.arange(world, device=dev), recv_counts.to(dev))
    return ts_recv, meta_recv[:, 0], src_rank, meta_recv[:, 1]


def route_back(values: torch.Tensor, src_rank: torch.Tensor, src_index: torch.Tensor, n_local: int,
               group=None) -> torch.Tensor:
    """Per-row results back to the rank and position each row came from
    (evm_dist_return)."""
    world = dist.get_world_size(group)
    dev = values.device
    send_counts = torch.bincount(src_rank, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    pay = torch.stack([src_index, values.to(torch.int64)], 1).contiguous()  # (already grouped by source)
    got = torch.empty((sum(rc), 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(got.view(-1), pay.view(-1), [2 * c for c in rc], [2 * c for c in sc], group=group)
    out = torch.zeros(n_local, dtype=torch.int64, device=dev)
    out[got[:, 0]] = got[:, 1]
    return out.to(values.dtype)


def gather_roots(root: torch.Tensor, present: torch.Tensor, omap: OwnerMap, group=None):
    """evm_dist_gather_roots: every rank's local roots (n_local of them) ->
    every global owner's (root int32, present bool); a split owner's root is
    the XOR of its partial roots, present if any part is."""
    world = dist.get_world_size(group)
    dev = root.device
    per = omap.hot_base + int(omap.hot.size) if omap.hot.size else omap.dir.per
    mine = torch.zeros(per, dtype=torch.int64, device=dev)
    mine[: root.numel()] = (root.to(torch.int64) & 0xFFFFFFFF) | (present.to(torch.int64) << 32)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    allr = torch.stack(parts).cpu().numpy()  # [rank, slot]
    g = allr[omap.dir.dest, omap.dir.local]
    for h, o in enumerate(omap.hot.tolist()):
        col = allr[:, omap.hot_base + h]
        x = 0
        for v in col:
            x ^= int(v) & 0xFFFFFFFF
        g[o] = x | (int(any((v >> 32) != 0 for v in col)) << 32)
    x = g & 0xFFFFFFFF
    x = np.where(x >= 2 ** 31, x - 2 ** 32, x)
    return torch.from_numpy(x.astype(np.int32)).to(dev), torch.from_numpy((g >> 32) != 0).to(dev)


def all_gather_var(t: torch.Tensor, group=None):
    """All-gather of a 1-D tensor whose length differs per rank -> list of
    the ranks' tensors."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sz = [int(x.item()) for x in sizes]
    cap = max(max(sz), 1)
    pad = torch.zeros(cap, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return [p[:k] for p, k in zip(parts, sz)]


def gather_leaf_parts(off: torch.Tensor, code: torch.Tensor, xr: torch.Tensor, group=None):
    """Every rank's partial leaf lists of the split owners (off int64[nh+1]
    from 0, code int64[L], xr int[L]) -> [(off, code, xr)] per rank
    (evm_dist_merge_trees gathers the same lists)."""
    nh = off.numel() - 1
    payload = torch.cat([off.to(torch.int64), code.to(torch.int64), xr.to(torch.int64)])
    out = []
    for a in all_gather_var(payload, group):
        L = (a.numel() - (nh + 1)) // 2
        out.append((a[: nh + 1], a[nh + 1: nh + 1 + L], a[nh + 1 + L:].to(torch.int32)))
    return out


def lex_order(key: torch.Tensor) -> torch.Tensor:
    """Permutation sorting rows of an int64 [m, k] key matrix lexicographically
    (stable passes from the last column)."""
    order = torch.arange(key.shape[0], device=key.device)
    for c in range(key.shape[1] - 1, -1, -1):
        order = order[torch.argsort(key[order, c], stable=True)]
    return order


def gather_selection(sel_off: torch.Tensor, sel_id: torch.Tensor, sel_key: torch.Tensor, group=None):
    """evm_dist_merge_select: each rank's share of the split owners' getMessages
    rows (sel_off int64[nh+1], sel_id int64[m], sel_key int64[m, 3] = the
    rows' order keys) -> (off, ids) of every split owner's rows from all ranks
    in timestamp order (ORDER BY "timestamp", index.ts:101; equal keys: lower
    rank first), the same on every rank."""
    nh = sel_off.numel() - 1
    payload = torch.cat([sel_off.to(torch.int64), sel_id.to(torch.int64), sel_key.to(torch.int64).reshape(-1)])
    owners, ranks, ids, keys = [], [], [], []
    for r, a in enumerate(all_gather_var(payload, group)):
        po = a[: nh + 1]
        m = int(po[-1].item())
        ids.append(a[nh + 1: nh + 1 + m])
        keys.append(a[nh + 1 + m: nh + 1 + 4 * m].reshape(m, 3))
        counts = po[1:] - po[:-1]
        owners.append(torch.repeat_interleave(torch.arange(nh, device=a.device), counts))
        ranks.append(torch.full((m,), r, dtype=torch.int64, device=a.device))
    owner = torch.cat(owners)
    ids = torch.cat(ids)
    keys = torch.cat(keys)
    order = lex_order(torch.cat([owner[:, None], keys, torch.cat(ranks)[:, None]], 1))
    counts = torch.bincount(owner, minlength=nh)
    off = torch.zeros(nh + 1, dtype=torch.int64, device=ids.device)
    off[1:] = torch.cumsum(counts, 0)
    return off, ids[order]


# ---------------------------------------------------------------------------
# Client: ONE owner's applyMessages batch over every rank (SURVEY 8(e), config
# 5-C).  The LWW decisions of applyMessages.ts:26-131 are per cell, so every
# row of a cell goes to one rank (in global batch order) and each cell's
# running max stays exact; the global __message PK case (one timestamp in two
# cells) is checked on the rank the timestamp hash picks, so every copy of one
# timestamp meets there; the tree is the XOR-combination of the per-rank
# partial trees (insertIntoMerkleTree is order-independent).
# ---------------------------------------------------------------------------
EVM_OK, EVM_ECOLLISION = 0, 3


def split_apply(ts: torch.Tensor, cell: torch.Tensor, n_cells: int, apply_local, check_local, group=None):
    """applyMessages of one owner's batch split over the ranks by cell
    (sharded.split_apply's plan: evm_dist_ts_dest / cell_dest / route /
    return / split_winners / agree_status).

    ts (n, stride) uint8 / cell (n,) int: this rank's slice of the batch; the
    batch is the ranks' slices in rank order.
    apply_local(ts_r, cell_r) -> (flags u8[n_r], winner int[n_cells] index
        into ts_r or -1, partial, status);
    check_local(ts_t, cell_t) -> bool: a timestamp with two cells.
    Returns (flags u8[n] of this rank's slice, winner int64[n_cells] = global
    batch index or -1, partial, status); status is the same on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = ts.device
    n = ts.shape[0]
    cell64 = cell.to(torch.int64)
    # the global PK check, by timestamp hash
    t_t, c_t, _, _ = route_by_owner(ts, cell64, ts_dest(ts, world), group=group)
    collide = bool(check_local(t_t, c_t)) if t_t.shape[0] else False
    # the LWW decisions, by cell
    ts_c, cell_c, src_rank, src_idx = route_by_owner(ts, cell64, cell_dest(cell64, world), group=group)
    flags_c, win_c, part, st = apply_local(ts_c, cell_c)
    status = torch.tensor([max(int(st), EVM_ECOLLISION if collide else EVM_OK)], dtype=torch.int64, device=dev)
    dist.all_reduce(status, op=dist.ReduceOp.MAX, group=group)
    status = int(status.item())
    if status != EVM_OK:
        return torch.zeros(n, dtype=torch.uint8, device=dev), None, None, status
    flags = route_back(flags_c.to(torch.int64), src_rank, src_idx, n, group=group).to(torch.uint8)
    # winners: local index -> global batch index (rank-major)
    sizes = torch.tensor([n], dtype=torch.int64, device=dev)
    alls = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(alls, sizes, group=group)
    base = torch.cumsum(torch.cat(alls), 0) - torch.cat(alls)
    gidx = base.index_select(0, src_rank) + src_idx
    w = win_c.to(torch.int64)
    mine = cell_dest(torch.arange(n_cells, device=dev), world) == rank
    glob = torch.where((w >= 0) & mine, gidx.index_select(0, w.clamp(min=0)) if gidx.numel() else w,
                       torch.full_like(w, -1))
    dist.all_reduce(glob, op=dist.ReduceOp.MAX, group=group)
    return flags, glob, part, status
