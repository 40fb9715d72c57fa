"""Owner-sharded multi-GPU plumbing (one process per GPU, torch.distributed).

Owners are independent in the whole hot path: each owner is its own client
database for applyMessages (applyMessages.ts:26-131) and the server keys
rows and trees by userId (apps/server/src/index.ts:64-75).  So the engine
scales by owner: rank = owner mod world (owner ids are dense integers the
host assigns, e.g. from murmur3(ownerId)), and

* messages that arrive on the wrong rank are routed with ONE all_to_all of
  counts and ONE all_to_all of payload (RCCL over xGMI on MI355X; gloo on
  CPU for tests).  Receive buffers are ordered by source rank and keep each
  source's order, so the global batch order (rank-major) is preserved --
  which the reference's first-occurrence rules depend on;
* per-owner roots are all-gathered (RCCL has no XOR reduction; nothing needs
  one: every owner lives on exactly one rank).

Hot owners (a skewed owner distribution, BASELINE config 5: Zipf 1.2, the
top owner ~18 % of all messages) would pin one rank.  `OwnerMap` splits
them: a hot owner lives on every rank, and each of its messages goes to the
rank a hash of its timestamp bytes picks.  Every copy of one (owner,
timestamp) therefore lands on one rank, so the server's INSERT OR IGNORE
dedup (index.ts:154) stays exact per rank; the owner's Merkle tree is the
XOR-combination of its per-rank partial trees (insertIntoMerkleTree is
order-independent, merkleTree.test.ts:30-42): partial roots XOR together
(`gather_hot_roots`), partial leaf lists merge on the device
(`merge_hot_trees`, evm_tree_merge).

This module is the torch.distributed formulation (gloo on CPU for the
multi-process tests, RCCL through torch on GPUs).  The product path for a
caller without torch is the same plan behind the C ABI: evm_dist_route /
take / gather_roots / hot_owners / split / merge_trees / merge_select /
return / split_winners (include/evm.h), driven by evolu_amd/sharded.py.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def owner_rank(owner: torch.Tensor, world: int) -> torch.Tensor:
    return (owner % world).to(torch.int64)


def local_owner(owner: torch.Tensor, world: int) -> torch.Tensor:
    """Dense per-rank owner id (owner // world)."""
    return (owner // world).to(torch.int32)


def ts_route_hash(ts: torch.Tensor) -> torch.Tensor:
    """A fixed 63-bit mix of the 46 timestamp bytes of each row (routing only:
    equal timestamps -> equal hashes)."""
    n, stride = ts.shape
    b = ts[:, :46].to(torch.int64)
    h = torch.zeros(n, dtype=torch.int64, device=ts.device)
    for k in range(0, 46, 7):  # 7 bytes per step: no sign trouble in int64
        w = torch.zeros(n, dtype=torch.int64, device=ts.device)
        for j in range(k, min(k + 7, 46)):
            w = w | (b[:, j] << (8 * (j - k)))
        h = ((h * 1000003) ^ w) & 0x7FFFFFFFFFFFFFFF
    return h


class OwnerMap:
    """Global owner id -> (rank, local owner id).

    A cold owner o lives on rank o % world as local owner o // world.  Hot
    owner hot[h] lives on every rank as local owner `per + h` (per = the
    cold slots per rank) and takes the messages whose timestamp hash picks
    that rank."""

    def __init__(self, n_owners: int, world: int, rank: int, hot: Optional[torch.Tensor] = None):
        self.n_owners = n_owners
        self.world = world
        self.rank = rank
        self.per = (n_owners + world - 1) // world
        self.hot = (hot if hot is not None else torch.zeros(0, dtype=torch.int64)).to(torch.int64).sort().values
        self.n_local = self.per + int(self.hot.numel())

    def is_hot(self, owner: torch.Tensor) -> torch.Tensor:
        if self.hot.numel() == 0:
            return torch.zeros_like(owner, dtype=torch.bool)
        hot = self.hot.to(owner.device)
        i = torch.searchsorted(hot, owner.to(torch.int64)).clamp(max=hot.numel() - 1)
        return hot[i] == owner

    def dest(self, owner: torch.Tensor, ts: torch.Tensor) -> torch.Tensor:
        d = (owner.to(torch.int64) % self.world)
        hot = self.is_hot(owner)
        if bool(hot.any()):
            d = torch.where(hot, ts_route_hash(ts) % self.world, d)
        return d

    def local(self, owner: torch.Tensor) -> torch.Tensor:
        """Local owner ids of messages this rank received."""
        loc = owner.to(torch.int64) // self.world
        hot = self.is_hot(owner)
        if bool(hot.any()):
            h = torch.searchsorted(self.hot.to(owner.device), owner.to(torch.int64))
            loc = torch.where(hot, self.per + h, loc)
        return loc.to(torch.int32)


def owner_counts(owner: torch.Tensor, n_owners: int, group=None) -> torch.Tensor:
    """Messages per global owner over all ranks (all_reduce of local counts)."""
    c = torch.bincount(owner.to(torch.int64), minlength=n_owners)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(c, group=group)
    return c


def hot_owners(counts: torch.Tensor, world: int, share: float = 0.25) -> torch.Tensor:
    """Owners holding more than `share` of one rank's fair share of messages."""
    if world <= 1:
        return torch.zeros(0, dtype=torch.int64)
    fair = float(counts.sum().item()) / world
    return torch.nonzero(counts > share * fair).flatten()  # (on the counts' device)


def route_by_owner(ts: torch.Tensor, owner: torch.Tensor, group=None, dest: Optional[torch.Tensor] = None
                   ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """All-to-all routing of messages to their owner's rank.

    ts: (n, stride) uint8 timestamp rows, owner: (n,) int64 global owner ids,
    both on this rank; dest: the rank of every message (default owner %
    world; OwnerMap.dest splits hot owners).  Returns (ts_recv, owner_recv,
    src_rank, src_index): the messages this rank owns, in global batch
    order, with where they came from (to send per-message results back with
    `route_back`).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = ts.device
    n, stride = ts.shape
    if dest is None:
        dest = owner_rank(owner, world)
    order = torch.argsort(dest, stable=True)
    send_counts = torch.bincount(dest, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc = send_counts.tolist()
    rc = recv_counts.tolist()
    m = sum(rc)
    ts_send = ts.index_select(0, order).contiguous()
    ts_recv = torch.empty((m, stride), dtype=ts.dtype, device=dev)
    # uint8 rows travel as int64 words when the stride allows (fewer, larger elements)
    if stride % 8 == 0:
        dist.all_to_all_single(ts_recv.view(torch.int64).view(-1), ts_send.view(torch.int64).view(-1),
                               [c * stride // 8 for c in rc], [c * stride // 8 for c in sc], group=group)
    else:
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
    """Returns per-message results (e.g. flags) to the rank and position each
    message came from (inverse of `route_by_owner`)."""
    world = dist.get_world_size(group)
    dev = values.device
    order = torch.argsort(src_rank, stable=True)  # already grouped by source; keeps it explicit
    send_counts = torch.bincount(src_rank, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    pay = torch.stack([src_index.index_select(0, order), values.index_select(0, order).to(torch.int64)], 1).contiguous()
    got = torch.empty((sum(rc), 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(got.view(-1), pay.view(-1), [2 * c for c in rc], [2 * c for c in sc], group=group)
    out = torch.zeros(n_local, dtype=torch.int64, device=dev)
    out[got[:, 0]] = got[:, 1]
    return out.to(values.dtype)


def gather_roots(root: torch.Tensor, present: torch.Tensor, n_owners_global: int, group=None):
    """All-gather of per-owner roots: local owner j of rank r is global owner
    j * world + r.  Returns (root int32[n_owners_global], present bool[...])."""
    world = dist.get_world_size(group)
    dev = root.device
    per = (n_owners_global + world - 1) // world
    pad_r = torch.zeros(per, dtype=torch.int64, device=dev)
    pad_r[: root.numel()] = root.to(torch.int64) | (present.to(torch.int64) << 32)
    allr = [torch.empty_like(pad_r) for _ in range(world)]
    dist.all_gather(allr, pad_r, group=group)
    g = torch.stack(allr, 1).reshape(-1)[:n_owners_global]  # row j = local owner j of every rank
    return (g & 0xFFFFFFFF).to(torch.int64).to(torch.int32), (g >> 32) != 0


def gather_hot_roots(root: torch.Tensor, present: torch.Tensor, omap: OwnerMap, group=None):
    """Roots of the split owners: the XOR of the per-rank partial roots
    (present if any part is).  root/present: this rank's local roots."""
    nh = int(omap.hot.numel())
    dev = root.device
    mine = torch.stack([root[omap.per:omap.per + nh].to(torch.int64) & 0xFFFFFFFF,
                        present[omap.per:omap.per + nh].to(torch.int64)], 1).contiguous()
    allp = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(allp, mine, group=group)
    x = torch.zeros(nh, dtype=torch.int64, device=dev)
    p = torch.zeros(nh, dtype=torch.bool, device=dev)
    for t in allp:
        x = x ^ t[:, 0]
        p = p | (t[:, 1] != 0)
    x = torch.where(x >= 2 ** 31, x - 2 ** 32, x)
    return x.to(torch.int32), p


def all_gather_var(t: torch.Tensor, group=None):
    """All-gather of a 1-D tensor whose length differs per rank -> list of
    the ranks' tensors (same device: RCCL device-to-device, gloo on CPU)."""
    world = dist.get_world_size(group)
    home = t.device
    if dist.get_backend(group) == "gloo" and home.type != "cpu":
        t = t.cpu()  # gloo (the CPU tests, ranks sharing one GPU) gathers host tensors
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sz = [int(x.item()) for x in sizes]
    cap = max(max(sz), 1)
    pad = torch.zeros(cap, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return [p[:k].to(home) for p, k in zip(parts, sz)]


def gather_leaf_parts(off: torch.Tensor, code: torch.Tensor, xr: torch.Tensor, group=None):
    """Every rank's partial leaf lists of the split owners (off int64[nh+1]
    from 0, code int64[L], xr int32/int64[L]) -> [(off, code, xr)] per rank,
    in one variable-size all-gather (device buffers stay on the device)."""
    nh = off.numel() - 1
    L = code.numel()
    payload = torch.cat([off.to(torch.int64), code.to(torch.int64), xr.to(torch.int64)])
    out = []
    for a in all_gather_var(payload, group):
        L = (a.numel() - (nh + 1)) // 2
        out.append((a[: nh + 1], a[nh + 1: nh + 1 + L], a[nh + 1 + L:].to(torch.int32)))
    return out


def merge_hot_trees(eng, trees, omap: OwnerMap, group=None):
    """Full trees of the split owners on every rank: the per-rank partial
    leaf lists of the hot local owners (evm_tree_slice, device) are
    all-gathered over RCCL and XOR-merged on the device (evm_tree_from_device_
    leaves + evm_tree_merge).  Returns an engine Trees with one owner per hot
    owner (in omap.hot order)."""
    nh = int(omap.hot.numel())
    off, code, xr = trees.slice_device(omap.per, nh)
    merged = None
    for po, pc, px in gather_leaf_parts(off, code, xr, group):
        part = eng.tree_from_device_leaves(po, pc, px)
        merged = part if merged is None else eng.tree_merge(merged, part)
    return merged


def lex_order(key: torch.Tensor) -> torch.Tensor:
    """Permutation sorting rows of an int64 [m, k] key matrix lexicographically
    (stable passes from the last column)."""
    order = torch.arange(key.shape[0], device=key.device)
    for c in range(key.shape[1] - 1, -1, -1):
        order = order[torch.argsort(key[order, c], stable=True)]
    return order


def gather_selection(sel_off: torch.Tensor, sel_id: torch.Tensor, sel_key: torch.Tensor, group=None):
    """getMessages rows of owners split over ranks: each rank selected its
    share (sel_off int64[nh+1], sel_id int64[m], sel_key int64[m, 3] = the
    rows' order keys); returns (off, ids) of every split owner's rows from all
    ranks in timestamp order (ORDER BY "timestamp", index.ts:101), the same
    on every rank."""
    nh = sel_off.numel() - 1
    payload = torch.cat([sel_off.to(torch.int64), sel_id.to(torch.int64), sel_key.to(torch.int64).reshape(-1)])
    owners, ids, keys = [], [], []
    for a in all_gather_var(payload, group):
        po = a[: nh + 1]
        m = int(po[-1].item())
        ids.append(a[nh + 1: nh + 1 + m])
        keys.append(a[nh + 1 + m: nh + 1 + 4 * m].reshape(m, 3))
        counts = po[1:] - po[:-1]
        owners.append(torch.repeat_interleave(torch.arange(nh, device=a.device), counts))
    owner = torch.cat(owners)
    ids = torch.cat(ids)
    keys = torch.cat(keys)
    order = lex_order(torch.cat([owner[:, None], keys], 1))
    counts = torch.bincount(owner, minlength=nh)
    off = torch.zeros(nh + 1, dtype=torch.int64, device=ids.device)
    off[1:] = torch.cumsum(counts, 0)
    return off, ids[order]


def split_get_messages(eng, store, client_local, client_hot, node: torch.Tensor, omap: OwnerMap, group=None):
    """getMessages (index.ts:173-202) for every local owner when hot owners
    are split over ranks.  A cold owner lives on one rank: its diff is the
    one of its full tree.  A hot owner's diff must be the diff of its FULL
    server tree against the client's full tree -- a diff of a partial tree is
    not the diff of the whole -- so the partial trees are merged first
    (merge_hot_trees), the diff is computed on the merge (identical on every
    rank), each rank selects its share after that bound (with the NOT LIKE
    node filter) and the shares merge in timestamp order.

    client_local: Trees over the local owners (the client trees of the cold
    owners; the hot slots are ignored); client_hot: Trees of the hot owners'
    full client trees, omap.hot order; node: uint8 [n_local * 16].
    Returns (diff int64[n_local] with the hot slots' full-tree diffs,
    cold (off, ids) over local owners -- hot slots empty -- and hot (off,
    ids) over omap.hot, all ranks' rows merged)."""
    nh = int(omap.hot.numel())
    diff = eng.merkle_diff(store.tree(), client_local)
    if nh:
        merged = merge_hot_trees(eng, store.tree(), omap, group)
        diff[omap.per: omap.per + nh] = eng.merkle_diff(merged, client_hot)
        merged.free()
    active = torch.ones(omap.n_local, dtype=torch.uint8, device=diff.device)
    active[omap.per: omap.per + nh] = 0
    off_c, ids_c, _ = store.select_after(diff, node, active=active)
    if not nh:
        return diff, (off_c, ids_c), None
    hot_only = torch.zeros_like(active)
    hot_only[omap.per: omap.per + nh] = 1
    off_h, ids_h, key_h = store.select_after(diff, node, active=hot_only, keys=True)
    part_off = off_h[omap.per: omap.per + nh + 1] - off_h[omap.per]
    return diff, (off_c, ids_c), gather_selection(part_off, ids_h, key_h, group)


# ---------------------------------------------------------------------------
# Client hot-owner split: ONE owner's applyMessages
# batch over every rank.  The LWW decisions of applyMessages.ts:26-131 are per
# cell, so sending every message of a cell to one rank (in global batch order)
# keeps each cell's running max exact; the global __message PK case (one
# timestamp in two cells) is checked on the rank a hash of the timestamp picks,
# so every copy of one timestamp meets there; the tree is the XOR-combination
# of the per-rank partial trees (insertIntoMerkleTree is order-independent).
# ---------------------------------------------------------------------------
EVM_OK, EVM_ECOLLISION = 0, 3


def cell_dest(cell: torch.Tensor, world: int) -> torch.Tensor:
    """Rank of each cell of a split owner (a fixed mix of the cell id)."""
    c = cell.to(torch.int64) & 0xFFFFFFFF
    return (((c * 0x9E3779B1) & 0xFFFFFFFF) >> 8) % world


def split_apply(ts: torch.Tensor, cell: torch.Tensor, n_cells: int, apply_local, check_local, group=None):
    """applyMessages of one owner's batch split over the ranks by cell.

    ts (n, stride) uint8 / cell (n,) int: this rank's slice of the batch; the
    batch is the ranks' slices in rank order.
    apply_local(ts_r, cell_r) -> (flags u8[n_r], winner int[n_cells] index
        into ts_r or -1, partial, status) -- evm_apply_batch from an empty
        tree on this rank's cells (the partial tree is the caller's to merge,
        `merge_partial_tree`);
    check_local(ts_t, cell_t) -> bool: a timestamp with two cells
        (evm_cross_cell_check).
    Returns (flags u8[n] of this rank's slice, winner int64[n_cells] = global
    batch index or -1, partial, status); status is the same on every rank
    (EVM_ECOLLISION if any rank found a cross-cell timestamp)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = ts.device
    n = ts.shape[0]
    cell64 = cell.to(torch.int64)
    # the global PK check, by timestamp hash
    t_t, c_t, _, _ = route_by_owner(ts, cell64, group=group, dest=ts_route_hash(ts) % world)
    collide = bool(check_local(t_t, c_t)) if t_t.shape[0] else False
    # the LWW decisions, by cell
    ts_c, cell_c, src_rank, src_idx = route_by_owner(ts, cell64, group=group, dest=cell_dest(cell64, world))
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
    glob = torch.where((w >= 0) & mine, gidx.index_select(0, w.clamp(min=0)) if gidx.numel() else w, torch.full_like(w, -1))
    dist.all_reduce(glob, op=dist.ReduceOp.MAX, group=group)
    return flags, glob, part, status


def merge_partial_tree(eng, tree_in, part, group=None):
    """The owner's new tree on every rank: its prior tree merged with every
    rank's partial tree (leaf lists all-gathered, XOR-merged on the device by
    evm_tree_merge; the leaves never leave the device except where gloo
    itself needs host tensors)."""
    merged = tree_in
    for po, pc, px in gather_leaf_parts(*part.slice_device(0, part.n_owners), group):
        p = eng.tree_from_device_leaves(po, pc, px)
        merged = eng.tree_merge(merged, p)
    return merged
