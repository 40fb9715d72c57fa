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


def route_by_owner(ts: torch.Tensor, owner: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                                                                  torch.Tensor]:
    """All-to-all routing of messages to their owner's rank.

    ts: (n, stride) uint8 timestamp rows, owner: (n,) int64 global owner ids,
    both on this rank.  Returns (ts_recv, owner_recv, src_rank, src_index):
    the messages this rank owns, in global batch order, with where they came
    from (to send per-message results back with `route_back`).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = ts.device
    n, stride = ts.shape
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
