"""Hot-owner split (evolu_amd/dist.py: the evm_dist_hot_owners / evm_dist_split
plan restated over torch.distributed) on CPU with gloo, world_size 2.

A skewed owner mix (BASELINE config 5: one owner holds half the messages,
with redeliveries), owners by murmur3(userId) mod world, is routed with the
hot owner split by murmur3(timestamp) mod world (local id hot_base + h).
Checked against one unsharded server (the oracle's verbatim-SQL
addMessages): the per-message INSERT decisions routed back to their origin,
the XOR-combined roots of the split owner, and its tree rebuilt from the
per-rank partial leaf maps."""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_OWNERS = 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _messages(rank, per_rank=160):
    from oracle import evolu_oracle as O
    from tests import workloads as W

    rng = random.Random(500 + rank)
    out = []
    for k in range(per_rank):
        o = 0 if rng.random() < 0.5 else rng.randrange(1, N_OWNERS)
        t = O.timestamp_to_string(W.T0 + rng.randrange(0, 40) * 7919, rng.randrange(3), "%016x" % (o * 7 + rng.randrange(2)))
        out.append((o, t))
    out += [out[i] for i in range(0, per_rank, 9)]  # redeliveries
    return out


def _leaves(tree, prefix=""):
    """Leaf map {key: xor} of a literal trie: nodes whose hash is not the XOR
    of their children's (inserts end there)."""
    out = {}
    for c in "012":
        if c in tree:
            out.update(_leaves(tree[c], prefix + c))
    if prefix:
        kids = 0
        for c in "012":
            if c in tree:
                kids ^= tree[c]["hash"]
        own = (tree["hash"] ^ kids) & 0xFFFFFFFF
        if own or not any(c in tree for c in "012"):
            out[prefix] = own
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from evolu_amd import dist as D
        from evolu_amd.engine import encode_timestamps
        from oracle import evolu_oracle as O

        from tests.test_dist import _user_ids

        msgs = _messages(rank)
        ts = torch.from_numpy(encode_timestamps([t for _, t in msgs]))
        owner = torch.tensor([o for o, _ in msgs], dtype=torch.int64)
        counts = D.owner_counts(owner, N_OWNERS)
        hot = D.hot_owners(counts, world)
        omap = D.OwnerMap(D.Directory(_user_ids(N_OWNERS), world), rank, hot)
        ts_r, own_r, src_rank, src_idx = D.route_by_owner(ts, owner, omap.dest(owner, ts))
        loc = omap.local(own_r)
        got = [(int(o), bytes(ts_r[i, :46].numpy()).decode()) for i, o in enumerate(own_r)]
        db = O.ServerDb()
        ins = []
        for (o, t), lo in zip(got, loc.tolist()):
            g = []
            db.add_messages(db.get_merkle_tree("l%d" % lo), "l%d" % lo, [(t, b"")], g)
            ins += g
        ins_back = D.route_back(torch.tensor(ins, dtype=torch.int64), src_rank, src_idx, len(msgs))
        roots = torch.tensor([db.get_merkle_tree("l%d" % j).get("hash", 0) for j in range(omap.n_local)],
                             dtype=torch.int32)
        present = torch.tensor(["hash" in db.get_merkle_tree("l%d" % j) for j in range(omap.n_local)])
        groot, gpres = D.gather_roots(roots, present, omap)
        hroot, hpres = groot[torch.from_numpy(hot)], gpres[torch.from_numpy(hot)]
        partial = {int(h): _leaves(db.get_merkle_tree("l%d" % (omap.hot_base + k)))
                   for k, h in enumerate(omap.hot.tolist())}
        q.put((rank, hot.tolist(), ins_back.tolist(), hroot.tolist(), hpres.tolist(), partial))
    finally:
        dist.destroy_process_group()


def test_hot_owner_split_gloo_world2():
    from oracle import evolu_oracle as O

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time

    res = {}
    deadline = time.time() + 240
    while len(res) < world:
        try:
            r = q.get(timeout=2)
            res[r[0]] = r[1:]
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail("a rank failed: exit codes %s" % [p.exitcode for p in procs])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][0] == [0] and res[1][0] == [0]  # owner 0 is the hot one
    # the unsharded server over the global batch order (rank-major)
    db = O.ServerDb()
    for r in range(world):
        ins = []
        for o, t in _messages(r):
            g = []
            db.add_messages(db.get_merkle_tree("u%d" % o), "u%d" % o, [(t, b"")], g)
            ins += g
        assert res[r][1] == ins
    want = db.get_merkle_tree("u0")
    for r in range(world):
        assert res[r][3] == [True] and res[r][2] == [O.to_int32(want["hash"])]
    # the split owner's tree from its partial leaf maps (XOR-combined)
    merged = {}
    for r in range(world):
        for k, x in res[r][4][0].items():
            merged[k] = merged.get(k, 0) ^ x
    assert O.merkle_tree_to_string(O.tree_from_leaves({k: O.to_int32(x) for k, x in merged.items()})) == \
        O.merkle_tree_to_string(want)
