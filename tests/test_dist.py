"""Owner-sharded routing (evolu_amd/dist.py) on CPU with gloo, world_size 2:
routing preserves global batch order, round-trips per-message results, and
sharded server ingest == unsharded ingest (checked with the oracle)."""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _messages(rank, n_owners=7, per_rank=60):
    """Each rank receives requests for random owners; the global batch order is
    rank-major (rank 0's messages, then rank 1's)."""
    from oracle import evolu_oracle as O
    from tests import workloads as W

    rng = random.Random(1000 + rank)
    out = []
    for k in range(per_rank):
        o = rng.randrange(n_owners)
        t = O.timestamp_to_string(W.T0 + rng.randrange(0, 5) * 1000, rng.randrange(3), "%016x" % (o * 7 + 1))
        out.append((o, t))
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import numpy as np

        from evolu_amd import dist as D
        from evolu_amd.engine import encode_timestamps
        from oracle import evolu_oracle as O

        msgs = _messages(rank)
        ts = torch.from_numpy(encode_timestamps([t for _, t in msgs]))
        owner = torch.tensor([o for o, _ in msgs], dtype=torch.int64)
        ts_r, own_r, src_rank, src_idx = D.route_by_owner(ts, owner)
        # every received message is ours, in global batch order
        assert bool(((own_r % world) == rank).all())
        allm = [_messages(r) for r in range(world)]
        want = [(o, t) for r in range(world) for (o, t) in allm[r] if o % world == rank]
        got = [(int(o), bytes(ts_r[i, :46].numpy()).decode()) for i, o in enumerate(own_r)]
        assert got == want
        # per-message results come back to their origin
        vals = (own_r * 3 + 1).to(torch.int64)
        back = D.route_back(vals, src_rank, src_idx, len(msgs))
        assert back.tolist() == [o * 3 + 1 for o, _ in msgs]
        # sharded ingest == unsharded ingest: oracle server per rank on routed rows
        db = O.ServerDb()
        ins = []
        for o, t in got:
            g = []
            db.add_messages(db.get_merkle_tree("u%d" % o), "u%d" % o, [(t, b"")], g)
            ins += g
        ins_back = D.route_back(torch.tensor(ins, dtype=torch.int64), src_rank, src_idx, len(msgs))
        trees = {o: O.merkle_tree_to_string(db.get_merkle_tree("u%d" % o)) for o in set(o for o, _ in got)}
        # roots all-gathered
        n_owners = 7
        local = [j * world + rank for j in range((n_owners - rank + world - 1) // world)]
        roots = torch.tensor([db.get_merkle_tree("u%d" % o).get("hash", 0) for o in local], dtype=torch.int32)
        present = torch.tensor(["hash" in db.get_merkle_tree("u%d" % o) for o in local])
        groot, gpres = D.gather_roots(roots, present, n_owners)
        q.put((rank, ins_back.tolist(), trees, groot.tolist(), gpres.tolist()))
    finally:
        dist.destroy_process_group()


def test_owner_sharding_gloo_world2():
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
    # unsharded reference over the global batch order
    db = O.ServerDb()
    want_ins = {}
    for r in range(world):
        ins = []
        for o, t in _messages(r):
            g = []
            db.add_messages(db.get_merkle_tree("u%d" % o), "u%d" % o, [(t, b"")], g)
            ins += g
        want_ins[r] = ins
    for r in range(world):
        assert res[r][0] == want_ins[r]
        for o, j in res[r][1].items():
            assert j == O.merkle_tree_to_string(db.get_merkle_tree("u%d" % o))
    groot, gpres = res[0][2], res[0][3]
    for o in range(7):
        t = db.get_merkle_tree("u%d" % o)
        assert gpres[o] == ("hash" in t) and (not gpres[o] or groot[o] == t["hash"])
