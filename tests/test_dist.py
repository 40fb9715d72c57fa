"""Owner-sharded routing (evolu_amd/dist.py: the evm_dist_* plan restated over
torch.distributed) on CPU with gloo, world_size 2: owners by
murmur3(userId) mod world with dense local ids (evm_dist_directory), routing
preserves global batch order, per-message results round-trip, sharded server
ingest == unsharded ingest (checked with the oracle), roots all-gathered."""
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


def _user_ids(n):
    """userId strings (21 chars, initDbModel.ts:21-22) as uint8 [n, 21]."""
    import numpy as np

    return np.frombuffer(b"".join(b"u%020d" % g for g in range(n)), dtype=np.uint8).reshape(n, 21)


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
        from evolu_amd import dist as D
        from evolu_amd.engine import encode_timestamps
        from oracle import evolu_oracle as O

        msgs = _messages(rank)
        n_owners = 7
        ts = torch.from_numpy(encode_timestamps([t for _, t in msgs]))
        owner = torch.tensor([o for o, _ in msgs], dtype=torch.int64)
        dirx = D.Directory(_user_ids(n_owners), world)
        want_dest = [O.murmur3_32(b"u%020d" % g) % world for g in range(n_owners)]
        assert dirx.dest.tolist() == want_dest
        omap = D.OwnerMap(dirx, rank)
        ts_r, own_r, src_rank, src_idx = D.route_by_owner(ts, owner, omap.dest(owner, ts))
        # every received message is ours, in global batch order
        assert all(want_dest[int(o)] == rank for o in own_r)
        allm = [_messages(r) for r in range(world)]
        want = [(o, t) for r in range(world) for (o, t) in allm[r] if want_dest[o] == rank]
        got = [(int(o), bytes(ts_r[i, :46].numpy()).decode()) for i, o in enumerate(own_r)]
        assert got == want
        loc = omap.local(own_r).tolist()
        glob = omap.owners_here().tolist()
        assert all(glob[lo] == int(o) for lo, o in zip(loc, own_r))
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
        # roots all-gathered (local id j holds global owner glob[j])
        roots = torch.tensor([db.get_merkle_tree("u%d" % g).get("hash", 0) if g >= 0 else 0 for g in glob],
                             dtype=torch.int32)
        present = torch.tensor([g >= 0 and "hash" in db.get_merkle_tree("u%d" % g) for g in glob])
        groot, gpres = D.gather_roots(roots, present, omap)
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


def test_murmur3_rows_matches_oracle():
    """dist.murmur3_rows (the partition's hash, vectorised) == the oracle's
    murmur3_32 (pinned by the reference snapshot 4179357717 and imurmurhash
    vectors) for every length 0..50 and the 46-byte timestamps."""
    import numpy as np

    from evolu_amd import dist as D
    from oracle import evolu_oracle as O

    rng = np.random.default_rng(7)
    for L in range(0, 51):
        rows = rng.integers(32, 127, (40, L)).astype(np.uint8)
        got = D.murmur3_rows(rows)
        assert [int(x) for x in got] == [O.murmur3_32(bytes(r)) for r in rows], L
    ts = np.frombuffer(b"2022-07-03T08:02:00.000Z-0000-c6a4a4a9fb3a73b4", dtype=np.uint8).reshape(1, 46)
    assert int(D.murmur3_rows(ts)[0]) == O.murmur3_32(ts.tobytes())
