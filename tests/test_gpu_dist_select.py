"""Split-owner getMessages through the engine (dist.split_get_messages): two
ranks (gloo) sharing the GPU.  The hot owner's partial trees are merged on
the device (evm_tree_slice -> all-gather -> evm_tree_from_device_leaves ->
evm_tree_merge), the diff is taken on the merged tree, each rank selects its
share (evm_store_select_after with order keys) and the shares merge in
timestamp order -- against one unsharded server (oracle, index.ts:173-202)."""
import os

import numpy as np
import pytest
import torch.distributed as dist

from tests.test_dist_hot import N_OWNERS, _free_port, _messages
from tests.test_dist_select import _client_tree, _node

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q):
    import torch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from evolu_amd import dist as D
        from evolu_amd.engine import Engine, encode_timestamps
        from oracle import evolu_oracle as O

        eng = Engine(0)
        msgs = _messages(rank)
        ts = torch.from_numpy(encode_timestamps([t for _, t in msgs]))
        owner = torch.tensor([o for o, _ in msgs], dtype=torch.int64)
        omap = D.OwnerMap(N_OWNERS, world, rank, D.hot_owners(D.owner_counts(owner, N_OWNERS), world))
        ts_r, own_r, src_rank, src_idx = D.route_by_owner(ts, owner, dest=omap.dest(owner, ts))
        gid = (src_rank * 100000 + src_idx).tolist()
        lown = eng.dev(omap.local(own_r).numpy().astype(np.uint32))
        store = eng.store_new(omap.n_local)
        store.ingest(eng.dev(ts_r.numpy()), lown, rank * 1_000_000)
        hot = omap.hot.tolist()
        client = []
        for j in range(omap.n_local):
            if j < omap.per:
                o = j * world + rank
                client.append(O.merkle_tree_to_string(_client_tree(o)) if o < N_OWNERS and o not in hot else "{}")
            else:
                client.append("{}")
        client_local = eng.tree_from_json(client)
        client_hot = eng.tree_from_json([O.merkle_tree_to_string(_client_tree(o)) for o in hot])
        nodes = [(_node(j * world + rank) if j < omap.per else _node(hot[j - omap.per])) for j in range(omap.n_local)]
        node = eng.dev(np.frombuffer("".join(nodes).encode(), dtype=np.uint8).copy())
        diff, (off_c, ids_c), (off_h, ids_h) = D.split_get_messages(eng, store, client_local, client_hot, node, omap)
        diff, off_c, ids_c = diff.cpu().tolist(), off_c.cpu().tolist(), ids_c.cpu().tolist()
        off_h, ids_h = off_h.cpu().tolist(), ids_h.cpu().tolist()
        cold = {}
        for j in range(omap.per):
            o = j * world + rank
            if o < N_OWNERS and o not in hot:
                cold[o] = (None if diff[j] < 0 else diff[j], ids_c[off_c[j]:off_c[j + 1]])
        hot_res = {o: (None if diff[omap.per + k] < 0 else diff[omap.per + k], ids_h[off_h[k]:off_h[k + 1]])
                   for k, o in enumerate(hot)}
        q.put((rank, cold, hot_res, gid))
        store.free()
        eng.close()
    finally:
        dist.destroy_process_group()


def test_engine_split_get_messages_vs_unsharded():
    import torch.multiprocessing as mp

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
    deadline = time.time() + 200
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
    gids = {r: res[r][2] for r in range(world)}

    def to_gid(eid):  # engine id = rank * 1e6 + routed index on that rank
        return gids[eid // 1_000_000][eid % 1_000_000]

    db = O.ServerDb()
    for r in range(world):
        for i, (o, t) in enumerate(_messages(r)):
            db.add_messages(db.get_merkle_tree("u%d" % o), "u%d" % o, [(t, str(r * 100000 + i).encode())])
    want = {}
    for o in range(N_OWNERS):
        d, rows = db.get_messages(db.get_merkle_tree("u%d" % o), _client_tree(o), "u%d" % o, _node(o))
        want[o] = (d, [int(c) for _, c in rows])
    assert set(res[0][1]) == {0} and res[0][1] == res[1][1]
    got = {}
    for r in range(world):
        for o, (d, ids) in list(res[r][0].items()) + list(res[r][1].items()):
            got[o] = (d, [to_gid(e) for e in ids])
    assert got == want
