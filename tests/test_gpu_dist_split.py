"""Client hot-owner split through the engine: two ranks (gloo, CPU routing)
sharing the GPU, each running evm_apply_batch on its cells and
evm_cross_cell_check on its timestamp-hash share; the merged result against
the C restatement's unsharded applyMessages (flags, winners, tree JSON)."""
import os

import numpy as np
import pytest
import torch.distributed as dist

from tests.test_dist_client_split import CELLS, N, _free_port, _stream

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, collide, q):
    import torch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from evolu_amd import dist as D
        from evolu_amd.engine import Engine

        eng = Engine(0)
        ts_all, cell_all = _stream(collide)
        cut = N // 2
        sl = slice(0, cut) if rank == 0 else slice(cut, N)
        ts = torch.from_numpy(np.ascontiguousarray(ts_all[sl]))
        cell = torch.from_numpy(cell_all[sl].astype(np.int64))

        def apply_local(t, c):
            f, w, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(t.numpy()),
                                             eng.dev(c.numpy().astype(np.uint32)), CELLS, raise_on_error=False)
            return f.cpu(), w.cpu().to(torch.int64), tree, st

        def check_local(t, c):
            return eng.cross_cell_check(eng.dev(t.numpy()), eng.dev(c.numpy().astype(np.uint32)), CELLS)

        flags, winner, part, st = D.split_apply(ts, cell, CELLS, apply_local, check_local)
        js = None
        if st == 0:
            js = D.merge_partial_tree(eng, eng.tree_new(1), part).to_json(0)
        q.put((rank, st, flags.tolist(), None if winner is None else winner.tolist(), js))
        eng.close()
    finally:
        dist.destroy_process_group()


def _run(collide):
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, collide, q)) for r in range(world)]
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
    return res


def test_engine_client_split_vs_unsharded():
    from oracle import c_oracle as CO

    res = _run(False)
    ts, cell = _stream(False)
    st, flags, winner, js = CO.apply(ts, cell, CELLS)
    assert st == 0
    cut = N // 2
    for r in range(2):
        assert res[r][0] == 0
        assert res[r][2] == winner.tolist()
        assert res[r][3] == js
    assert res[0][1] == flags[:cut].tolist() and res[1][1] == flags[cut:].tolist()


def test_engine_client_split_collision():
    res = _run(True)
    assert res[0][0] == 3 and res[1][0] == 3
