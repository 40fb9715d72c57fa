"""Client hot-owner split (evolu_amd/dist.py split_apply; SURVEY 8(e) config
5-C) on CPU with gloo, world_size 2.

One owner's applyMessages batch (Zipf-free config-5 stream: bursts of equal
millis across nodes, ~1 % upper-case nodes, 10 % redeliveries, half stale)
is cut into two rank slices; the ranks route it by cell, decide locally and
route the flags back.  The local step is the C restatement (oracle/c) of
applyMessages standing in for the engine, so this checks the split itself:
against one unsharded applyMessages over the whole batch, the per-message
flags of every slice, the winners as global batch indices, the tree as the
XOR-merge of the per-rank partial trees, and a cross-cell timestamp planted
across the two slices making both ranks report EVM_ECOLLISION."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, CELLS = 6000, 300


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(collide: bool):
    from evolu_amd import synth

    ts, _, cell = synth.config5(1, N, cells_per_owner=CELLS, seed_config=55)
    cell = cell.astype(np.uint32)
    if collide:  # one timestamp of slice 0 again in slice 1, under another cell
        ts = ts.copy()
        ts[N - 7] = ts[11]
        cell = cell.copy()
        cell[N - 7] = (cell[11] + 1) % CELLS
    return ts, cell


def _leaves(tree, prefix=""):
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


def _worker(rank, world, port, collide, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from evolu_amd import dist as D
        from oracle import c_oracle as CO

        ts_all, cell_all = _stream(collide)
        cut = N // 2
        sl = slice(0, cut) if rank == 0 else slice(cut, N)
        ts = torch.from_numpy(np.ascontiguousarray(ts_all[sl]))
        cell = torch.from_numpy(cell_all[sl].astype(np.int64))

        def apply_local(t, c):
            st, f, w, js = CO.apply(t.numpy(), c.numpy().astype(np.uint32), CELLS)
            return torch.from_numpy(f.copy()), torch.from_numpy(w.astype(np.int64)), js, st

        def check_local(t, c):
            seen = {}
            for row, cc in zip(t.numpy(), c.tolist()):
                k = bytes(row[:46])
                if seen.setdefault(k, cc) != cc:
                    return True
            return False

        flags, winner, part, st = D.split_apply(ts, cell, CELLS, apply_local, check_local)
        q.put((rank, st, flags.tolist(), None if winner is None else winner.tolist(),
               None if part is None else _leaves(json.loads(part))))
    finally:
        dist.destroy_process_group()


def _run(collide):
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
    return res


def test_client_split_matches_unsharded_apply():
    from oracle import c_oracle as CO

    res = _run(False)
    ts, cell = _stream(False)
    st, flags, winner, js = CO.apply(ts, cell, CELLS)
    assert st == 0
    cut = N // 2
    assert res[0][0] == 0 and res[1][0] == 0
    assert res[0][1] == flags[:cut].tolist()
    assert res[1][1] == flags[cut:].tolist()
    assert res[0][2] == winner.tolist() and res[1][2] == winner.tolist()
    merged = {}
    for r in range(2):
        for k, v in res[r][3].items():
            merged[k] = merged.get(k, 0) ^ v
    want = _leaves(json.loads(js))
    assert {k: v for k, v in merged.items()} == want


def test_client_split_cross_cell_collision_on_every_rank():
    from oracle import c_oracle as CO

    res = _run(True)
    ts, cell = _stream(True)
    assert CO.apply(ts, cell, CELLS)[0] == 3  # the unsharded reference case: EVM_ECOLLISION
    assert res[0][0] == 3 and res[1][0] == 3
