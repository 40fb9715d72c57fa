"""applyMessages parity on both device paths (streaming fast path / sort path),
multi-owner batches, wide minute ranges, and BASELINE-size cross-checks."""
import random

import numpy as np
import pytest

from oracle import evolu_oracle as O
from tests import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.set_option(1, 0)
    e.close()


def _run(eng, msgs, cells, path, cell_owner=None, n_owners=1, tree_json=None):
    from evolu_amd import _lib as L

    eng.set_option(L.OPT_CLIENT_PATH, path)
    cid = {c: i for i, c in enumerate(cells)}
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype=np.uint32)
    tin = eng.tree_from_json(tree_json or ["{}"] * n_owners)
    co = None if cell_owner is None else eng.dev(np.array(cell_owner, dtype=np.uint32))
    flags, winner, tout, st = eng.apply_batch(tin, eng.timestamps([m["timestamp"] for m in msgs]), eng.dev(cell),
                                              len(cells), cell_owner=co)
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    return flags.cpu().numpy(), winner.cpu().numpy(), tout


def _check(msgs, cells, flags, winner, dec):
    from evolu_amd import _lib as L

    for i, (ups, xr, _) in enumerate(dec):
        assert bool(flags[i] & L.MSG_UPS) == ups, i
        assert bool(flags[i] & L.MSG_XOR) == xr, i
    last = {}
    for i, m in enumerate(msgs):
        if dec[i][0]:
            last[(m["table"], m["row"], m["column"])] = i
    assert [int(w) for w in winner] == [last.get(c, -1) for c in cells]


@pytest.mark.parametrize("path", [1, 2])
@pytest.mark.parametrize("seed", range(4))
def test_both_paths_vs_oracle(eng, path, seed):
    msgs, cells = W.client_batch(100 + seed, n=600, n_cells=5 + 7 * seed)
    db = O.ClientDb()
    dec = []
    want = O.apply_messages(db, {}, msgs, dec)
    flags, winner, tout = _run(eng, msgs, cells, path)
    _check(msgs, cells, flags, winner, dec)
    assert tout.to_json(0) == O.merkle_tree_to_string(want)


def test_general_path_many_cells(eng):
    # > 2048 cells: the sort path is chosen automatically
    rng = random.Random(9)
    nodes = [W.node_id(rng) for _ in range(5)]
    tss = W.hlc_timestamps(rng, 6000, nodes)
    cells = [("t", "r%d" % i, "c") for i in range(2500)]
    msgs = [{"timestamp": t, "table": "t", "row": "r%d" % rng.randrange(2500), "column": "c", "value": i}
            for i, t in enumerate(tss)]
    msgs += [dict(rng.choice(msgs)) for _ in range(300)]
    db = O.ClientDb()
    dec = []
    want = O.apply_messages(db, {}, msgs, dec)
    flags, winner, tout = _run(eng, msgs, cells, 0)
    _check(msgs, cells, flags, winner, dec)
    assert tout.to_json(0) == O.merkle_tree_to_string(want)


@pytest.mark.parametrize("path", [1, 2])
def test_wide_minute_range_and_short_keys(eng, path):
    # spans > 4 fold windows and mixed key lengths -> the sort-based fold
    rng = random.Random(4)
    nodes = [W.node_id(rng) for _ in range(3)]
    tss = []
    for base in (0, 50 * 60000, W.T0, W.T0 + 200 * 86400000):
        tss += W.hlc_timestamps(rng, 150, nodes, t0=base, span=20 * 86400000)
    cells = [("t", "r", "c%d" % i) for i in range(40)]
    msgs = [{"timestamp": t, "table": "t", "row": "r", "column": "c%d" % rng.randrange(40), "value": i}
            for i, t in enumerate(tss)]
    rng.shuffle(msgs)
    db = O.ClientDb()
    dec = []
    want = O.apply_messages(db, {}, msgs, dec)
    flags, winner, tout = _run(eng, msgs, cells, path)
    _check(msgs, cells, flags, winner, dec)
    assert tout.to_json(0) == O.merkle_tree_to_string(want)


def test_multi_owner_batch(eng):
    # cells of 6 owners in one launch == 6 independent applyMessages calls
    rng = random.Random(21)
    all_msgs, all_cells, owner_of_cell, per_owner = [], [], [], []
    for o in range(6):
        msgs, cells = W.client_batch(300 + o, n=200, n_cells=6)
        cells = [("o%d_%s" % (o, c[0]), c[1], c[2]) for c in cells]
        msgs = [dict(m, table="o%d_%s" % (o, m["table"])) for m in msgs]
        per_owner.append((msgs, cells))
        all_cells += cells
        owner_of_cell += [o] * len(cells)
    for msgs, _ in per_owner:
        all_msgs += msgs
    rng.shuffle(all_msgs)
    flags, winner, tout = _run(eng, all_msgs, all_cells, 0, cell_owner=owner_of_cell, n_owners=6)
    for o, (msgs, cells) in enumerate(per_owner):
        mine = [m for m in all_msgs if m["table"].startswith("o%d_" % o)]
        db = O.ClientDb()
        dec = []
        want = O.apply_messages(db, {}, mine, dec)
        idx = [i for i, m in enumerate(all_msgs) if m["table"].startswith("o%d_" % o)]
        from evolu_amd import _lib as L

        for k, i in enumerate(idx):
            assert bool(flags[i] & L.MSG_UPS) == dec[k][0] and bool(flags[i] & L.MSG_XOR) == dec[k][1]
        assert tout.to_json(o) == O.merkle_tree_to_string(want)


@pytest.mark.parametrize("n", [1_000_000, 10_000_000])
def test_fast_vs_sort_path_at_scale(eng, n):
    """BASELINE config-2 sizes: two independent device algorithms must agree
    bit for bit (flags, winners, every leaf), and the tree's root must equal
    the XOR of the hashes of the XOR-flagged messages (size-independent)."""
    import torch

    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(n, 1000, seed_config=2)
    # add stale + exact redeliveries so every branch is taken at scale
    rng = np.random.default_rng(5)
    dup = rng.integers(0, n, size=n // 50)
    ts_np = np.concatenate([ts_np, ts_np[dup]])
    cell_np = np.concatenate([cell_np, cell_np[dup]])
    ts = eng.dev(ts_np)
    cell = eng.dev(cell_np)
    res = []
    for path in (1, 2):
        eng.set_option(L.OPT_CLIENT_PATH, path)
        flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, 1000)
        off, code, xr = tree.leaves()
        res.append((flags.cpu().numpy(), winner.cpu().numpy(), code, xr, tree.roots()))
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    (f1, w1, c1, x1, r1), (f2, w2, c2, x2, r2) = res
    assert np.array_equal(f1, f2) and np.array_equal(w1, w2)
    assert np.array_equal(c1, c2) and np.array_equal(x1, x2)
    assert r1[0][0] == r2[0][0]
    # root == XOR of the XOR-flagged messages' hashes (independent of the fold)
    recs, _ = eng.pack(ts)
    hashes = recs[:, 2].cpu().numpy().view(np.uint32).reshape(-1, 2)[:, 1]
    sel = (f1 & L.MSG_XOR) != 0
    want = np.bitwise_xor.reduce(hashes[sel].astype(np.uint32)) if sel.any() else 0
    assert np.array([r1[0][0]], dtype=np.int32).view(np.uint32)[0] == np.uint32(want)
    # every message whose timestamp is new to its cell is XORed; exact dups of the max never are
    assert (f1 & L.MSG_BAD).sum() == 0
    del ts, cell
    torch.cuda.empty_cache()


def test_redelivery_storm_oversize_bucket(eng):
    """20k copies of one message overflow an LDS hash bucket: the exact global
    check takes over; a copy in another cell is still a collision."""
    from evolu_amd import _lib as L

    ts = "2024-03-01T10:00:00.000Z-0000-00000000000000aa"
    older = "2024-03-01T09:59:59.999Z-0000-00000000000000aa"
    newer = "2024-03-01T10:00:00.001Z-0000-00000000000000aa"
    # exact redeliveries of the cell max are no-ops; a stale one re-XORs (toggles)
    strings = [older] + [ts] * 20000 + [newer, ts, ts]
    cell = np.zeros(len(strings), dtype=np.uint32)
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.timestamps(strings), eng.dev(cell), 2)
    f = flags.cpu().numpy()
    db = O.ClientDb()
    dec = []
    want = O.apply_messages(db, {}, [{"timestamp": s, "table": "t", "row": "r", "column": "c", "value": 0}
                                     for s in strings], dec)
    assert list(f) == [(1 if u else 0) | (2 if x else 0) for u, x, _ in dec]
    assert list(f[:3]) == [3, 3, 0] and list(f[-3:]) == [3, 2, 2]
    assert list(winner.cpu().numpy()) == [20001, -1]
    assert tree.to_json(0) == O.merkle_tree_to_string(want)
    cell[-1] = 1
    _, _, tree, st = eng.apply_batch(eng.tree_new(1), eng.timestamps(strings), eng.dev(cell), 2, raise_on_error=False)
    assert st == L.EVM_ECOLLISION


def test_collision_detected_at_scale(eng):
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(2_000_000, 1000, seed_config=7)
    ts_np = np.concatenate([ts_np, ts_np[123456:123457]])
    cell_np = np.concatenate([cell_np, (cell_np[123456:123457] + 1) % 1000])
    _, _, _, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts_np), eng.dev(cell_np), 1000, raise_on_error=False)
    assert st == L.EVM_ECOLLISION


@pytest.mark.parametrize("copies", [2, 7, 30, 60])
def test_cross_cell_check_hash_classes(eng, copies):
    """The partitioned cross-cell check settles one pair of a hash class per
    round: a timestamp redelivered `copies` times in one cell is no collision
    (the result equals the sort path's); one more copy in another cell, placed
    last, is found whatever the class size (above XP_MAX_ROUNDS the exact
    global check takes over)."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(200_000, 1000, seed_config=11)
    rng = np.random.default_rng(copies)
    picks = rng.integers(0, len(ts_np), size=5)
    extra_ts = np.concatenate([np.repeat(ts_np[p:p + 1], copies, axis=0) for p in picks])
    extra_cell = np.concatenate([np.repeat(cell_np[p:p + 1], copies) for p in picks])
    ts2 = np.concatenate([ts_np, extra_ts])
    cell2 = np.concatenate([cell_np, extra_cell])
    perm = rng.permutation(len(ts2))
    ts2, cell2 = ts2[perm], cell2[perm]
    res = []
    for path in (1, 2):
        eng.set_option(L.OPT_CLIENT_PATH, path)
        flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts2), eng.dev(cell2), 1000)
        off, code, xr = tree.leaves()
        res.append((flags.cpu().numpy(), winner.cpu().numpy(), code, xr))
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    for a, b in zip(*res):
        assert np.array_equal(a, b)
    # one copy of the last class in another cell: a collision
    ts3 = np.concatenate([ts2, ts_np[picks[-1]:picks[-1] + 1]])
    cell3 = np.concatenate([cell2, (cell_np[picks[-1]:picks[-1] + 1] + 1) % 1000])
    _, _, _, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts3), eng.dev(cell3), 1000, raise_on_error=False)
    assert st == L.EVM_ECOLLISION
