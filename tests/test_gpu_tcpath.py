"""The streaming tc path of applyMessages (evm_client.hip TP1-TP3, the default
for one owner with <= 2,048 cells): decisions from tc = millis << 16 |
counter, and a tie (equal tc against its cell's running max: equal millis +
counter from two nodes, or a redelivery of the cell's max) decided inside the
walk by the two timestamps' node ranks -- no redo.  Checked against the
oracle (applyMessages.ts:26-131, verbatim SQL), the C restatement at the
headline's own stream and size, and bit for bit against the sort path."""
import random

import numpy as np
import torch
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


def _has_tie(msgs, prior=None):
    """Some message's tc equals its cell's running max tc (node ranks decide)."""
    run = dict(prior or {})
    for m in msgs:
        c = (m["table"], m["row"], m["column"])
        ms, ctr, _ = O.parse_canonical(m["timestamp"])
        tc = (ms << 16) | ctr
        t = run.get(c)
        if t is not None and tc == t:
            return True
        if t is None or tc > t:
            run[c] = tc
    return False


def _apply(eng, msgs, cells, path, prior=None, tree_json="{}"):
    from evolu_amd import _lib as L

    cid = {c: i for i, c in enumerate(cells)}
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype=np.uint32)
    kw = {}
    if prior is not None:
        kw["prior_ts"] = eng.timestamps([prior.get(c, "") for c in cells])
        kw["prior_present"] = eng.dev(np.array([c in prior for c in cells], dtype=np.uint8))
    eng.set_option(L.OPT_CLIENT_PATH, path)
    s0 = eng.stats()
    flags, winner, tree, st = eng.apply_batch(eng.tree_from_json([tree_json]),
                                              eng.timestamps([m["timestamp"] for m in msgs]), eng.dev(cell),
                                              len(cells), raise_on_error=False, **kw)
    s1 = eng.stats()
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    ran = {"tc": s1["tc_batches"] - s0["tc_batches"], "redo": s1["tc_redos"] - s0["tc_redos"]}
    return st, flags.cpu().numpy(), winner.cpu().numpy(), tree, ran


def _oracle(msgs, cells, prior=None):
    db = O.ClientDb()
    tree = {}
    if prior:
        # the prior rows: one message per cell holding that cell's max
        tree = O.apply_messages(db, {}, [{"timestamp": t, "table": c[0], "row": c[1], "column": c[2], "value": "p"}
                                         for c, t in prior.items()])
    dec = []
    want = O.apply_messages(db, tree, msgs, dec)
    flags = np.array([(1 if u else 0) | (2 if x else 0) for u, x, _ in dec], dtype=np.uint8)
    last = {}
    for i, m in enumerate(msgs):
        if dec[i][0]:
            last[(m["table"], m["row"], m["column"])] = i
    return flags, np.array([last.get(c, -1) for c in cells]), want, tree


def _distinct_batch(seed, n=3000, n_cells=40, nodes=6):
    """Timestamps with distinct (millis, counter): no tie possible."""
    rng = random.Random(seed)
    node_ids = [W.node_id(rng, upper=(k % 2 == 1)) for k in range(nodes)]
    ms = rng.sample(range(W.T0, W.T0 + 3600_000 * 24), n)
    cells = [("t%d" % (i % 3), "r%d" % (i // 3), "c") for i in range(n_cells)]
    msgs = [{"timestamp": O.timestamp_to_string(m, rng.randrange(3), rng.choice(node_ids)),
             "table": cells[k][0], "row": cells[k][1], "column": cells[k][2], "value": i}
            for i, (m, k) in enumerate(zip(ms, [rng.randrange(n_cells) for _ in range(n)]))]
    # stale redeliveries (older than the cell's max): XOR toggles, still no tie
    for _ in range(200):
        i = rng.randrange(len(msgs))
        msgs.insert(rng.randrange(i, len(msgs)) + 1, dict(msgs[i]))
    return msgs, cells


@pytest.mark.parametrize("seed", range(3))
def test_tc_path_without_ties_vs_oracle(eng, seed):
    msgs, cells = _distinct_batch(seed)
    tie = _has_tie(msgs)
    st, flags, winner, tree, ran = _apply(eng, msgs, cells, 3)
    f, w, want, _ = _oracle(msgs, cells)
    assert st == 0
    assert np.array_equal(flags, f) and np.array_equal(winner, w)
    assert tree.to_json(0) == O.merkle_tree_to_string(want)
    assert ran == {"tc": 1, "redo": 0}


@pytest.mark.parametrize("seed", range(4))
def test_tc_path_with_ties_and_case_vs_oracle(eng, seed):
    """Equal millis across nodes, mixed-case node ids, exact + stale
    redeliveries: the ties are decided by node rank inside the walk."""
    msgs, cells = W.client_batch(700 + seed, n=800, n_cells=7)
    st, flags, winner, tree, ran = _apply(eng, msgs, cells, 3)
    f, w, want, _ = _oracle(msgs, cells)
    assert st == 0
    assert np.array_equal(flags, f) and np.array_equal(winner, w)
    assert tree.to_json(0) == O.merkle_tree_to_string(want)
    assert ran == {"tc": 1, "redo": 0}
    if seed == 0:
        assert _has_tie(msgs)  # (the stream does exercise ties)


def test_tc_path_prior_rows(eng):
    """Prior maxima: below, above and equal (an exact redelivery of the prior)."""
    msgs, cells = _distinct_batch(11, n=1500, n_cells=30)
    rng = random.Random(3)
    prior = {}
    for c in cells[:20]:
        mine = [m["timestamp"] for m in msgs if (m["table"], m["row"], m["column"]) == c]
        ms, ctr, node = O.parse_canonical(rng.choice(mine))
        prior[c] = O.timestamp_to_string(ms + rng.choice([-1, 1]) * rng.randrange(1, 5000), ctr, node)
    ptc = {c: (O.parse_canonical(t)[0] << 16) | O.parse_canonical(t)[1] for c, t in prior.items()}
    _, _, _, t0 = _oracle([], cells, prior)
    st, flags, winner, tree, ran = _apply(eng, msgs, cells, 3, prior=prior, tree_json=O.merkle_tree_to_string(t0))
    f, w, want, _ = _oracle(msgs, cells, prior)
    assert st == 0 and np.array_equal(flags, f) and np.array_equal(winner, w)
    assert ran == {"tc": 1, "redo": 0}
    assert tree.to_json(0) == O.merkle_tree_to_string(want)
    # an exact redelivery of a prior max is a tie against the prior row: a no-op
    c0 = cells[0]
    msgs2 = msgs + [{"timestamp": prior[c0], "table": c0[0], "row": c0[1], "column": c0[2], "value": "dup"}]
    st, flags, winner, tree, ran = _apply(eng, msgs2, cells, 3, prior=prior)
    f, w, _, _ = _oracle(msgs2, cells, prior)
    assert st == 0 and np.array_equal(flags, f) and np.array_equal(winner, w)
    assert ran == {"tc": 1, "redo": 0} and _has_tie(msgs2, ptc)


@pytest.mark.parametrize("cells", [1, 7, 1000, 2048])
def test_tc_path_vs_sort_path_at_scale(eng, cells):
    """2M messages (config-2 generator): the tc path (no ties in these
    streams) bit for bit against the sort path; one cell is the hot-cell
    extreme (every row in one segment of the scan)."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(2_000_000, cells, seed_config=40 + cells)
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    res = []
    for path in (3, 2):
        eng.set_option(L.OPT_CLIENT_PATH, path)
        s0 = eng.stats()
        flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, cells)
        s1 = eng.stats()
        off, code, xr = tree.leaves()
        res.append((flags.cpu().numpy(), winner.cpu().numpy(), code, xr, s1["tc_batches"] - s0["tc_batches"],
                    s1["tc_redos"] - s0["tc_redos"]))
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    (f1, w1, c1, x1, tc1, r1), (f2, w2, c2, x2, _, _) = res
    assert np.array_equal(f1, f2) and np.array_equal(w1, w2)
    assert np.array_equal(c1, c2) and np.array_equal(x1, x2)
    assert tc1 + r1 == 1


def test_tc_path_redeliveries_at_scale(eng):
    """10M messages + 2 % exact/stale redeliveries: whichever way the tc path
    goes (a redelivered cell max is a tie), the result equals the sort path."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(10_000_000, 1000, seed_config=2)
    rng = np.random.default_rng(5)
    dup = rng.integers(0, len(ts_np), size=len(ts_np) // 50)
    ts_np = np.concatenate([ts_np, ts_np[dup]])
    cell_np = np.concatenate([cell_np, cell_np[dup]])
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    out = []
    for path in (0, 2):
        eng.set_option(L.OPT_CLIENT_PATH, path)
        flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, 1000)
        out.append((flags.cpu().numpy(), winner.cpu().numpy(), tree.leaves()[1], tree.leaves()[2]))
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)


def test_tc_path_bad_input(eng):
    from evolu_amd import _lib as L

    msgs, cells = _distinct_batch(5, n=500, n_cells=10)
    strings = [m["timestamp"] for m in msgs]
    strings[17] = strings[17].replace("T", "t")  # not canonical
    cid = {c: i for i, c in enumerate(cells)}
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype=np.uint32)
    eng.set_option(L.OPT_CLIENT_PATH, 3)
    flags, _, tree, st = eng.apply_batch(eng.tree_new(1), eng.timestamps(strings), eng.dev(cell), len(cells),
                                         raise_on_error=False)
    assert st == L.EVM_ENONCANON and tree is None
    f = flags.cpu().numpy()
    assert f[17] == L.MSG_BAD and (np.delete(f, 17) == 0).all()
    cell[3] = len(cells)  # a cell id out of range
    _, _, tree, st = eng.apply_batch(eng.tree_new(1), eng.timestamps([m["timestamp"] for m in msgs]), eng.dev(cell),
                                     len(cells), raise_on_error=False)
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    assert st == L.EVM_EINVAL


@pytest.mark.parametrize("cells", [1, 64, 1000])
def test_tc_path_ascending_stream(eng, cells):
    """Batch order = timestamp order (what a client receives: ORDER BY
    timestamp): every row is a new maximum of its cell, so every row goes
    through the walk; bit for bit against the sort path."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(1_000_000, cells, seed_config=70 + cells)
    order = np.argsort(ts_np[:, :29].copy().view("S29").ravel(), kind="stable")
    ts_np, cell_np = ts_np[order], cell_np[order]
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    res = []
    for path in (3, 2):
        eng.set_option(L.OPT_CLIENT_PATH, path)
        flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, cells)
        res.append((flags.cpu().numpy(), winner.cpu().numpy(), tree.leaves()[1], tree.leaves()[2]))
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
    assert (res[0][0] & L.MSG_UPS).mean() > 0.5  # mostly new maxima


@pytest.mark.parametrize("n", [1_250_001, 999_937, 65])
def test_tc_path_ragged_size_keeps_dense_fold(eng, n):
    """A batch whose size is not a multiple of 64 takes the dense minute fold
    (the tail lanes of the last wave must not widen the minute bounds), and
    equals the sort path."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(max(n, 1000), 1000, seed_config=77)
    ts, cell = eng.dev(ts_np[:n]), eng.dev(cell_np[:n])
    eng.set_option(L.OPT_CLIENT_PATH, 3)
    eng.prof_enable(True)
    eng.prof_reset()
    f1, w1, t1, st = eng.apply_batch(eng.tree_new(1), ts, cell, 1000, raise_on_error=False)
    rep = eng.prof_report()
    eng.prof_enable(False)
    if st == L.EVM_OK:  # (the tc path's fused check + dense fold, not the sort-based fold)
        assert "k_xf_dedup" in rep and "k_xf_blocks" in rep, sorted(rep)
        assert "k_cl_fold_ck" not in rep, sorted(rep)
    eng.set_option(L.OPT_CLIENT_PATH, 2)
    f2, w2, t2, _ = eng.apply_batch(eng.tree_new(1), ts, cell, 1000)
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    if st == L.EVM_OK:
        assert torch.equal(f1, f2) and torch.equal(w1, w2)
        assert t1.to_json(0) == t2.to_json(0)


def test_tc_path_headline_stream_vs_c_oracle(eng):
    """The stream and size bench.py times (BASELINE config 2: 10M messages,
    1,000 cells, 64 nodes, seed 2) through the tc path only, bit for bit
    against the C restatement of applyMessages: flags, winners, tree JSON."""
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from oracle import c_oracle as CO

    ts_np, cell_np = synth.config2(10_000_000, 1000, seed_config=2)
    st_w, f_w, w_w, js_w = CO.apply(ts_np, cell_np, 1000)
    assert st_w == 0
    eng.set_option(L.OPT_CLIENT_PATH, 3)
    s0 = eng.stats()
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts_np), eng.dev(cell_np), 1000)
    s1 = eng.stats()
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    assert s1["tc_batches"] - s0["tc_batches"] == 1 and s1["tc_redos"] == s0["tc_redos"]
    assert np.array_equal(flags.cpu().numpy(), f_w)
    assert np.array_equal(winner.cpu().numpy(), w_w)
    assert tree.to_json(0) == js_w


@pytest.mark.parametrize("n,cells,nodes", [(2_000_000, 1000, 64), (1_000_000, 50, 4), (300_000, 1, 8)])
def test_tc_path_adversarial_client_stream_vs_c_oracle(eng, n, cells, nodes):
    """BASELINE config 5 on the client side: one owner, equal-millis bursts
    (counter and node tie-breaks), 10 % redeliveries (half after a newer
    write: the XOR toggle; the rest ties with the cell max), ~1 % upper-case
    nodes.  Ties are decided inside the walk (no redo), bit for bit against
    the C restatement."""
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from oracle import c_oracle as CO

    ts_np, cell_np = synth.client_adversarial(n, cells, nodes, seed_config=5)
    st_w, f_w, w_w, js_w = CO.apply(ts_np, cell_np, cells)
    assert st_w == 0
    eng.set_option(L.OPT_CLIENT_PATH, 3)
    s0 = eng.stats()
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts_np), eng.dev(cell_np), cells)
    s1 = eng.stats()
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    assert s1["tc_batches"] - s0["tc_batches"] == 1 and s1["tc_redos"] == s0["tc_redos"]
    assert np.array_equal(flags.cpu().numpy(), f_w)
    assert np.array_equal(winner.cpu().numpy(), w_w)
    assert tree.to_json(0) == js_w
    if cells > 1:
        assert ((f_w & L.MSG_XOR) == 0).sum() > 0  # the stream has exact redeliveries of cell maxima (ties)


def test_tc_path_tie_list_overflow_redoes_exactly(eng):
    """More than 512 rows of one range tied at a cell's range max (700 nodes
    sending at the same millisecond, counter 0, inside the second range of
    1,024 rows: the first is cut into geometric pieces): TP1's list overflows
    and the exact walk path answers -- the result is still exact."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    rng = np.random.default_rng(9)
    n = 4096
    ms = synth.BENCH_T0 + rng.integers(0, 10_000, n)
    ms[1100:1800] = synth.BENCH_T0 + 50_000  # 700 rows, one millisecond, above everything else (one range)
    nodes = synth.random_nodes(rng, n)
    ts_np = synth.format_timestamps(ms, np.zeros(n, dtype=np.int64), nodes)
    cell_np = np.zeros(n, dtype=np.uint32)
    cell_np[::7] = 1
    cell_np[1100:1800] = 0
    from oracle import c_oracle as CO

    st_w, f_w, w_w, js_w = CO.apply(ts_np, cell_np, 2)
    eng.set_option(L.OPT_CLIENT_PATH, 3)
    s0 = eng.stats()
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts_np), eng.dev(cell_np), 2)
    s1 = eng.stats()
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    assert s1["tc_redos"] - s0["tc_redos"] == 1
    assert np.array_equal(flags.cpu().numpy(), f_w) and np.array_equal(winner.cpu().numpy(), w_w)
    assert tree.to_json(0) == js_w


# ---------------------------------------------------------------------------
# The fused cross-cell check + Merkle fold (k_xf_*): minute buckets, the fold
# of every row with the walk's exact redeliveries XORed out again, and the
# batches it hands to the exact walk path (xf_redo) -- each against the C
# restatement of applyMessages.
# ---------------------------------------------------------------------------
def _c_vs_tc(eng, ts_np, cell_np, cells, redo):
    from evolu_amd import _lib as L
    from oracle import c_oracle as CO

    st_w, f_w, w_w, js_w = CO.apply(ts_np, cell_np, cells)
    eng.set_option(L.OPT_CLIENT_PATH, 3)
    s0 = eng.stats()
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts_np), eng.dev(cell_np), cells,
                                              raise_on_error=False)
    s1 = eng.stats()
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    assert (s1["tc_redos"] - s0["tc_redos"], s1["tc_batches"] - s0["tc_batches"]) == ((1, 0) if redo else (0, 1))
    if st_w != 0:
        return st, st_w
    assert st == 0
    assert np.array_equal(flags.cpu().numpy(), f_w) and np.array_equal(winner.cpu().numpy(), w_w)
    assert tree.to_json(0) == js_w
    return st, st_w


@pytest.mark.parametrize("minutes", [1, 3, 700])
def test_xf_narrow_minute_span(eng, minutes):
    """A batch over fewer minutes than buckets: each minute is split over
    buckets by hash bits, its XOR combined from every bucket; with exact and
    stale redeliveries (the walk's no-op rows XORed out of the fold)."""
    from evolu_amd import synth

    rng = np.random.default_rng(minutes)
    n = 1_000_000
    ms = synth.BENCH_T0 + rng.integers(0, minutes * 60_000, n)
    nodes = synth.random_nodes(rng, 16)
    ts_np = synth.format_timestamps(ms, rng.integers(0, 4, n), nodes[rng.integers(0, 16, n)])
    cell_np = rng.integers(0, 300, n).astype(np.uint32)
    dup = rng.integers(0, n, n // 20)  # 5 % redeliveries
    ts_np = np.concatenate([ts_np, ts_np[dup]])
    cell_np = np.concatenate([cell_np, cell_np[dup]])
    # (every copy of a timestamp in its first copy's cell: no cross-cell twins)
    key = ts_np[:, :46].copy().view("S46").ravel()
    _, first, inv = np.unique(key, return_index=True, return_inverse=True)
    cell_np = cell_np[first][inv].astype(np.uint32)
    _c_vs_tc(eng, ts_np, cell_np, 300, redo=False)


def test_xf_collision_redoes_exactly(eng):
    """One timestamp in two different cells (the global __message PK): the
    fingerprints match across cells, the exact walk path confirms the collision."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(200_000, 100, seed_config=91)
    ts_np = np.concatenate([ts_np, ts_np[1234:1235]])
    cell_np = np.concatenate([cell_np, np.array([(cell_np[1234] + 1) % 100], dtype=np.uint32)])
    st, st_w = _c_vs_tc(eng, ts_np, cell_np, 100, redo=True)
    assert st == L.EVM_ECOLLISION and st_w != 0


def test_xf_wide_span_redoes_exactly(eng):
    """A batch over more than XF_SPAN_MAX (131,072) minutes: the exact walk path."""
    from evolu_amd import synth

    rng = np.random.default_rng(4)
    n = 300_000
    ms = synth.BENCH_T0 + rng.integers(0, 200 * 86_400_000, n)
    ts_np = synth.format_timestamps(ms, np.zeros(n, dtype=np.int64), synth.random_nodes(rng, n))
    _c_vs_tc(eng, ts_np, rng.integers(0, 64, n).astype(np.uint32), 64, redo=True)


def test_xf_skewed_minute_overflows_to_exact(eng):
    """Half the batch in one minute of a 30-day batch: that minute's bucket
    overflows its capacity and the exact walk path answers."""
    from evolu_amd import synth

    rng = np.random.default_rng(6)
    n = 2_000_000
    ms = synth.BENCH_T0 + rng.integers(0, 30 * 86_400_000, n)
    ms[: n // 2] = synth.BENCH_T0 + 5 * 86_400_000 + rng.integers(0, 60_000, n // 2)
    ts_np = synth.format_timestamps(ms, np.zeros(n, dtype=np.int64), synth.random_nodes(rng, n))
    _c_vs_tc(eng, ts_np, rng.integers(0, 1000, n).astype(np.uint32), 1000, redo=True)


def test_xf_mixed_key_lengths_redo(eng):
    """Minutes on both sides of 3^16 (2051-11-05): two base-3 key lengths, so
    leaf order is not minute order -- the exact walk path's sort-based fold."""
    from evolu_amd import synth

    rng = np.random.default_rng(8)
    n = 100_000
    edge = 3 ** 16 * 60_000
    ms = edge + rng.integers(-3_600_000, 3_600_000, n)
    ts_np = synth.format_timestamps(ms, np.zeros(n, dtype=np.int64), synth.random_nodes(rng, 32)[rng.integers(0, 32, n)])
    _c_vs_tc(eng, ts_np, rng.integers(0, 50, n).astype(np.uint32), 50, redo=True)


@pytest.mark.parametrize("case", ["counter", "year2045"])
def test_tc_path_far_rows_vs_c_oracle(eng, case):
    """Rows outside TP1's packed word (counter >= 256, or millis >= 2^41:
    after 2039-09) travel as TP_FAR with their tc in the side array: the
    walk and the fused check read them from there; still one tc batch, no
    redo, bit-exact against the C restatement."""
    from evolu_amd import synth

    rng = np.random.default_rng(12)
    n = 400_000
    t0 = synth.BENCH_T0 if case == "counter" else 2_378_000_000_000  # (2045-05: same base-3 key length as 2024)
    ms = t0 + rng.integers(0, 20 * 86_400_000, n)
    ctr = np.zeros(n, dtype=np.int64)
    if case == "counter":
        far = rng.random(n) < 0.02
        ctr[far] = rng.integers(256, 0xffff, far.sum())
    nodes = synth.random_nodes(rng, 32)
    ts_np = synth.format_timestamps(ms, ctr, nodes[rng.integers(0, 32, n)])
    # (every far row marks its cell for TP1's rescan, whose match list holds
    # 512 rows per range: all-far batches over few cells)
    cells = 700 if case == "counter" else 200
    cell_np = rng.integers(0, cells, n).astype(np.uint32)
    key = ts_np[:, :46].copy().view("S46").ravel()
    _, first, inv = np.unique(key, return_index=True, return_inverse=True)
    cell_np = cell_np[first][inv].astype(np.uint32)  # (no cross-cell twins)
    _c_vs_tc(eng, ts_np, cell_np, cells, redo=False)
