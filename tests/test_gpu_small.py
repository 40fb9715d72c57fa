"""The small-batch client path (EVM_OPT_CLIENT_PATH 4; the auto choice for
<= 262,144 messages over more than 2,048 cells): applyMessages
(applyMessages.ts:26-131) in five kernels and one status read, against the C
restatement (flags, winners, tree JSON) and the sort path; long cells (more
than 32 rows: a workgroup each, LDS sort + blocked max scan) and its
hand-offs to the sort path (a cell of more than 4,096 rows, minutes wider
than the dense window, two base-3 key lengths) give the same answers."""
import numpy as np
import pytest

from oracle import c_oracle as CO
from oracle import evolu_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.set_option(1, 0)
    e.close()


def _apply(eng, ts, cell, n_cells, path, tree_in="{}", prior=None, prior_present=None):
    from evolu_amd import _lib as L

    eng.set_option(L.OPT_CLIENT_PATH, path)
    try:
        tin = eng.tree_from_json([tree_in])
        pt = None if prior is None else eng.dev(prior)
        pp = None if prior_present is None else eng.dev(prior_present.astype(np.uint8))
        flags, winner, tout, st = eng.apply_batch(tin, eng.dev(ts), eng.dev(cell.astype(np.uint32)), n_cells,
                                                  prior_ts=pt, prior_present=pp, raise_on_error=False)
        return st, flags.cpu().numpy(), winner.cpu().numpy(), (tout.to_json(0) if tout is not None else None)
    finally:
        eng.set_option(L.OPT_CLIENT_PATH, 0)


def _stats(eng):
    s = eng.stats()
    return s["small_batches"], s["small_fallbacks"]


def test_config1_stream_vs_c_oracle(eng):
    """BASELINE config 1 (the todo app's messages in send order, ~55k cells):
    the auto choice takes the small path, bit-exact against the oracle."""
    from evolu_amd import synth

    ts, cell, cells, _ = synth.config1(100_000)
    n_cells = len(cells)
    st_o, f_o, w_o, js_o = CO.apply(ts, cell, n_cells)
    b0, _ = _stats(eng)
    st, f, w, js = _apply(eng, ts, cell, n_cells, 0)
    assert _stats(eng)[0] == b0 + 1
    assert st == st_o == 0
    assert np.array_equal(f, f_o) and np.array_equal(w, w_o) and js == js_o


@pytest.mark.parametrize("n,n_cells,seed", [(1, 1, 1), (100, 40, 2), (5000, 3000, 3), (60_000, 20_000, 4)])
def test_random_batches_with_prior_vs_c_oracle(eng, n, n_cells, seed):
    """Shuffled streams with redeliveries, equal millis across nodes and a
    prior max per cell (SELECT ... ORDER BY timestamp DESC LIMIT 1)."""
    from evolu_amd import synth

    ts, _, cell = synth.config5(1, max(n, 50), cells_per_owner=n_cells, seed_config=seed)
    ts, cell = ts[:n], cell[:n].astype(np.uint32)
    rng = np.random.default_rng(seed)
    # priors (stored rows, none of them a batch timestamp): from another stream
    # over the same time span -- some cells' prior max is older than their
    # batch rows, some newer
    other, _, _ = synth.config5(1, max(n_cells, 50), cells_per_owner=n_cells, seed_config=seed + 100)
    prior = other[rng.integers(0, len(other), n_cells)].copy()
    present = rng.random(n_cells) < 0.5
    st_o, f_o, w_o, js_o = CO.apply(ts, cell, n_cells, prior, present)
    st, f, w, js = _apply(eng, ts, cell, n_cells, 4, prior=prior, prior_present=present)
    assert st == st_o
    if st == 0:
        assert np.array_equal(f, f_o) and np.array_equal(w, w_o) and js == js_o


def test_tree_in_merge_matches_sort_path(eng):
    """A second batch onto the first batch's tree: the leaf merge (equal keys
    XOR-combine) gives the sort path's tree, and the oracle's for both
    batches at once."""
    from evolu_amd import synth

    ts, cell, cells, _ = synth.config1(30_000, seed_config=7)
    n_cells = len(cells)
    st1, _, _, js1 = _apply(eng, ts[:12_000], cell[:12_000], n_cells, 4)
    assert st1 == 0
    st_s, f_s, w_s, js_s = _apply(eng, ts[12_000:], cell[12_000:], n_cells, 2, tree_in=js1)
    st_m, f_m, w_m, js_m = _apply(eng, ts[12_000:], cell[12_000:], n_cells, 4, tree_in=js1)
    assert st_s == st_m == 0
    assert np.array_equal(f_m, f_s) and js_m == js_s
    assert js_m == CO.tree_json(ts)  # every message of both batches is new: all XORed once


def test_collision_and_noncanonical(eng):
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts, cell, cells, _ = synth.config1(4000, seed_config=8)
    n_cells = len(cells)
    t2, c2 = ts.copy(), cell.copy()
    t2[3000] = t2[10]
    c2[3000] = (c2[10] + 1) % n_cells  # one timestamp under two cells: the PK case
    st, _, _, _ = _apply(eng, t2, c2, n_cells, 4)
    assert st == L.EVM_ECOLLISION == CO.apply(t2, c2, n_cells)[0]
    t3 = ts.copy()
    t3[77, 5] = ord("x")
    st, f, _, _ = _apply(eng, t3, cell, n_cells, 4)
    assert st == L.EVM_ENONCANON
    assert f[77] == L.MSG_BAD and (f[:77] == 0).all()


def test_long_cells_and_fallbacks_give_the_same_answers(eng):
    """A cell of 40 rows (one wave of k_sm_long_wave) and one of 300 rows (a
    workgroup of k_sm_long sorts it in LDS) stay on the small path; a cell of
    5,000 rows (> 4,096) and minutes 60 days apart
    hand the batch to the sort path (small_fallbacks counts them); every
    result exact."""
    from evolu_amd import synth

    ts, cell = synth.config2(12_000, 3000, seed_config=11)  # (unique timestamps)
    cell = cell.astype(np.uint32)
    cell[:40] = 5  # a long cell
    cell[40:340] = 6  # a longer one
    b0, f0 = _stats(eng)
    st_o, f_o, w_o, js_o = CO.apply(ts, cell, 3000)
    st, f, w, js = _apply(eng, ts, cell, 3000, 4)
    assert _stats(eng) == (b0 + 1, f0)
    assert st == st_o == 0 and np.array_equal(f, f_o) and np.array_equal(w, w_o) and js == js_o
    cell2 = cell.copy()
    cell2[1000:6000] = 7  # too long for LDS
    st_o, f_o, w_o, js_o = CO.apply(ts, cell2, 3000)
    st, f, w, js = _apply(eng, ts, cell2, 3000, 4)
    assert _stats(eng) == (b0 + 1, f0 + 1)
    assert st == st_o == 0 and np.array_equal(f, f_o) and np.array_equal(w, w_o) and js == js_o
    t2 = ts.copy()
    late = O.timestamp_to_string(O.parse_canonical(bytes(ts[0][:46]).decode())[0] + 60 * 86_400_000, 0,
                                 "00000000000000aa")
    t2[9, :46] = np.frombuffer(late.encode(), dtype=np.uint8)
    cell3 = (np.arange(len(ts)) % 3000).astype(np.uint32)
    st_o, f_o, w_o, js_o = CO.apply(t2, cell3, 3000)
    st, f, w, js = _apply(eng, t2, cell3, 3000, 4)
    assert _stats(eng) == (b0 + 1, f0 + 2)
    assert st == st_o == 0 and np.array_equal(f, f_o) and np.array_equal(w, w_o) and js == js_o
