"""BASELINE-size parity: the HIP engine against the C restatement of the
reference (oracle/c), bit for bit -- per-message flags, per-cell winners and
the whole Merkle tree JSON -- on config-2 streams with stale and exact
redeliveries; and server ingest on a config-3-shaped stream."""
import numpy as np
import pytest

from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("n,cells", [(1_000_000, 1000), (10_000_000, 1000), (300_000, 7)])
def test_apply_vs_c_oracle(eng, n, cells):
    from evolu_amd import synth

    ts, cell = synth.config2(n, cells, seed_config=2)
    rng = np.random.default_rng(n)
    dup = rng.integers(0, n, size=n // 50)  # redeliveries: mostly stale (toggle), some of the cell max (no-op)
    ts = np.concatenate([ts, ts[dup]])
    cell = np.concatenate([cell, cell[dup]])
    st, f_want, w_want, js_want = CO.apply(ts, cell, cells)
    assert st == 0
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts), eng.dev(cell), cells)
    assert np.array_equal(flags.cpu().numpy(), f_want)
    assert np.array_equal(winner.cpu().numpy(), w_want)
    assert tree.to_json(0) == js_want


def test_server_ingest_vs_c_oracle(eng):
    from evolu_amd import synth

    ts, owner, _ = synth.config3(n_owners=5000, per_owner=200, seed_config=3)
    rng = np.random.default_rng(1)
    dup = rng.integers(0, len(ts), size=len(ts) // 10)  # redeliveries
    ts = np.concatenate([ts, ts[dup]])
    owner = np.concatenate([owner, owner[dup]])
    half = len(ts) // 2
    srv = CO.Server(5000, len(ts))
    store = eng.store_new(5000)
    for a, b in ((0, half), (half, len(ts))):
        st, f_want = srv.ingest(ts[a:b], owner[a:b])
        assert st == 0
        f, _ = store.ingest(eng.dev(ts[a:b]), eng.dev(owner[a:b]), a)
        assert np.array_equal(f.cpu().numpy(), f_want)
    tree = store.tree()
    for o in range(0, 5000, 97):
        assert tree.to_json(o) == srv.tree_json(o)
