"""BASELINE config 5 at test scale: Zipf-1.2 owners, bursts of equal millis
across nodes (ties broken by counter then node bytes), ~1 % upper-case node
ids, 10 % redeliveries (stale ones toggle the Merkle XOR).  The engine
against the C restatement of the reference (oracle/c), bit for bit: server
ingest flags and trees; client applyMessages flags, winners and trees per
owner (multi-owner sort path) and for the hottest owner alone (streaming
path)."""
import numpy as np
import pytest

from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu

N_OWNERS, N, CELLS = 400, 240_000, 50


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def stream():
    from evolu_amd import synth

    return synth.config5(N_OWNERS, N, cells_per_owner=CELLS, seed_config=5)


def test_server_ingest_adversarial(eng, stream):
    ts, owner, _ = stream
    srv = CO.Server(N_OWNERS, len(ts))
    st, want = srv.ingest(ts, owner)
    assert st == 0
    store = eng.store_new(N_OWNERS)
    got, st = store.ingest(eng.dev(ts), eng.dev(owner), 0)
    assert st == 0
    assert np.array_equal(got.cpu().numpy(), want)
    tree = store.tree()
    counts = np.bincount(owner, minlength=N_OWNERS)
    for o in list(np.argsort(-counts)[:5]) + list(range(0, N_OWNERS, 37)):
        assert tree.to_json(int(o)) == srv.tree_json(int(o)), o


def test_client_apply_adversarial_per_owner(eng, stream):
    ts, owner, cell = stream
    n_cells = N_OWNERS * CELLS
    cell_owner = np.repeat(np.arange(N_OWNERS, dtype=np.uint32), CELLS)
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(N_OWNERS), eng.dev(ts), eng.dev(cell), n_cells,
                                              cell_owner=eng.dev(cell_owner))
    assert st == 0
    f = flags.cpu().numpy()
    w = winner.cpu().numpy()
    counts = np.bincount(owner, minlength=N_OWNERS)
    for o in list(np.argsort(-counts)[:3]) + list(range(1, N_OWNERS, 53)):
        idx = np.nonzero(owner == o)[0]
        st, fw, ww, js = CO.apply(ts[idx], cell[idx] - o * CELLS, CELLS)
        assert st == 0
        assert np.array_equal(f[idx], fw), o
        gw = w[o * CELLS:(o + 1) * CELLS]
        assert np.array_equal(np.where(gw >= 0, np.searchsorted(idx, gw), -1), ww), o
        assert tree.to_json(int(o)) == js, o


def test_client_streaming_path_hot_owner(eng, stream):
    """The hottest owner alone through the streaming path (one owner, 50 cells)."""
    from evolu_amd import _lib as L

    ts, owner, cell = stream
    o = int(np.argmax(np.bincount(owner)))
    idx = np.nonzero(owner == o)[0]
    lts, lcell = np.ascontiguousarray(ts[idx]), (cell[idx] - o * CELLS).astype(np.uint32)
    st, fw, ww, js = CO.apply(lts, lcell, CELLS)
    assert st == 0
    eng.set_option(L.OPT_CLIENT_PATH, 1)
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(lts), eng.dev(lcell), CELLS)
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    assert st == 0
    assert np.array_equal(flags.cpu().numpy(), fw)
    assert np.array_equal(winner.cpu().numpy(), ww)
    assert tree.to_json(0) == js
