"""addMessages is one transaction (apps/server/src/index.ts:147-169: BEGIN ...
COMMIT, ROLLBACK on any throw).  A batch with owners too big for the
per-owner LDS path is ingested in two phases (LDS path, then the sort path
for the big owners); a failure in the second phase must leave the store and
its trees exactly as they were, and report no inserted message."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import os

    from evolu_amd.engine import Engine

    os.environ["EVM_TEST_HOOKS"] = "1"  # include/evm_test.h: the fault hook answers only with it set
    e = Engine(0)
    yield e
    _fault(e, 0)
    e.close()
    del os.environ["EVM_TEST_HOOKS"]


def _fault(eng, mode):
    """include/evm_test.h evm_test_fault (test-only, outside the product ABI)."""
    from evolu_amd import _lib as L

    L.check(L.load().evm_test_fault(eng.h, mode), "evm_test_fault")


def _snapshot(store):
    off, ids = store.messages()
    toff, code, xr = store.tree().leaves()
    return off.copy(), ids.copy(), toff.copy(), code.copy(), xr.copy()


def _batch(seed, n_owners=64):
    from evolu_amd import synth

    # Zipf sizes: a few owners above the 4,096-message LDS capacity
    ts, owner, _ = synth.config5(n_owners, 60_000, zipf_s=1.2, seed_config=seed)
    return ts, owner


def test_split_ingest_rolls_back_on_phase2_failure(eng):
    from evolu_amd import _lib as L

    n_owners = 64
    ts_a, own_a = _batch(41, n_owners)
    ts_b, own_b = _batch(42, n_owners)
    assert np.bincount(own_b, minlength=n_owners).max() > 4096  # the split path is taken
    eng.set_option(L.OPT_SERVER_PATH, 3)  # big owners through the sort path (no key-range segments)
    store = eng.store_new(n_owners)
    store.ingest(eng.dev(ts_a), eng.dev(own_a), 0)
    before = _snapshot(store)
    flags = eng.dev(np.full(len(ts_b), 0x55, dtype=np.uint8))
    _fault(eng, 1)
    _, st = store.ingest(eng.dev(ts_b), eng.dev(own_b), len(ts_a), flags=flags, raise_on_error=False)
    _fault(eng, 0)
    eng.set_option(L.OPT_SERVER_PATH, 0)
    assert st == L.EVM_ENOMEM
    after = _snapshot(store)
    for x, y in zip(before, after):
        assert np.array_equal(x, y)
    assert int(flags.cpu().numpy().astype(np.int64).sum()) == 0, "no message reported as inserted"
    # the retry succeeds and equals the all-sort-path ingest of the same two batches
    f_ok, st = store.ingest(eng.dev(ts_b), eng.dev(own_b), len(ts_a), raise_on_error=False)
    assert st == L.EVM_OK
    ref = eng.store_new(n_owners)
    eng.set_option(L.OPT_SERVER_PATH, 2)
    ref.ingest(eng.dev(ts_a), eng.dev(own_a), 0)
    f_ref, _ = ref.ingest(eng.dev(ts_b), eng.dev(own_b), len(ts_a))
    eng.set_option(L.OPT_SERVER_PATH, 0)
    assert np.array_equal(f_ok.cpu().numpy(), f_ref.cpu().numpy())
    for x, y in zip(_snapshot(store), _snapshot(ref)):
        assert np.array_equal(x, y)
    store.free()
    ref.free()


def test_steady_state_makes_no_allocations(eng):
    """Repeated ingests into fresh stores (the server bench step) reuse the
    engine's freed device blocks and its workspace: no allocation call after
    the first rounds."""
    n_owners = 64
    ts, own = _batch(43, n_owners)
    dts, down = eng.dev(ts), eng.dev(own)
    for _ in range(3):
        s = eng.store_new(n_owners)
        s.ingest(dts, down, 0)
        s.free()
    a = eng.stats()
    for _ in range(5):
        s = eng.store_new(n_owners)
        s.ingest(dts, down, 0)
        s.free()
    b = eng.stats()
    assert b["workspace_regrows"] == a["workspace_regrows"]
    assert b["block_allocs"] == a["block_allocs"]
    assert b["scratch_pool_allocs"] == a["scratch_pool_allocs"]


def test_merge_guard_refuses_overlapping_keys(eng):
    """The merge (k_svo_b) places rows assuming the segment's stored and new
    keys are disjoint.  With K5's check against the stored rows switched off
    (evm_test_fault 2, include/evm_test.h) a redelivered stored timestamp reaches the merge as
    a new row: the guard must return EVM_ESTATE -- not fault, not commit --
    leave the store as it was and report nothing inserted; the same batch
    then ingests normally."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    n_owners = 200
    ts, own, _ = synth.config3(n_owners, 300, request=300, seed_config=71)
    half = len(ts) // 2
    store = eng.store_new(n_owners)
    store.ingest(eng.dev(ts[:half]), eng.dev(own[:half]), 0)
    before = _snapshot(store)
    # the second half plus a redelivery of every 7th stored row, in their owners' requests
    rng = np.random.default_rng(5)
    redo = np.arange(0, half, 7)
    ts_b = np.concatenate([ts[half:], ts[redo]])
    own_b = np.concatenate([own[half:], own[redo]])
    order = np.argsort(own_b, kind="stable")  # requests stay runs of one owner
    ts_b, own_b = ts_b[order], own_b[order]
    del rng
    for path in (0, 3):  # segments of one owner; the LDS path without segments
        eng.set_option(L.OPT_SERVER_PATH, path)
        flags = eng.dev(np.full(len(ts_b), 0x55, dtype=np.uint8))
        _fault(eng, 2)
        _, st = store.ingest(eng.dev(ts_b), eng.dev(own_b), 10_000_000, flags=flags, raise_on_error=False)
        _fault(eng, 0)
        assert st == L.EVM_ESTATE
        assert int(flags.cpu().numpy().astype(np.int64).sum()) == 0, "no message reported as inserted"
        for x, y in zip(before, _snapshot(store)):
            assert np.array_equal(x, y)
    eng.set_option(L.OPT_SERVER_PATH, 0)
    f_ok, st = store.ingest(eng.dev(ts_b), eng.dev(own_b), 10_000_000, raise_on_error=False)
    assert st == L.EVM_OK
    ref = eng.store_new(n_owners)
    eng.set_option(L.OPT_SERVER_PATH, 2)
    ref.ingest(eng.dev(ts[:half]), eng.dev(own[:half]), 0)
    f_ref, _ = ref.ingest(eng.dev(ts_b), eng.dev(own_b), 10_000_000)
    eng.set_option(L.OPT_SERVER_PATH, 0)
    assert np.array_equal(f_ok.cpu().numpy(), f_ref.cpu().numpy())
    assert int((f_ok.cpu().numpy() & L.MSG_INS).astype(bool).sum()) == len(ts) - half
    for x, y in zip(_snapshot(store), _snapshot(ref)):
        assert np.array_equal(x, y)
    store.free()
    ref.free()


def test_fault_hook_refused_without_test_env(eng):
    """The fault hook is not on the product ABI: without EVM_TEST_HOOKS=1 it
    refuses (EVM_EINVAL) and the context keeps its checks."""
    import os

    from evolu_amd import _lib as L

    del os.environ["EVM_TEST_HOOKS"]
    try:
        assert L.load().evm_test_fault(eng.h, 2) == L.EVM_EINVAL
    finally:
        os.environ["EVM_TEST_HOOKS"] = "1"
    assert L.load().evm_test_fault(eng.h, 0) == L.EVM_OK
