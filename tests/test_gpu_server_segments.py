"""Key-range segments of big owners (evm_server.hip k_seg_*): an owner whose
share of a batch exceeds the LDS capacity (4,096) is cut at sampled minute
splitters into segments that each fit the per-owner LDS kernels.  Checked
bit for bit against the global sort path (EVM_OPT_SERVER_PATH 2) and the
unsegmented LDS path (3: big owners through the sort path) -- flags, stored
rows in (owner, timestamp) order, every leaf -- over two ingests (the second
against a non-empty store, whose rows and leaves the segments must each copy
exactly once), on Zipf-skewed, bursty and mixed-key-length batches."""
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
    e.set_option(2, 0)
    e.close()


def _run(eng, path, n_owners, ts_np, owner_np, cut):
    from evolu_amd import _lib as L

    eng.set_option(L.OPT_SERVER_PATH, path)
    store = eng.store_new(n_owners)
    fl = []
    for a, b in ((0, cut), (cut, len(ts_np))):
        f, st = store.ingest(eng.dev(ts_np[a:b]), eng.dev(owner_np[a:b]), a)
        assert st == L.EVM_OK
        fl.append(f.cpu().numpy().copy())
    off, ids = store.messages()
    toff, code, xr = store.tree().leaves()
    store.free()
    eng.set_option(L.OPT_SERVER_PATH, 0)
    return np.concatenate(fl), off, ids, toff, code, xr


def _same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("n_owners,n,seed", [(200, 600_000, 1), (2000, 2_000_000, 2), (5, 300_000, 3)])
def test_zipf_segments_vs_sort_path(eng, n_owners, n, seed):
    from evolu_amd import synth

    ts_np, owner_np, _ = synth.config5(n_owners, n, seed_config=60 + seed)
    assert np.bincount(owner_np).max() > 4096
    cut = len(ts_np) * 3 // 5
    seg = _run(eng, 0, n_owners, ts_np, owner_np, cut)
    _same(seg, _run(eng, 2, n_owners, ts_np, owner_np, cut))
    _same(seg, _run(eng, 3, n_owners, ts_np, owner_np, cut))


def test_burst_minute_overflows_to_sort_path(eng):
    """A big owner with 6,000 messages in one minute: that segment cannot fit,
    so the owner goes to the sort path while the other owners' segments commit."""
    rng = random.Random(5)
    strings, owner = [], []
    nodes = [W.node_id(rng) for _ in range(8)]
    burst = [O.timestamp_to_string(W.T0 + 120_000 + rng.randrange(60_000), rng.randrange(3), rng.choice(nodes))
             for _ in range(6000)]
    spread = W.hlc_timestamps(rng, 9000, nodes, span=3 * 86_400_000)
    for o, ms in ((0, burst + spread), (1, W.hlc_timestamps(rng, 8000, nodes[:3], span=86_400_000)),
                  (2, W.hlc_timestamps(rng, 500, nodes[:2]))):
        ms = ms + ms[:100]  # redeliveries
        strings += ms
        owner += [o] * len(ms)
    perm = list(range(len(strings)))
    rng.shuffle(perm)
    strings = [strings[i] for i in perm]
    owner_np = np.array([owner[i] for i in perm], dtype=np.uint32)
    ts_np = eng.timestamps(strings).cpu().numpy()
    cut = len(strings) // 2
    seg = _run(eng, 0, 3, ts_np, owner_np, cut)
    _same(seg, _run(eng, 2, 3, ts_np, owner_np, cut))


def test_mixed_key_lengths_disable_segments(eng):
    """A batch whose minutes have base-3 keys of two lengths (a 1990 timestamp)
    is not segmented (code order != minute order across lengths): big owners
    take the sort path, results unchanged."""
    rng = random.Random(6)
    nodes = [W.node_id(rng) for _ in range(4)]
    ms = W.hlc_timestamps(rng, 9000, nodes, span=86_400_000)
    old = [O.timestamp_to_string(631_152_000_000 + k * 61_000, 0, nodes[0]) for k in range(30)]  # 1990
    strings = ms + old + ms[:50]
    rng.shuffle(strings)
    owner_np = np.zeros(len(strings), dtype=np.uint32)
    owner_np[::7] = 1
    ts_np = eng.timestamps(strings).cpu().numpy()
    cut = len(strings) // 3
    seg = _run(eng, 0, 2, ts_np, owner_np, cut)
    _same(seg, _run(eng, 2, 2, ts_np, owner_np, cut))


def test_unsampled_key_length_falls_back(eng):
    """One 1990 timestamp at a batch position the plan does not sample (the
    interleaved-owner plan reads every 16th row's minute, no minutes pass):
    the big owners are cut from the sampled range, K5 reports the second key
    length, and the batch takes the sort path -- results unchanged."""
    rng = random.Random(8)
    nodes = [W.node_id(rng) for _ in range(4)]
    strings = W.hlc_timestamps(rng, 12000, nodes, span=86_400_000)
    rng.shuffle(strings)
    strings.insert(17, O.timestamp_to_string(631_152_000_000, 0, nodes[1]))  # 17 % 16 != 0: never sampled
    owner_np = (np.arange(len(strings)) % 3 == 0).astype(np.uint32)
    owner_np[17] = 0
    ts_np = eng.timestamps(strings).cpu().numpy()
    cut = len(strings) // 2
    _same(_run(eng, 0, 2, ts_np, owner_np, cut), _run(eng, 2, 2, ts_np, owner_np, cut))


@pytest.mark.parametrize("burst", [2600, 5000])
def test_size_classes_with_burst_segment(eng, burst):
    """Many small owners (the batch takes the size-class passes: the one-wave
    128 kernel, 512, 1,024) plus a big owner whose burst minute makes one
    segment of burst/2+ messages per ingest (the 2,048 or the 4,096 class): equal to the
    sort path over two ingests."""
    rng = random.Random(burst)
    strings, owner = [], []
    nodes = [W.node_id(rng) for _ in range(8)]
    burst_ms = [O.timestamp_to_string(W.T0 + 240_000 + rng.randrange(60_000), rng.randrange(3), rng.choice(nodes))
                for _ in range(burst)]
    groups = [(0, burst_ms + W.hlc_timestamps(rng, 9000, nodes, span=3 * 86_400_000)),
              (1, W.hlc_timestamps(rng, 8000, nodes[:3], span=86_400_000))]
    groups += [(o, W.hlc_timestamps(rng, rng.randrange(5, 300), nodes[:2])) for o in range(2, 302)]
    for o, ms in groups:
        ms = ms + ms[: len(ms) // 20]  # redeliveries
        strings += ms
        owner += [o] * len(ms)
    perm = list(range(len(strings)))
    rng.shuffle(perm)
    strings = [strings[i] for i in perm]
    owner_np = np.array([owner[i] for i in perm], dtype=np.uint32)
    ts_np = eng.timestamps(strings).cpu().numpy()
    cut = len(strings) // 2
    eng.prof_enable(True)
    eng.prof_reset()
    seg = _run(eng, 0, 302, ts_np, owner_np, cut)
    ran = set(eng.prof_report())
    eng.prof_enable(False)
    assert any("k_svo_a<128" in k for k in ran), ran
    assert any(("k_svo_a<2048" if burst < 4000 else "k_svo_a<SVO_CAP") in k for k in ran), ran
    _same(seg, _run(eng, 2, 302, ts_np, owner_np, cut))


@pytest.mark.parametrize("path", [0, 2])
def test_ten_bit_radix_digits_give_the_same_store(eng, path):
    """EVM_OPT_RADIX 2 (10-bit digits where they save a pass: the segment
    sort's ~19-bit ids in 2 passes instead of 3, the sort path's 40-bit leaf
    keys in 4 instead of 5) against the 8-bit one-sweep sort, bit for bit."""
    from evolu_amd import synth

    ts_np, owner_np, _ = synth.config5(3000, 1_500_000, seed_config=64)
    cut = len(ts_np) // 2
    base = _run(eng, path, 3000, ts_np, owner_np, cut)
    eng.set_option(4, 2)
    try:
        wide = _run(eng, path, 3000, ts_np, owner_np, cut)
    finally:
        eng.set_option(4, 1)
    _same(base, wide)
