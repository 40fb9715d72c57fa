"""The evm_dist_* C ABI (RCCL) on one GPU (world 1: every row routes to this
rank through RCCL's self send/recv): the exchange keeps batch order, the
take groups by local owner stably, the roots gather matches the trees.
Multi-rank routing order is covered by the gloo tests of the same algorithm
(tests/test_dist.py); 8-GPU runs are the driver's."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def dist(eng):
    from evolu_amd.engine import Dist, dist_unique_id

    d = Dist(eng, dist_unique_id(), 0, 1)
    yield d
    d.free()


def _rows(n, n_owners, seed):
    from evolu_amd import synth

    ts, _ = synth.config2(n, 1000, seed_config=seed)
    rng = np.random.default_rng(seed)
    owner = rng.integers(0, n_owners, n).astype(np.uint32)
    aux = rng.integers(0, 1 << 31, n).astype(np.uint32)
    return ts, owner, aux


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 300_000])
def test_route_take_keeps_order(eng, dist, n):
    ts, owner, aux = _rows(max(n, 1000), 37, n + 1)
    ts, owner, aux = ts[:n], owner[:n], aux[:n]
    got = dist.route(eng.dev(ts), eng.dev(owner), eng.dev(aux))
    assert got == n
    t2, o2, a2, src, g = dist.take()
    assert g is None
    assert np.array_equal(t2.cpu().numpy(), ts)
    assert np.array_equal(o2.cpu().numpy().view(np.uint32), owner)
    assert np.array_equal(a2.cpu().numpy().view(np.uint32), aux)
    assert np.array_equal(src.cpu().numpy(), np.arange(n, dtype=np.int64))  # source rank 0, index i


@pytest.mark.parametrize("group", [1, 5, 8, 64])
def test_take_grouped_by_local_owner(eng, dist, group):
    n = 250_000
    ts, owner, aux = _rows(n, group, 7 + group)
    assert dist.route(eng.dev(ts), eng.dev(owner), eng.dev(aux)) == n
    t2, o2, a2, src, goff = dist.take(group=group)
    order = np.argsort(owner, kind="stable")
    assert np.array_equal(src.cpu().numpy(), order)
    assert np.array_equal(t2.cpu().numpy(), ts[order])
    assert np.array_equal(a2.cpu().numpy().view(np.uint32), aux[order])
    want = np.concatenate([[0], np.cumsum(np.bincount(owner, minlength=group))])
    assert goff == list(want)
    # the staged rows can be taken again (ungrouped this time)
    t3, _, _, s3, _ = dist.take()
    assert np.array_equal(s3.cpu().numpy(), np.arange(n))


def test_bad_dest_and_group_overflow(eng, dist):
    from evolu_amd import _lib as L

    n = 10_000
    ts, owner, aux = _rows(n, 4, 3)
    dest = np.zeros(n, dtype=np.uint8)
    dest[77] = 1  # no rank 1 in a world of 1
    with pytest.raises(L.EngineError) as e:
        dist.route(eng.dev(ts), eng.dev(owner), None, dest=eng.dev(dest))
    assert e.value.status == L.EVM_EINVAL
    # the exchange completed without the bad row; the next route is clean
    assert dist.route(eng.dev(ts), eng.dev(owner), dest=eng.dev(np.zeros(n, dtype=np.uint8))) == n
    with pytest.raises(L.EngineError) as e:
        dist.take(group=3)  # owners 0..3 do not fit 3 groups
    assert e.value.status == L.EVM_EINVAL
    small = (torch.empty((10, 48), dtype=torch.uint8, device="cuda"), torch.empty(10, dtype=torch.int32, device="cuda"),
             None, None)
    with pytest.raises(L.EngineError) as e:
        dist.take(out=small)
    assert e.value.status == L.EVM_ECAPACITY


def test_gather_roots_matches_trees(eng, dist):
    from evolu_amd import synth

    n_owners = 1000
    ts, owner = synth.config3(n_owners, 20, seed_config=5)[:2]
    owner = owner.astype(np.uint32)
    owner[owner == 17] = 18  # an owner without messages: present = 0
    trees = eng.merkle_insert(eng.tree_new(n_owners), eng.dev(ts), eng.dev(owner))
    root, present = dist.gather_roots(trees, n_owners)
    r, p = trees.roots()
    assert np.array_equal(root.cpu().numpy(), r) and np.array_equal(present.cpu().numpy(), p)


def test_gather_roots_of_single_owner_trees(eng, dist):
    """One tree per local owner (the client path's per-owner batches): the
    local owners are the trees' owners in order, the rest absent."""
    from evolu_amd import synth

    ts, owner = synth.config3(4, 50, seed_config=9)[:2]
    trees = [eng.merkle_insert(eng.tree_new(1), eng.dev(ts[owner == o])) for o in range(3)]
    root, present = dist.gather_roots(trees, 5)
    want = [int(t.roots()[0][0]) for t in trees]
    assert root.cpu().tolist()[:3] == want and present.cpu().tolist() == [True, True, True, False, False]


def test_packed_wire_rebuilds_rows_exactly(eng, dist):
    """48-B rows travel as 32-B packed records (parsed tc, node, case mask) and
    are rebuilt byte for byte: mixed-case nodes, counters, dates across
    years.  A row outside the native domain cannot be rebuilt from the
    packed form, so its route travels raw and every byte arrives; a 56-B
    stride travels raw."""
    import random

    from oracle import evolu_oracle as O
    from tests import workloads as W

    rng = random.Random(4)
    strings = []
    for _ in range(5000):
        ms = rng.randrange(0, 2 ** 31 * 60000 - 1)
        node = W.node_id(rng, upper=rng.random() < 0.5)
        node = "".join(c.upper() if rng.random() < 0.3 else c for c in node)
        strings.append(O.timestamp_to_string(ms, rng.randrange(65536), node))
    ts = eng.timestamps(strings).cpu().numpy()
    owner = np.arange(len(strings), dtype=np.uint32) % 5
    assert dist.route(eng.dev(ts), eng.dev(owner)) == len(strings)
    t2, o2, _, src, _ = dist.take()
    assert np.array_equal(t2.cpu().numpy(), ts)
    # rows outside the native domain: the whole route goes raw, nothing is lost
    bad = ts.copy()
    bad[17, 3] = ord("x")  # not a date
    bad[4000, 26] = ord("g")  # not hex
    bad[:, 46] = 7  # padding bytes ride along in raw records
    assert dist.route(eng.dev(bad), eng.dev(owner)) == len(strings)
    t2, _, _, _, _ = dist.take()
    assert np.array_equal(t2.cpu().numpy(), bad)
    # raw records for a non-48 stride: bytes 46.. carry data and arrive unchanged
    ext = np.concatenate([ts, np.arange(len(ts) * 8, dtype=np.uint8).reshape(-1, 8)], 1)
    assert dist.route(eng.dev(ext), eng.dev(owner)) == len(strings)
    t3, _, _, _, _ = dist.take()
    assert np.array_equal(t3.cpu().numpy(), ext)


def test_route_larger_than_4gib_arrives_whole(eng, dist):
    """A route whose exchange is > 2^32 bytes (140M rows x 32-B records: the
    config-4 share of one GPU) arrives byte for byte through RCCL (the
    transfer is cut into pieces)."""
    from evolu_amd import synth

    gen = synth.DeviceSynth()
    dev = torch.device("cuda", 0)
    ts, owner, _ = gen.source(0xE7010004, 140_000, 1000, 1, 0, dev)
    n = dist.route(ts, owner)
    assert n == ts.shape[0]
    out = (torch.empty_like(ts), torch.empty_like(owner), None, None)
    t2, o2, _, _, _ = dist.take(aux=False, src=False, out=out)
    assert torch.equal(t2, ts) and torch.equal(o2, owner)
    del ts, owner, out, t2, o2
    torch.cuda.empty_cache()
