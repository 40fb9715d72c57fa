"""evm_dist_ingest: addMessages over a route's received records read where
they arrived (apps/server/src/index.ts:138-171 per owner) must be exactly
evm_server_ingest over the rows evm_dist_take rebuilds -- flags, stored rows
(ids = receive index), trees -- on loopback ranks, for every record format
(24-B, 32-B, raw after an invalid row), interleaved and run-ordered requests,
owners big enough to be cut into key-range segments or sent to the sort
path, split (hot) owners, every server path option, and redeliveries inside
and across slices."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SEED = 0xE7010006


def _slices(world, n_owners, grouped, seed):
    from evolu_amd import synth

    out = []
    for r in range(world):
        ts, _ = synth.config2(30_000, 1000, seed_config=seed + r)
        rng = np.random.default_rng(seed * 7 + r)
        n = len(ts)
        owner = rng.integers(2, n_owners, n).astype(np.uint32)
        owner[: n // 8] = 0  # ~7,500 rows over the ranks: above the LDS capacity (sort path)
        owner[n // 8: n // 8 + n // 20] = 1  # ~3,000: cut into key-range segments
        # redeliveries: inside this slice, and of the previous slice's rows (same owners)
        d, src = rng.integers(0, n, n // 10), rng.integers(0, n, n // 10)
        ts[d] = ts[src]
        owner[d] = owner[src]
        if r and out:
            k = min(2000, n)
            ts[:k] = out[-1][0][:k]
            owner[:k] = out[-1][1][:k]
        perm = np.argsort(owner, kind="stable") if grouped else rng.permutation(n)
        out.append((np.ascontiguousarray(ts[perm]), np.ascontiguousarray(owner[perm])))
    return out


def _run(world, grouped, need_src, invalid=False, hot=False, path=0, keep=False):
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.engine import run_loopback
    from evolu_amd.sharded import ShardedServer

    n_owners = 300
    ids = synth.config4_owner_ids(SEED, n_owners)
    slices = _slices(world, n_owners, grouped, 17 + world)
    if invalid:
        slices[-1][0][5, 3] = ord("x")  # not a date: every rank routes raw records

    def fn(r, eng, dd):
        if path:
            eng.set_option(L.OPT_SERVER_PATH, path)
        pad = np.zeros((n_owners, 24), dtype=np.uint8)
        pad[:, :21] = ids
        sv = ShardedServer(eng, dd, eng.dev(pad), 21)
        ts, owner = slices[r]
        if hot:
            sv.set_hot([0, 7])
        t_in = eng.dev(ts)
        n = dd.route(t_in, eng.dev(owner), need_src=need_src, keep_input=keep)
        a = eng.store_new(sv.n_local)
        st_a = L.EVM_OK
        fa = torch.empty(max(n, 1), dtype=torch.uint8, device=torch.device("cuda", eng.device))
        try:
            dd.ingest(a, r << 40, fa)
        except L.EngineError as e:
            st_a = e.status
        t2, o2, _, _, _ = dd.take(aux=False, src=False)  # (the route stays staged)
        b = eng.store_new(sv.n_local)
        fb, st_b = b.ingest(t2, o2, r << 40, raise_on_error=False)
        out = {"n": n, "st": (st_a, st_b), "flags": (fa[:n].cpu().numpy(), fb[:n].cpu().numpy())}
        if st_a == L.EVM_OK and st_b == L.EVM_OK:
            out["msgs"] = (a.messages(), b.messages())
            out["tree"] = tuple(tuple(x.cpu().numpy() for x in s.tree().slice_device(0, sv.n_local)) for s in (a, b))
            out["ins"] = int(((fa[:n] & L.MSG_INS) != 0).sum().item())
        a.free()
        b.free()
        sv.close()
        return out

    return run_loopback(world, fn)


def _check(res, ok=True):
    from evolu_amd import _lib as L

    for out in res:
        st_a, st_b = out["st"]
        assert st_a == st_b, out["st"]
        assert np.array_equal(out["flags"][0], out["flags"][1])
        if ok:
            assert st_a == L.EVM_OK
            (oa, ia), (ob, ib) = out["msgs"]
            assert np.array_equal(oa, ob) and np.array_equal(ia, ib)
            for x, y in zip(*out["tree"]):
                assert np.array_equal(x, y)
            assert 0 < out["ins"] < out["n"]  # redeliveries ignored


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("grouped", [False, True])
@pytest.mark.parametrize("need_src", [False, True])
def test_dist_ingest_is_take_plus_ingest(world, grouped, need_src):
    _check(_run(world, grouped, need_src))


def test_dist_ingest_hot_owners():
    _check(_run(2, True, False, hot=True))


@pytest.mark.parametrize("path", [2, 3, 4])
def test_dist_ingest_server_paths(path):
    _check(_run(2, False, False, path=path))


def test_dist_ingest_raw_records_flag_the_culprit():
    from evolu_amd import _lib as L

    res = _run(2, False, False, invalid=True)
    _check(res, ok=False)
    assert any(out["st"][0] == L.EVM_ENONCANON for out in res)


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("grouped", [False, True])
def test_keep_input_route_equals_copied_route(world, grouped):
    """EVM_ROUTE_KEEP_INPUT: this rank's own rows are neither parsed nor
    copied by the route; take and ingest read them from the caller's rows.
    Flags, stored rows and trees equal the route that copies them, and take
    + ingest equals the dist ingest."""
    a = _run(world, grouped, False, keep=True)
    _check(a)
    b = _run(world, grouped, False, keep=False)
    for x, y in zip(a, b):
        assert x["n"] == y["n"] and x["st"] == y["st"]
        assert np.array_equal(x["flags"][0], y["flags"][0])
        for u, v in zip(x["msgs"][0], y["msgs"][0]):
            assert np.array_equal(u, v)
        for u, v in zip(x["tree"][0], y["tree"][0]):
            assert np.array_equal(u, v)


def test_keep_input_invalid_own_row_is_flagged_by_the_ingest():
    """With the own rows left unparsed, a row of them outside the native
    domain does not send the route raw: the ingest finds it (EVM_ENONCANON,
    the row flagged EVM_MSG_BAD), exactly as take + evm_server_ingest."""
    from evolu_amd import _lib as L

    res = _run(1, False, False, invalid=True, keep=True)
    _check(res, ok=False)
    st_a, _ = res[0]["st"]
    assert st_a == L.EVM_ENONCANON
    assert res[0]["flags"][0][5] == L.MSG_BAD
