"""The evm_dist_* C ABI at world 2 and 3 on one GPU: loopback ranks (one
thread, context and HIP stream each, evm_dist_hub) run the same partitions,
count exchange, grouped take, directory and root gather as RCCL would, with
device-to-device copies for the transfers.  Checked against a numpy model of
the routing and against the unsharded C restatement of the server
(apps/server/src/index.ts:138-202) -- the config-4 path end to end."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as CO
from oracle import evolu_oracle as O

pytestmark = pytest.mark.gpu

SEED = 0xE7010004


def _loop(world, fn):
    from evolu_amd.engine import run_loopback

    return run_loopback(world, fn)


def _slices(world, n_per, n_owners, seed):
    from evolu_amd import synth

    out = []
    for r in range(world):
        n = n_per[r] if isinstance(n_per, list) else n_per
        ts, _ = synth.config2(max(n, 1000), 1000, seed_config=seed + r)
        ts = ts[:n]
        rng = np.random.default_rng(seed * 10 + r)
        owner = rng.integers(0, n_owners, len(ts)).astype(np.uint32)
        aux = rng.integers(0, 1 << 31, len(ts)).astype(np.uint32)
        out.append((ts, owner, aux))
    return out


def _expected(slices, world, r, key):
    """Rows for rank r in (source rank, source order): ts, owner, aux, src."""
    parts = []
    for s, (ts, owner, aux) in enumerate(slices):
        sel = np.flatnonzero(key(owner) == r)
        parts.append((ts[sel], owner[sel], aux[sel], (np.int64(s) << 32) | sel.astype(np.int64)))
    return [np.concatenate([p[k] for p in parts]) for k in range(4)]


@pytest.mark.parametrize("world,n_per", [(2, 100_000), (3, [0, 70_001, 4097]), (2, [1, 0])])
def test_route_take_keeps_global_order(world, n_per):
    slices = _slices(world, n_per, 41, 11)

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        n = dd.route(eng.dev(ts), eng.dev(owner), eng.dev(aux))
        t2, o2, a2, src, _ = dd.take()
        return n, t2.cpu().numpy(), o2.cpu().numpy().view(np.uint32), a2.cpu().numpy().view(np.uint32), src.cpu().numpy()

    res = _loop(world, fn)
    for r in range(world):
        ts, owner, aux, src = _expected(slices, world, r, lambda o: o % world)
        n, t2, o2, a2, s2 = res[r]
        assert n == len(ts)
        assert np.array_equal(t2[:n], ts) and np.array_equal(o2[:n], owner)
        assert np.array_equal(a2[:n], aux) and np.array_equal(s2[:n].astype(np.int64), src)


def test_grouped_take_and_roots_world2():
    world, n_owners = 2, 37
    slices = _slices(world, 60_000, n_owners, 5)
    per = (n_owners + world - 1) // world

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        dd.route(eng.dev(ts), eng.dev(owner), eng.dev(aux))
        t2, o2, _, src, goff = dd.take(group=per)
        # this rank's owners' trees from their rows, then every owner's root
        lo = (o2.to(torch.int64) // world).to(torch.int32)
        tree = eng.merkle_insert(eng.tree_new(per), t2.contiguous(), lo.contiguous())
        root, present = dd.gather_roots(tree, n_owners)
        return t2.cpu().numpy(), src.cpu().numpy(), goff, root.cpu().numpy(), present.cpu().numpy()

    res = _loop(world, fn)
    all_ts = np.concatenate([s[0] for s in slices])
    all_owner = np.concatenate([s[1] for s in slices])
    for r in range(world):
        ts, owner, _, src = _expected(slices, world, r, lambda o: o % world)
        order = np.argsort(owner // world, kind="stable")
        t2, s2, goff, root, present = res[r]
        assert np.array_equal(t2, ts[order]) and np.array_equal(s2.astype(np.int64), src[order])
        want = np.concatenate([[0], np.cumsum(np.bincount(owner // world, minlength=per))])
        assert goff == list(want)
        for o in range(0, n_owners, 5):
            js = CO.tree_json(all_ts[all_owner == o])
            assert root[o] == O.merkle_tree_from_string(js).get("hash", 0)
            assert bool(present[o]) == (js != "{}")


def test_directory_route_and_roots_world3():
    """Owner g -> rank murmur3(userId_g) mod 3 (the reference hash), dense
    local ids; the route delivers local ids; roots come back per global owner."""
    from evolu_amd import synth

    world, n_owners = 3, 500
    ids = synth.config4_owner_ids(SEED, n_owners)
    dest_want = np.array([O.murmur3_32(bytes(r)) % world for r in ids])
    local_want = np.zeros(n_owners, dtype=np.int64)
    for r in range(world):
        local_want[dest_want == r] = np.arange((dest_want == r).sum())
    slices = _slices(world, 30_000, n_owners, 9)

    def fn(r, eng, dd):
        pad = np.zeros((n_owners, 24), dtype=np.uint8)
        pad[:, :21] = ids
        dest, local = dd.directory((eng.dev(pad), 21))
        ts, owner, aux = slices[r]
        dd.route(eng.dev(ts), eng.dev(owner), eng.dev(aux))
        t2, o2, a2, src, _ = dd.take()
        tree = eng.merkle_insert(eng.tree_new(dd.n_local), t2.contiguous(), o2.contiguous())
        root, present = dd.gather_roots(tree, n_owners)
        return (dest.cpu().numpy(), local.cpu().numpy(), dd.n_local, t2.cpu().numpy(), o2.cpu().numpy(),
                src.cpu().numpy(), root.cpu().numpy(), present.cpu().numpy())

    res = _loop(world, fn)
    all_ts = np.concatenate([s[0] for s in slices])
    all_owner = np.concatenate([s[1] for s in slices])
    for r in range(world):
        dest, local, n_local, t2, o2, s2, root, present = res[r]
        assert np.array_equal(dest, dest_want) and np.array_equal(local, local_want)
        assert n_local == (dest_want == r).sum()
        ts, owner, _, src = _expected(slices, world, r, lambda o: dest_want[o])
        assert np.array_equal(t2, ts) and np.array_equal(o2, local_want[owner])
        for o in range(0, n_owners, 7):
            js = CO.tree_json(all_ts[all_owner == o])
            assert root[o] == O.merkle_tree_from_string(js).get("hash", 0)
            assert bool(present[o]) == (js != "{}")


def test_invalid_row_anywhere_sends_every_rank_raw():
    """A row outside the native domain on rank 1 only: every rank's route
    falls back to raw records, and every byte of every row arrives."""
    world = 2
    slices = _slices(world, 20_000, 11, 21)
    ts1 = slices[1][0]
    ts1[123, 3] = ord("x")  # not a date
    ts1[124, 26] = ord("g")  # not hex
    for ts, _, _ in slices:
        ts[:, 46] = 0x5A  # pad bytes: only raw records carry them

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        dd.route(eng.dev(ts), eng.dev(owner), eng.dev(aux))
        t2, _, _, _, _ = dd.take()
        return t2.cpu().numpy()

    res = _loop(world, fn)
    for r in range(world):
        ts, _, _, _ = _expected(slices, world, r, lambda o: o % world)
        assert np.array_equal(res[r], ts)


def test_one_rank_unaligned_every_rank_raw_and_8b_take():
    """Rank 1's rows sit at an 8-B but not 16-B aligned address (the API only
    asks stride % 8 == 0): it cannot pack, says so in its count words, and
    every rank sends raw records -- the record sizes agree, every row arrives.
    Then a packed route taken into an 8-B aligned output (8-B stores)."""
    world = 2
    slices = _slices(world, 20_000, 13, 23)

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        t = eng.dev(ts)
        if r == 1:  # the same rows one 8-B word into a larger buffer
            flat = torch.zeros(t.numel() + 8, dtype=torch.uint8, device=t.device)
            flat[8:].copy_(t.reshape(-1))
            t = flat[8:].view(-1, 48)
            assert t.data_ptr() % 16 == 8
        dd.route(t, eng.dev(owner), eng.dev(aux))
        raw = dd.take()[0].cpu().numpy()
        n = dd.route(eng.dev(ts), eng.dev(owner), eng.dev(aux))
        buf = torch.zeros((n + 1) * 48 + 8, dtype=torch.uint8, device=t.device)
        out_ts = buf[8:8 + n * 48].view(n, 48)
        out = (out_ts, torch.empty(max(n, 1), dtype=torch.int32, device=t.device), None, None)
        t8 = dd.take(aux=False, src=False, out=out)[0].cpu().numpy()
        return raw, t8

    res = _loop(world, fn)
    for r in range(world):
        ts, _, _, _ = _expected(slices, world, r, lambda o: o % world)
        raw, t8 = res[r]
        assert np.array_equal(raw, ts)
        assert np.array_equal(t8[:, :46], ts[:, :46])


def test_mixed_strides_are_refused_on_every_rank():
    """Raw records at two strides cannot be exchanged: every rank returns
    EVM_EINVAL before any data moves, and the next route works."""
    from evolu_amd import _lib as L

    world = 2
    slices = _slices(world, 3000, 5, 41)

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        t = eng.dev(ts)
        wide = torch.zeros((t.shape[0], 56), dtype=torch.uint8, device=t.device)
        wide[:, :48] = t
        st = None
        try:
            dd.route(wide if r == 0 else t, eng.dev(owner))
        except L.EngineError as e:
            st = e.status
        return st, dd.route(t, eng.dev(owner))

    res = _loop(world, fn)
    assert res[0][0] == L.EVM_EINVAL and res[1][0] == L.EVM_EINVAL
    assert res[0][1] + res[1][1] == 6000


@pytest.mark.parametrize("raw", [False, True])
def test_empty_rank_stride_is_a_wildcard(raw):
    """A rank with no rows votes for no record format and no stride: its
    stride (56) neither sends the others raw nor fails the route as mixed
    strides.  raw=True: another rank holds a row outside the native domain, so
    every rank sends raw records at 48 B -- the empty rank receives them at
    the senders' stride."""
    world = 3
    slices = _slices(world, [20_000, 15_000, 0], 11, 61)
    if raw:
        slices[1][0][77, 3] = ord("x")  # not a date: raw records everywhere

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        if r == 2:
            t = torch.zeros((0, 56), dtype=torch.uint8, device=torch.device("cuda", eng.device))
            o = torch.zeros(0, dtype=torch.int32, device=t.device)
            n = dd.route(t, o)
        else:
            n = dd.route(eng.dev(ts), eng.dev(owner))
        t2 = dd.take(aux=False, src=False)[0].cpu().numpy()
        return n, t2

    res = _loop(world, fn)
    for r in range(world):
        ts, _, _, _ = _expected(slices, world, r, lambda o: o % world)
        n, t2 = res[r]
        assert n == len(ts)
        assert np.array_equal(t2[:, :46], ts[:, :46])


def test_local_failure_is_agreed_not_hung():
    """Rank 1 passes a bad stride: it returns EVM_EINVAL, rank 0 EVM_EDIST,
    nobody waits; the next route of both succeeds.  Same for gather_roots."""
    from evolu_amd import _lib as L

    world = 2
    slices = _slices(world, 5000, 8, 31)

    def fn(r, eng, dd):
        ts, owner, aux = slices[r]
        t = eng.dev(ts)
        bad = t[:, :40] if r == 1 else t  # stride 40 < 46
        st1 = None
        try:
            dd.route(bad.contiguous(), eng.dev(owner))
        except L.EngineError as e:
            st1 = e.status
        n = dd.route(t, eng.dev(owner))
        tree = eng.tree_new(2)
        st2 = None
        try:
            dd.gather_roots([tree] * (3 if r == 0 else 1), 8)  # rank 0: 6 local owners > 4
        except L.EngineError as e:
            st2 = e.status
        root, _ = dd.gather_roots(tree, 8)
        return st1, n, st2

    res = _loop(world, fn)
    assert res[1][0] == L.EVM_EINVAL and res[0][0] == L.EVM_EDIST
    assert res[0][1] + res[1][1] == 10_000
    assert res[0][2] == L.EVM_EINVAL and res[1][2] == L.EVM_EDIST


def test_device_generator_matches_numpy_twin():
    from evolu_amd import synth

    gen = synth.DeviceSynth()
    dev = torch.device("cuda", 0)
    O_, P, G = 301, 100, 3
    for s in range(G):
        ts, owner, keep = gen.source(SEED, O_, P, G, s, dev, keep=True)
        t_np, o_np, k_np = synth.config4_source(SEED, O_, P, G, s)
        assert np.array_equal(ts.cpu().numpy(), t_np)
        assert np.array_equal(owner.cpu().numpy().view(np.uint32), o_np)
        assert np.array_equal(keep.cpu().numpy().astype(bool), k_np)
    lst = np.array([0, 5, 300, 17], dtype=np.int64)
    ts, li, keep = gen.owners(SEED, O_, P, G, torch.from_numpy(lst), dev)
    t_np, l_np, k_np = synth.config4_owners(SEED, P, G, lst)
    assert np.array_equal(ts.cpu().numpy(), t_np) and np.array_equal(keep.cpu().numpy().astype(bool), k_np)
    assert np.array_equal(li.cpu().numpy().view(np.uint32), l_np)
    ids = gen.owner_ids(SEED, 1000, dev)
    assert np.array_equal(ids.cpu().numpy()[:, :21], synth.config4_owner_ids(SEED, 1000))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_server_vs_unsharded_c_oracle(world):
    """Config 4 in miniature through evolu_amd.sharded.ShardedServer on
    loopback ranks: each rank's slice = one request per owner of the job,
    owners sharded by murmur3(userId) mod world.  Against ONE unsharded C
    restatement of the server: INSERT OR IGNORE flags per owner, every
    owner's tree (JSON) and root, the diff against the client tree and the
    getMessages rows (timestamp > syncTs(diff), NOT LIKE '%' || node)."""
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.sharded import ShardedServer

    O_, P = 240, 60
    ids = synth.config4_owner_ids(SEED, O_)
    sources = [synth.config4_source(SEED, O_, P, world, s) for s in range(world)]
    # the unsharded reference: every source's requests in rank order
    srv = CO.Server(O_, O_ * P)
    cli = CO.Server(O_, O_ * P)
    for ts, owner, keep in sources:
        st, _ = srv.ingest(ts, owner)
        assert st == 0
        st, _ = cli.ingest(ts[keep], owner[keep])
        assert st == 0
    node_of = {o: synth.config4_messages(SEED, P, [o], [0])[0][0, 30:46].tobytes().decode() for o in range(O_)}

    def fn(r, eng, dd):
        pad = np.zeros((O_, 24), dtype=np.uint8)
        pad[:, :21] = ids
        sv = ShardedServer(eng, dd, eng.dev(pad), 21)
        ts, owner, keep = sources[r]
        t_r, o_r, f = sv.ingest(eng.dev(ts), eng.dev(owner), id_base=r << 40)
        here = sv.owners_here.cpu().numpy()
        # client trees of the local owners from their known messages (any rank's slices)
        cts, cown = [], []
        for s_ts, s_owner, s_keep in sources:
            m = s_keep & np.isin(s_owner, here)
            cts.append(s_ts[m])
            cown.append(np.searchsorted(here, s_owner[m]).astype(np.uint32))
        client = eng.merkle_insert(eng.tree_new(sv.n_local), eng.dev(np.concatenate(cts)), eng.dev(np.concatenate(cown)))
        node = eng.dev(np.frombuffer("".join(node_of[int(g)] for g in here).encode(), dtype=np.uint8).copy())
        diff, off, sel = sv.select(client, node)
        root, present = sv.roots()
        trees = [sv.store.tree().to_json(j) for j in range(sv.n_local)]
        ins = np.bincount(o_r.cpu().numpy()[(f.cpu().numpy() & L.MSG_INS) != 0], minlength=sv.n_local)
        rows = t_r.cpu().numpy()
        sel_rows = [rows[(sel[int(off[j]):int(off[j + 1])] - (r << 40)).cpu().numpy()] for j in range(sv.n_local)]
        sv.close()
        return here, ins, diff.cpu().numpy(), sel_rows, trees, root.cpu().numpy(), present.cpu().numpy()

    res = _loop(world, fn)
    covered = set()
    for r in range(world):
        here, ins, diff, sel_rows, trees, root, present = res[r]
        for j, g in enumerate(here):
            g = int(g)
            covered.add(g)
            assert ins[j] == P  # all distinct: every message inserted once
            assert trees[j] == srv.tree_json(g)
            d = srv.diff(cli, g)
            assert diff[j] == d
            sync = O.timestamp_to_string(d, 0, "0000000000000000") if d >= 0 else None
            all_rows = np.concatenate([s[0][s[1] == g] for s in sources])
            strs = sorted(bytes(x[:46]).decode() for x in all_rows)
            want = [] if sync is None else [s for s in strs if s > sync and not s.lower().endswith(node_of[g])]
            assert [bytes(x[:46]).decode() for x in sel_rows[j]] == want
        assert np.array_equal(res[r][5], res[0][5])  # every rank holds every owner's root
    assert covered == set(range(O_))
    for g in range(0, O_, 13):
        js = srv.tree_json(g)
        assert res[0][5][g] == O.merkle_tree_from_string(js).get("hash", 0) and bool(res[0][6][g])


@pytest.mark.parametrize("world", [2, 3])
def test_config4_bench_loopback_self_check(world):
    """bench.py's config-4 rank (the N-GPU default) on loopback ranks, small:
    its own self-check must pass on every rank."""
    import argparse

    import bench

    a = argparse.Namespace(c4_owners=4000, c4_per_owner=100, steps=2, warmup=1, c4_sample=300)
    out = bench.config4_loopback(a, world)
    assert out["parity_checked"] is True
    for r in range(world):
        d = out["self_check_rank%d" % r]
        assert d["received"] == d["expected"] and d["sample_owners"] > 0
        assert d["inserted"] and d["roots"] and d["diffs"] and d["selections"]


@pytest.mark.parametrize("world", [2, 3])
def test_config5_bench_loopback_self_check(world):
    """bench.py's config-5 rank (BASELINE config 5 at N GPUs: Zipf owners,
    the hot ones split over every rank, merged selections) on loopback ranks,
    small: its self-check -- sampled cold owners and every split owner
    recomputed unsharded -- must pass on every rank and must cover split
    owners and selected rows."""
    import argparse

    import bench

    a = argparse.Namespace(c5_owners=3000, c5_messages=400_000, steps=2, warmup=1, c5_sample=120, c5_share=0.1)
    out = bench.config5_loopback(a, world)
    assert out["parity_checked"] is True
    assert out["config"]["n_split_owners"] >= 1
    for r in range(world):
        d = out["self_check_rank%d" % r]
        assert d["split_owners_checked"] >= 1 and d["sample_owners"] > 0 and d["selected_rows"] > 0
        assert d["inserted"] and d["roots"] and d["diffs"] and d["split_trees"] and d["selections"]


def test_config5c_bench_loopback_self_check():
    """bench.py's client split leg (one owner's batch split by cell over 2
    loopback ranks) against the whole batch applied unsharded."""
    import argparse

    import bench

    a = argparse.Namespace(c5c_messages=200_000, c5c_cells=300, steps=2, warmup=1)
    out = bench.client_split_loopback(a, 2)
    assert out["parity_checked"] is True
    for r in range(2):
        d = out["self_check_rank%d" % r]
        assert d["flags"] and d["winners"] and d["tree"] and d["batch_rows"] == 400_000


@pytest.mark.parametrize("world", [2, 3])
def test_torch_plan_is_the_c_abi_partition(world):
    """evolu_amd/dist.py (the torch.distributed restatement the gloo CPU tests
    prove exact) assigns every row the destination rank and local id the C
    ABI does: directory, hot owners, hot_base, the split owners' rows by
    timestamp hash, cells by cell hash, the global-PK timestamp ranks."""
    from evolu_amd import dist as D
    from evolu_amd import synth

    O_, N = 60, 40_000
    ts, owner, cell = synth.config5(O_, N, seed_config=77)
    owner = owner.astype(np.uint32)
    ids = np.frombuffer(b"".join(b"x%020d" % g for g in range(O_)), dtype=np.uint8).reshape(O_, 21)
    cut = [N * r // world for r in range(world + 1)]
    dirx = D.Directory(ids, world)
    hot_py = D.hot_owners(torch.from_numpy(np.bincount(owner, minlength=O_)), world, 0.25)

    def fn(r, eng, dd):
        pad = np.zeros((O_, 24), dtype=np.uint8)
        pad[:, :21] = ids
        dest, local = dd.directory((eng.dev(pad), 21))
        t_in, o_in = eng.dev(ts[cut[r]:cut[r + 1]]), eng.dev(owner[cut[r]:cut[r + 1]])
        hot = dd.hot_owners(o_in, O_, 0.25)
        base = dd.split(hot, O_)
        dd.route(t_in, o_in, aux=eng.dev(np.arange(cut[r], cut[r + 1], dtype=np.uint32)))
        _, lo, gi, _, _ = dd.take()
        tsd = dd.ts_dest(t_in)
        cd = dd.cell_dest(eng.dev(cell[cut[r]:cut[r + 1]].astype(np.uint32)))
        return (dest.cpu().numpy(), local.cpu().numpy(), hot, base, lo.cpu().numpy(), gi.cpu().numpy(),
                tsd.cpu().numpy(), cd.cpu().numpy())

    res = _loop(world, fn)
    assert hot_py.size >= 1
    for r in range(world):
        dest, local, hot, base, lo, gi, tsd, cd = res[r]
        assert np.array_equal(dest, dirx.dest) and np.array_equal(local, dirx.local)
        assert np.array_equal(hot, hot_py)
        omap = D.OwnerMap(dirx, r, hot_py)
        assert base == omap.hot_base
        t_all = torch.from_numpy(ts)
        o_all = torch.from_numpy(owner.astype(np.int64))
        want_dest = omap.dest(o_all, t_all).numpy()
        # the rows this rank received: exactly those the plan sends here, in global order, same local ids
        mine = np.flatnonzero(want_dest == r)
        assert np.array_equal(gi.view(np.uint32).astype(np.int64), mine)
        assert np.array_equal(lo, omap.local(o_all[mine]).numpy())
        sl = slice(cut[r], cut[r + 1])
        assert np.array_equal(tsd, D.ts_dest(t_all[sl], world).numpy())
        assert np.array_equal(cd, D.cell_dest(torch.from_numpy(cell[sl].astype(np.int64)), world).numpy())


@pytest.mark.parametrize("mixed", [False, True])
def test_narrow_records_route(mixed):
    """evm_dist_route_ex with EVM_ROUTE_NO_SRC and no aux: 24-B records, every
    row arrives byte-exact with its owner; sources cannot be taken and the
    return path refuses (on every rank).  One rank asking for sources
    (mixed): every rank sends 32-B records and sources work again."""
    from evolu_amd import _lib as L

    world = 2
    slices = _slices(world, 30_000, 17, 29)

    def fn(r, eng, dd):
        ts, owner, _ = slices[r]
        need = mixed and r == 1
        n = dd.route(eng.dev(ts), eng.dev(owner), need_src=need)
        t2, o2, _, _, _ = dd.take(aux=False, src=False)
        got = (n, t2.cpu().numpy(), o2.cpu().numpy().view(np.uint32))
        st_take = st_ret = None
        try:
            dd.take(aux=False, src=True)
        except L.EngineError as e:
            st_take = e.status
        try:
            dd.send_back(torch.zeros(n, dtype=torch.int32, device=t2.device), len(ts))
        except L.EngineError as e:
            st_ret = e.status
        return got, st_take, st_ret

    res = _loop(world, fn)
    for r in range(world):
        ts, owner, _, _ = _expected(slices, world, r, lambda o: o % world)
        (n, t2, o2), st_take, st_ret = res[r]
        assert n == len(ts) and np.array_equal(t2[:, :46], ts[:, :46]) and np.array_equal(o2, owner)
        if mixed:
            assert st_take is None and st_ret is None
        else:
            assert st_take == L.EVM_EINVAL and st_ret in (L.EVM_EINVAL, L.EVM_EDIST)


@pytest.mark.parametrize("directory", [False, True])
def test_narrow_grouped_take(directory):
    """A 24-B route (three arrays, the owner column written as the receiver
    uses it) taken grouped by local owner, with and without a directory:
    rows, owners and group bounds as the 32-B route would give them."""
    from evolu_amd import synth

    world, n_owners = 3, 61
    ids = synth.config4_owner_ids(SEED, n_owners)
    dest_want = np.array([O.murmur3_32(bytes(r)) % world for r in ids]) if directory else np.arange(n_owners) % world
    local_want = np.zeros(n_owners, dtype=np.int64)
    for r in range(world):
        local_want[dest_want == r] = np.arange((dest_want == r).sum())
    if not directory:
        local_want = np.arange(n_owners) // world
    slices = _slices(world, [20_000, 33_333, 7], n_owners, 13)
    groups = int(local_want.max()) + 1

    def fn(r, eng, dd):
        if directory:
            pad = np.zeros((n_owners, 24), dtype=np.uint8)
            pad[:, :21] = ids
            dd.directory((eng.dev(pad), 21))
        ts, owner, _ = slices[r]
        n = dd.route(eng.dev(ts), eng.dev(owner), need_src=False)
        t2, o2, _, _, goff = dd.take(group=groups, aux=False, src=False)
        return n, t2.cpu().numpy(), o2.cpu().numpy().view(np.uint32), goff

    res = _loop(world, fn)
    for r in range(world):
        ts, owner, _, _ = _expected(slices, world, r, lambda o: dest_want[o])
        lo = local_want[owner]
        order = np.argsort(lo, kind="stable")
        n, t2, o2, goff = res[r]
        assert n == len(ts)
        assert np.array_equal(t2[:, :46], ts[order][:, :46])
        # the owner column: local ids with a directory, global ids without (as evm_dist_take documents)
        assert np.array_equal(o2, (lo if directory else owner)[order].astype(np.uint32))
        assert goff == list(np.concatenate([[0], np.cumsum(np.bincount(lo, minlength=groups))]))
