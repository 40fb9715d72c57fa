"""Server ingest/select parity (apps/server/src/index.ts) against the oracle's
verbatim-SQL server (sqlite3)."""
import json
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
    e.close()


def _requests(seed, n_owners=9, n_req=40, t0=W.T0):
    """Requests (userId, [timestamps]) with duplicates inside and across requests."""
    rng = random.Random(seed)
    owners = ["%021x" % rng.getrandbits(84) for _ in range(n_owners)]
    pools = {}
    for o in owners:
        nodes = [W.node_id(rng, upper=rng.random() < 0.3) for _ in range(3)]
        base = rng.choice([t0, t0, 0, 3 * 60000])  # short keys for some owners
        pools[o] = W.hlc_timestamps(rng, 80, nodes, t0=base, span=rng.choice([600_000, 3 * 86_400_000]))
    reqs = []
    for _ in range(n_req):
        o = rng.choice(owners)
        k = rng.randrange(0, 12)
        msgs = [rng.choice(pools[o]) for _ in range(k)]
        reqs.append((o, msgs))
    return owners, pools, reqs


def _run_batches(eng, owners, batches):
    """batches: list of lists of requests.  Returns (store, per-message flags, ids->ts)."""
    oid = {o: i for i, o in enumerate(owners)}
    store = eng.store_new(len(owners))
    flags_all, id_ts = [], {}
    base = 0
    for reqs in batches:
        strings = [t for _, ms in reqs for t in ms]
        own = [oid[o] for o, ms in reqs for _ in ms]
        for k, t in enumerate(strings):
            id_ts[base + k] = t
        f, st = store.ingest(eng.timestamps(strings), eng.dev(np.array(own, dtype=np.uint32)), base)
        flags_all.append(f.cpu().numpy()[: len(strings)])
        base += len(strings)
    return store, flags_all, id_ts


def _oracle(owners, batches):
    db = O.ServerDb()
    ins_all = []
    for reqs in batches:
        ins = []
        for o, ms in reqs:
            got = []
            db.add_messages(db.get_merkle_tree(o), o, [(t, b"") for t in ms], got)
            ins += got
        ins_all.append(ins)
    return db, ins_all


@pytest.mark.parametrize("seed", range(4))
def test_ingest_vs_oracle(eng, seed):
    from evolu_amd import _lib as L

    owners, pools, reqs = _requests(seed)
    batches = [reqs[:15], reqs[15:16], reqs[16:]]
    store, flags, id_ts = _run_batches(eng, owners, batches)
    db, ins = _oracle(owners, batches)
    for f, want in zip(flags, ins):
        assert [bool(x & L.MSG_INS) for x in f] == want
    tree = store.tree()
    for i, o in enumerate(owners):
        assert tree.to_json(i) == O.merkle_tree_to_string(db.get_merkle_tree(o)), o
    # stored rows in (owner, timestamp) order == the message table
    off, ids = store.messages()
    for i, o in enumerate(owners):
        rows = db.conn.execute('SELECT "timestamp" FROM "message" WHERE "userId" = ? ORDER BY "timestamp"',
                               (o,)).fetchall()
        assert [id_ts[int(k)] for k in ids[off[i]:off[i + 1]]] == [r[0] for r in rows]


@pytest.mark.parametrize("seed,path", [(s, p) for s in range(4) for p in (0, 1)])
def test_select_vs_oracle(eng, seed, path):
    from evolu_amd import _lib as L

    eng.set_option(L.OPT_SELECT_PATH, path)  # 0: one-pass keep/rank/emit, 1: three passes
    owners, pools, reqs = _requests(100 + seed)
    store, flags, id_ts = _run_batches(eng, owners, [reqs])
    db, _ = _oracle(owners, [reqs])
    rng = random.Random(seed)
    client_json, nodes, want = [], [], []
    for o in owners:
        # the client knows a random subset (incl. nothing / everything)
        mode = rng.random()
        have = [t for t in pools[o] if (mode > 0.8 or (mode > 0.2 and rng.random() < 0.7))]
        ct = {}
        for t in have:
            ct = O.insert_into_merkle_tree(ct, O.parse_canonical(t))
        cj = O.merkle_tree_to_string(ct)
        node = rng.choice([t[30:] for t in pools[o]] + [W.node_id(rng)])
        if rng.random() < 0.3:
            node = node.swapcase()  # LIKE is ASCII case-insensitive
        client_json.append(cj)
        nodes.append(node)
        try:
            d, rows = db.get_messages(db.get_merkle_tree(o), ct, o, node)
            want.append((-1 if d is None else d, [r[0] for r in rows]))
        except O.RangeErrorJS:
            want.append((-2, []))
    client = eng.tree_from_json(client_json)
    node_arr = eng.dev(np.frombuffer("".join(nodes).encode(), dtype=np.uint8).copy())
    diff, off, ids = store.select(client, node_arr)
    eng.set_option(L.OPT_SELECT_PATH, 0)
    diff, off, ids = diff.cpu().numpy(), off.cpu().numpy(), ids.cpu().numpy()
    for i in range(len(owners)):
        assert int(diff[i]) == want[i][0]
        assert [id_ts[int(k)] for k in ids[off[i]:off[i + 1]]] == want[i][1]


def test_select_paths_agree_many_tiles(eng):
    """The one-pass selection (look-back over 2,048-candidate tiles) against
    the keep / scan / emit passes on a store of 2M rows: offsets, ids and
    order keys identical; a capacity below the selection returns
    EVM_ECAPACITY with the needed count from both."""
    import ctypes as C

    import torch

    from evolu_amd import _lib as L
    from evolu_amd import synth

    dev = torch.device("cuda", 0)
    O_, P = 20_000, 100
    gen = synth.DeviceSynth()
    ts, own, _ = gen.source(0xE7010007, O_, P, 1, 0, dev)
    store = eng.store_new(O_)
    store.ingest(ts, own, 0)
    rng = np.random.default_rng(5)
    tsn = ts.cpu().numpy()
    # bounds: none / before everything / mid-stream (the owner's rows' millis); requesters: a node of the
    # owner's rows (excluded) or a stranger
    by = np.argsort(own.cpu().numpy(), kind="stable")
    first_row = tsn[by.reshape(O_, P)[:, 0]]
    bound = rng.choice([-1, 0, 1], O_).astype(np.int64)
    mid = np.array([O.parse_canonical(bytes(r[:46]).decode())[0] for r in tsn[by.reshape(O_, P)[:, P // 2]]])
    bound = np.where(bound == 1, mid, bound)
    node = np.where(rng.random(O_)[:, None] < 0.5, first_row[:, 30:46],
                    np.frombuffer(b"0123456789abcdef", dtype=np.uint8)[None, :]).astype(np.uint8)
    b_d, n_d = eng.dev(bound), eng.dev(np.ascontiguousarray(node).reshape(-1))
    res = []
    for path in (0, 1):
        eng.set_option(L.OPT_SELECT_PATH, path)
        off, ids, key = store.select_after(b_d, n_d, keys=True)
        res.append((off.cpu().numpy(), ids.cpu().numpy(), key.cpu().numpy()))
        # capacity below the selection
        k = ids.numel()
        assert k > 4096
        o2 = torch.empty(O_ + 1, dtype=torch.int64, device=dev)
        i2 = torch.empty(k // 2, dtype=torch.int64, device=dev)
        nsel = C.c_uint64()
        st = eng.lib.evm_store_select_after(eng.h, store.h, b_d.data_ptr(), n_d.data_ptr(), None, o2.data_ptr(),
                                            i2.data_ptr(), None, k // 2, C.byref(nsel))
        assert st == L.EVM_ECAPACITY and nsel.value == k
    eng.set_option(L.OPT_SELECT_PATH, 0)
    for x, y in zip(res[0], res[1]):
        assert np.array_equal(x, y)
    store.free()


def test_ingest_noncanonical_and_empty(eng):
    from evolu_amd import _lib as L

    store = eng.store_new(2)
    f, st = store.ingest(eng.timestamps([]), eng.dev(np.zeros(0, dtype=np.uint32)))
    assert st == 0 and store.n_messages == 0
    good = "2024-01-01T00:00:00.000Z-0000-0000000000000001"
    bad = "2022-02-30T00:00:00.000Z-0000-0000000000000001"
    f, st = store.ingest(eng.timestamps([good, bad]), eng.dev(np.array([0, 1], dtype=np.uint32)), raise_on_error=False)
    assert st == L.EVM_ENONCANON and list(f.cpu().numpy()) == [0, L.MSG_BAD]
    assert store.n_messages == 0
    assert store.tree().to_json(0) == "{}"


def test_ingest_many_owners_scale(eng):
    """config-3 shape at reduced size: every (owner, ts) once, all inserted;
    roots == XOR of the owners' hashes; a second ingest of the same batch
    inserts nothing and leaves every tree unchanged."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, owner_np, _ = synth.config3(n_owners=2000, per_owner=500)
    ts, own = eng.dev(ts_np), eng.dev(owner_np)
    store = eng.store_new(2000)
    f, _ = store.ingest(ts, own, 0)
    assert (f.cpu().numpy() == L.MSG_INS).all()
    r1, p1 = store.tree().roots()
    recs, _ = eng.pack(ts)
    h = recs[:, 2].cpu().numpy().view(np.uint32).reshape(-1, 2)[:, 1]
    want = np.zeros(2000, dtype=np.uint32)
    np.bitwise_xor.at(want, owner_np, h)
    assert np.array_equal(r1.view(np.uint32), want) and p1.all()
    f2, _ = store.ingest(ts, own, len(ts_np))
    assert (f2.cpu().numpy() == 0).all() and store.n_messages == len(ts_np)
    r2, _ = store.tree().roots()
    assert np.array_equal(r1, r2)


@pytest.mark.parametrize("run", [3, 64, 65, 200])
def test_ingest_tie_runs(eng, run):
    """Runs of equal (owner, millis, counter) with distinct nodes (mixed case):
    ordered by the node bytes; runs longer than the tie fix-up's limit take
    the full-field sort.  Checked against the oracle's message table."""
    from evolu_amd import _lib as L

    rng = random.Random(run)
    owners = ["%021x" % rng.getrandbits(84) for _ in range(3)]
    reqs = []
    for k, o in enumerate(owners):
        nodes = {W.node_id(rng, upper=rng.random() < 0.5) for _ in range(run)}
        ms = [O.timestamp_to_string(W.T0 + 7 * k, 3, nd) for nd in nodes]
        ms += [O.timestamp_to_string(W.T0 + 7 * k + 1, 0, nd) for nd in list(nodes)[:5]]
        rng.shuffle(ms)
        reqs.append((o, ms + ms[:3]))  # in-request duplicates too
    store, flags, id_ts = _run_batches(eng, owners, [reqs])
    db, ins = _oracle(owners, [reqs])
    assert [bool(x & L.MSG_INS) for x in flags[0]] == ins[0]
    off, ids = store.messages()
    for i, o in enumerate(owners):
        rows = db.conn.execute('SELECT "timestamp" FROM "message" WHERE "userId" = ? ORDER BY "timestamp"',
                               (o,)).fetchall()
        assert [id_ts[int(k)] for k in ids[off[i]:off[i + 1]]] == [r[0] for r in rows]
    tree = store.tree()
    for i, o in enumerate(owners):
        assert tree.to_json(i) == O.merkle_tree_to_string(db.get_merkle_tree(o))


@pytest.mark.parametrize("seed", range(3))
def test_store_since_resend_range(eng, seed):
    """receive.ts:118-124: SELECT * FROM "__message" WHERE "timestamp" > ?
    ORDER BY "timestamp", with ? = timestampToString(createSyncTimestamp(d)),
    on a store mirroring each owner's message table (sqlite3 as the checker)."""
    import sqlite3

    owners, pools, reqs = _requests(300 + seed)
    store, flags, id_ts = _run_batches(eng, owners, [reqs])
    db, _ = _oracle(owners, [reqs])
    rng = random.Random(seed)
    since = []
    for o in owners:
        ts_o = sorted(t for t in pools[o])
        pick = rng.random()
        if pick < 0.15:
            since.append(-1)
        elif pick < 0.3:
            since.append(0)
        else:
            since.append(O.parse_canonical(rng.choice(ts_o))[0] + rng.choice([-1, 0, 0, 1]))
    off, ids = store.since(torch_tensor(eng, since))
    off, ids = off.cpu().numpy(), ids.cpu().numpy()
    for i, o in enumerate(owners):
        if since[i] < 0:
            assert off[i + 1] == off[i]
            continue
        bound = O.timestamp_to_string(since[i], 0, "0000000000000000")
        rows = db.conn.execute('SELECT "timestamp" FROM "message" WHERE "userId" = ? AND "timestamp" > ? '
                               'ORDER BY "timestamp"', (o, bound)).fetchall()
        assert [id_ts[int(k)] for k in ids[off[i]:off[i + 1]]] == [r[0] for r in rows]


def torch_tensor(eng, values):
    import torch

    return torch.tensor(values, dtype=torch.int64, device=eng.device)


@pytest.mark.parametrize("n_owners,per_owner,req_size", [(3000, 300, 1), (3000, 300, 50), (20000, 1000, 100),
                                                        (50, 3000, 100), (3, 5000, 100)])
def test_owner_lds_path_vs_sort_path(eng, n_owners, per_owner, req_size):
    """The per-owner LDS ingest (K5) and the global sort path are independent
    device algorithms: on config-3-shaped batches with redeliveries, fed in
    two ingests (the second one against a non-empty store and trees), they
    must agree bit for bit -- flags, stored rows in (owner, timestamp) order,
    and every leaf of every tree."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, owner_np, _ = synth.config3(n_owners=n_owners, per_owner=per_owner, seed_config=11, request=req_size)
    rng = np.random.default_rng(n_owners)
    dup = rng.integers(0, len(ts_np), size=len(ts_np) // 20)
    ts_np = np.concatenate([ts_np, ts_np[dup]])
    owner_np = np.concatenate([owner_np, owner_np[dup]])
    half = len(ts_np) * 2 // 3
    res = []
    for path in (1, 2):
        eng.set_option(L.OPT_SERVER_PATH, path)
        store = eng.store_new(n_owners)
        fl = []
        for a, b in ((0, half), (half, len(ts_np))):
            f, st = store.ingest(eng.dev(ts_np[a:b]), eng.dev(owner_np[a:b]), a)
            fl.append(f.cpu().numpy().copy())
        off, ids = store.messages()
        toff, code, xr = store.tree().leaves()
        res.append((np.concatenate(fl), off, ids, toff, code, xr))
        store.free()
    eng.set_option(L.OPT_SERVER_PATH, 0)
    for x, y in zip(res[0], res[1]):
        assert np.array_equal(x, y)
    # every distinct (owner, timestamp) is inserted exactly once (config-3 nodes are per owner)
    assert (res[0][0] == L.MSG_INS).sum() == len(np.unique(np.ascontiguousarray(ts_np[:, :46]).view("S46")))


def test_owner_lds_path_bursts_vs_oracle(eng):
    """Owners whose timestamps crowd a few milliseconds (plus far outliers):
    the LDS path's counting sort overflows its buckets and the bitonic
    network orders the share; equal (millis, counter) with distinct nodes are
    ordered by the node bytes.  Checked against the verbatim-SQL oracle and
    against the global sort path."""
    from evolu_amd import _lib as L

    rng = random.Random(77)
    owners = ["%021x" % rng.getrandbits(84) for _ in range(12)]
    reqs = []
    for o in owners:
        nodes = [W.node_id(rng, upper=rng.random() < 0.3) for _ in range(8)]
        ms = [O.timestamp_to_string(W.T0 + rng.randrange(1000), rng.randrange(4), rng.choice(nodes)) for _ in range(300)]
        ms += [O.timestamp_to_string(W.T0 + 10 * 86_400_000 + k, 0, nodes[0]) for k in range(2)]
        ms += ms[:20]  # redeliveries
        rng.shuffle(ms)
        reqs.append((o, ms))
    got = []
    for path in (1, 2):
        eng.set_option(L.OPT_SERVER_PATH, path)
        store, flags, id_ts = _run_batches(eng, owners, [reqs[:6], reqs[6:]])
        off, ids = store.messages()
        tree = store.tree()
        got.append(([list(f) for f in flags], [id_ts[int(k)] for k in ids], [tree.to_json(i) for i in range(len(owners))]))
        store.free()
    eng.set_option(L.OPT_SERVER_PATH, 0)
    assert got[0] == got[1]
    db, ins = _oracle(owners, [reqs[:6], reqs[6:]])
    assert [[bool(x & L.MSG_INS) for x in f] for f in got[0][0]] == ins
    for i, o in enumerate(owners):
        assert got[0][2][i] == O.merkle_tree_to_string(db.get_merkle_tree(o))
    want_rows = []
    for o in owners:
        want_rows += [r[0] for r in db.conn.execute(
            'SELECT "timestamp" FROM "message" WHERE "userId" = ? ORDER BY "timestamp"', (o,)).fetchall()]
    assert got[0][1] == want_rows


@pytest.mark.parametrize("run", [40, 100])
def test_big_owner_tie_runs(eng, run):
    """An owner above the LDS capacity (its messages go through the sort path
    as a sub-batch after the other owners commit) whose batch holds a run of
    `run` equal (millis, counter) timestamps with distinct mixed-case nodes:
    a run above the tie ranking's limit takes the full-field sort over the
    sub-batch.  Flags, row order and trees against the C restatement."""
    from evolu_amd import _lib as L
    from oracle import c_oracle as CO

    rng = random.Random(900 + run)
    strings, owner = [], []
    nodes = [W.node_id(rng, upper=rng.random() < 0.3) for _ in range(6)]
    big = W.hlc_timestamps(rng, 5000, nodes, span=600_000)
    tie = [O.timestamp_to_string(W.T0 + 123_456, 7, W.node_id(rng, upper=rng.random() < 0.5)) for _ in range(run)]
    mine = big + tie + tie[:5]  # redeliveries inside the batch
    rng.shuffle(mine)
    strings += mine
    owner += [0] * len(mine)
    for o in (1, 2):
        small = W.hlc_timestamps(rng, 300, [W.node_id(rng) for _ in range(3)])
        strings += small
        owner += [o] * len(small)
    perm = list(range(len(strings)))
    rng.shuffle(perm)
    strings = [strings[i] for i in perm]
    owner = np.array([owner[i] for i in perm], dtype=np.uint32)
    ts_np = eng.timestamps(strings).cpu().numpy()
    srv = CO.Server(3, len(strings))
    st, want = srv.ingest(ts_np, owner)
    assert st == 0
    store = eng.store_new(3)
    got, st = store.ingest(eng.dev(ts_np), eng.dev(owner), 0)
    assert st == 0
    assert np.array_equal(got.cpu().numpy(), want)
    off, ids = store.messages()
    for o in range(3):
        rows = sorted({s for s, w in zip(strings, owner) if w == o})
        assert [strings[int(k)] for k in ids[off[o]:off[o + 1]]] == rows
        assert store.tree().to_json(o) == srv.tree_json(o)
    assert ((got.cpu().numpy() & L.MSG_INS) != 0).sum() == sum(len({s for s, w in zip(strings, owner) if w == o})
                                                         for o in range(3))


def _check_prefix_xor(eng, tree):
    """The tree's prefix XOR (written by K5 for a gapped tree, by the empty
    store's copy kernel, or by the scan after a merge) against its own leaves: every owner's root is
    the XOR of its leaves, and a diff with the same leaves rebuilt through
    evm_tree_from_leaves (whose prefix is a scan) finds nothing at any level."""
    from evolu_amd import _lib as L

    r, _ = tree.roots()  # (read as the tree is: gapped -- owner-local prefix -- or compact)
    off, code, xr = tree.leaves()
    px = np.concatenate([[0], np.bitwise_xor.accumulate(xr.astype(np.int32))]).astype(np.int32)
    o = off.astype(np.int64)
    assert np.array_equal(r, px[o[1:]] ^ px[o[:-1]])
    same = eng.tree_from_leaves(off, code, xr)
    assert (eng.merkle_diff(tree, same).cpu().numpy() == L.DIFF_NONE).all()


@pytest.mark.parametrize("seed", [0, 1])
def test_merge_paths_by_segment_size(eng, seed):
    """Round 2 into a non-empty store through every merge shape (k_svo_b<true>):
    a segment whose stored + new rows and leaves fit the LDS source map
    (<= 4,096: written once in output order), one that exceeds it (stored
    rows first, new rows into the gaps), small ones, a new owner and an owner
    with no new rows -- with redeliveries of stored rows (equal tree leaves
    XOR-combined) -- against the C oracle of addMessages
    (apps/server/src/index.ts:138-171): flags, stored rows, trees."""
    from evolu_amd import _lib as L
    from oracle import c_oracle as CO

    rng = random.Random(7100 + seed)
    day = 86_400_000
    # owner: (stored rows, new rows); minutes spread so the leaf lists are long too
    shape = {0: (3000, 1000), 1: (3600, 600), 2: (200, 100), 3: (0, 50), 4: (100, 0)}
    r1, r2 = [], []
    for o, (ns, nn) in shape.items():
        nodes = [W.node_id(rng, upper=rng.random() < 0.3) for _ in range(4)]
        old = W.hlc_timestamps(rng, ns, nodes, span=5 * day) if ns else []
        new = W.hlc_timestamps(rng, nn, [W.node_id(rng) for _ in range(3)], span=5 * day) if nn else []
        redo = [rng.choice(old) for _ in range(nn // 10)] if old and nn else []
        r1 += [(s, o) for s in old]
        r2 += [(s, o) for s in new + redo]
    rng.shuffle(r1)
    rng.shuffle(r2)
    srv = CO.Server(len(shape), len(r1) + len(r2))
    store = eng.store_new(len(shape))
    got_all = []
    for batch, base in ((r1, 0), (r2, 1 << 40)):
        ts_np = eng.timestamps([s for s, _ in batch]).cpu().numpy()
        own = np.array([o for _, o in batch], dtype=np.uint32)
        st, want = srv.ingest(ts_np, own)
        assert st == 0
        got, st = store.ingest(eng.dev(ts_np), eng.dev(own), base)
        assert st == 0
        got_all.append(got.cpu().numpy())
        assert np.array_equal(got_all[-1], want)
        _check_prefix_xor(eng, store.tree())
    assert (got_all[1] & L.MSG_INS).astype(bool).sum() == sum(nn for _, nn in shape.values())
    off, ids = store.messages()
    both = r1 + r2
    id_of = {}
    for k, (s, o) in enumerate(r1):
        id_of.setdefault((s, o), k)
    for k, (s, o) in enumerate(r2):
        id_of.setdefault((s, o), (1 << 40) + k)
    for o in shape:
        rows = sorted({s for s, w in both if w == o})
        assert [int(k) for k in ids[off[o]:off[o + 1]]] == [id_of[(s, o)] for s in rows]
        assert store.tree().to_json(o) == srv.tree_json(o)
    assert store.n_messages == len(set(both))


def _is_gapped(eng, tree):
    import ctypes as C

    from evolu_amd import _lib as L

    p = C.c_void_p()
    return eng.lib.evm_tree_device(tree.h, C.byref(p), C.byref(p), C.byref(p)) == L.EVM_EINVAL


def test_gapped_tree_reads_equal_compact(eng):
    """An ingest into an empty store of one request per owner, every message
    inserted, leaves a GAPPED tree (each owner's leaves where K5 wrote them,
    owner-local prefix XOR; no copy pass).  Its roots and diffs, read gapped,
    equal the same reads after it is compacted, and the compacted leaves
    equal the sort path's tree; a second ingest into that store (which
    compacts first) equals the sort path's two ingests."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    n_owners, per = 400, 250
    ts, own, millis = synth.config3(n_owners, per, request=per, seed_config=91)
    ts2, own2, _ = synth.config3(n_owners, per, request=per, seed_config=92)
    store = eng.store_new(n_owners)
    f, _ = store.ingest(eng.dev(ts), eng.dev(own), 0)
    assert int((f.cpu().numpy() & L.MSG_INS).astype(bool).sum()) == len(ts)
    tree = store.tree()
    assert _is_gapped(eng, tree)
    # client trees: each owner's first 90 % by time (config 3)
    o64 = own.astype(np.int64)
    order = np.lexsort((millis, o64))
    rank = np.empty(len(order), dtype=np.int64)
    cnt = np.bincount(o64, minlength=n_owners)
    rank[order] = np.arange(len(order)) - (np.cumsum(cnt) - cnt)[o64[order]]
    keep = rank < (0.9 * cnt[o64]).astype(np.int64)
    client = eng.merkle_insert(eng.tree_new(n_owners), eng.dev(np.ascontiguousarray(ts[keep])),
                               eng.dev(np.ascontiguousarray(own[keep])))
    r_gap, p_gap = tree.roots()
    d_gap = eng.merkle_diff(tree, client).cpu().numpy()
    d_gap_rev = eng.merkle_diff(client, tree).cpu().numpy()
    node = eng.dev(np.frombuffer(b"0123456789abcdef" * n_owners, dtype=np.uint8).copy())
    s_diff, s_off, s_ids = store.select(client, node)
    s_diff, s_off, s_ids = s_diff.cpu().numpy(), s_off.cpu().numpy(), s_ids.cpu().numpy()
    assert _is_gapped(eng, tree)  # (diff, roots and select read it as it is)
    off, code, xr = tree.leaves()  # compacts
    assert not _is_gapped(eng, tree)
    r_c, p_c = tree.roots()
    assert np.array_equal(r_gap, r_c) and np.array_equal(p_gap, p_c)
    assert np.array_equal(d_gap, eng.merkle_diff(tree, client).cpu().numpy())
    assert np.array_equal(d_gap_rev, eng.merkle_diff(client, tree).cpu().numpy())
    assert (d_gap >= 0).all()
    # against the sort path
    eng.set_option(L.OPT_SERVER_PATH, 2)
    ref = eng.store_new(n_owners)
    ref.ingest(eng.dev(ts), eng.dev(own), 0)
    eng.set_option(L.OPT_SERVER_PATH, 0)
    ro, rc, rx = ref.tree().leaves()
    assert np.array_equal(off, ro) and np.array_equal(code, rc) and np.array_equal(xr, rx)
    r_ref, _ = ref.tree().roots()
    assert np.array_equal(r_ref, r_gap)
    d2, o2, i2 = ref.select(client, node)
    assert np.array_equal(d2.cpu().numpy(), s_diff) and np.array_equal(o2.cpu().numpy(), s_off)
    assert np.array_equal(i2.cpu().numpy(), s_ids)
    for o in (0, 7, n_owners - 1):
        assert tree.to_json(o) == ref.tree().to_json(o)
    # a second round: the gapped store compacts, then merges
    fresh = eng.store_new(n_owners)
    fresh.ingest(eng.dev(ts), eng.dev(own), 0)
    assert _is_gapped(eng, fresh.tree())
    fa, _ = fresh.ingest(eng.dev(ts2), eng.dev(own2), 1 << 40)
    eng.set_option(L.OPT_SERVER_PATH, 2)
    fb, _ = ref.ingest(eng.dev(ts2), eng.dev(own2), 1 << 40)
    eng.set_option(L.OPT_SERVER_PATH, 0)
    assert np.array_equal(fa.cpu().numpy(), fb.cpu().numpy())
    for x, y in zip(fresh.tree().leaves(), ref.tree().leaves()):
        assert np.array_equal(x, y)
    for x, y in zip(fresh.messages(), ref.messages()):
        assert np.array_equal(x, y)
    for t in (store, ref, fresh):
        t.free()
    client.free()
