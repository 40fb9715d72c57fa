"""GPU parity tests of libevm against the CPU oracle (run on the MI355X box)."""
import json
import os
import random

import numpy as np
import pytest

from oracle import evolu_oracle as O
from tests import workloads as W

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
JSV = json.load(open(os.path.join(GOLD, "js_vectors.json")))
SNAP = json.load(open(os.path.join(GOLD, "reference_snapshots.json")))
MT = SNAP["merkleTree.test.ts.snap"]
NODE1 = "0000000000000001"


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


def _recs(eng, strings, stride=48):
    from evolu_amd import engine as E

    ts = eng.timestamps(strings, stride)
    out, st = eng.pack(ts)
    r = out.cpu().numpy()
    tc = r[:, 0].view(np.uint64)
    node = r[:, 1].view(np.uint64)
    w = r[:, 2:].copy().view(np.uint32)  # meta, hash, minute, aux
    return tc, node, w[:, 0], w[:, 1], w[:, 2], st


# ------------------------------------------------------------------ K1 pack
@pytest.mark.parametrize("stride", [48, 46, 47, 64])
def test_pack_js_vectors(eng, stride):
    from evolu_amd import _lib as L

    vs = JSV["timestamps"]
    tc, node, meta, h, minute, st = _recs(eng, [v["s"] for v in vs], stride)
    for i, v in enumerate(vs):
        native = v["millis"] < (2**31) * 60000
        if not native:
            assert meta[i] & L.META_RANGE
            continue
        assert meta[i] & L.META_VALID, v["s"]
        assert int(tc[i]) == (v["millis"] << 16) | v["counter"]
        assert int(node[i]) == int(v["node"], 16)
        assert int(meta[i]) & L.META_CASEMASK == sum(1 << k for k, c in enumerate(v["node"]) if c in "ABCDEF")
        assert int(h[i]) == v["hash"], v["s"]
        assert int(minute[i]) == O.to_int32(v["millis"] / 1000 / 60)


def test_pack_snapshot_hash(eng):
    s = O.timestamp_to_string(*O.create_sync_timestamp())
    _, _, meta, h, _, st = _recs(eng, [s])
    assert st == 0 and int(h[0]) == 4179357717


def test_pack_flags_noncanonical(eng):
    from evolu_amd import _lib as L

    good = "2024-01-01T00:00:00.000Z-0000-0000000000000001"
    bad = [
        "2024-01-01T00:00:00.000Z-00a0-0000000000000001",  # lower-case counter
        "2022-02-30T00:00:00.000Z-0000-0000000000000001",  # V8 lenient Feb-30
        "2024-02-29T24:00:00.000Z-0000-0000000000000001",  # hour 24
        "2024-13-01T00:00:00.000Z-0000-0000000000000001",
        "2024-01-01T00:00:60.000Z-0000-0000000000000001",
        "2024-01-01T00:00:00.000Z-0000-000000000000000g",
        "2024-01-01 00:00:00.000Z-0000-0000000000000001",
        "+02024-01-01T00:00:00.000Z-0000-000000000000001",
        "short",
    ]
    ranged = ["1969-12-31T23:59:59.999Z-0000-0000000000000001", "6053-01-23T02:08:00.000Z-0000-0000000000000001"]
    tc, node, meta, h, minute, st = _recs(eng, [good] + bad + ranged)
    assert st == L.EVM_ENONCANON
    assert meta[0] & L.META_VALID
    for i in range(1, 1 + len(bad)):
        assert meta[i] & L.META_NONCANON and not meta[i] & L.META_VALID
        with pytest.raises(O.NonCanonical):
            O.parse_canonical(([good] + bad)[i])
    for i in range(1 + len(bad), 1 + len(bad) + len(ranged)):
        assert meta[i] & L.META_RANGE


def test_pack_random_vs_oracle(eng):
    rng = random.Random(7)
    strings = []
    for _ in range(5000):
        m = rng.randrange(0, (2**31) * 60000)
        strings.append(O.timestamp_to_string(m, rng.randrange(65536), W.node_id(rng, rng.random() < 0.3)))
    tc, node, meta, h, minute, st = _recs(eng, strings)
    assert st == 0
    for i, s in enumerate(strings):
        m, c, n = O.parse_canonical(s)
        assert int(h[i]) == O.murmur3_32(s.encode())
        assert int(tc[i]) == (m << 16) | c and int(minute[i]) == m // 60000


# --------------------------------------------------------------- Merkle trie
def _oracle_tree(ts_list):
    t = {}
    for s in ts_list:
        t = O.insert_into_merkle_tree(t, O.parse_canonical(s))
    return t


def test_merkle_insert_snapshots(eng):
    ts1 = O.timestamp_to_string(0, 0, NODE1)
    ts2 = O.timestamp_to_string(1656873738591, 0, NODE1)
    e = eng.tree_new(1)
    assert e.to_json(0) == "{}"
    a = eng.merkle_insert(e, eng.timestamps([ts1]))
    assert json.loads(a.to_json(0)) == MT["insertIntoMerkleTree 1"]
    b = eng.merkle_insert(e, eng.timestamps([ts2]))
    assert json.loads(b.to_json(0)) == MT["insertIntoMerkleTree 2"]
    ab = eng.merkle_insert(a, eng.timestamps([ts2]))
    ba = eng.merkle_insert(b, eng.timestamps([ts1]))
    assert json.loads(ab.to_json(0)) == MT["insertIntoMerkleTree 3"]
    assert ab.to_json(0) == ba.to_json(0) == O.merkle_tree_to_string(_oracle_tree([ts1, ts2]))
    r, p = ab.roots()
    assert p[0] and r[0] == 1335454297
    both = eng.merkle_insert(e, eng.timestamps([ts1, ts2]))
    assert both.to_json(0) == ab.to_json(0)


def test_merkle_insert_js_trees(eng):
    for t in JSV["trees"]:
        strings = [O.timestamp_to_string(m, c, n) for m, c, n in t["ops"]]
        got = eng.merkle_insert(eng.tree_new(1), eng.timestamps(strings)).to_json(0)
        assert got == t["json"]
        assert eng.tree_from_json([t["json"]]).to_json(0) == t["json"]


def test_merkle_insert_multi_owner_random(eng):
    rng = random.Random(11)
    n_owners = 37
    strings, owners = [], []
    for o in range(n_owners):
        nodes = [W.node_id(rng) for _ in range(3)]
        base = rng.choice([0, 5 * 60000, W.T0, 2582803260000 - 600000])  # short, 16 and 17-digit keys
        for s in W.hlc_timestamps(rng, rng.randrange(0, 60), nodes, t0=base, span=7200_000):
            strings.append(s)
            owners.append(o)
            if rng.random() < 0.2:  # duplicate -> XOR cancels, nodes stay with hash 0
                strings.append(s)
                owners.append(o)
    perm = list(range(len(strings)))
    rng.shuffle(perm)
    strings = [strings[i] for i in perm]
    owners = [owners[i] for i in perm]
    trees = eng.merkle_insert(eng.tree_new(n_owners), eng.timestamps(strings),
                              eng.dev(np.array(owners, dtype=np.uint32)))
    for o in range(n_owners):
        want = O.merkle_tree_to_string(_oracle_tree([s for s, oo in zip(strings, owners) if oo == o]))
        assert trees.to_json(o) == want
    # incremental insert == one-shot insert
    half = len(strings) // 2
    t1 = eng.merkle_insert(eng.tree_new(n_owners), eng.timestamps(strings[:half]),
                           eng.dev(np.array(owners[:half], dtype=np.uint32)))
    t2 = eng.merkle_insert(t1, eng.timestamps(strings[half:]), eng.dev(np.array(owners[half:], dtype=np.uint32)))
    for o in range(n_owners):
        assert t2.to_json(o) == trees.to_json(o)


def test_tree_json_rejects_unproducible(eng):
    from evolu_amd import _lib as L
    from evolu_amd._lib import EngineError

    for bad in ['{"hash":1}', '{"0":{"hash":1}}', '{"0":{"hash":1},"hash":2}', '{"0":{}, "hash":0}',
                '{"3":{"hash":1},"hash":1}', '{"0":{"hash":1.5},"hash":1}', '[]']:
        with pytest.raises(EngineError) as ei:
            eng.tree_from_json([bad])
        assert ei.value.status == L.EVM_ETREE


def test_diff_snapshots(eng):
    ts = O.timestamp_to_string(1656873738591, 0, NODE1)
    e = eng.tree_new(1)
    mt = eng.merkle_insert(e, eng.timestamps([ts]))
    assert int(eng.merkle_diff(e, e).cpu()[0]) == -1
    assert int(eng.merkle_diff(e, mt).cpu()[0]) == 1656873720000
    assert int(eng.merkle_diff(mt, e).cpu()[0]) == 1656873720000


def test_diff_random_vs_oracle(eng):
    rng = random.Random(5)
    n_owners = 200
    A, B = [], []
    for o in range(n_owners):
        nodes = [W.node_id(rng) for _ in range(3)]
        base = rng.choice([0, 120000, W.T0, W.T0, W.T0, 2582803260000 - 60000])
        pool = W.hlc_timestamps(rng, rng.randrange(0, 40), nodes, t0=base, span=rng.choice([600_000, 86_400_000]))
        a = [s for s in pool if rng.random() < 0.9]
        b = [s for s in pool if rng.random() < 0.9]
        if rng.random() < 0.2:
            b = list(a)
        if rng.random() < 0.2 and a:
            b = a + [a[0], a[0]]  # XOR cancellation: equal root hash but extra hash-0 nodes? no: same set
        A.append(a)
        B.append(b)
    sa = [s for o in range(n_owners) for s in A[o]]
    oa = [o for o in range(n_owners) for _ in A[o]]
    sb = [s for o in range(n_owners) for s in B[o]]
    ob = [o for o in range(n_owners) for _ in B[o]]
    ta = eng.merkle_insert(eng.tree_new(n_owners), eng.timestamps(sa), eng.dev(np.array(oa, dtype=np.uint32)))
    tb = eng.merkle_insert(eng.tree_new(n_owners), eng.timestamps(sb), eng.dev(np.array(ob, dtype=np.uint32)))
    got = eng.merkle_diff(ta, tb).cpu().numpy()
    for o in range(n_owners):
        try:
            want = O.diff_merkle_trees(_oracle_tree(A[o]), _oracle_tree(B[o]))
            want = -1 if want is None else want
        except O.RangeErrorJS:
            want = -2
        assert int(got[o]) == want, (o, A[o], B[o])


def test_diff_from_json_trees(eng):
    # hand-built trees incl. hash-0 nodes and XOR cancellation along the greedy path
    cases = [
        ("{}", '{"0":{"hash":0},"hash":0}'),
        ('{"1":{"0":{"hash":5},"1":{"hash":6},"hash":3},"hash":3}', '{"1":{"0":{"hash":6},"1":{"hash":5},"hash":3},"hash":3}'),
        ('{"1":{"0":{"hash":5},"1":{"hash":6},"hash":3},"2":{"hash":1},"hash":2}', '{"1":{"0":{"hash":6},"1":{"hash":5},"hash":3},"hash":3}'),
        ('{"1":{"2":{"hash":7},"hash":4},"hash":4}', '{"1":{"2":{"hash":7},"hash":7},"hash":7}'),
    ]
    for a, b in cases:
        ta, tb = eng.tree_from_json([a]), eng.tree_from_json([b])
        want = O.diff_merkle_trees(json.loads(a), json.loads(b))
        assert int(eng.merkle_diff(ta, tb).cpu()[0]) == (-1 if want is None else want)
        assert ta.to_json(0) == a.replace(" ", "") and tb.to_json(0) == b


# -------------------------------------------------------------- applyMessages
def _oracle_apply(msgs, prior_msgs=()):
    db = O.ClientDb()
    tree = O.apply_messages(db, {}, list(prior_msgs))
    dec = []
    tree2 = O.apply_messages(db, tree, msgs, dec)
    return db, tree, tree2, dec


def _engine_apply(eng, msgs, cells, prior_msgs=(), prior_tree_json="{}"):
    cid = {c: i for i, c in enumerate(cells)}
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype=np.uint32)
    prior_ts, prior_present = None, None
    if prior_msgs:
        pdb = O.ClientDb()
        O.apply_messages(pdb, {}, list(prior_msgs))
        mx = [pdb.cell_max(*c) for c in cells]
        prior_ts = eng.timestamps([m or "" for m in mx])
        prior_present = eng.dev(np.array([m is not None for m in mx], dtype=np.uint8))
    tin = eng.tree_from_json([prior_tree_json])
    flags, winner, tout, st = eng.apply_batch(tin, eng.timestamps([m["timestamp"] for m in msgs]), eng.dev(cell),
                                              len(cells), prior_ts=prior_ts, prior_present=prior_present)
    return flags.cpu().numpy(), winner.cpu().numpy(), tout


@pytest.mark.parametrize("seed", range(6))
def test_apply_batch_vs_oracle(eng, seed):
    from evolu_amd import _lib as L

    msgs, cells = W.client_batch(seed, n=300 + 100 * seed, n_cells=3 + 4 * seed)
    prior = []
    if seed % 2:
        prior, _ = W.client_batch(1000 + seed, n=80, n_cells=3 + 4 * seed, t0=W.T0 - 1800_000)
        # prior rows must use the same cells
        prior = [dict(m, table=cells[i % len(cells)][0], row=cells[i % len(cells)][1], column=cells[i % len(cells)][2])
                 for i, m in enumerate(prior)]
        # a stale redelivery of a prior row and an exact redelivery of a cell max
        msgs.insert(3, dict(prior[0]))
    db, t_prior, t_want, dec = _oracle_apply(msgs, prior)
    flags, winner, tout = _engine_apply(eng, msgs, cells, prior, O.merkle_tree_to_string(t_prior))
    for i, (ups, xr, ins) in enumerate(dec):
        assert bool(flags[i] & L.MSG_UPS) == ups, i
        assert bool(flags[i] & L.MSG_XOR) == xr, i
    last_ups = {}
    for i, m in enumerate(msgs):
        if dec[i][0]:
            last_ups[(m["table"], m["row"], m["column"])] = i
    for c, cell in enumerate(cells):
        assert int(winner[c]) == last_ups.get(cell, -1)
    assert tout.to_json(0) == O.merkle_tree_to_string(t_want)
    # the final user table value == the winner's value
    for c, cell in enumerate(cells):
        if winner[c] >= 0:
            row = db.conn.execute('SELECT "%s" FROM "%s" WHERE id = ?' % (cell[2], cell[0]), (cell[1],)).fetchone()
            assert row[0] == msgs[winner[c]]["value"]


def test_apply_batch_collision_and_noncanonical(eng):
    from evolu_amd import _lib as L

    ts = "2024-01-01T00:00:00.000Z-0000-0000000000000001"
    cells = [("t", "r", "a"), ("t", "r", "b")]
    msgs = [{"timestamp": ts, "table": "t", "row": "r", "column": "a", "value": 1},
            {"timestamp": ts, "table": "t", "row": "r", "column": "b", "value": 2}]
    cell = eng.dev(np.array([0, 1], dtype=np.uint32))
    _, _, tout, st = eng.apply_batch(eng.tree_new(1), eng.timestamps([m["timestamp"] for m in msgs]), cell, 2,
                                     raise_on_error=False)
    assert st == L.EVM_ECOLLISION and tout is None
    # same cell twice: fine (exact redelivery is a no-op)
    flags, winner, tout, st = eng.apply_batch(eng.tree_new(1), eng.timestamps([ts, ts]),
                                              eng.dev(np.array([0, 0], dtype=np.uint32)), 2)
    assert list(flags.cpu().numpy()) == [3, 0] and list(winner.cpu().numpy()) == [0, -1]
    bad = "2024-01-01T00:00:00.000Z-00a0-0000000000000001"
    flags, _, tout, st = eng.apply_batch(eng.tree_new(1), eng.timestamps([ts, bad]),
                                         eng.dev(np.array([0, 1], dtype=np.uint32)), 2, raise_on_error=False)
    assert st == L.EVM_ENONCANON and list(flags.cpu().numpy()) == [0, L.MSG_BAD]
