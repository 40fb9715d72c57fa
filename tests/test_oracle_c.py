"""Pins the C restatement (large-N checker, CPU baseline) to the Python oracle."""
import random

import numpy as np
import pytest

from oracle import c_oracle as CO
from oracle import evolu_oracle as O
from tests import workloads as W


def _arena(strings):
    from evolu_amd.engine import encode_timestamps

    return encode_timestamps(strings)


def test_murmur_vectors():
    import json
    import os

    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "js_vectors.json")))
    for v in d["timestamps"][:500]:
        assert CO.lib().evo_murmur3(v["s"].encode(), 46) == v["hash"]


@pytest.mark.parametrize("seed", range(5))
def test_apply_matches_python_oracle(seed):
    msgs, cells = W.client_batch(seed, n=500, n_cells=4 + 5 * seed)
    prior = []
    if seed % 2:
        prior, _ = W.client_batch(900 + seed, n=60, n_cells=4 + 5 * seed, t0=W.T0 - 3600_000)
        prior = [dict(m, table=cells[i % len(cells)][0], row=cells[i % len(cells)][1],
                      column=cells[i % len(cells)][2]) for i, m in enumerate(prior)]
    db = O.ClientDb()
    t0 = O.apply_messages(db, {}, prior)
    dec = []
    want = O.apply_messages(db, t0, msgs, dec)
    cid = {c: i for i, c in enumerate(cells)}
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype=np.uint32)
    pts, pp = None, None
    if prior:
        pdb = O.ClientDb()
        O.apply_messages(pdb, {}, prior)
        mx = [pdb.cell_max(*c) for c in cells]
        pts = _arena([m or "x" * 46 for m in mx])
        pp = np.array([m is not None for m in mx], dtype=np.uint8)
    st, flags, winner, js = CO.apply(_arena([m["timestamp"] for m in msgs]), cell, len(cells), pts, pp)
    assert st == 0
    assert [(bool(f & 1), bool(f & 2)) for f in flags] == [(u, x) for u, x, _ in dec]
    # the C oracle folds only this batch's XORs: compare with the batch-only tree
    tb = {}
    for m, (u, x, _) in zip(msgs, dec):
        if x:
            tb = O.insert_into_merkle_tree(tb, O.parse_canonical(m["timestamp"]))
    assert js == O.merkle_tree_to_string(tb)


def test_server_matches_python_oracle():
    rng = random.Random(3)
    owners = ["u%d" % i for i in range(6)]
    db = O.ServerDb()
    srv = CO.Server(6, 10000)
    for b in range(5):
        strings, own = [], []
        for _ in range(rng.randrange(1, 8)):
            o = rng.randrange(6)
            k = rng.randrange(0, 20)
            ts = [O.timestamp_to_string(W.T0 + rng.randrange(0, 50) * 997, rng.randrange(2), "%016x" % o)
                  for _ in range(k)]
            got = []
            db.add_messages(db.get_merkle_tree(owners[o]), owners[o], [(t, b"") for t in ts], got)
            strings += ts
            own += [o] * k
            st, f = srv.ingest(_arena(ts), np.array([o] * k, dtype=np.uint32))
            assert st == 0 and [bool(x) for x in f] == got
    for o in range(6):
        assert srv.tree_json(o) == O.merkle_tree_to_string(db.get_merkle_tree(owners[o]))


def test_tree_json_and_diff():
    rng = random.Random(8)
    for _ in range(20):
        pool = W.hlc_timestamps(rng, rng.randrange(1, 30), [W.node_id(rng)], t0=rng.choice([0, W.T0]))
        t = {}
        for s in pool:
            t = O.insert_into_merkle_tree(t, O.parse_canonical(s))
        assert CO.tree_json(_arena(pool)) == O.merkle_tree_to_string(t)
