"""applyMessages against a __message table that already holds rows
(applyMessages.ts:42-45,104-119; PK "timestamp", initDbModel.ts:44).

Batch 2 runs on the state batch 1 left: the cells' current maxima (prior_ts,
applyMessages.ts:34-40) and the stored rows that hold one of batch 2's
timestamps (the caller's SELECT ... WHERE "timestamp" IN (...)).  A stored
row of the message's own cell is ordinary LWW state; one of another cell is
the global-PK case the engine must report (EVM_ECOLLISION)."""
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
    e.set_option(1, 0)
    e.close()


def _stored_rows(db, batch):
    """SELECT "timestamp", "table", "row", "column" FROM "__message" WHERE "timestamp" IN (...)"""
    tss = sorted({m["timestamp"] for m in batch})
    rows = []
    for k in range(0, len(tss), 500):
        chunk = tss[k:k + 500]
        q = 'SELECT "timestamp", "table", "row", "column" FROM "__message" WHERE "timestamp" IN (%s)' % ",".join(
            "?" * len(chunk))
        rows += db.conn.execute(q, chunk).fetchall()
    return rows


def _apply2(eng, db, tree1, batch, path):
    """batch 2 through the engine on db's state -> (status, flags, winner, tree json, cells)."""
    from evolu_amd import _lib as L

    cells = []
    cid = {}
    for m in batch:
        c = (m["table"], m["row"], m["column"])
        if c not in cid:
            cid[c] = len(cells)
            cells.append(c)
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in batch], dtype=np.uint32)
    prior = [db.cell_max(*c) for c in cells]
    pp = np.array([p is not None for p in prior], dtype=np.uint8)
    rows = _stored_rows(db, batch)
    s_ts = eng.timestamps([r[0] for r in rows]) if rows else None
    s_cell = eng.dev(np.array([cid.get((r[1], r[2], r[3]), 0xFFFFFFFF) for r in rows], dtype=np.uint32)) \
        if rows else None
    eng.set_option(L.OPT_CLIENT_PATH, path)
    flags, winner, tout, st = eng.apply_batch(
        eng.tree_from_json([O.merkle_tree_to_string(tree1)]), eng.timestamps([m["timestamp"] for m in batch]),
        eng.dev(cell), len(cells), prior_ts=eng.timestamps([p or "" for p in prior]), prior_present=eng.dev(pp),
        raise_on_error=False, stored_ts=s_ts, stored_cell=s_cell)
    eng.set_option(L.OPT_CLIENT_PATH, 0)
    return st, flags.cpu().numpy(), winner.cpu().numpy(), (tout.to_json(0) if tout is not None else None), cells, rows


def _two_batches(seed, cross):
    rng = random.Random(seed)
    b1, _ = W.client_batch(seed, n=400, n_cells=9)
    b2, _ = W.client_batch(seed + 1000, n=300, n_cells=12, t0=W.T0 + 1800_000)
    # redeliveries of batch-1 rows inside batch 2 (their own cells: ordinary state)
    for _ in range(40):
        b2.insert(rng.randrange(len(b2) + 1), dict(rng.choice(b1)))
    if cross:
        # one batch-1 timestamp re-sent under another cell
        m = dict(rng.choice(b1))
        m["column"] = "otherColumn"
        b2.insert(rng.randrange(len(b2) + 1), m)
    return b1, b2


@pytest.mark.parametrize("path", [1, 2])
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_stored_rows_own_cell_vs_oracle(eng, path, seed):
    from evolu_amd import _lib as L

    b1, b2 = _two_batches(seed, cross=False)
    db = O.ClientDb()
    tree1 = O.apply_messages(db, {}, b1)
    st, flags, winner, tjson, cells, rows = _apply2(eng, db, tree1, b2, path)
    assert rows, "the batch must hit stored rows"
    assert st == L.EVM_OK
    dec = []
    want = O.apply_messages(db, tree1, b2, dec)
    for i, (ups, xr, _) in enumerate(dec):
        assert bool(flags[i] & L.MSG_UPS) == ups and bool(flags[i] & L.MSG_XOR) == xr, i
    last = {}
    for i, m in enumerate(b2):
        if dec[i][0]:
            last[(m["table"], m["row"], m["column"])] = i
    assert [int(w) for w in winner] == [last.get(c, -1) for c in cells]
    assert tjson == O.merkle_tree_to_string(want)


@pytest.mark.parametrize("path", [1, 2])
def test_stored_row_of_another_cell_is_a_collision(eng, path):
    """The reference ignores the INSERT (ON CONFLICT DO NOTHING) and freezes
    that cell's running max; the engine must not apply the batch."""
    from evolu_amd import _lib as L

    b1, b2 = _two_batches(21, cross=True)
    db = O.ClientDb()
    tree1 = O.apply_messages(db, {}, b1)
    st, _, _, tjson, _, rows = _apply2(eng, db, tree1, b2, path)
    assert st == L.EVM_ECOLLISION and tjson is None
    # the in-batch check alone cannot see it: batch 2 holds that timestamp once
    i = next(k for k, m in enumerate(b2) if m["column"] == "otherColumn")
    assert sum(m["timestamp"] == b2[i]["timestamp"] for m in b2) == 1
    assert any(r[0] == b2[i]["timestamp"] and r[3] != "otherColumn" for r in rows)
    # and the reference indeed ignores that message's INSERT while XORing it
    dec = []
    O.apply_messages(db, tree1, b2, dec)
    assert dec[i][1] and not dec[i][2], "XOR taken, INSERT ignored (applyMessages.ts:104-119)"


def test_stored_rows_at_scale(eng):
    """1M-message batch with 20k stored rows of its own cells: no collision;
    one stored row relabelled to another cell: collision (both paths)."""
    from evolu_amd import _lib as L
    from evolu_amd import synth

    ts_np, cell_np = synth.config2(1_000_000, 1000, seed_config=31)
    rng = np.random.default_rng(3)
    pick = rng.choice(len(ts_np), size=20000, replace=False)
    s_ts = eng.dev(ts_np[pick])
    s_cell_np = cell_np[pick].copy()
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    for path in (1, 2):
        eng.set_option(L.OPT_CLIENT_PATH, path)
        _, _, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, 1000, raise_on_error=False, stored_ts=s_ts,
                                         stored_cell=eng.dev(s_cell_np))
        assert st == L.EVM_OK
        bad = s_cell_np.copy()
        bad[12345] = (bad[12345] + 1) % 1000
        _, _, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, 1000, raise_on_error=False, stored_ts=s_ts,
                                         stored_cell=eng.dev(bad))
        assert st == L.EVM_ECOLLISION
        bad[12345] = 0xFFFFFFFF  # a cell the batch does not touch
        _, _, tree, st = eng.apply_batch(eng.tree_new(1), ts, cell, 1000, raise_on_error=False, stored_ts=s_ts,
                                         stored_cell=eng.dev(bad))
        assert st == L.EVM_ECOLLISION
    eng.set_option(L.OPT_CLIENT_PATH, 0)
