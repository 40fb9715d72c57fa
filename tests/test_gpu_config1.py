"""BASELINE config 1 at full size: one owner's todo-schema stream
(examples/nextjs/pages/index.tsx:23-34, db.ts:268-300 mutation shapes;
evolu_amd/synth.config1), 100k CrdtMessages over ~55k cells -- merged by
applyMessages on the GPU (the sort path: > 2,048 cells) against the Python
oracle (applyMessages.ts control flow, reference SQL verbatim in sqlite3):
every message's upsert / XOR decision, every cell's winner, and the
MerkleTree JSON byte for byte."""
import numpy as np
import pytest

from oracle import evolu_oracle as O

pytestmark = pytest.mark.gpu


def _oracle(ts, cell, cells, values):
    msgs = []
    for i in range(len(cell)):
        t, r, c = cells[cell[i]]
        msgs.append({"timestamp": ts[i, :46].tobytes().decode(), "table": t, "row": r, "column": c, "value": values[i]})
    db = O.ClientDb()
    dec = []
    tree = O.apply_messages(db, {}, msgs, dec)
    return msgs, dec, tree


def test_config1_full_size_vs_oracle():
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.engine import Engine

    ts, cell, cells, values = synth.config1(100_000)
    assert len(cells) > 2048
    msgs, dec, want = _oracle(ts, cell, cells, values)
    eng = Engine(0)
    flags, winner, tree, st = eng.apply_batch(eng.tree_new(1), eng.dev(ts), eng.dev(cell), len(cells))
    assert st == L.EVM_OK
    f = flags.cpu().numpy()
    exp = np.array([(1 if u else 0) | (2 if x else 0) for u, x, _ in dec], dtype=np.uint8)
    assert np.array_equal(f, exp)
    last = np.full(len(cells), -1, dtype=np.int64)
    for i, (u, _, _) in enumerate(dec):
        if u:
            last[cell[i]] = i
    assert np.array_equal(winner.cpu().numpy().astype(np.int64), last)
    assert tree.to_json(0) == O.merkle_tree_to_string(want)
    eng.close()


def test_config1_redelivered_on_prior_state():
    """The second half of the stream applied on the state the first half left
    (prior cell maxima + the first half's tree), with 5 % of the first half
    re-sent inside it (stale redeliveries toggle, exact ones are no-ops)."""
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.engine import Engine

    ts, cell, cells, values = synth.config1(40_000, seed_config=101)
    half = 20_000
    rng = np.random.default_rng(1)
    red = rng.choice(half, size=1000, replace=False)
    ts2 = np.concatenate([ts[half:], ts[red]])
    cell2 = np.concatenate([cell[half:], cell[red]])
    perm = rng.permutation(len(ts2))
    ts2, cell2 = ts2[perm], cell2[perm]
    vals2 = [values[half + i] if i < len(ts) - half else values[red[i - (len(ts) - half)]] for i in perm]
    msgs1, _, tree1 = _oracle(ts[:half], cell[:half], cells, values[:half])
    db = O.ClientDb()
    O.apply_messages(db, {}, msgs1)
    # the second batch's own cell numbering, with the prior maxima
    used = sorted(set(cell2.tolist()))
    remap = {c: k for k, c in enumerate(used)}
    c2 = np.array([remap[c] for c in cell2], dtype=np.uint32)
    prior = [db.cell_max(*cells[c]) for c in used]
    msgs2 = [{"timestamp": ts2[i, :46].tobytes().decode(), "table": cells[cell2[i]][0], "row": cells[cell2[i]][1],
              "column": cells[cell2[i]][2], "value": vals2[i]} for i in range(len(ts2))]
    dec = []
    want = O.apply_messages(db, tree1, msgs2, dec)
    eng = Engine(0)
    from evolu_amd.engine import encode_timestamps

    flags, winner, tree, st = eng.apply_batch(
        eng.tree_from_json([O.merkle_tree_to_string(tree1)]), eng.dev(ts2), eng.dev(c2), len(used),
        prior_ts=eng.dev(encode_timestamps([p or "" for p in prior])),
        prior_present=eng.dev(np.array([p is not None for p in prior], dtype=np.uint8)))
    assert st == L.EVM_OK
    exp = np.array([(1 if u else 0) | (2 if x else 0) for u, x, _ in dec], dtype=np.uint8)
    assert np.array_equal(flags.cpu().numpy(), exp)
    assert (exp == 2).sum() > 0 and (exp == 0).sum() > 0  # stale toggles and no-op redeliveries both occur
    assert tree.to_json(0) == O.merkle_tree_to_string(want)
    eng.close()
