"""evm_apply_batch_async / evm_apply_wait (applyMessages as a task,
applyMessages.ts:26-31): batches enqueued back to back, then waited, give
exactly what the synchronous call gives -- including the cases the wait has
to finish on the host (a tie redone by the exact walk path, a non-empty tree
merged, a bad timestamp, a batch the streaming path does not take)."""
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


def _sync(eng, tree_json, ts, cell, C):
    f, w, t, st = eng.apply_batch(eng.tree_from_json([tree_json]), ts, cell, C, raise_on_error=False)
    return st, f.cpu().numpy(), w.cpu().numpy(), (t.to_json(0) if t is not None else None)


def _dev_batch(eng, msgs, cells):
    cid = {c: i for i, c in enumerate(cells)}
    return (eng.timestamps([m["timestamp"] for m in msgs]),
            eng.dev(np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype=np.uint32)))


def test_pipelined_batches_equal_sync(eng):
    import torch

    from evolu_amd import synth

    # (batches large enough that one batch's second-stream work -- the fused
    # check + fold reads TP1's per-row words -- still runs while the next
    # batch's TP1 writes its own: they must not share a buffer)
    n = 2_000_000
    batches = []
    for k in range(4):
        ts_np, cell_np = synth.config2(n, 500, seed_config=60 + k)
        batches.append((eng.dev(ts_np), eng.dev(cell_np)))
    trees_in = [eng.tree_new(1) for _ in batches]
    outs = [(torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(500, dtype=torch.int32, device="cuda"))
            for _ in batches]
    pend = [eng.apply_batch_async(trees_in[k], ts, cell, 500, *outs[k]) for k, (ts, cell) in enumerate(batches)]
    for k, p in enumerate(pend):
        f, w, t, st = p.wait()
        want = _sync(eng, "{}", batches[k][0], batches[k][1], 500)
        assert st == want[0] == 0
        assert np.array_equal(f.cpu().numpy(), want[1]) and np.array_equal(w.cpu().numpy(), want[2])
        assert t.to_json(0) == want[3]


def test_async_redo_merge_bad_and_general(eng):
    import torch

    # a tie (equal millis + counter, two nodes, one cell) -> the exact walk path at the wait
    msgs, cells = W.client_batch(901, n=700, n_cells=5)
    ts, cell = _dev_batch(eng, msgs, cells)
    prior_tree = O.merkle_tree_to_string(O.apply_messages(O.ClientDb(), {}, W.client_batch(902, n=50, n_cells=5)[0]))
    for tree_json in ("{}", prior_tree):  # empty: the speculative tree; non-empty: merged at the wait
        f = torch.empty(len(msgs), dtype=torch.uint8, device="cuda")
        w = torch.empty(len(cells), dtype=torch.int32, device="cuda")
        tin = eng.tree_from_json([tree_json])
        p = eng.apply_batch_async(tin, ts, cell, len(cells), f, w)
        fo, wo, t, st = p.wait(raise_on_error=False)
        want = _sync(eng, tree_json, ts, cell, len(cells))
        assert st == want[0] == 0
        assert np.array_equal(fo.cpu().numpy(), want[1]) and np.array_equal(wo.cpu().numpy(), want[2])
        assert t.to_json(0) == want[3]
    # a bad timestamp: ENONCANON at the wait, only the culprit flagged
    strings = [m["timestamp"] for m in msgs]
    strings[5] = strings[5][:-1] + "g"
    ts_bad = eng.timestamps(strings)
    f = torch.empty(len(msgs), dtype=torch.uint8, device="cuda")
    w = torch.empty(len(cells), dtype=torch.int32, device="cuda")
    fo, _, t, st = eng.apply_batch_async(eng.tree_new(1), ts_bad, cell, len(cells), f, w).wait(raise_on_error=False)
    from evolu_amd import _lib as L

    assert st == L.EVM_ENONCANON and t is None
    assert fo.cpu().numpy()[5] == L.MSG_BAD and (np.delete(fo.cpu().numpy(), 5) == 0).all()
    # > 2,048 cells: the sort path, finished inside the async call
    many = [("t", "r%d" % i, "c") for i in range(3000)]
    import zlib

    mm = [{"timestamp": m["timestamp"], "table": "t", "row": "r%d" % (zlib.crc32(m["timestamp"].encode()) % 3000),
           "column": "c", "value": i} for i, m in enumerate(msgs)]
    ts2, cell2 = _dev_batch(eng, mm, many)
    f = torch.empty(len(mm), dtype=torch.uint8, device="cuda")
    w = torch.empty(len(many), dtype=torch.int32, device="cuda")
    fo, wo, t, st = eng.apply_batch_async(eng.tree_new(1), ts2, cell2, len(many), f, w).wait()
    want = _sync(eng, "{}", ts2, cell2, len(many))
    assert np.array_equal(fo.cpu().numpy(), want[1]) and t.to_json(0) == want[3]
