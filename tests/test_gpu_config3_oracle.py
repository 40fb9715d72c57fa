"""The config-3 bench path pinned directly against the C restatement of the
server (apps/server/src/index.ts:138-171 addMessages: INSERT OR IGNORE on
(timestamp, userId), XOR into the owner's tree iff inserted), at the bench's
own shape: 20,000 owners x 1,000 messages, one SyncRequest per owner -- the
shape that runs K5 with the rows parsed in the workgroup
(`k_svo_a<1024, true>`), asserted from the engine's kernel report.

Round 2 is the steady state (bench.py `reingest`): per owner 900 new
timestamps and 100 redeliveries of round-1 rows, shuffled inside the
owner's request, into the store round 1 left -- the LDS-staged merge
(`k_svo_b<true>`).  Checked: every row's INSERT flag, the stored rows of
sampled owners byte for byte in timestamp order, sampled trees as JSON, and
the stored-row count."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu

O_, P = 20_000, 1000
SEED = 0xE7010003


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


def _ran(eng, fn):
    eng.prof_enable(True)
    eng.prof_reset()
    out = fn()
    torch.cuda.synchronize()
    rep = eng.prof_report()
    eng.prof_enable(False)
    return out, rep


def test_config3_shape_and_reingest_vs_c_oracle(eng):
    from evolu_amd import _lib as L
    from evolu_amd import synth

    dev = torch.device("cuda", 0)
    gen = synth.DeviceSynth()
    t1, o1, _ = gen.source(SEED, O_, P, 1, 0, dev)  # one request (run) per owner, 1,000 messages each
    t2n, o2n, _ = gen.source(SEED + 1, O_, P, 1, 0, dev)
    ts1, own1 = t1.cpu().numpy(), o1.cpu().numpy().astype(np.uint32)
    by1 = ts1[np.argsort(own1, kind="stable")].reshape(O_, P, 48)  # every owner's 1,000 round-1 rows
    # round 2: per owner 900 new timestamps + 100 redeliveries of its round-1 rows, shuffled in the run
    rng = np.random.default_rng(3)
    t2n_np, o2n_np = t2n.cpu().numpy(), o2n.cpu().numpy()
    new = t2n_np[np.argsort(o2n_np, kind="stable")].reshape(O_, P, 48)[:, :900]
    redo = by1[np.arange(O_)[:, None], rng.integers(0, P, (O_, 100))]
    run = np.concatenate([new, redo], 1)
    perm = np.argsort(rng.random((O_, P)), axis=1)
    ts2 = run[np.arange(O_)[:, None], perm].reshape(-1, 48)
    own2 = np.repeat(np.arange(O_, dtype=np.uint32), P)
    ts1, ts2 = np.ascontiguousarray(ts1), np.ascontiguousarray(ts2)
    srv = CO.Server(O_, 2 * O_ * P)
    st, f1_want = srv.ingest(ts1, own1)
    assert st == 0
    st, f2_want = srv.ingest(ts2, own2)
    assert st == 0

    store = eng.store_new(O_)
    (f1, st1), rep1 = _ran(eng, lambda: store.ingest(t1, o1, 0))
    assert st1 == 0 and "(k_svo_a<1024, true>)" in rep1, sorted(rep1)
    # the empty store's commit: nothing -- K5 left the rows and a gapped tree in place
    assert "k_svo_copy" not in rep1 and "k_svo_b<false>" not in rep1, sorted(rep1)
    from tests.test_gpu_server import _check_prefix_xor, _is_gapped

    assert _is_gapped(eng, store.tree())

    _check_prefix_xor(eng, store.tree())
    assert np.array_equal(f1.cpu().numpy(), f1_want)
    (f2, st2), rep2 = _ran(eng, lambda: store.ingest(eng.dev(ts2), eng.dev(own2), 1 << 40))
    assert st2 == 0 and "k_svo_b<true>" in rep2, sorted(rep2)
    assert "(k_svo_a<1024, true, SVO_THREADS, true>)" in rep2, sorted(rep2)  # tree searches in LDS
    f2 = f2.cpu().numpy()
    assert np.array_equal(f2, f2_want)
    assert (f2 & L.MSG_INS).astype(bool).sum() == O_ * 900  # every redelivery ignored
    n_ins = int((f1_want & L.MSG_INS).astype(bool).sum() + (f2_want & L.MSG_INS).astype(bool).sum())
    assert store.n_messages == n_ins
    # the stored rows of sampled owners, in timestamp order, byte for byte
    off, ids = store.messages()
    for o in range(0, O_, 41):
        got = []
        for i in ids[int(off[o]):int(off[o + 1])]:
            i = int(i)
            got.append(bytes(ts2[i & ((1 << 40) - 1), :46] if i >> 40 else ts1[i, :46]))
        want = sorted({bytes(r[:46]) for r in by1[o]} | {bytes(r[:46]) for r in ts2[o * P:(o + 1) * P]})
        assert got == want, o
    tree = store.tree()
    for o in range(0, O_, 97):
        assert tree.to_json(o) == srv.tree_json(o)
    store.free()
