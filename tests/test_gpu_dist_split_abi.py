"""Hot-owner and cell splits through the evm_dist_* C ABI (SURVEY 8(e),
BASELINE config 5) on loopback ranks (one thread, context and stream each,
one GPU), against the unsharded C restatement:

* server: a Zipf(1.2) round over owners sharded murmur3(userId) mod world
  (evm_dist_directory), the hot ones
  (evm_dist_hot_owners) split over every rank by timestamp hash
  (evm_dist_split): INSERT OR IGNORE counts per owner, every owner's root
  (evm_dist_gather_roots XORs the split ones), the split owners' full trees
  (evm_dist_merge_trees), their diffs against the client trees and their
  getMessages rows merged in timestamp order (evm_dist_merge_select) --
  apps/server/src/index.ts:138-202 for one unsharded server;
* client: one owner's applyMessages batch split by cell
  (evolu_amd.sharded.split_apply): flags back to the source rows
  (evm_dist_return), global winners (evm_dist_split_winners), the merged
  tree, and a cross-cell PK collision agreed by every rank
  (applyMessages.ts:26-131)."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as CO
from oracle import evolu_oracle as O

pytestmark = pytest.mark.gpu


def _loop(world, fn):
    from evolu_amd.engine import run_loopback

    return run_loopback(world, fn)


def _cuts(n, world):
    return [n * r // world for r in range(world + 1)]


@pytest.mark.parametrize("world", [2, 3])
def test_hot_owner_split_server_vs_unsharded_c_oracle(world):
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.sharded import ShardedServer

    O_, N = 40, 30_000
    ts, owner, _ = synth.config5(O_, N, seed_config=71)
    owner = owner.astype(np.uint32)
    rng = np.random.default_rng(5)
    keep = rng.random(len(ts)) < 0.6  # what the clients already hold
    srv, cli = CO.Server(O_, len(ts)), CO.Server(O_, len(ts))
    assert srv.ingest(ts, owner)[0] == 0 and cli.ingest(ts[keep], owner[keep])[0] == 0
    cut = _cuts(len(ts), world)
    node_of = {g: "%016x" % (0x1234_5678_9ABC_0000 + g) for g in range(O_)}
    counts = np.bincount(owner, minlength=O_)
    want_hot = np.flatnonzero(counts > 0.25 * len(ts) / world)
    assert want_hot.size >= 1  # Zipf 1.2: the top owners

    def fn(r, eng, dd):
        ids = np.zeros((O_, 24), dtype=np.uint8)
        ids[:, :21] = np.frombuffer(b"".join(b"u%020d" % g for g in range(O_)), dtype=np.uint8).reshape(O_, 21)
        sv = ShardedServer(eng, dd, eng.dev(ids), 21)
        t_in, o_in = eng.dev(ts[cut[r]:cut[r + 1]]), eng.dev(owner[cut[r]:cut[r + 1]])
        hot = sv.split_hot(o_in, share=0.25)
        t_r, o_r, f = sv.ingest(t_in, o_in, id_base=r << 40)
        glob = sv.local_owners().cpu().numpy()
        # client trees per local id (hot slots: the split owner's full client tree)
        rows, slots = [], []
        for j, g in enumerate(glob):
            if g >= 0:
                m = keep & (owner == g)
                rows.append(ts[m])
                slots.append(np.full(m.sum(), j, dtype=np.uint32))
        client = eng.merkle_insert(eng.tree_new(sv.n_local), eng.dev(np.concatenate(rows)),
                                   eng.dev(np.concatenate(slots)))
        node = eng.dev(np.frombuffer("".join(node_of[int(g)] if g >= 0 else "0" * 16 for g in glob).encode(),
                                     dtype=np.uint8).copy())
        diff, (off, sel), (hoff, hsel) = sv.select(client, node)
        root, present = sv.roots()
        full = dd.merge_trees(sv.store.tree(), sv.hot_base, len(hot))
        full_js = [full.to_json(h) for h in range(len(hot))]
        ins = np.bincount(o_r.cpu().numpy()[(f.cpu().numpy() & L.MSG_INS) != 0], minlength=sv.n_local)
        out = dict(hot=hot, base=sv.hot_base, glob=glob, rows=t_r.cpu().numpy(), ins=ins, diff=diff.cpu().numpy(),
                   off=off.cpu().numpy(), sel=sel.cpu().numpy(), hoff=hoff.cpu().numpy(), hsel=hsel.cpu().numpy(),
                   root=root.cpu().numpy(), present=present.cpu().numpy(), full=full_js)
        sv.close()
        return out

    res = _loop(world, fn)
    hot = res[0]["hot"]
    assert np.array_equal(hot, want_hot)
    for r in range(world):
        assert np.array_equal(res[r]["hot"], hot)

    def row_str(i):
        q, k = int(i) >> 40, int(i) & ((1 << 40) - 1)
        return bytes(res[q]["rows"][k][:46]).decode()

    def expected(g, d):
        if d < 0:
            return []
        sync = O.timestamp_to_string(d, 0, "0000000000000000")
        strs = sorted({bytes(x[:46]).decode() for x in ts[owner == g]})
        return [s for s in strs if s > sync and not s.lower().endswith(node_of[g])]

    inserted = np.zeros(O_, dtype=np.int64)
    for r in range(world):
        x = res[r]
        for j, g in enumerate(x["glob"]):
            if g < 0:
                continue
            inserted[g] += x["ins"][j]
            if j >= x["base"]:  # split owner: its full-tree diff on every rank
                h = j - x["base"]
                d = srv.diff(cli, int(g))
                assert x["diff"][j] == d
                got = [row_str(i) for i in x["hsel"][x["hoff"][h]:x["hoff"][h + 1]]]
                assert got == expected(int(g), d)
                assert x["full"][h] == srv.tree_json(int(g))
            else:
                d = srv.diff(cli, int(g))
                assert x["diff"][j] == d
                got = [row_str(i) for i in x["sel"][x["off"][j]:x["off"][j + 1]]]
                assert got == expected(int(g), d)
        assert np.array_equal(x["root"], res[0]["root"])
    # INSERT OR IGNORE: each distinct (owner, timestamp) inserted exactly once over all ranks
    for g in range(O_):
        assert inserted[g] == len({bytes(x[:46]) for x in ts[owner == g]})
        js = srv.tree_json(g)
        assert res[0]["root"][g] == O.merkle_tree_from_string(js).get("hash", 0)
        assert bool(res[0]["present"][g]) == (js != "{}")


@pytest.mark.parametrize("world,collide", [(2, False), (3, False), (2, True)])
def test_cell_split_apply_vs_unsharded_c_oracle(world, collide):
    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.sharded import split_apply

    CELLS, N = 300, 40_000
    ts, _, cell = synth.config5(1, N, cells_per_owner=CELLS, seed_config=57)
    cell = cell.astype(np.uint32)
    if collide:  # one timestamp again under another cell, in another rank's slice
        ts = ts.copy()
        ts[len(ts) - 7] = ts[11]
        cell = cell.copy()
        cell[len(ts) - 7] = (cell[11] + 1) % CELLS
    st_o, flags_o, win_o, js_o = CO.apply(ts, cell, CELLS)
    cut = _cuts(len(ts), world)

    def fn(r, eng, dd):
        t, c = eng.dev(ts[cut[r]:cut[r + 1]]), eng.dev(cell[cut[r]:cut[r + 1]].view(np.int32))
        flags, winner, tree, st = split_apply(eng, dd, t, c, CELLS, tree_in=eng.tree_new(1))
        return (st, flags.cpu().numpy(), None if winner is None else winner.cpu().numpy(),
                None if tree is None else tree.to_json(0))

    res = _loop(world, fn)
    if collide:
        assert st_o == L.EVM_ECOLLISION
        assert all(x[0] == L.EVM_ECOLLISION for x in res)
        return
    assert st_o == 0
    flags = np.concatenate([x[1] for x in res])
    assert np.array_equal(flags, flags_o)
    for x in res:
        assert x[0] == 0
        assert np.array_equal(x[2], win_o.astype(np.int64))
        assert x[3] == js_o


def test_merge_select_orders_shares_and_return_restores_positions():
    """Index math on its own: three ranks' sorted shares of 4 groups (one
    empty, equal keys across ranks -> lower rank first) merge in key order;
    evm_dist_return sends each received row's value to its source index."""
    world = 3
    rng = np.random.default_rng(3)
    shares = []
    for r in range(world):
        counts = rng.integers(0, 6, 4)
        counts[2] = 0
        keys, ids = [], []
        for g, k in enumerate(counts):
            kk = np.sort(rng.integers(0, 8, k)) * 10 + g
            keys += [(int(v), 0, 0) for v in kk]
            ids += [(r << 40) | len(ids) + j for j in range(k)]
        off = np.concatenate([[0], np.cumsum(counts)]) + 5  # off[0] need not be 0
        shares.append((off, np.array(ids, dtype=np.int64), np.array(keys, dtype=np.int64).reshape(-1, 3)))

    def fn(r, eng, dd):
        off, ids, keys = shares[r]
        pad_ids = np.concatenate([np.zeros(5, dtype=np.int64), ids])
        pad_keys = np.concatenate([np.zeros((5, 3), dtype=np.int64), keys])
        o, i = dd.merge_select(eng.dev(off), eng.dev(pad_ids), eng.dev(pad_keys.reshape(-1)))
        # return path: route rows to rank (row % world), send row*7+r back
        n = 50 + r
        rows = np.zeros((n, 48), dtype=np.uint8)
        own = np.arange(n, dtype=np.uint32)
        dd.route(eng.dev(rows), eng.dev(own), dest=eng.dev((own % world).astype(np.uint8)))
        _, o2, _, src, _ = dd.take()
        back = dd.send_back((o2.to(torch.int64) * 7 + r).to(torch.int32), n)
        return o.cpu().numpy(), i.cpu().numpy(), back.cpu().numpy()

    res = _loop(world, fn)
    for g in range(4):
        rows = []
        for r, (off, ids, keys) in enumerate(shares):
            a, b = off[g] - 5, off[g + 1] - 5
            rows += [(int(keys[k][0]), r, int(ids[k])) for k in range(a, b)]
        want = [x[2] for x in sorted(rows)]
        for r in range(world):
            o, i, _ = res[r]
            assert list(i[o[g]:o[g + 1]]) == want
    for r in range(world):
        n = 50 + r
        back = res[r][2]
        assert list(back) == [k * 7 + (k % world) for k in range(n)]


@pytest.mark.parametrize("world,cross", [(2, False), (3, False), (2, True)])
def test_cell_split_apply_on_prior_state_vs_oracle(world, cross):
    """The split on a non-empty DB (applyMessages.ts:34-45,93-119): batch 2
    runs on the state batch 1 left -- every cell's current max and the
    __message rows holding a batch-2 timestamp, the same on every rank.
    Redeliveries of batch-1 rows are no-ops or XOR toggles exactly as in one
    process; a batch-1 timestamp re-sent under another cell is the global-PK
    case on every rank."""
    from evolu_amd import _lib as L
    from evolu_amd.sharded import split_apply
    from tests.test_gpu_apply_stored import _stored_rows, _two_batches

    b1, b2 = _two_batches(21 + world, cross)
    db = O.ClientDb()
    tree1 = O.apply_messages(db, {}, b1)
    cells, cid = [], {}
    for m in b2:
        c = (m["table"], m["row"], m["column"])
        if c not in cid:
            cid[c] = len(cells)
            cells.append(c)
    cell = np.array([cid[(m["table"], m["row"], m["column"])] for m in b2], dtype=np.uint32)
    prior = [db.cell_max(*c) for c in cells]
    pp = np.array([p is not None for p in prior], dtype=np.uint8)
    rows = _stored_rows(db, b2)
    assert rows and pp.any()
    s_cell = np.array([cid.get((r[1], r[2], r[3]), 0xFFFFFFFF) for r in rows], dtype=np.uint32)
    dec = []
    want = O.apply_messages(db, tree1, b2, dec)
    cut = _cuts(len(b2), world)
    strs = [m["timestamp"] for m in b2]
    tree1_js = O.merkle_tree_to_string(tree1)

    def fn(r, eng, dd):
        t = eng.timestamps(strs[cut[r]:cut[r + 1]])
        c = eng.dev(cell[cut[r]:cut[r + 1]].view(np.int32))
        flags, winner, tree, st = split_apply(
            eng, dd, t, c, len(cells), tree_in=eng.tree_from_json([tree1_js]),
            prior_ts=eng.timestamps([p or "" for p in prior]), prior_present=eng.dev(pp),
            stored_ts=eng.timestamps([x[0] for x in rows]), stored_cell=eng.dev(s_cell))
        return (st, flags.cpu().numpy(), None if winner is None else winner.cpu().numpy(),
                None if tree is None else tree.to_json(0))

    res = _loop(world, fn)
    if cross:
        assert all(x[0] == L.EVM_ECOLLISION for x in res)
        return
    flags = np.concatenate([x[1] for x in res])
    for i, (ups, xr, _) in enumerate(dec):
        assert bool(flags[i] & L.MSG_UPS) == ups and bool(flags[i] & L.MSG_XOR) == xr, i
    last = {}
    for i, m in enumerate(b2):
        if dec[i][0]:
            last[(m["table"], m["row"], m["column"])] = i
    for x in res:
        assert x[0] == L.EVM_OK
        assert [int(w) for w in x[2]] == [last.get(c, -1) for c in cells]
        assert x[3] == O.merkle_tree_to_string(want)
