"""getMessages for an owner split over ranks (evolu_amd/dist.py: the
evm_dist_merge_trees / merge_select plan over torch.distributed), gloo on CPU,
world_size 2, against one unsharded server (the oracle's verbatim SQL,
apps/server/src/index.ts:173-202).

The split owner's diff must be the diff of its FULL server tree (the merge
of the per-rank partial leaf maps, gather_leaf_parts) against the client's
full tree; each rank then selects its share after that bound with the
NOT LIKE node filter, and the shares merge in timestamp order
(gather_selection).  The local step is the oracle (a ServerDb per rank)."""
import os
import random

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_dist_hot import N_OWNERS, _free_port, _leaves, _messages


def _client_tree(o):
    """The client's tree of owner o: every third message of that owner missing."""
    from oracle import evolu_oracle as O

    tree = {}
    k = 0
    for r in range(2):
        for oo, t in _messages(r):
            if oo == o:
                if k % 3:
                    tree = O.insert_into_merkle_tree(tree, O.parse_canonical(t))
                k += 1
    return tree


def _node(o):
    return "%016x" % (o * 7)  # one of the owner's two nodes: its rows are filtered out


def _key(ts):
    from oracle import evolu_oracle as O

    m, c, n = O.parse_canonical(ts)
    return [(m << 16) | c, int(n, 16), 0]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from evolu_amd import dist as D
        from evolu_amd.engine import encode_timestamps, key_code, key_string
        from oracle import evolu_oracle as O

        msgs = _messages(rank)
        ts = torch.from_numpy(encode_timestamps([t for _, t in msgs]))
        owner = torch.tensor([o for o, _ in msgs], dtype=torch.int64)
        from tests.test_dist import _user_ids

        omap = D.OwnerMap(D.Directory(_user_ids(N_OWNERS), world), rank,
                          D.hot_owners(D.owner_counts(owner, N_OWNERS), world))
        ts_r, own_r, src_rank, src_idx = D.route_by_owner(ts, owner, omap.dest(owner, ts))
        loc = omap.local(own_r).tolist()
        gid = (src_rank * 100000 + src_idx).tolist()  # global message ids
        db = O.ServerDb()
        for i, lo in enumerate(loc):
            t = bytes(ts_r[i, :46].numpy()).decode()
            db.add_messages(db.get_merkle_tree("l%d" % lo), "l%d" % lo, [(t, str(gid[i]).encode())])
        nh = int(omap.hot.size)
        # cold owners: their whole tree is here
        cold = {}
        for j, o in enumerate(omap.owners_here()[:omap.hot_base].tolist()):
            if o < 0:
                continue
            d, rows = db.get_messages(db.get_merkle_tree("l%d" % j), _client_tree(o), "l%d" % j, _node(o))
            cold[o] = (d, [int(c) for _, c in rows])
        # hot owners: merge the partial leaf maps, diff the full trees, select shares, merge shares
        offs, codes, xrs = [0], [], []
        for k in range(nh):
            lv = _leaves(db.get_merkle_tree("l%d" % (omap.hot_base + k)))
            for key in sorted(lv, key=key_code):
                codes.append(key_code(key))
                xrs.append(O.to_int32(lv[key]))
            offs.append(len(codes))
        parts = D.gather_leaf_parts(torch.tensor(offs), torch.tensor(codes, dtype=torch.int64),
                                    torch.tensor(xrs, dtype=torch.int32))
        sel_off, sel_id, sel_key, diffs = [0], [], [], []
        for k, o in enumerate(omap.hot.tolist()):
            merged = {}
            for po, pc, px in parts:
                for c, x in zip(pc[po[k]:po[k + 1]].tolist(), px[po[k]:po[k + 1]].tolist()):
                    merged[key_string(c)] = merged.get(key_string(c), 0) ^ x
            full = O.tree_from_leaves({key: O.to_int32(x) for key, x in merged.items()})
            d = O.diff_merkle_trees(full, _client_tree(o))
            diffs.append(d)
            if d is not None:
                since = O.timestamp_to_string(*O.create_sync_timestamp(d))
                rows = db.conn.execute(O._SQL_SELECT_MESSAGES, ("l%d" % (omap.hot_base + k), since,
                                                                _node(o))).fetchall()
                for t, c in rows:
                    sel_id.append(int(c))
                    sel_key.append(_key(t))
            sel_off.append(len(sel_id))
        hoff, hids = D.gather_selection(torch.tensor(sel_off), torch.tensor(sel_id, dtype=torch.int64),
                                        torch.tensor(sel_key, dtype=torch.int64).reshape(-1, 3))
        hot = {o: (diffs[k], hids[hoff[k]:hoff[k + 1]].tolist()) for k, o in enumerate(omap.hot.tolist())}
        q.put((rank, cold, hot))
    finally:
        dist.destroy_process_group()


def test_split_owner_get_messages_gloo_world2():
    from oracle import evolu_oracle as O

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time

    res = {}
    deadline = time.time() + 240
    while len(res) < world:
        try:
            r = q.get(timeout=2)
            res[r[0]] = r[1:]
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs) or time.time() > deadline:
                for p in procs:
                    p.kill()
                pytest.fail("a rank failed: exit codes %s" % [p.exitcode for p in procs])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # the unsharded server, global batch order (rank-major), content = global id
    db = O.ServerDb()
    for r in range(world):
        for i, (o, t) in enumerate(_messages(r)):
            db.add_messages(db.get_merkle_tree("u%d" % o), "u%d" % o, [(t, str(r * 100000 + i).encode())])
    want = {}
    for o in range(N_OWNERS):
        d, rows = db.get_messages(db.get_merkle_tree("u%d" % o), _client_tree(o), "u%d" % o, _node(o))
        want[o] = (d, [int(c) for _, c in rows])
    assert set(res[0][1]) == {0}  # owner 0 is the split one
    assert res[0][1] == res[1][1]  # every rank holds the merged selection
    got = dict(res[0][1])
    for r in range(world):
        got.update(res[r][0])
    assert got == want
    assert want[0][0] is not None and len(want[0][1]) > 10
