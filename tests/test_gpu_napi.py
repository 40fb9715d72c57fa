"""The N-API addon + JS entry points (js/) on the GPU, driven from node 12,
against the oracle: the reference-side binding works end to end."""
import json
import os
import random
import shutil
import subprocess

import pytest

from oracle import evolu_oracle as O
from tests import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _build_addon():
    js = os.path.join(ROOT, "js")
    out = os.path.join(js, "evm_napi.node")
    if not os.path.exists(out):
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DNODE_GYP_MODULE_NAME=evm_napi",
                        "-I/usr/include/node", "-I" + os.path.join(ROOT, "include"), os.path.join(js, "evm_napi.cpp"),
                        "-o", out, "-L" + os.path.join(ROOT, "evolu_amd"), "-levm",
                        "-Wl,-rpath,$ORIGIN/../evolu_amd"], check=True)
    return out


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists("/usr/include/node/node_api.h"),
                    reason="node / N-API headers not present")
def test_js_entry_points(tmp_path):
    _build_addon()
    n1 = "0000000000000001"
    ts1, ts2 = O.timestamp_to_string(0, 0, n1), O.timestamp_to_string(1656873738591, 0, n1)
    cases = {"insert": [{"tree": "{}", "timestamps": [ts1]}, {"tree": "{}", "timestamps": [ts2]},
                        {"tree": O.merkle_tree_to_string(O.insert_into_merkle_tree({}, O.parse_canonical(ts1))),
                         "timestamps": [ts2]}],
             "diff": [{"a": "{}", "b": "{}"},
                      {"a": "{}", "b": O.merkle_tree_to_string(O.insert_into_merkle_tree({}, O.parse_canonical(ts2)))}]}
    # applyMessages cases with prior rows
    apply_cases, expects = [], []
    for seed in range(4):
        msgs, cells = W.client_batch(500 + seed, n=200, n_cells=6)
        prior, _ = W.client_batch(600 + seed, n=30, n_cells=6, t0=W.T0 - 600_000)
        prior = list({m["timestamp"]: m for m in prior}.values())  # one cell per stored timestamp
        prior = [dict(m, table=cells[i % 6][0], row=cells[i % 6][1], column=cells[i % 6][2])
                 for i, m in enumerate(prior)]
        rng = random.Random(seed)
        # redeliveries of stored rows (their own cells), and in case 3 one stored
        # timestamp under another cell: the reference ignores that INSERT -> null
        for m in rng.sample(prior, 8):
            msgs.insert(rng.randrange(len(msgs) + 1), dict(m))
        if seed == 3:
            msgs.insert(50, dict(prior[4], column="otherColumn"))
        db = O.ClientDb()
        t0 = O.apply_messages(db, {}, prior)
        cell_max = {json.dumps([c[0], c[1], c[2]], separators=(",", ":")): db.cell_max(*c) for c in cells}
        stored = [{"timestamp": r[0], "table": r[1], "row": r[2], "column": r[3]} for r in db.conn.execute(
            'SELECT "timestamp", "table", "row", "column" FROM "__message"').fetchall()]
        dec = []
        t1 = O.apply_messages(db, t0, msgs, dec)
        ups = {}
        for m, (u, x, _) in zip(msgs, dec):
            if u:
                ups[json.dumps([m["table"], m["row"], m["column"]], separators=(",", ":"))] = m["value"]
        ins = [m["timestamp"] for m, (u, x, _) in zip(msgs, dec) if x]
        apply_cases.append({"tree": O.merkle_tree_to_string(t0), "messages": msgs, "stored": stored,
                            "cellMax": {k: v for k, v in cell_max.items() if v is not None}})
        expects.append({"tree": O.merkle_tree_to_string(t1), "upserts": ups, "inserts": ins} if seed < 3 else
                       {"tree": None, "upserts": {}, "inserts": []})
    cases["apply"] = apply_cases
    # server
    rng = random.Random(2)
    n_owners = 4
    pools = [W.hlc_timestamps(rng, 40, [W.node_id(rng) for _ in range(2)]) for _ in range(n_owners)]
    batches = []
    for _ in range(3):
        batches.append([{"owner": o, "messages": [{"timestamp": rng.choice(pools[o])} for _ in range(rng.randrange(8))]}
                        for o in [rng.randrange(n_owners) for _ in range(5)]])
    sdb = O.ServerDb()
    want_ins = []
    for b in batches:
        got = []
        for r in b:
            u = "u%d" % r["owner"]
            g = []
            sdb.add_messages(sdb.get_merkle_tree(u), u, [(m["timestamp"], b"") for m in r["messages"]], g)
            got += g
        want_ins.append(got)
    client = [O.merkle_tree_to_string(O.insert_into_merkle_tree({}, O.parse_canonical(p[0]))) for p in pools]
    node_ids = [p[1][30:] for p in pools]
    since = [None, 0, O.parse_canonical(sorted(pools[2])[10])[0], O.parse_canonical(sorted(pools[3])[-1])[0] + 1]
    cases["server"] = {"nOwners": n_owners, "batches": batches, "clientTrees": client, "nodeIds": node_ids,
                       "since": since}
    # receive fold: ok, drift, duplicate node
    rcases, rwant = [], []
    for k, mode in enumerate(["ok", "drift", "dup"]):
        node = "000000000000000%d" % (k + 1)
        now = W.T0 + 1000
        ts = W.hlc_timestamps(rng, 50, [W.node_id(rng) for _ in range(3)], t0=W.T0 - 5000, span=4000)
        if mode == "drift":
            ts.insert(20, O.timestamp_to_string(now + 60001, 0, W.node_id(rng)))
        if mode == "dup":
            ts.insert(30, O.timestamp_to_string(W.T0, 5, node))
        clock = {"millis": W.T0 - 7000, "counter": 3, "node": node}
        rcases.append({"clock": clock, "timestamps": ts, "now": now})
        t = (clock["millis"], clock["counter"], node)
        want = None
        for i, s_ in enumerate(ts):
            try:
                t = O.receive_timestamp(t, O.parse_canonical(s_), now, 60000)
            except O.TimestampError as e:
                want = {"ok": False, "type": e.kind, "index": i}
                break
        rwant.append(want or {"ok": True, "clock": {"millis": t[0], "counter": t[1], "node": node}})
    cases["receive"] = rcases
    f = tmp_path / "cases.json"
    f.write_text(json.dumps(cases))
    out = subprocess.run(["node", os.path.join(ROOT, "js", "test_evm.js"), str(f)], check=True,
                         capture_output=True, text=True, timeout=300).stdout
    res = json.loads(out.strip().splitlines()[-1])  # (RCCL prints its banner on stdout first)
    snap = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_snapshots.json")))["merkleTree.test.ts.snap"]
    assert [json.loads(t) for t in res["insert"]] == [snap["insertIntoMerkleTree 1"], snap["insertIntoMerkleTree 2"],
                                                     snap["insertIntoMerkleTree 3"]]
    assert res["diff"] == [None, 1656873720000]
    assert len(res["apply"]) == len(expects) == len(res["applyAsync"])
    for got, got_async, want in zip(res["apply"], res["applyAsync"], expects):
        assert got == want
        assert got_async == want  # Promise<Either>: Right, the same writes
    assert res["server"]["ins"] == want_ins
    for o in range(n_owners):
        assert res["server"]["trees"][o] == O.merkle_tree_to_string(sdb.get_merkle_tree("u%d" % o))
    for key in ("get", "getAsync"):
        for o in range(n_owners):
            d, rows = sdb.get_messages(sdb.get_merkle_tree("u%d" % o), json.loads(client[o]), "u%d" % o, node_ids[o])
            assert res["server"][key]["diff"][o] == d
            assert len(res["server"][key]["ids"][o]) == len(rows)
    assert res["server"]["insAsync"] == want_ins
    assert res["server"]["treesAsync"] == res["server"]["trees"]
    assert res["server"]["getAsync"]["ids"] == res["server"]["get"]["ids"]
    # evm_dist_* through the addon at world 1
    assert res["dist"]["sameOrder"] is True
    assert res["dist"]["roots"] == res["dist"]["treeHashes"]
    # a device error reaches the caller as Left(UnknownError), not as a throw
    assert res["leftOnError"]["_tag"] == "Left" and res["leftOnError"]["left"]["type"] == "UnknownError"
    # storedRows is required: without it a stored timestamp under another cell is invisible
    assert res["noStoredRows"] == "TypeError"
    assert res["noStoredRowsAsync"] == "UnknownError:TypeError"
    id_ts = [m["timestamp"] for b in batches for r in b for m in r["messages"]]
    for o in range(n_owners):
        rows = [] if since[o] is None else sdb.conn.execute(
            'SELECT "timestamp" FROM "message" WHERE "userId" = ? AND "timestamp" > ? ORDER BY "timestamp"',
            ("u%d" % o, O.timestamp_to_string(since[o], 0, "0000000000000000"))).fetchall()
        assert [id_ts[int(k)] for k in res["server"]["since"][o]] == [r[0] for r in rows]
    for got, want in zip(res["receive"], rwant):
        if want["ok"]:
            assert got == want
        else:
            assert (got["ok"], got["type"], got["index"]) == (False, want["type"], want["index"])


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists("/usr/include/node/node_api.h"),
                    reason="node / N-API headers not present")
@pytest.mark.parametrize("world", [2, 3])
def test_js_dist_split_loopback(tmp_path, world):
    """js/evolu_evm.js Dist on loopback ranks (worker threads, one GPU):
    applyMessagesSplit (one owner's batch split by cell) and the server's
    hot-owner split (directory, splitHot, route, getMessagesSplit,
    gatherRoots) against the unsharded C restatement."""
    import numpy as np

    from evolu_amd import synth
    from oracle import c_oracle as CO

    _build_addon()
    ts, _, cell = synth.config5(1, 6000, cells_per_owner=120, seed_config=58)
    st_o, flags_o, win_o, js_o = CO.apply(ts, cell.astype(np.uint32), 120)
    strs = [bytes(r[:46]).decode() for r in ts]
    O_ = 24
    sts, sown, _ = synth.config5(O_, 8000, seed_config=72)
    sstr = [bytes(r[:46]).decode() for r in sts]
    rng = np.random.default_rng(9)
    keep = rng.random(len(sts)) < 0.5
    srv, cli = CO.Server(O_, len(sts)), CO.Server(O_, len(sts))
    assert srv.ingest(sts, sown.astype(np.uint32))[0] == 0
    assert cli.ingest(sts[keep], sown[keep].astype(np.uint32))[0] == 0
    node_of = ["%016x" % (0xABCD_0000_0000_0000 + g) for g in range(O_)]
    cases = {"world": world,
             "apply": {"timestamps": strs, "cells": [int(c) for c in cell], "nCells": 120},
             "server": {"userIds": ["user%016d" % g for g in range(O_)], "timestamps": sstr,
                        "owners": [int(o) for o in sown],
                        "clientTrees": [CO.tree_json(sts[keep & (sown == g)]) for g in range(O_)],
                        "nodeIds": node_of}}
    # a batch on a non-empty DB (applyMessages.ts:34-45): batch 1 applied by the oracle, batch 2 split
    from tests import workloads as W

    b1, _ = W.client_batch(71, n=400, n_cells=9)
    b2, _ = W.client_batch(72, n=300, n_cells=12, t0=W.T0 + 1800_000)
    prng = np.random.default_rng(4)
    for k in prng.choice(len(b1), 40, replace=False):  # redeliveries of batch-1 rows
        b2.insert(int(prng.integers(0, len(b2) + 1)), dict(b1[int(k)]))
    pdb = O.ClientDb()
    ptree = O.apply_messages(pdb, {}, b1)
    pcells, pcid = [], {}
    for m in b2:
        c = (m["table"], m["row"], m["column"])
        if c not in pcid:
            pcid[c] = len(pcells)
            pcells.append(c)
    from tests.test_gpu_apply_stored import _stored_rows

    prows = _stored_rows(pdb, b2)
    cases["applyPrior"] = {"timestamps": [m["timestamp"] for m in b2],
                           "cells": [pcid[(m["table"], m["row"], m["column"])] for m in b2], "nCells": len(pcells),
                           "treeJson": O.merkle_tree_to_string(ptree), "prior": [pdb.cell_max(*c) for c in pcells],
                           "stored": [{"timestamp": r[0], "cell": pcid.get((r[1], r[2], r[3]), 0xFFFFFFFF)}
                                      for r in prows]}
    pdec = []
    pwant = O.apply_messages(pdb, ptree, b2, pdec)
    f = tmp_path / "cases.json"
    f.write_text(json.dumps(cases))
    out = subprocess.run(["node", os.path.join(ROOT, "js", "test_dist_split.js"), str(f)], check=True,
                         capture_output=True, text=True, timeout=300).stdout
    res = json.loads(out.strip().splitlines()[-1])
    assert st_o == 0
    assert sum((x["apply"]["flags"] for x in res), []) == [int(v) for v in flags_o]
    for x in res:
        assert x["apply"]["status"] == 0 and x["apply"]["winner"] == [int(v) for v in win_o]
        assert x["apply"]["tree"] == js_o
    assert prows
    pflags = sum((x["applyPrior"]["flags"] for x in res), [])
    for i, (ups, xr, _) in enumerate(pdec):
        assert bool(pflags[i] & 1) == ups and bool(pflags[i] & 2) == xr, i
    plast = {}
    for i, m in enumerate(b2):
        if pdec[i][0]:
            plast[(m["table"], m["row"], m["column"])] = i
    for x in res:
        assert x["applyPrior"]["status"] == 0
        assert x["applyPrior"]["winner"] == [plast.get(c, -1) for c in pcells]
        assert x["applyPrior"]["tree"] == O.merkle_tree_to_string(pwant)
    counts = np.bincount(sown, minlength=O_)
    want_hot = [int(g) for g in np.flatnonzero(counts > 0.25 * len(sts) / world)]
    assert want_hot and all(x["server"]["hot"] == want_hot for x in res)

    def row(i):
        q, k = int(i) // 2 ** 40, int(i) % 2 ** 40
        return res[q]["server"]["rows"][k]

    def expected(g, d):
        if d is None:
            return []
        sync = O.timestamp_to_string(d, 0, "0000000000000000")
        return [s for s in sorted({sstr[i] for i in np.flatnonzero(sown == g)})
                if s > sync and not s.lower().endswith(node_of[g])]

    seen = set()
    for x in res:
        sv = x["server"]
        for j, g in enumerate(sv["glob"]):
            if g < 0:
                continue
            d = srv.diff(cli, g)
            d = None if d == -1 else d
            assert sv["diff"][j] == d
            if j >= sv["hotBase"]:
                got = [row(i) for i in sv["hotIds"][j - sv["hotBase"]]]
            else:
                got = [row(i) for i in sv["ids"][j]]
                seen.add(g)
            assert got == expected(g, d)
        for g in range(O_):
            h = O.merkle_tree_from_string(srv.tree_json(g)).get("hash", 0)
            assert sv["root"][g] == h
    assert seen | set(want_hot) == set(range(O_))
    for x in res:  # Dist.addRouted (evm_dist_ingest) == Server.addMessages over the routed rows
        ri = x["routedIngest"]
        assert ri["status"] == 0 and ri["sameFlags"] and ri["sameTrees"] and ri["n"] == len(x["server"]["rows"])


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists("/usr/include/node/node_api.h"),
                    reason="node / N-API headers not present")
def test_js_sync_server_round_equals_server_db(tmp_path):
    """The whole POST handler through the addon (js/evolu_evm.js SyncServer ->
    evm_sync_round): calls of SyncRequest bodies -- several requests of one
    user in one call (rounds), a body that does not parse, an absent client
    tree -- against the oracle's ServerDb.sync (index.ts:204-251) of the same
    bodies in the same order: the same response bytes, 500 where it throws."""
    import base64

    from tests.test_gpu_wire import REQ, _expected, _requests

    _build_addon()
    bodies = _requests(9, n_users=10, n_req=40)
    rng = random.Random(4)
    node = W.node_id(rng)
    ts = W.hlc_timestamps(rng, 6, [node])
    bodies.insert(7, b"\x0a\x05ab")  # truncated: parseBody throws
    bodies.insert(13, REQ(messages=[dict(timestamp=t, content=b"q") for t in ts], userId="no-tree",
                          nodeId=node).SerializeToString())  # merkleTree absent: JSON.parse("") throws
    calls = [bodies[:17], bodies[17:30], bodies[30:]]
    f = tmp_path / "sync.json"
    f.write_text(json.dumps({"users": 16, "calls": [[base64.b64encode(b).decode() for b in c] for c in calls]}))
    run = subprocess.run(["node", os.path.join(ROOT, "js", "test_sync.js"), str(f)], check=True,
                         capture_output=True, text=True, timeout=300)
    got = json.loads(run.stdout.strip().splitlines()[-1])
    want = _expected(bodies)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        if w in ("500", "ParseBodyError"):
            assert g == 500, i
        else:
            assert g is not None and base64.b64decode(g) == w, i
