// Loopback ranks through the JS Dist (worker threads, one GPU): the hot-owner
// split of a server round and one owner's applyMessages split by cell, on the
// cases tests/test_gpu_napi.py prepares; prints every rank's results as JSON
// (the pytest side compares them with the unsharded C restatement).
"use strict";
const fs = require("fs");
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");

if (isMainThread) {
  const cases = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
  const { Dist } = require("./evolu_evm.js");
  const world = cases.world;
  const hub = Dist.loopbackHub(world);
  const results = new Array(world);
  let left = world;
  let failed = false;
  for (let r = 0; r < world; r++) {
    const w = new Worker(__filename, { workerData: { hub, rank: r, world, cases } });
    w.on("message", (m) => { results[r] = m; });
    w.on("error", (e) => {
      failed = true;
      process.stderr.write("rank " + r + ": " + String(e && e.stack) + "\n");
      Dist.abortHub(hub); // the other ranks' collectives return instead of waiting
    });
    w.on("exit", () => {
      if (--left === 0) {
        Dist.freeHub(hub);
        if (failed) process.exit(1);
        process.stdout.write("\n" + JSON.stringify(results) + "\n");
      }
    });
  }
} else {
  const { Engine, Server, Dist } = require("./evolu_evm.js");
  const { hub, rank, world, cases } = workerData;
  const eng = new Engine(0);
  const d = new Dist(eng, { hub }, rank, world);
  const out = {};
  // client: one owner's batch split by cell
  const a = cases.apply;
  const cut = (n) => [Math.floor((n * rank) / world), Math.floor((n * (rank + 1)) / world)];
  {
    const [lo, hi] = cut(a.timestamps.length);
    const r = d.applyMessagesSplit(a.timestamps.slice(lo, hi), a.cells.slice(lo, hi), a.nCells);
    out.apply = { status: r.status, flags: Array.from(r.flags), winner: r.winner, tree: r.tree };
  }
  // the same on a non-empty DB: the cells' maxima and the stored rows of batch 2's timestamps
  if (cases.applyPrior) {
    const b = cases.applyPrior;
    const [lo, hi] = cut(b.timestamps.length);
    const r = d.applyMessagesSplit(b.timestamps.slice(lo, hi), b.cells.slice(lo, hi), b.nCells, b.treeJson,
      { prior: b.prior, stored: b.stored });
    out.applyPrior = { status: r.status, flags: Array.from(r.flags), winner: r.winner, tree: r.tree };
  }
  // server: owners by murmur3(userId) % world, the hot ones split over every rank
  const s = cases.server;
  {
    const [lo, hi] = cut(s.timestamps.length);
    const dir = d.directory(s.userIds);
    const hot = d.splitHot(s.owners.slice(lo, hi), s.userIds.length, 0.25);
    const routed = d.route(s.timestamps.slice(lo, hi), s.owners.slice(lo, hi));
    const srv = new Server(eng, d.nLocal);
    srv.nextId = rank * 2 ** 40;
    const ins = srv.addMessages(routed.timestamps.map((t, i) => ({ owner: routed.owner[i], messages: [{ timestamp: t }] })));
    // the same rows from the received records themselves (evm_dist_ingest)
    const srv2 = new Server(eng, d.nLocal);
    const r2 = d.addRouted(srv2, rank * 2 ** 40);
    let sameTrees = true;
    for (let j = 0; j < d.nLocal; j++) sameTrees = sameTrees && srv.merkleTree(j) === srv2.merkleTree(j);
    out.routedIngest = { status: r2.status, sameFlags: JSON.stringify(r2.inserted) === JSON.stringify(ins), sameTrees,
      n: r2.inserted.length };
    srv2.close();
    // global owner of every local id (-1: unused)
    const glob = new Array(d.nLocal).fill(-1);
    for (let g = 0; g < s.userIds.length; g++) if (dir.dest[g] === rank) glob[dir.local[g]] = g;
    for (let j = 0; j < glob.length; j++) if (glob[j] >= 0 && hot.includes(glob[j])) glob[j] = -1;
    hot.forEach((g, h) => { glob[d.hotBase + h] = g; });
    const trees = glob.map((g) => (g >= 0 ? s.clientTrees[g] : "{}"));
    const nodes = glob.map((g) => (g >= 0 ? s.nodeIds[g] : "0000000000000000"));
    const got = d.getMessagesSplit(srv, trees, nodes);
    const roots = d.gatherRoots(srv, s.userIds.length);
    out.server = { hot: Array.from(hot), hotBase: d.hotBase, glob, rows: routed.timestamps, diff: got.diff,
      ids: got.ids, hotIds: got.hotIds, root: Array.from(roots.root), present: Array.from(roots.present) };
    srv.close();
  }
  d.close();
  eng.close();
  parentPort.postMessage(out);
}
