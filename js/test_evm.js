// Runs the JS entry points on cases prepared by tests/test_gpu_napi.py and
// prints the results as JSON (the pytest side compares them with the oracle).
"use strict";
const fs = require("fs");
const { Engine, Server, Dist } = require("./evolu_evm.js");

const cases = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
const eng = new Engine(0);
const out = {};

// merkleTree.test.ts-shaped checks
out.insert = cases.insert.map((c) => eng.insertIntoMerkleTree(c.tree, c.timestamps));
out.diff = cases.diff.map((c) => {
  try {
    return eng.diffMerkleTrees(c.a, c.b);
  } catch (e) {
    return e instanceof RangeError ? "RangeError" : String(e);
  }
});

// applyMessages with an in-memory Database stand-in
function fakeDb(c) {
  const max = new Map(Object.entries(c.cellMax));
  const upserts = {};
  const inserts = [];
  const db = {
    cellMax: (t, r, col) => max.get(JSON.stringify([t, r, col])) || null,
    // SELECT "timestamp", "table", "row", "column" FROM "__message" WHERE "timestamp" IN (...)
    storedRows: (tss) => { const s = new Set(tss); return c.stored.filter((r) => s.has(r.timestamp)); },
    upsert: (t, r, col, v) => { upserts[JSON.stringify([t, r, col])] = v; },
    insertMessage: (m) => inserts.push(m.timestamp),
  };
  return { db, upserts, inserts };
}
out.apply = cases.apply.map((c) => {
  const f = fakeDb(c);
  const tree = eng.applyMessages(f.db, c.tree, c.messages);
  return { tree, upserts: f.upserts, inserts: f.inserts };
});

// server addMessages / getMessages
const srv = new Server(eng, cases.server.nOwners);
out.server = { ins: cases.server.batches.map((b) => srv.addMessages(b)) };
out.server.trees = [];
for (let o = 0; o < cases.server.nOwners; o++) out.server.trees.push(srv.merkleTree(o));
out.server.get = srv.getMessages(cases.server.clientTrees, cases.server.nodeIds);
out.server.since = srv.messagesSince(cases.server.since);
// receive.ts:45-66 clock fold
out.receive = cases.receive.map((c) => eng.receiveMessages(c.clock, c.timestamps, c.now));
srv.close();

// the async entry points: Promise<Either<UnknownError, ...>>, all in flight at once
async function asyncPart() {
  const fs_ = cases.apply.map((c) => fakeDb(c));
  const es = await Promise.all(cases.apply.map((c, i) => eng.applyMessagesAsync(fs_[i].db, c.tree, c.messages)));
  out.applyAsync = es.map((e, i) => (e._tag === "Right" ? { tree: e.right, upserts: fs_[i].upserts, inserts: fs_[i].inserts } : e));
  const s2 = new Server(eng, cases.server.nOwners);
  out.server.insAsync = [];
  for (const b of cases.server.batches) {
    const e = await s2.addMessagesAsync(b);
    out.server.insAsync.push(e._tag === "Right" ? e.right : e);
  }
  out.server.treesAsync = [];
  for (let o = 0; o < cases.server.nOwners; o++) out.server.treesAsync.push(s2.merkleTree(o));
  const g = await s2.getMessagesAsync(cases.server.clientTrees, cases.server.nodeIds);
  out.server.getAsync = g._tag === "Right" ? g.right : g;
  // multi-GPU plumbing at world 1 (RCCL self exchange): rows keep batch order; roots = the trees' hashes
  const d = new Dist(eng, Dist.uniqueId(), 0, 1);
  const rts = cases.server.batches.flat().flatMap((r) => r.messages.map((m) => m.timestamp));
  const rown = cases.server.batches.flat().flatMap((r) => r.messages.map(() => r.owner));
  const routed = d.route(rts, rown, rown.map((o, i) => i * 7));
  out.dist = {
    sameOrder: routed.timestamps.join() === rts.join() && Array.from(routed.owner).join() === rown.join() &&
      Array.from(routed.src).join() === rts.map((_, i) => i).join() &&
      Array.from(routed.aux).join() === rown.map((o, i) => i * 7).join(),
    roots: (({ root, present }) => Array.from(root, (x, i) => (present[i] ? x : null)))(
      d.gatherRoots(s2, cases.server.nOwners)),
    treeHashes: out.server.treesAsync.map((t) => { const h = JSON.parse(t).hash; return h === undefined ? null : h; }),
  };
  d.close();
  // an owner id beyond the store's owner count: the engine refuses the batch -> Left
  const addon = require("./evm_napi.node");
  out.leftOnError = await addon.serverIngestAsync(eng.ctx, s2.store, new Uint8Array(48), 48, new Uint32Array([99]), 0);
  s2.close();
  // an adapter without storedRows is refused, not run blind (applyMessages.ts:42-45)
  const c0 = cases.apply[0];
  const noStored = Object.assign({}, fakeDb(c0).db);
  delete noStored.storedRows;
  try {
    eng.applyMessages(noStored, c0.tree, c0.messages);
    out.noStoredRows = "accepted";
  } catch (e) {
    out.noStoredRows = e instanceof TypeError ? "TypeError" : String(e);
  }
  const e2 = await eng.applyMessagesAsync(noStored, c0.tree, c0.messages);
  out.noStoredRowsAsync = e2._tag === "Left" ? e2.left.type + ":" + e2.left.error.constructor.name : "Right";
}
asyncPart().then(() => {
  eng.close();
  process.stdout.write("\n" + JSON.stringify(out) + "\n");
}, (e) => {
  process.stderr.write(String(e && e.stack) + "\n");
  process.exit(1);
});
