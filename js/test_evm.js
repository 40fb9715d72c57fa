// Runs the JS entry points on cases prepared by tests/test_gpu_napi.py and
// prints the results as JSON (the pytest side compares them with the oracle).
"use strict";
const fs = require("fs");
const { Engine, Server } = require("./evolu_evm.js");

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
out.apply = cases.apply.map((c) => {
  const max = new Map(Object.entries(c.cellMax));
  const upserts = {};
  const inserts = [];
  const db = {
    cellMax: (t, r, col) => max.get(JSON.stringify([t, r, col])) || null,
    upsert: (t, r, col, v) => { upserts[JSON.stringify([t, r, col])] = v; },
    insertMessage: (m) => inserts.push(m.timestamp),
  };
  const tree = eng.applyMessages(db, c.tree, c.messages);
  return { tree, upserts, inserts };
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
eng.close();
process.stdout.write(JSON.stringify(out));
