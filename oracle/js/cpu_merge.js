// cpu_merge.js -- CPU BASELINE and TEST INFRASTRUCTURE (never the product).
//
// The reference merge restated in plain JavaScript and run by node on the
// GPU box's host cores (bench.py cpu_baseline, "kind": "port", 1 thread, as
// the reference's single DB worker):
//   timestampFromString / timestampToString ... packages/evolu/src/timestamp.ts:43-55
//   timestampToHash ........................... timestamp.ts:87-88 (murmurhash@2.0.1 v3 = MurmurHash3_x86_32;
//                                               here Debian's imurmurhash 0.1.4, the same function)
//   insertIntoMerkleTree ...................... merkleTree.ts:8-50 (persistent object spreads)
//   applyMessages ............................. applyMessages.ts:78-124, the three SQL statements
//                                               replaced by Maps with the same results: the cell's max
//                                               timestamp (:34-40), the __message PRIMARY KEY (:41-45),
//                                               the user-table upsert (:94-101).
// Without SQLite this is FASTER than the reference (no wa-sqlite, no IndexedDB).
//
// Usage: node cpu_merge.js TS_FILE CELL_FILE N BUDGET_SECONDS [--check]
//   TS_FILE: N rows of 48 bytes (46-byte timestamp + 2 pad); CELL_FILE: N uint32 LE cell ids.
//   Applies messages 0.. in batch order until all N are done or the budget is spent.
//   Prints {"done", "seconds", "rate", "root"}; --check adds "flags" (1 = upsert, 2 = Merkle XOR)
//   and "tree" (JSON.stringify of the final MerkleTree).
"use strict";
const fs = require("fs");
const MurmurHash3 = require("/usr/share/nodejs/imurmurhash");

function timestampFromString(s) {
  const a = s.split("-");
  return { millis: Date.parse(a.slice(0, 3).join("-")), counter: parseInt(a[3], 16), node: a[4] };
}
function timestampToString(t) {
  return [new Date(t.millis).toISOString(), t.counter.toString(16).toUpperCase().padStart(4, "0"), t.node].join("-");
}
function timestampToHash(t) {
  return MurmurHash3(timestampToString(t)).result();
}
function insertKey(tree, key, hash) {
  if (key.length === 0) return tree;
  const c = key[0];
  const n = tree[c] || {};
  return { ...tree, [c]: { ...n, ...insertKey(n, key.slice(1), hash), hash: n.hash ^ hash } };
}
function insertIntoMerkleTree(t, tree) {
  const key = Number((t.millis / 1000 / 60) | 0).toString(3);
  const hash = timestampToHash(t);
  return insertKey({ ...tree, hash: tree.hash ^ hash }, key, hash);
}

function main() {
  const [tsFile, cellFile, nArg, budgetArg] = process.argv.slice(2);
  const check = process.argv.includes("--check");
  const n = Number(nArg);
  const budget = Number(budgetArg);
  const tsBuf = fs.readFileSync(tsFile);
  const cellBuf = fs.readFileSync(cellFile);
  const cells = new Uint32Array(cellBuf.buffer, cellBuf.byteOffset, n);
  const cellMax = new Map();
  const messagePk = new Set();
  const userCell = new Map();
  const flags = check ? [] : null;
  let tree = {};
  const t0 = process.hrtime.bigint();
  let i = 0;
  for (; i < n; i++) {
    if ((i & 255) === 0 && i > 0 && Number(process.hrtime.bigint() - t0) / 1e9 > budget) break;
    const ts = tsBuf.toString("latin1", 48 * i, 48 * i + 46);
    const cell = cells[i];
    const t = cellMax.get(cell);
    const ups = t === undefined || t < ts; // applyMessages.ts:93
    if (ups) userCell.set(cell, i);
    const xor = t === undefined || t !== ts; // :105
    if (xor) {
      if (!messagePk.has(ts)) {
        // INSERT ... ON CONFLICT DO NOTHING took: the row joins the cell
        messagePk.add(ts);
        if (t === undefined || ts > t) cellMax.set(cell, ts);
      }
      tree = insertIntoMerkleTree(timestampFromString(ts), tree); // :114-119
    }
    if (check) flags.push((ups ? 1 : 0) | (xor ? 2 : 0));
  }
  const seconds = Number(process.hrtime.bigint() - t0) / 1e9;
  const out = { done: i, seconds, rate: i / seconds, root: tree.hash === undefined ? null : tree.hash };
  if (check) {
    out.flags = flags;
    out.tree = JSON.stringify(tree);
  }
  process.stdout.write(JSON.stringify(out) + "\n");
}

main();
