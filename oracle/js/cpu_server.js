// cpu_server.js -- CPU BASELINE and TEST INFRASTRUCTURE (never the product).
//
// The sync server's hot path (apps/server/src/index.ts) restated in plain
// JavaScript, run by node on the GPU box's host cores (bench.py, config 3):
//   per SyncRequest (one owner, its messages in batch order), sync = (:204-216)
//     getMerkleTree ...... :121-136  JSON.parse of the owner's stored tree
//     addMessages ........ :138-171  INSERT OR IGNORE (timestamp, userId) -> a Set;
//                                    insertIntoMerkleTree iff inserted; JSON.stringify
//                                    of the tree back into the "merkleTree" table
//     getMessages ........ :173-202  diffMerkleTrees(tree, JSON.parse(request tree)),
//                                    then the owner's rows with timestamp > syncTs(diff)
//                                    AND NOT LIKE '%' || nodeId, ORDER BY timestamp
//   timestamp.ts:43-55,87-88 / merkleTree.ts:8-91 as in cpu_merge.js (murmur3 =
//   Debian's imurmurhash 0.1.4, the same function as murmurhash@2.0.1).
// SQLite is replaced by Maps/arrays (FASTER than better-sqlite3 would be).
//
// Usage: node cpu_server.js TS_FILE OWNER_FILE N BUDGET_SECONDS THREADS
//   TS_FILE: N rows of 48 bytes; OWNER_FILE: N uint32 owner ids; requests are the
//   runs of one owner in batch order.  The client tree of an owner is built
//   (untimed) from its first 90 % of messages by timestamp, as bench.py's GPU
//   step does.  THREADS > 1: worker_threads, owners split owner % THREADS.
//   Prints {"done", "requests", "seconds", "rate", "threads"}.
"use strict";
const fs = require("fs");
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");
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
const getKeys = (tree) => Object.keys(tree).filter((x) => x !== "hash");
function keyToTimestamp(key) {
  const fullkey = key + "0".repeat(16 - key.length);
  return parseInt(fullkey, 3) * 1000 * 60;
}
function diffMerkleTrees(tree1, tree2) {
  if (tree1.hash === tree2.hash) return null;
  let node1 = tree1;
  let node2 = tree2;
  let k = "";
  for (;;) {
    const keys = Array.from(new Set([...getKeys(node1), ...getKeys(node2)])).sort();
    const diffkey = keys.find((key) => (node1[key] || {}).hash !== (node2[key] || {}).hash);
    if (!diffkey) return keyToTimestamp(k);
    k += diffkey;
    node1 = node1[diffkey] || {};
    node2 = node2[diffkey] || {};
  }
}
const NODE = "0123456789abcdef"; // the requester's nodeId (bench.py's GPU step uses the same)

// the rows of the owners this thread serves (owner % threads === me), in batch order
function load(tsFile, ownerFile, n, threads, me) {
  const tsBuf = fs.readFileSync(tsFile);
  const ob = fs.readFileSync(ownerFile);
  const all = new Uint32Array(ob.buffer, ob.byteOffset, n);
  const ts = [];
  const own = [];
  for (let i = 0; i < n; i++) {
    if (all[i] % threads !== me) continue;
    ts.push(tsBuf.toString("latin1", 48 * i, 48 * i + 46));
    own.push(all[i]);
  }
  return { ts, owner: Uint32Array.from(own) };
}

// requests (owner runs) of the owners this thread serves; an owner's client
// tree (the request's merkleTree JSON) is built on its first request, untimed
function prepare(d, threads, me) {
  const reqs = [];
  const byOwner = new Map();
  for (let i = 0; i < d.ts.length; ) {
    const o = d.owner[i];
    let j = i + 1;
    while (j < d.ts.length && d.owner[j] === o) j++;
    if (o % threads === me) {
      reqs.push([o, i, j]);
      if (!byOwner.has(o)) byOwner.set(o, []);
      for (let k = i; k < j; k++) byOwner.get(o).push(d.ts[k]);
    }
    i = j;
  }
  const client = new Map();
  const clientTree = (o) => {
    if (!client.has(o)) {
      const s = byOwner.get(o).slice().sort();
      let tree = {};
      for (let k = 0; k < Math.floor(0.9 * s.length); k++) tree = insertIntoMerkleTree(timestampFromString(s[k]), tree);
      client.set(o, JSON.stringify(tree));
    }
    return client.get(o);
  };
  return { reqs, clientTree };
}

function serve(d, p, budget) {
  const stored = new Set(); // "message" PRIMARY KEY(timestamp, userId)
  const rows = new Map(); // owner -> its timestamps
  const trees = new Map(); // "merkleTree" table: owner -> JSON
  let done = 0;
  let nreq = 0;
  let selected = 0;
  let prep = 0n; // client-tree building: the request's input, not server work
  const t0 = process.hrtime.bigint();
  for (const [o, a, b] of p.reqs) {
    if (nreq > 0 && Number(process.hrtime.bigint() - t0 - prep) / 1e9 > budget) break;
    const c0 = process.hrtime.bigint();
    const clientJson = p.clientTree(o);
    prep += process.hrtime.bigint() - c0;
    let tree = trees.has(o) ? JSON.parse(trees.get(o)) : {}; // getMerkleTree
    if (!rows.has(o)) rows.set(o, []);
    const mine = rows.get(o);
    for (let i = a; i < b; i++) {
      const key = d.ts[i] + "|" + o;
      if (!stored.has(key)) { // INSERT OR IGNORE ... changes === 1
        stored.add(key);
        mine.push(d.ts[i]);
        tree = insertIntoMerkleTree(timestampFromString(d.ts[i]), tree);
      }
    }
    trees.set(o, JSON.stringify(tree)); // INSERT OR REPLACE INTO "merkleTree"
    const diff = diffMerkleTrees(tree, JSON.parse(clientJson)); // getMessages
    if (diff !== null) {
      const since = timestampToString({ millis: diff, counter: 0, node: "0000000000000000" });
      const sel = mine.filter((t) => t > since && !t.toLowerCase().endsWith(NODE)).sort();
      selected += sel.length;
    }
    done += b - a;
    nreq++;
  }
  const seconds = Number(process.hrtime.bigint() - t0 - prep) / 1e9;
  return { done, requests: nreq, seconds, selected };
}

if (isMainThread) {
  const [tsFile, ownerFile, nArg, budgetArg, thrArg] = process.argv.slice(2);
  const n = Number(nArg);
  const budget = Number(budgetArg);
  const threads = Math.max(1, Number(thrArg || 1));
  if (threads === 1) {
    const d = load(tsFile, ownerFile, n, 1, 0);
    const r = serve(d, prepare(d, 1, 0), budget);
    process.stdout.write(JSON.stringify({ ...r, rate: r.done / r.seconds, threads: 1 }) + "\n");
  } else {
    // every worker loads and prepares, then all start serving together
    const sab = new SharedArrayBuffer(4);
    const gate = new Int32Array(sab);
    const res = [];
    let ready = 0;
    const ws = [];
    for (let w = 0; w < threads; w++) {
      const wk = new Worker(__filename, { workerData: { tsFile, ownerFile, n, budget, threads, me: w, sab } });
      wk.on("message", (m) => {
        if (m === "ready") {
          if (++ready === threads) {
            Atomics.store(gate, 0, 1);
            Atomics.notify(gate, 0);
          }
          return;
        }
        res.push(m);
        if (res.length === threads) {
          const done = res.reduce((s, r) => s + r.done, 0);
          const seconds = Math.max(...res.map((r) => r.seconds));
          const requests = res.reduce((s, r) => s + r.requests, 0);
          process.stdout.write(JSON.stringify({ done, requests, seconds, rate: done / seconds, threads }) + "\n");
        }
      });
      ws.push(wk);
    }
  }
} else {
  const w = workerData;
  const d = load(w.tsFile, w.ownerFile, w.n, w.threads, w.me);
  const p = prepare(d, w.threads, w.me);
  const gate = new Int32Array(w.sab);
  parentPort.postMessage("ready");
  Atomics.wait(gate, 0, 0);
  parentPort.postMessage(serve(d, p, w.budget));
}
