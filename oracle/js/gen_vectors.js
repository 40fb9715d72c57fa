// Golden-vector generator (TEST INFRASTRUCTURE, run in the build container
// only).  It pins the Python oracle's emulation of JavaScript semantics with
// the real thing: V8's Date#toISOString / Date.parse, ToInt32 on `|0` and `^`,
// Number#toString(3), parseInt(s, 3), JSON.stringify key order -- and pins
// murmur3 with an independent implementation (Debian imurmurhash 0.1.4,
// MurmurHash3_x86_32, the algorithm of npm murmurhash@2.0.1 that the
// reference calls at packages/evolu/src/timestamp.ts:87-88).
//
// Usage: node oracle/js/gen_vectors.js > tests/golden/js_vectors.json
"use strict";
const MurmurHash3 = require("/usr/share/nodejs/imurmurhash");

// splitmix64 over BigInt, identical to tests' Python twin.
function makeRng(seed) {
  let s = BigInt.asUintN(64, BigInt(seed));
  return function next() {
    s = BigInt.asUintN(64, s + 0x9e3779b97f4a7c15n);
    let z = s;
    z = BigInt.asUintN(64, (z ^ (z >> 30n)) * 0xbf58476d1ce4e5b9n);
    z = BigInt.asUintN(64, (z ^ (z >> 27n)) * 0x94d049bb133111ebn);
    return z ^ (z >> 31n);
  };
}
const rng = makeRng(0xe7010000);
const below = (n) => Number(rng() % BigInt(n));

const hex = "0123456789abcdef";
function nodeId(upperProb) {
  let s = "";
  for (let i = 0; i < 16; i++) {
    let c = hex[below(16)];
    if (below(100) < upperProb) c = c.toUpperCase();
    s += c;
  }
  return s;
}
// The string form of timestamp.ts:43-48 (restated).
const tsString = (millis, counter, node) =>
  [new Date(millis).toISOString(), counter.toString(16).toUpperCase().padStart(4, "0"), node].join("-");
const mm3 = (s) => MurmurHash3(s).result();
const minuteKey = (millis) => Number((millis / 1000 / 60) | 0).toString(3);

// --- 1. timestamp strings + hashes over eras that stress the date math.
const spans = [
  [0, 86400000 * 3],
  [860934420000 - 86400000, 860934420000 + 86400000], // 16-digit key boundary (1997)
  [1704067200000, 1704067200000 + 30 * 86400000], // bench window (2024)
  [951782400000 - 86400000 * 2, 951782400000 + 86400000 * 2], // 2000-02-29
  [2582803260000 - 86400000, 2582803260000 + 86400000], // 17-digit key boundary (2051)
  [0, 253402300799999], // whole 4-digit-year range
];
const timestamps = [];
for (const [lo, hi] of spans) {
  for (let i = 0; i < 400; i++) {
    const millis = lo + below(hi - lo);
    const counter = below(4) === 0 ? 65535 - below(3) : below(65536);
    const node = nodeId(i % 5 === 0 ? 30 : 0);
    const s = tsString(millis, counter, node);
    timestamps.push({ s, millis, counter, node, hash: mm3(s), key: minuteKey(millis) });
  }
}
// Minute boundaries.
for (const k of [1, 2, 3, 8, 9, 26, 27, 14348906, 14348907, 43046720, 43046721]) {
  for (const d of [-1, 0, 1]) {
    const millis = k * 60000 + d;
    if (millis < 0) continue;
    const s = tsString(millis, 0, "0000000000000000");
    timestamps.push({ s, millis, counter: 0, node: "0000000000000000", hash: mm3(s), key: minuteKey(millis) });
  }
}

// --- 2. Date.parse behaviour on lenient forms (the engine flags these).
const lenient = [
  "2022-02-30T00:00:00.000Z",
  "2022-02-29T00:00:00.000Z",
  "2024-02-29T24:00:00.000Z",
  "2024-13-01T00:00:00.000Z",
  "2024-01-01T00:00:60.000Z",
  "2024-01-01T00:00:00.000Z",
].map((s) => ({ s, parsed: Date.parse(s) }));

// --- 3. Small tries: literal restatement of a persistent base-3 XOR trie.
function insertPath(tree, key, h) {
  if (key.length === 0) return tree;
  const c = key[0];
  const n = tree[c] || {};
  return { ...tree, [c]: { ...n, ...insertPath(n, key.slice(1), h), hash: n.hash ^ h } };
}
function insertTs(tree, millis, counter, node) {
  const h = mm3(tsString(millis, counter, node));
  return insertPath({ ...tree, hash: tree.hash ^ h }, minuteKey(millis), h);
}
const trees = [];
for (let t = 0; t < 40; t++) {
  let tree = {};
  const ops = [];
  const n = 1 + below(t < 10 ? 4 : 40);
  const base = t % 3 === 0 ? below(5) * 60000 : 1704067200000 + below(3) * 86400000;
  for (let i = 0; i < n; i++) {
    const millis = base + below(t % 2 ? 600000 : 86400000);
    const counter = below(3);
    const node = "000000000000000" + below(3);
    ops.push([millis, counter, node]);
    tree = insertTs(tree, millis, counter, node);
    if (below(4) === 0) {
      // double insert: XOR cancels, node stays present with hash 0
      ops.push([millis, counter, node]);
      tree = insertTs(tree, millis, counter, node);
    }
  }
  trees.push({ ops, json: JSON.stringify(tree) });
}

// --- 4. parseInt(padEnd(16,'0'),3) * 60000 for keys of several lengths.
const keyMillis = ["", "0", "1", "2", "10", "12", "1211121022121110", "2222222222222222"].map((k) => ({
  k,
  millis: parseInt(k + "0".repeat(16 - k.length), 3) * 1000 * 60,
}));

process.stdout.write(JSON.stringify({ timestamps, lenient, trees, keyMillis }));
