// Golden vectors for lenient timestamp strings (TEST INFRASTRUCTURE, run in
// the build container only): what the reference's server does with a
// timestamp that is not canonical.  apps/server/src/index.ts:151-159 stores
// the raw string and XORs insertIntoMerkleTree(timestampFromString(raw));
// timestampFromString (packages/evolu/src/timestamp.ts:50-55) is
//   a = s.split("-"); millis = Date.parse(a.slice(0, 3).join("-")),
//   counter = parseInt(a[3], 16), node = a[4]
// and the tree insert hashes timestampToString of that (timestamp.ts:43-48),
// whose toISOString throws a RangeError on an invalid date (500 for the
// whole request, index.ts:166-169).
//
// Each vector: the raw string and either the canonical string the tree sees
// (timestampToString(timestampFromString(raw))) or "RangeError".  Raw strings
// are ISO-like dates with fields at and past their limits (V8 rolls a day 29-31
// over into the next month and accepts hour 24 at :00:00.000), both cases of
// 'T'/'Z', and lower/upper-case counters.
//
// Usage: node oracle/js/gen_lenient.js > tests/golden/js_lenient.json
"use strict";

let s = 0x2545f4914f6cdd1dn;
const next = () => {
  s = BigInt.asUintN(64, s + 0x9e3779b97f4a7c15n);
  let z = s;
  z = BigInt.asUintN(64, (z ^ (z >> 30n)) * 0xbf58476d1ce4e5b9n);
  z = BigInt.asUintN(64, (z ^ (z >> 27n)) * 0x94d049bb133111ebn);
  return z ^ (z >> 31n);
};
const below = (n) => Number(next() % BigInt(n));
const pick = (a) => a[below(a.length)];
const pad = (v, w) => String(v).padStart(w, "0");

const fromString = (str) => {
  const a = str.split("-");
  return { millis: Date.parse(a.slice(0, 3).join("-")).valueOf(), counter: parseInt(a[3], 16), node: a[4] };
};
const toString = (t) =>
  [new Date(t.millis).toISOString(), t.counter.toString(16).toUpperCase().padStart(4, "0"), t.node].join("-");

const hex = "0123456789abcdef";
const out = [];
for (let k = 0; k < 6000; k++) {
  const y = pick([1970, 1999, 2000, 2023, 2024, 2051, 2100, 2400, 9999, 1904 + below(200)]);
  const mo = pick([0, 1, 2, 2, 2, 4, 6, 9, 11, 12, 13, 1 + below(12)]);
  const d = pick([0, 1, 28, 29, 29, 30, 30, 31, 31, 32, 1 + below(31)]);
  const hh = pick([0, 12, 23, 24, 24, 25, below(24)]);
  const mi = pick([0, 0, 59, 60, below(60)]);
  const ss = pick([0, 0, 59, 60, below(60)]);
  const ms = pick([0, 0, 1, 999, below(1000)]);
  const T = below(8) === 0 ? "t" : "T";
  const Z = below(8) === 0 ? "z" : "Z";
  let ctr = pad(below(65536).toString(16), 4);
  ctr = below(3) === 0 ? ctr : ctr.toUpperCase();
  let node = "";
  for (let i = 0; i < 16; i++) node += hex[below(16)];
  if (below(4) === 0) node = node.toUpperCase();
  const raw = `${pad(y, 4)}-${pad(mo, 2)}-${pad(d, 2)}${T}${pad(hh, 2)}:${pad(mi, 2)}:${pad(ss, 2)}.${pad(ms, 3)}${Z}-${ctr}-${node}`;
  let canonical;
  try {
    canonical = toString(fromString(raw));
  } catch (e) {
    canonical = e instanceof RangeError ? "RangeError" : "Error";
  }
  out.push({ raw, canonical });
}
process.stdout.write(JSON.stringify({ node: process.version, vectors: out }));
