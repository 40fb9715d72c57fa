// Runs SyncServer.sync (the POST handler of apps/server/src/index.ts over one
// native round per call) on bodies prepared by tests/test_gpu_napi.py and
// prints per body the response (base64), 500, or null, as JSON.
"use strict";
const fs = require("fs");
const { Engine, SyncServer } = require("./evolu_evm.js");

const cases = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
const eng = new Engine(0);
const srv = new SyncServer(eng, cases.users);
const out = [];
for (const call of cases.calls) {
  const res = srv.sync(call.map((b) => Buffer.from(b, "base64")));
  res.forEach((r) => out.push(r === null || r === 500 ? r : Buffer.from(r).toString("base64")));
}
srv.close();
eng.close();
console.log(JSON.stringify(out));
