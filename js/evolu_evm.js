// evolu_evm.js -- reference-shaped JS entry points over the N-API addon.
//
// Drop-in for the hot path of packages/evolu and apps/server (reference @
// 2025-01-31): the same inputs and outputs as the reference functions, batched.
//   insertIntoMerkleTree ... merkleTree.ts:31-50   (many timestamps at once)
//   diffMerkleTrees ........ merkleTree.ts:63-91
//   applyMessages .......... applyMessages.ts:26-131 (decisions on the GPU; the
//                            SQL writes stay with the caller's Database)
//   Server#addMessages ..... apps/server/src/index.ts:138-171
//   Server#getMessages ..... apps/server/src/index.ts:173-202
//   Engine#receiveMessages . receive.ts:45-66 (the HLC fold over a batch)
//   Engine#messagesSince ... receive.ts:118-124 (resend range, via a Server store)
//   SyncRequest / SyncResponse fromBinary / toBinary .. protobuf.ts:60-171
// Trees cross this boundary as MerkleTree JSON (types.ts:80-84), the format
// the reference persists and sends.  Results the engine does not model
// (non-canonical timestamps, a timestamp in two cells) return `null` so the
// caller runs the reference code for that batch.
"use strict";
const addon = require("./evm_napi.node");

const STRIDE = 48;
const EVM_OK = 0;
const EVM_ENONCANON = 2;
const EVM_ECOLLISION = 3;
const MSG_UPS = 1;
const MSG_XOR = 2;
const MSG_INS = 4;

function encodeTimestamps(strings) {
  const out = new Uint8Array(strings.length * STRIDE);
  strings.forEach((s, i) => {
    const o = i * STRIDE;
    if (s.length !== 46) {
      out.fill(0xff, o, o + 46); // cannot be canonical: the engine flags it
      return;
    }
    for (let k = 0; k < 46; k++) {
      const c = s.charCodeAt(k);
      out[o + k] = c < 128 ? c : 0xff;
    }
  });
  return out;
}

class Engine {
  constructor(device = 0) {
    this.ctx = addon.create(device);
  }
  close() {
    if (this.ctx) addon.destroy(this.ctx);
    this.ctx = null;
  }
  _tree(json) {
    return addon.treeFromJson(this.ctx, [json]);
  }
  _json(tree) {
    const s = addon.treeToJson(this.ctx, tree, 0);
    addon.treeFree(this.ctx, tree);
    return s;
  }

  // merkleTree.ts:31-50, for a list of timestamps (order-independent)
  insertIntoMerkleTree(treeJson, timestamps) {
    const t = this._tree(treeJson);
    const out = addon.insert(this.ctx, t, encodeTimestamps(timestamps), STRIDE, null);
    addon.treeFree(this.ctx, t);
    return this._json(out);
  }

  // merkleTree.ts:63-91 -> null (option.none) | millis; throws RangeError like keyToTimestamp
  diffMerkleTrees(aJson, bJson) {
    const a = this._tree(aJson);
    const b = this._tree(bJson);
    const d = addon.diff(this.ctx, a, b)[0];
    addon.treeFree(this.ctx, a);
    addon.treeFree(this.ctx, b);
    if (d === -2) throw new RangeError("Invalid count value");
    return d === -1 ? null : d;
  }

  // applyMessages.ts:26-131.  db: { cellMax(table, row, column) -> string|null,
  // storedRows(timestamps) -> [{timestamp, table, row, column}] (required: the
  // "__message" rows holding one of the batch's timestamps, PK "timestamp",
  // initDbModel.ts:44), upsert(table, row, column, value), insertMessage(message) }.
  // Returns the new MerkleTree JSON, or null when the batch needs the reference path
  // (a non-canonical timestamp, or one timestamp under two cells in the batch or
  // against a stored row: the reference then ignores that INSERT, :104-119).
  // An adapter without storedRows is refused (TypeError; Left in the async form):
  // the engine could not see a stored timestamp under another cell and would
  // return other upserts and XORs than the reference, with no error.
  applyMessages(db, treeJson, messages) {
    const args = this._applyArgs(db, treeJson, messages);
    const r = addon.applyBatch(this.ctx, ...args);
    addon.treeFree(this.ctx, args[0]);
    return this._applyWrites(db, messages, r);
  }

  // the same, the GPU work on a libuv worker thread: Promise<Either<UnknownError, json|null>>
  // (the reference's Effect-returning shape, types.ts:317-399)
  async applyMessagesAsync(db, treeJson, messages) {
    let args;
    try {
      args = this._applyArgs(db, treeJson, messages);
    } catch (error) {
      return { _tag: "Left", left: { type: "UnknownError", error } };
    }
    const e = await addon.applyBatchAsync(this.ctx, ...args);
    addon.treeFree(this.ctx, args[0]);
    if (e._tag === "Left") return e;
    return { _tag: "Right", right: this._applyWrites(db, messages, e.right) };
  }

  _applyArgs(db, treeJson, messages) {
    if (typeof db.storedRows !== "function")
      throw new TypeError("applyMessages: the db adapter must provide storedRows(timestamps) " +
        "(the __message rows of the batch's timestamps, applyMessages.ts:42-45)");
    const ids = new Map();
    const cells = [];
    const cell = new Uint32Array(messages.length);
    const key = (m) => JSON.stringify([m.table, m.row, m.column]);
    messages.forEach((m, i) => {
      const k = key(m);
      let c = ids.get(k);
      if (c === undefined) {
        c = cells.length;
        ids.set(k, c);
        cells.push(m);
      }
      cell[i] = c;
    });
    // the cells' current maxima: SELECT "timestamp" ... ORDER BY "timestamp" DESC LIMIT 1 (applyMessages.ts:34-40)
    const prior = cells.map((m) => db.cellMax(m.table, m.row, m.column));
    const priorPresent = Uint8Array.from(prior.map((p) => (p == null ? 0 : 1)));
    let storedTs = null;
    let storedCell = null;
    const rows = db.storedRows(Array.from(new Set(messages.map((m) => m.timestamp))));
    if (rows.length) {
      storedTs = encodeTimestamps(rows.map((r) => r.timestamp));
      // a row of a cell the batch does not touch: any id >= the cell count
      storedCell = Uint32Array.from(rows, (r) => { const c = ids.get(key(r)); return c === undefined ? 0xffffffff : c; });
    }
    return [this._tree(treeJson), encodeTimestamps(messages.map((m) => m.timestamp)), STRIDE, cell, cells.length,
      encodeTimestamps(prior.map((p) => (p == null ? "" : p))), priorPresent, storedTs, storedCell];
  }

  _applyWrites(db, messages, r) {
    if (r.status === EVM_ENONCANON || r.status === EVM_ECOLLISION) return null;
    // the same statements the reference runs, in batch order: the final upsert
    // of every cell, and INSERT ... ON CONFLICT DO NOTHING of every XOR message
    r.winner.forEach((i) => {
      if (i >= 0) db.upsert(messages[i].table, messages[i].row, messages[i].column, messages[i].value);
    });
    messages.forEach((m, i) => {
      if (r.flags[i] & MSG_XOR) db.insertMessage(m);
    });
    return this._json(r.tree);
  }
}

Engine.prototype.receiveMessages = function (clock, timestamps, now, maxDrift = 60000) {
  // receive.ts:45-66: fold receiveTimestamp over the batch; clock = {millis, counter, node}.
  // -> { ok: true, clock } | { ok: false, type, index, next }
  const r = addon.receiveFold(this.ctx, encodeTimestamps(timestamps), STRIDE, clock.millis, clock.counter, clock.node,
    now, maxDrift);
  if (r.error === 0) return { ok: true, clock: { millis: r.millis, counter: r.counter, node: clock.node } };
  const type = ["", "TimestampDriftError", "TimestampDuplicateNodeError", "TimestampCounterOverflowError"][r.error];
  return { ok: false, type, index: r.index, next: r.next };
};

// protobuf.ts:60-171 (protobuf-ts MessageType shape): fromBinary / toBinary
const PB_REQUEST = 1;
const PB_RESPONSE = 2;
function pbMessages(r, body) {
  const dec = new TextDecoder();
  const out = [];
  for (let i = 0; i < r.tsLen.length; i++) {
    out.push({
      timestamp: dec.decode(body.subarray(r.tsOff[i], r.tsOff[i] + r.tsLen[i])),
      content: r.content.slice(r.contentOff[i], r.contentOff[i + 1]),
    });
  }
  return out;
}
function pbEncode(kind, m) {
  const msgs = m.messages || [];
  const ts = encodeTimestamps(msgs.map((x) => x.timestamp));
  if (msgs.some((x) => x.timestamp.length !== 46)) throw new RangeError("timestamps must be 46 chars");
  const off = new Float64Array(msgs.length + 1);
  msgs.forEach((x, i) => { off[i + 1] = off[i] + x.content.length; });
  const content = new Uint8Array(off[msgs.length]);
  msgs.forEach((x, i) => content.set(x.content, off[i]));
  return addon.pbEncode(kind, ts, content, off, m.userId || "", m.nodeId || "", m.merkleTree || "");
}
const SyncRequest = {
  fromBinary(body) {
    const r = addon.pbDecode(PB_REQUEST, body);
    return { messages: pbMessages(r, body), userId: r.userId, nodeId: r.nodeId, merkleTree: r.merkleTree };
  },
  toBinary(m) { return pbEncode(PB_REQUEST, m); },
};
const SyncResponse = {
  fromBinary(body) {
    const r = addon.pbDecode(PB_RESPONSE, body);
    return { messages: pbMessages(r, body), merkleTree: r.merkleTree };
  },
  toBinary(m) { return pbEncode(PB_RESPONSE, m); },
};

// apps/server/src/index.ts: one store for many owners (userIds)
class Server {
  constructor(engine, nOwners) {
    this.engine = engine;
    this.store = addon.storeNew(engine.ctx, nOwners);
    this.nOwners = nOwners;
    this.nextId = 0;
  }
  close() {
    addon.storeFree(this.engine.ctx, this.store);
  }
  // addMessages for a batch of requests: [{owner, messages: [{timestamp}]}] -> per message inserted flags
  addMessages(requests) {
    const [ts, own] = this._ingestArgs(requests);
    const r = addon.serverIngest(this.engine.ctx, this.store, ts, STRIDE, own, this.nextId);
    return this._ingested(r, own.length);
  }
  // -> Promise<Either<UnknownError, flags|null>>; the id range is reserved before the await
  async addMessagesAsync(requests) {
    const [ts, own] = this._ingestArgs(requests);
    const base = this.nextId;
    this.nextId += own.length;
    const e = await addon.serverIngestAsync(this.engine.ctx, this.store, ts, STRIDE, own, base);
    if (e._tag === "Left") return e;
    return { _tag: "Right", right: e.right.status !== EVM_OK ? null : Array.from(e.right.flags, (f) => (f & MSG_INS) !== 0) };
  }
  _ingestArgs(requests) {
    const ts = [];
    const own = [];
    requests.forEach((r) => r.messages.forEach((m) => { ts.push(m.timestamp); own.push(r.owner); }));
    return [encodeTimestamps(ts), Uint32Array.from(own)];
  }
  _ingested(r, n) {
    if (r.status !== EVM_OK) return null;
    this.nextId += n;
    return Array.from(r.flags, (f) => (f & MSG_INS) !== 0);
  }
  merkleTree(owner) {
    return addon.treeToJson(this.engine.ctx, addon.storeTree(this.store), owner);
  }
  // getMessages for every owner: clientTrees[o] JSON, nodeIds[o] -> { diff[o], ids[o][], errors[o] }
  getMessages(clientTreesJson, nodeIds) {
    const [c, node] = this._selectArgs(clientTreesJson, nodeIds);
    try {
      return this._selected(addon.serverSelect(this.engine.ctx, this.store, c, node));
    } finally {
      addon.treeFree(this.engine.ctx, c);
    }
  }
  // -> Promise<Either<UnknownError, { diff, ids, errors }>>
  async getMessagesAsync(clientTreesJson, nodeIds) {
    const [c, node] = this._selectArgs(clientTreesJson, nodeIds);
    const e = await addon.serverSelectAsync(this.engine.ctx, this.store, c, node);
    addon.treeFree(this.engine.ctx, c);
    return e._tag === "Left" ? e : { _tag: "Right", right: this._selected(e.right) };
  }
  _selectArgs(clientTreesJson, nodeIds) {
    if (clientTreesJson.length !== this.nOwners || nodeIds.length !== this.nOwners)
      throw new RangeError("one client tree and one nodeId per owner slot");
    nodeIds.forEach((n) => {
      // a NodeId is 16 hex chars (types.ts:42); any other string would shift every later owner's slice
      if (typeof n !== "string" || !/^[0-9a-f]{16}$/i.test(n)) throw new RangeError("nodeId must be 16 hex chars");
    });
    return [addon.treeFromJson(this.engine.ctx, clientTreesJson), Uint8Array.from(Buffer.from(nodeIds.join(""), "latin1"))];
  }
  _selected(r) {
    const ids = [];
    for (let o = 0; o < this.nOwners; o++) ids.push(Array.from(r.ids.subarray(r.off[o], r.off[o + 1])));
    // diffMerkleTrees throws RangeError at a 17-digit key (merkleTree.ts:55-61), which fails that
    // owner's request (index.ts:185 -> 500): errors[o] holds it, and that owner selects nothing
    const errors = Array.from(r.diff, (d) => (d === -2 ? new RangeError("Invalid count value") : null));
    return { diff: Array.from(r.diff, (d) => (d === -1 || d === -2 ? null : d)), ids, errors };
  }
  // receive.ts:118-124 over this store as a "__message" mirror: since[o] millis | null -> ids[o][]
  messagesSince(since) {
    const s = Float64Array.from(since, (d) => (d == null ? -1 : d));
    const r = addon.storeSince(this.engine.ctx, this.store, s);
    const ids = [];
    for (let o = 0; o < this.nOwners; o++) ids.push(Array.from(r.ids.subarray(r.off[o], r.off[o + 1])));
    return ids;
  }
}

// apps/server/src/index.ts:218-248, the whole POST handler for a batch of
// request bodies: one native round (evm_sync_round) -- parseBody, the userId
// directory, addMessages, getMessages and SyncResponse.toBinary on the device.
// sync(bodies: Uint8Array[]) -> per body the response bytes (Uint8Array), 500
// (the handler's res.status(500): a body that does not parse, a client tree
// merkleTreeFromString rejects, a RangeError of the diff), or null: not
// applied here -- a timestamp outside the engine's domain, a nodeId that is not
// 16 hex chars, a non-ASCII userId, or a user handed over (handOver): the
// reference's handler runs it.  A user with two requests in one call gets them
// in rounds, in order (the k-th request of every user in round k).
const EVM_EROUNDS = 11;
const SYNC_ANSWERED = 0;
const SYNC_500 = new Set([1 /* EVM_EINVAL */, 4 /* EVM_ERANGE */, 5 /* EVM_ETREE */]);
class SyncServer {
  constructor(engine, nUsers) {
    this.engine = engine;
    this.store = addon.storeNew(engine.ctx, nUsers);
    this.h = addon.syncCreate(engine.ctx, this.store);
  }
  close() {
    addon.syncDestroy(this.engine.ctx, this.h);
    addon.storeFree(this.engine.ctx, this.store);
  }
  handOver(userId, flag = true) {
    addon.syncUserFlag(this.engine.ctx, this.h, userId, flag ? 1 : 0);
  }
  sync(bodies) {
    const out = new Array(bodies.length).fill(null);
    if (!this._round(bodies, bodies.map((_, i) => i), out)) {
      const seen = new Map();
      const rounds = [];
      bodies.forEach((b, i) => {
        let u = null;
        try {
          u = SyncRequest.fromBinary(b).userId;
        } catch (e) {
          u = null;  // (answered 500 by the round)
        }
        const k = u === null ? 0 : (seen.get(u) || 0);
        if (u !== null) seen.set(u, k + 1);
        while (rounds.length <= k) rounds.push([]);
        rounds[k].push(i);
      });
      for (const idx of rounds) {
        if (!this._round(idx.map((i) => bodies[i]), idx, out)) throw new Error("syncRound: a userId twice in a round");
      }
    }
    return out;
  }
  _round(bodies, idx, out) {
    const off = new Float64Array(bodies.length + 1);
    bodies.forEach((b, i) => { off[i + 1] = off[i] + b.length; });
    const arena = new Uint8Array(off[bodies.length]);
    bodies.forEach((b, i) => arena.set(b, off[i]));
    const r = addon.syncRound(this.engine.ctx, this.h, arena, off);
    if (r.status === EVM_EROUNDS) return false;
    for (let k = 0; k < bodies.length; k++) {
      const code = r.results[k];
      if (code === SYNC_ANSWERED) out[idx[k]] = r.responses.slice(r.offsets[k], r.offsets[k + 1]);
      else if (SYNC_500.has(code)) out[idx[k]] = 500;
      else out[idx[k]] = null;
    }
    return true;
  }
}

// Multi-GPU owner sharding (evm_dist_*): one Engine + Dist per GPU process;
// rank 0 makes the id (Dist.uniqueId()) and hands it to the other processes.
// Owners live on rank owner % world, or -- after directory(userIds) -- on rank
// murmur3(userId) % world with dense local ids (SURVEY 8(e)).  Loopback ranks
// (Dist.loopbackHub(world), one worker thread each, one GPU) run the same
// collectives with device copies instead of xGMI.
class Dist {
  static uniqueId() {
    return addon.distUniqueId();
  }
  // a hub for `world` loopback ranks (a BigInt: hand it to the worker threads)
  static loopbackHub(world) {
    return addon.distHubNew(world);
  }
  static freeHub(hub) {
    addon.distHubFree(hub);
  }
  static abortHub(hub) {
    addon.distHubAbort(hub);
  }
  // id: a uniqueId (RCCL), or { hub } for a loopback rank
  constructor(engine, id, rank, world) {
    this.engine = engine;
    this.rank = rank;
    this.world = world;
    this.h = id && id.hub !== undefined ? addon.distInitLoopback(engine.ctx, id.hub, rank)
      : addon.distInit(engine.ctx, id, rank, world); // collective
    this.hotBase = 0;
    this.hot = new Uint32Array(0);
  }
  close() {
    addon.distFree(this.engine.ctx, this.h);
  }
  // owner directory from the userId strings (global owner id = index): -> { dest, local, nLocal }
  directory(userIds) {
    const len = userIds.length ? Buffer.byteLength(userIds[0], "latin1") : 1;
    const stride = (len + 7) & ~7;
    const ids = new Uint8Array(userIds.length * stride);
    userIds.forEach((u, i) => {
      if (Buffer.byteLength(u, "latin1") !== len) throw new RangeError("userIds must have one length");
      ids.set(Buffer.from(u, "latin1"), i * stride);
    });
    const r = addon.distDirectory(this.engine.ctx, this.h, ids, stride, len);
    this.nOwners = userIds.length;
    this.nLocal = r.nLocal;
    return r;
  }
  // collective: split the owners holding more than `share` of one rank's fair share of
  // this round's rows (owners: this rank's rows' global ids) over every rank.
  // Local ids afterwards: hotBase + h for split owner hot[h].  -> hot (Uint32Array)
  splitHot(owners, nOwnersGlobal, share = 0.25) {
    const hot = addon.distHotOwners(this.engine.ctx, this.h, Uint32Array.from(owners), nOwnersGlobal, share);
    this.hotBase = addon.distSplit(this.engine.ctx, this.h, hot, nOwnersGlobal);
    this.hot = hot;
    this.nLocal = this.hotBase + hot.length;
    return hot;
  }
  // collective: this rank's slice of a batch -> the rows of the owners this rank
  // serves, in global batch order: { timestamps, owner, aux, src } (src = rank * 2^32 + index;
  // owner: local ids once a directory or split is set).  dest (optional): the rank of every row.
  route(timestamps, owners, aux = null, dest = null) {
    const r = addon.distRoute(this.engine.ctx, this.h, encodeTimestamps(timestamps), STRIDE, Uint32Array.from(owners),
      aux ? Uint32Array.from(aux) : null, dest ? Uint8Array.from(dest) : null);
    const dec = new TextDecoder();
    const ts = [];
    for (let i = 0; i < r.owner.length; i++) ts.push(dec.decode(r.ts.subarray(i * STRIDE, i * STRIDE + 46)));
    return { timestamps: ts, owner: r.owner, aux: r.aux, src: r.src };
  }
  // addMessages (index.ts:138-171) of the last route's rows into `server` (this rank's
  // owners) from the received records themselves (evm_dist_ingest); row i of route()'s
  // result gets id idBase + i.  -> { status, inserted: boolean[] }
  addRouted(server, idBase = 0) {
    const r = addon.distIngest(this.engine.ctx, this.h, server.store, idBase);
    return { status: r.status, inserted: Array.from(r.flags, (f) => (f & 4) !== 0) };
  }
  // collective: every owner's root (split owners: the XOR of their partial roots)
  gatherRoots(server, nOwnersGlobal) {
    return addon.distGatherRoots(this.engine.ctx, this.h, addon.storeTree(server.store), nOwnersGlobal);
  }
  // collective: getMessages (index.ts:173-202) over a server whose owners are this rank's
  // local ids, with split owners: clientTreesJson[j] / nodeIds[j] per local id (the hot
  // slots: the split owner's client tree and requester, the same on every rank).
  // -> { diff[j], ids[j][] (this rank's rows), hotIds[h][] (every rank's rows, timestamp order) }
  getMessagesSplit(server, clientTreesJson, nodeIds) {
    const [c, node] = server._selectArgs(clientTreesJson, nodeIds);
    try {
      const r = addon.distSelectSplit(this.engine.ctx, this.h, server.store, c, node, this.hotBase, this.hot.length);
      const ids = [];
      for (let j = 0; j < server.nOwners; j++) ids.push(Array.from(r.ids.subarray(r.off[j], r.off[j + 1])));
      const hotIds = [];
      for (let h = 0; h < this.hot.length; h++) hotIds.push(Array.from(r.hotIds.subarray(r.hotOff[h], r.hotOff[h + 1])));
      return { diff: Array.from(r.diff, (d) => (d === -1 || d === -2 ? null : d)), ids, hotIds };
    } finally {
      addon.treeFree(this.engine.ctx, c);
    }
  }
  // collective: applyMessages (applyMessages.ts:26-131) of ONE owner's batch split over
  // the ranks by cell; each rank passes its slice (timestamps, cell ids < nCells).
  // state (optional, the owner's DB as the single-rank applyMessages reads it, the SAME on
  // every rank): { prior: per cell its current max timestamp or null (applyMessages.ts:34-40),
  // stored: [{ timestamp, cell }] the __message rows holding a batch timestamp (:42-45;
  // cell >= nCells: a cell the batch does not touch) }.
  // -> { status, flags (this slice), winner[c] (global batch index or -1), tree JSON | null }
  applyMessagesSplit(timestamps, cells, nCells, treeJson = "{}", state = null) {
    const t = addon.treeFromJson(this.engine.ctx, [treeJson]);
    try {
      const args = [this.engine.ctx, this.h, encodeTimestamps(timestamps), Uint32Array.from(cells), nCells, t];
      if (state) {
        const prior = state.prior || new Array(nCells).fill(null);
        args.push(encodeTimestamps(prior.map((p) => (p == null ? "" : p))),
          Uint8Array.from(prior.map((p) => (p == null ? 0 : 1))));
        // (a non-empty DB must say which of the batch's timestamps "__message" holds)
        if (!Array.isArray(state.stored))
          throw new TypeError("applyMessagesSplit: state.stored (the __message rows of the batch's timestamps) is required");
        const stored = state.stored;
        if (stored.length) {
          args.push(encodeTimestamps(stored.map((r) => r.timestamp)), Uint32Array.from(stored.map((r) => r.cell)));
        }
      }
      const r = addon.distSplitApply(...args);
      let tree = null;
      if (r.tree) {
        tree = addon.treeToJson(this.engine.ctx, r.tree, 0);
        addon.treeFree(this.engine.ctx, r.tree);
      }
      return { status: r.status, flags: r.flags, winner: Array.from(r.winner), tree };
    } finally {
      addon.treeFree(this.engine.ctx, t);
    }
  }
}

module.exports = { Engine, Server, SyncServer, Dist, SyncRequest, SyncResponse, encodeTimestamps, MSG_UPS, MSG_XOR,
  MSG_INS };
