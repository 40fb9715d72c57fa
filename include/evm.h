/*
 * evm.h -- C ABI of the MI355X batch-merge engine for Evolu's CRDT sync path.
 *
 * Plain C, plain pointers and sizes.  Every compute entry point takes DEVICE
 * pointers and runs on the context's HIP stream; `evm_copy_*` / `evm_dev_*`
 * let a caller without its own allocator (the N-API addon) stage host
 * buffers.  Every call returns an int status (EVM_OK == 0).  One context per
 * thread; the library keeps no global state.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to harrywebdev/evolu @ 2025-01-31):
 *
 *   evm_pack ............ timestamp.ts:50-55 timestampFromString +
 *                         timestamp.ts:87-88 timestampToHash (batched)
 *   evm_merkle_insert ... merkleTree.ts:31-50 insertIntoMerkleTree (batched,
 *                         many owners)
 *   evm_merkle_diff ..... merkleTree.ts:63-91 diffMerkleTrees (batched over
 *                         owners)
 *   evm_apply_batch ..... applyMessages.ts:26-131 applyMessages (LWW decisions
 *                         + Merkle fold; the SQL writes stay with the caller)
 *   evm_server_ingest ... apps/server/src/index.ts:138-171 addMessages
 *   evm_server_select ... apps/server/src/index.ts:173-202 getMessages
 *   evm_pb_* ............ protobuf.ts:60-171 SyncRequest / SyncResponse
 *                         fromBinary / toBinary (host codec)
 *   evm_store_since ..... receive.ts:106-142 handleMerkleTreesDiff's resend
 *                         range (SELECT ... "timestamp" > ? ORDER BY
 *                         "timestamp"), batched over owners
 *   evm_tree_to_json /
 *   evm_tree_from_json .. types.ts:80-84 merkleTreeToString / FromString
 *   evm_sync_round ...... apps/server/src/index.ts:204-251 the whole sync
 *                         request handler (parseBody, getMerkleTree,
 *                         addMessages, getMessages, toBinary), batched over
 *                         the requests of one round, bodies in and out
 */
#ifndef EVM_H
#define EVM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
enum evm_status {
  EVM_OK = 0,
  EVM_EINVAL = 1,     /* bad argument */
  EVM_ENONCANON = 2,  /* >= 1 timestamp outside the native domain (see EVM_META_*); nothing applied */
  EVM_ECOLLISION = 3, /* one timestamp in two cells of a batch (global __message PK); nothing applied */
  EVM_ERANGE = 4,     /* a diff reached a 17-digit key: the reference throws RangeError */
  EVM_ETREE = 5,      /* tree JSON is not a tree insertIntoMerkleTree can produce */
  EVM_EDEVICE = 6,    /* HIP error */
  EVM_ENOMEM = 7,     /* device allocation failed */
  EVM_ECAPACITY = 8,  /* output buffer too small */
  EVM_EDIST = 9,      /* RCCL missing or a collective failed (evm_dist_*) */
  EVM_ESTATE = 10,    /* a store invariant broke in a merge (stored and new keys not disjoint); nothing committed */
  EVM_EROUNDS = 11,   /* evm_sync_round: a userId in two requests of one call; nothing applied (split the call) */
  EVM_EHANDOVER = 12  /* evm_sync_round, per request: not modelled here (a nodeId that is not 16 hex chars, or a
                         user handed to the caller); nothing of it applied -- the caller's reference path runs it */
};

/* ---- packed timestamp record (32 bytes, device) -------------------------
 * tc    = millis << 16 | counter
 * node  = the 16 node hex digits as a 64-bit value (case folded)
 * meta  = EVM_META_* bits; low 16 bits: bit i set <=> node char i is 'A'-'F'
 * hash  = murmur3 of the canonical string (uint32; timestampToHash)
 * minute= floor(millis / 60000) == (millis/1000/60)|0 on the native domain
 * aux   = caller's per-message id copied through (cell or owner)          */
typedef struct evm_rec {
  uint64_t tc;
  uint64_t node;
  uint32_t meta;
  uint32_t hash;
  uint32_t minute;
  uint32_t aux;
} evm_rec;

#define EVM_META_CASEMASK 0x0000FFFFu
#define EVM_META_VALID 0x00010000u    /* canonical and 1970 <= t < 2^31 minutes */
#define EVM_META_NONCANON 0x00020000u /* not canonical: V8's lenient Date.parse forms etc. */
#define EVM_META_RANGE 0x00040000u    /* canonical, but before 1970 or at/after 2^31 minutes */

/* ---- per-message flag bits (uint8, device) ----------------------------- */
#define EVM_MSG_UPS 0x01u /* applyMessages.ts:93  upsert of the user-table cell executed */
#define EVM_MSG_XOR 0x02u /* applyMessages.ts:105 __message INSERT attempted + Merkle XOR */
#define EVM_MSG_INS 0x04u /* index.ts:154         INSERT OR IGNORE changed a row (+ XOR) */
#define EVM_MSG_BAD 0x80u /* timestamp outside the native domain */

/* ---- context ----------------------------------------------------------- */
typedef struct evm_ctx evm_ctx;

int evm_create(int device, evm_ctx** out);
void evm_destroy(evm_ctx* ctx);
const char* evm_strerror(int status);
/* Makes the calling thread use the context's GPU (a worker thread -- e.g. the
 * N-API addon's async work -- driving a context created on another thread).
 * A context is still used by one thread at a time. */
int evm_bind_thread(evm_ctx* ctx);
/* Allocation counters since evm_create: what a steady-state loop should keep
 * flat (every counter but workspace_bytes only grows). */
typedef struct evm_stats {
  uint64_t workspace_regrows;   /* the per-call scratch arena was reallocated (synchronising) */
  uint64_t workspace_bytes;     /* current arena size */
  uint64_t scratch_pool_allocs; /* scratch requests the arena could not hold (stream-ordered pool) */
  uint64_t scratch_pool_bytes;
  uint64_t block_allocs;        /* device blocks allocated for trees and stores (freed ones are reused) */
  uint64_t block_bytes;
  uint64_t tc_batches;          /* evm_apply_batch calls the streaming tc path finished */
  uint64_t tc_redos;            /* ... whose tie list overflowed and were redone by the exact walk path */
  uint64_t small_batches;       /* evm_apply_batch calls the small-batch path finished */
  uint64_t small_fallbacks;     /* ... it handed to the sort path (a cell of > 4,096 rows, minutes too wide) */
} evm_stats;
int evm_get_stats(const evm_ctx* ctx, evm_stats* out);
int evm_set_stream(evm_ctx* ctx, void* hip_stream); /* NULL: the HIP default stream; initially the context's own */
void* evm_get_stream(evm_ctx* ctx);
int evm_sync(evm_ctx* ctx);
/* tuning / test knobs */
#define EVM_OPT_CLIENT_PATH 1 /* evm_apply_batch: 0 auto (<= 2,048 cells: the streaming tc path; more cells: the \
                                 small-batch path up to 262,144 messages, else the sort path), 1 exact walk path, \
                                 2 sort path, 3 tc path (the exact walk path only when a range's tie list \
                                 overflows), 4 small-batch path (the sort path when it does not apply) */
#define EVM_OPT_OVERLAP 3     /* 1 (default): independent checks run on a second HIP stream inside a call; 0: one stream */
#define EVM_OPT_SERVER_PATH 2 /* evm_server_ingest: 0/1 per-owner LDS path, owners above its capacity cut into
                                 key-range segments; 2 force the sort path; 3 LDS path without the segments (owners
                                 above the capacity through the sort path); 4 as 0 with K5 reading packed 32-B
                                 records instead of parsing the rows itself (A/B) */
#define EVM_OPT_RADIX 4       /* radix sorts: 1 (default) one-sweep passes with decoupled look-back; 2 the same with \
                                 10-bit digits when that saves a pass; 0 histogram + scan + scatter per pass */
#define EVM_OPT_DIFF_GRID 6   /* evm_merkle_diff / select: k_diff workgroups per CU (0: one lane group per owner) */
#define EVM_OPT_SELECT_PATH 7 /* getMessages selection with a requester: 0 (default) keep + rank + emit in one pass \
                                 (look-back over candidate tiles), 1 keep / scan / emit passes (A/B) */
int evm_set_option(evm_ctx* ctx, int option, int64_t value);
/* kernel timing with HIP events on the context stream (for roofline reports) */
int evm_prof_enable(evm_ctx* ctx, int on);
int evm_prof_reset(evm_ctx* ctx);
/* time only the launches of one kernel (its report name); null or "" = all */
int evm_prof_only(evm_ctx* ctx, const char* kernel);
/* JSON {"kernel": [total_ms, launches], ...}; *len = bytes needed */
int evm_prof_report(evm_ctx* ctx, char* buf, size_t cap, size_t* len);
int evm_dev_alloc(evm_ctx* ctx, size_t bytes, void** out);
int evm_dev_free(evm_ctx* ctx, void* p);
int evm_copy_h2d(evm_ctx* ctx, void* dst_dev, const void* src_host, size_t bytes);
int evm_copy_d2h(evm_ctx* ctx, void* dst_host, const void* src_dev, size_t bytes);

/* ---- K1: parse + canonical check + murmur3 + minute (timestamp.ts) -------
 * ts: n timestamps of 46 significant bytes at `stride` bytes (46 or more;
 * 48 is the coalesced native layout).  aux may be NULL.  Writes out[n].
 * Returns EVM_ENONCANON if any record lacks EVM_META_VALID (out still full). */
int evm_pack(evm_ctx* ctx, const char* ts, size_t stride, size_t n, const uint32_t* aux, evm_rec* out);

/* ---- Merkle trees: per-owner leaf maps, device resident -----------------
 * A tree set holds one MerkleTree per owner as the sorted list of its leaves:
 * every key path that received >= 1 insert, with the XOR of the hashes that
 * ended there.  Node hashes, node presence and JSON all derive from it.
 * Leaf code = sum (digit_i + 1) * 4^(19 - i) over the base-3 key digits.   */
typedef struct evm_tree evm_tree;

int evm_tree_new(evm_ctx* ctx, uint32_t n_owners, evm_tree** out); /* all trees {} */
int evm_tree_from_leaves(evm_ctx* ctx, uint32_t n_owners, const uint64_t* owner_off_host,
                         const uint64_t* code_host, const int32_t* xor_host, evm_tree** out);
int evm_tree_free(evm_ctx* ctx, evm_tree* t);
/* The same from DEVICE arrays (off[n_owners + 1], code[off[n_owners]], xr):
 * how leaf lists gathered over RCCL become trees without a host copy.     */
int evm_tree_from_device_leaves(evm_ctx* ctx, uint32_t n_owners, const uint64_t* off_dev, const uint64_t* code_dev,
                                const int32_t* xr_dev, evm_tree** out);
/* Device copy of the leaves of owners [owner_lo, owner_lo + count): off[count
 * + 1] (rebased to 0), code / xr [*n_leaves <= cap] (EVM_ECAPACITY if not). */
int evm_tree_slice(evm_ctx* ctx, const evm_tree* t, uint32_t owner_lo, uint32_t count, uint64_t* off_dev,
                   uint64_t* code_dev, int32_t* xr_dev, uint64_t cap, uint64_t* n_leaves);
int evm_tree_info(const evm_tree* t, uint32_t* n_owners, uint64_t* n_leaves);
/* device views (valid until the tree is freed) */
int evm_tree_device(const evm_tree* t, const uint64_t** owner_off, const uint64_t** code, const int32_t** xr);
/* host copies: owner_off[n_owners+1], code[n_leaves], xr[n_leaves] (any may be NULL) */
int evm_tree_leaves(evm_ctx* ctx, const evm_tree* t, uint64_t* owner_off, uint64_t* code, int32_t* xr);
/* per owner root: hash (int32) and present (0: the tree is {}) -- host arrays */
int evm_tree_roots(evm_ctx* ctx, const evm_tree* t, int32_t* root_hash, uint8_t* present);
/* types.ts:80-81 JSON.stringify(tree of `owner`); *len = bytes needed (no NUL) */
int evm_tree_to_json(evm_ctx* ctx, const evm_tree* t, uint32_t owner, char* buf, size_t cap, size_t* len);
/* The same for many owners in one call, on the device (index.ts:160-163,:240
 * for every request of a round): owners[0..n) (device u32; NULL = owners
 * 0..n-1) -> their texts back to back in `out` (device, cap bytes), owner j's
 * at [off[j], off[j+1]) (off: device, n + 1 entries); *total = the bytes
 * needed.  out == NULL: only off and *total.  EVM_ECAPACITY when total > cap;
 * EVM_EINVAL for an owner id out of range. */
int evm_tree_to_json_batch(evm_ctx* ctx, const evm_tree* t, const uint32_t* owners, uint32_t n, char* out, size_t cap,
                           uint64_t* off, uint64_t* total);
/* types.ts:83-84, one JSON text per owner (host strings) */
int evm_tree_from_json(evm_ctx* ctx, uint32_t n_owners, const char* const* json, const size_t* lens, evm_tree** out);

/* merkleTree.ts:31-50, batched: XOR every timestamp into its owner's tree.
 * owner: device [n] (NULL: all owner 0).  *out is a new tree set.          */
int evm_merkle_insert(evm_ctx* ctx, const evm_tree* in, const char* ts, size_t stride, size_t n,
                      const uint32_t* owner, evm_tree** out);

/* Per owner: the tree holding the inserts of both a and b (leaf union, equal
 * keys XOR-combined) -- what insertIntoMerkleTree gives for the two insert
 * sets together, in any order (merkleTree.test.ts:30-42).  Combines the
 * partial trees of an owner whose messages were split over GPUs.          */
int evm_tree_merge(evm_ctx* ctx, const evm_tree* a, const evm_tree* b, evm_tree** out);

/* merkleTree.ts:63-91 for every owner o: diffMerkleTrees(a[o], b[o]).
 * millis: device int64[n_owners]; -1 = option.none, -2 = RangeError.       */
#define EVM_DIFF_NONE (-1)
#define EVM_DIFF_RANGE_ERROR (-2)
int evm_merkle_diff(evm_ctx* ctx, const evm_tree* a, const evm_tree* b, int64_t* millis);

/* ---- client: applyMessages.ts:26-131 -------------------------------------
 * Batch order is message order.  cell: device [n], dense ids < n_cells of
 * (table,row,column) per owner.  cell_owner: device [n_cells] or NULL (one
 * owner).  prior_ts: device, n_cells timestamps at prior_stride = the cell's
 * current max in __message (SELECT ... ORDER BY timestamp DESC LIMIT 1);
 * prior_present: device uint8 [n_cells] (NULL: no prior rows).
 * Outputs: flags[n] (EVM_MSG_UPS / EVM_MSG_XOR), winner[n_cells] (index of
 * the message whose upsert is final, -1 if none), *tree_out.
 * The caller then runs the upsert of each winner and
 * INSERT ... ON CONFLICT DO NOTHING of each XOR message, in batch order.   */
int evm_apply_batch(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n,
                    const uint32_t* cell, uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts,
                    size_t prior_stride, const uint8_t* prior_present, uint8_t* flags, int32_t* winner,
                    evm_tree** tree_out);

/* evm_apply_batch plus the rows ALREADY in __message that hold a batch
 * timestamp (applyMessages.ts:42-45: "timestamp" is the table's PRIMARY KEY,
 * initDbModel.ts:44), i.e. the caller's
 *   SELECT "timestamp", "table", "row", "column" FROM "__message"
 *   WHERE "timestamp" IN (<the batch's timestamps>)
 * stored_ts: device, n_stored timestamps at stored_stride; stored_cell:
 * device [n_stored], the row's cell in the batch's numbering, or any id >=
 * n_cells for a cell the batch does not touch.  A batch message whose
 * timestamp is stored under ANOTHER cell has its INSERT ignored and freezes
 * that cell's running max (applyMessages.ts:104-119): EVM_ECOLLISION, nothing
 * applied.  A stored row of the message's own cell is covered by prior_ts
 * (the cell's max is >= it).  n_stored == 0: exactly evm_apply_batch.
 * (With cell_owner, a stored row matching another owner's message is also
 * reported, conservatively.)                                               */
int evm_apply_batch_ex(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n,
                       const uint32_t* cell, uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts,
                       size_t prior_stride, const uint8_t* prior_present, const char* stored_ts, size_t stored_stride,
                       size_t n_stored, const uint32_t* stored_cell, uint8_t* flags, int32_t* winner,
                       evm_tree** tree_out);

/* Asynchronous evm_apply_batch_ex (applyMessages is a ReaderTaskEither,
 * applyMessages.ts:26-31): the batch is enqueued on the context stream and the
 * call returns at once, so the host prepares the next batch while the GPU
 * works; evm_apply_wait collects the status and the new tree.  Every input and
 * output buffer (and tree_in) must stay valid and untouched until the wait.
 * Batches the streaming path does not take (many owners, > 2,048 cells, empty)
 * and the rare redo cases (a tie, an oversized hash bucket, a wide minute
 * range) finish synchronously -- inside this call or the wait.  Each handle is
 * waited exactly once.                                                      */
typedef struct evm_pending evm_pending;
int evm_apply_batch_async(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n,
                          const uint32_t* cell, uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts,
                          size_t prior_stride, const uint8_t* prior_present, const char* stored_ts,
                          size_t stored_stride, size_t n_stored, const uint32_t* stored_cell, uint8_t* flags,
                          int32_t* winner, evm_pending** out);
/* -> the batch's status (as evm_apply_batch_ex); *tree_out on EVM_OK */
int evm_apply_wait(evm_ctx* ctx, evm_pending* p, evm_tree** tree_out);

/* The global __message PK check evm_apply_batch runs (applyMessages.ts:42-45,
 * 104-113: one timestamp in two cells of a batch), on its own: for a batch
 * whose cells are split over ranks (evolu_amd/dist.py split_apply), each rank
 * checks the messages routed to it by timestamp hash.  *found = 1 iff some
 * timestamp occurs with two different cells.                               */
int evm_cross_cell_check(evm_ctx* ctx, const char* ts, size_t stride, size_t n, const uint32_t* cell,
                         uint32_t n_cells, int32_t* found);

/* ---- client: receive.ts:45-66 receiveMessages -----------------------------
 * Folds timestampFromString(m.timestamp) of every message of a batch into
 * the local clock with timestamp.ts:125-165 receiveTimestamp, `now` fixed
 * for the batch (db.worker.ts:71), stopping at the first error exactly as
 * the reference's readerEither.traverseArray does.  ts: device.          */
#define EVM_CLOCK_OK 0
#define EVM_CLOCK_DRIFT 1          /* TimestampDriftError {next, now} */
#define EVM_CLOCK_DUPLICATE_NODE 2 /* TimestampDuplicateNodeError {node} */
#define EVM_CLOCK_OVERFLOW 3       /* TimestampCounterOverflowError */
typedef struct evm_clock_result {
  int32_t error;       /* EVM_CLOCK_* */
  uint32_t counter;    /* the new clock (when error == 0) */
  int64_t millis;
  int64_t error_index; /* message that failed, -1 */
  int64_t next;        /* TimestampDriftError.next */
} evm_clock_result;
int evm_receive_fold(evm_ctx* ctx, const char* ts, size_t stride, size_t n, int64_t local_millis,
                     uint32_t local_counter, const char* local_node, int64_t now, int64_t max_drift,
                     evm_clock_result* out);

/* ---- server: apps/server/src/index.ts -------------------------------------
 * A store holds, per owner (userId), the set of stored messages -- the
 * "message" table's PRIMARY KEY(timestamp, userId) -- sorted by timestamp
 * (string order), each with the caller's 64-bit message id, plus the owner's
 * MerkleTree ("merkleTree" table).  Device resident.                       */
typedef struct evm_store evm_store;

int evm_store_new(evm_ctx* ctx, uint32_t n_owners, evm_store** out);
int evm_store_free(evm_ctx* ctx, evm_store* s);
int evm_store_info(const evm_store* s, uint32_t* n_owners, uint64_t* n_messages);
/* the store's per-owner trees (borrowed; valid until the next ingest/free) */
const evm_tree* evm_store_tree(const evm_store* s);
/* host copies: owner_off[n_owners+1], id[n_messages] in (owner, timestamp) order */
int evm_store_messages(evm_ctx* ctx, const evm_store* s, uint64_t* owner_off, uint64_t* id);

/* index.ts:138-171 addMessages, batched over requests of many owners.
 * Batch order = index order (requests concatenated in arrival order).
 * owner: device [n] owner of each message.  Message i gets id id_base + i.
 * flags: device [n] -> EVM_MSG_INS where INSERT OR IGNORE changed a row
 * (first occurrence of (timestamp, owner) not already stored); exactly
 * those messages are XORed into their owner's tree.                        */
int evm_server_ingest(evm_ctx* ctx, evm_store* s, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                      uint64_t id_base, uint8_t* flags);

/* The same with the reference's per-request transactions (index.ts:147-169:
 * a throw rolls back that request only): an owner with a row outside the
 * native domain commits NOTHING -- owner_status[o] = 1 (device uint8
 * [n_owners]), its culprit rows flagged EVM_MSG_BAD, its other rows 0 --
 * and every other owner commits exactly as evm_server_ingest would.  Returns
 * EVM_OK (all committed), EVM_ENONCANON (the flagged owners did not, the rest
 * did), or an error (nothing committed).  A batch carries one request per
 * owner, as SyncServer's rounds do. */
int evm_server_ingest_ex(evm_ctx* ctx, evm_store* s, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                         uint64_t id_base, uint8_t* flags, uint8_t* owner_status);

/* index.ts:173-202 getMessages for one request per owner:
 * diff = diffMerkleTrees(store tree, client[o]); if Some(d), the owner's
 * messages with timestamp > timestampToString(createSyncTimestamp(d)) and
 * timestamp NOT LIKE '%' || node[o] (ASCII case-insensitive suffix), in
 * timestamp order.  node: device, 16 bytes per owner (the requester's
 * nodeId; 16 hex chars); active: device uint8 [n_owners] (NULL: all).
 * Outputs (device): diff[n_owners] (EVM_DIFF_NONE / millis / RANGE_ERROR),
 * sel_off[n_owners + 1], sel_id[cap]; *n_sel = total selected.            */
/* receive.ts:118-124 (client resend after a diff) / index.ts:98-102 without
 * the node filter: per owner o with since[o] >= 0, the stored messages with
 * timestamp > timestampToString(createSyncTimestamp(since[o])), in timestamp
 * order.  A store fed with the client's inserted messages (owner 0) mirrors
 * its "__message" table.  since: device int64 [n_owners] (< 0: none).
 * Outputs as evm_server_select: sel_off[n_owners + 1], sel_id[cap], *n_sel.  */
int evm_store_since(evm_ctx* ctx, const evm_store* s, const int64_t* since, uint64_t* sel_off, uint64_t* sel_id,
                    uint64_t cap, uint64_t* n_sel);

int evm_server_select(evm_ctx* ctx, const evm_store* s, const evm_tree* client, const char* node,
                      const uint8_t* active, int64_t* diff, uint64_t* sel_off, uint64_t* sel_id, uint64_t cap,
                      uint64_t* n_sel);

/* The selection half of getMessages (index.ts:189-197, stmt :98-102) with the
 * bound given: per owner o with bound[o] >= 0, the rows with timestamp >
 * timestampToString(createSyncTimestamp(bound[o])) and (node != NULL)
 * timestamp NOT LIKE '%' || node[o], in timestamp order.  For an owner whose
 * rows are split over GPUs the bound is the diff of its FULL trees (computed
 * once, on the merged tree), and each GPU selects its share; sel_key
 * (device, 3 x u64 per selected row, may be NULL) receives each row's order
 * key (tc, node ranks hi, lo) so the shares merge in timestamp order.      */
int evm_store_select_after(evm_ctx* ctx, const evm_store* s, const int64_t* bound, const char* node,
                           const uint8_t* active, uint64_t* sel_off, uint64_t* sel_id, uint64_t* sel_key,
                           uint64_t cap, uint64_t* n_sel);

/* ---------------------------------------------------------------- wire codec
 * protobuf.proto SyncRequest / SyncResponse (protobuf.ts:60-171), HOST
 * buffers (this is the request body the server receives, index.ts:115, and
 * the response it sends, index.ts:239).  Encoding omits proto3 defaults and
 * writes fields in number order (protobuf-ts toBinary); decoding skips
 * unknown fields and rejects truncated / ill-typed input (EVM_EINVAL).     */
#define EVM_PB_SYNC_REQUEST 1
#define EVM_PB_SYNC_RESPONSE 2
typedef struct evm_pb_sync {
  uint64_t n_messages;
  uint64_t content_bytes;      /* sum of the messages' content lengths */
  uint64_t user_off, user_len; /* SyncRequest.userId, as bytes of buf */
  uint64_t node_off, node_len; /* SyncRequest.nodeId */
  uint64_t tree_off, tree_len; /* merkleTree (JSON) */
  uint64_t nonstd_ts;          /* messages whose timestamp is not 46 bytes */
} evm_pb_sync;
/* Pass 1: sizes and the string fields' positions. */
int evm_pb_scan(int kind, const uint8_t* buf, size_t len, evm_pb_sync* info);
/* Pass 2: timestamps into the engine's arena (ts[n * stride]; a timestamp
 * that is not 46 bytes is written as 0xFF bytes so the engine flags it;
 * optional ts_len[n] and ts_off[n] = the original string's bytes in buf),
 * contents concatenated (content_off[n + 1]; content may be NULL to get
 * offsets only). */
int evm_pb_split(int kind, const uint8_t* buf, size_t len, char* ts, size_t stride, uint32_t* ts_len,
                 uint64_t* ts_off, uint64_t* content_off, uint8_t* content);
/* Encode n messages (ts rows of ts_len[i] bytes, NULL: 46; contents by
 * content_off) + the string fields (user/node only for a request).  out NULL
 * or too small: *out_len = bytes needed (EVM_ECAPACITY if out was given). */
int evm_pb_encode(int kind, const char* ts, size_t stride, const uint32_t* ts_len, size_t n,
                  const uint64_t* content_off, const uint8_t* content, const char* user, size_t user_len,
                  const char* node, size_t node_len, const char* tree, size_t tree_len, uint8_t* out, size_t cap,
                  size_t* out_len);
/* Batches of bodies on host threads (a server round, index.ts:224-248 per
 * request; EVM_HOST_THREADS caps the threads).  Bodies are arena[off[k] ..
 * off[k + 1]).  scan: per body its evm_pb_sync and status (EVM_EINVAL = the
 * reference's parseBody throw).  split: the bodies with status 0 into one
 * timestamp arena / content arena, body k's messages from global index
 * msg_base[k] and content byte content_base[k] (content_off: N + 1 global
 * entries; ts_off: offsets into the arena). */
int evm_pb_scan_batch(int kind, const uint8_t* arena, const uint64_t* off, uint32_t n, evm_pb_sync* info,
                      int32_t* status);
int evm_pb_split_batch(int kind, const uint8_t* arena, const uint64_t* off, uint32_t n, const int32_t* status,
                       const uint64_t* msg_base, const uint64_t* content_base, char* ts, size_t stride,
                       uint32_t* ts_len, uint64_t* ts_off, uint64_t* content_off, uint8_t* content);
/* SyncResponse bodies (index.ts:235-245) for n requests: request r's
 * messages are the ids sel_id[sel_off[r] .. sel_off[r + 1]) (a getMessages
 * selection); id -> log segment s = the last with seg_base[s] <= id, row =
 * id - seg_base[s] (or seg_row[s][that], when seg_row[s] is not NULL): its
 * 46-B timestamp at seg_ts[s] + row * stride, its content
 * seg_content[s][seg_coff[s][row] .. seg_coff[s][row + 1]); the merkleTree
 * text json[json_off[r] .. json_off[r + 1]).  Responses back to back in out
 * (out_off: n + 1 entries; out NULL: sizes only). */
/* SyncRequest bodies for n requests (the client side's toBinary,
 * sync.worker.ts:102; the bench's synthetic rounds): request r's messages
 * are ts rows [msg_off[r], msg_off[r + 1]) with contents by content_off; its
 * userId / nodeId / merkleTree the strings [x_off[r], x_off[r + 1]) of the
 * user / node / tree arenas.  out NULL: out_off (n + 1) only. */
int evm_pb_encode_requests(uint32_t n, const uint64_t* msg_off, const char* ts, size_t stride,
                           const uint64_t* content_off, const uint8_t* content, const char* user,
                           const uint64_t* user_off, const char* node, const uint64_t* node_off, const char* tree,
                           const uint64_t* tree_off, uint8_t* out, uint64_t* out_off);
int evm_pb_encode_responses(uint32_t n, const uint64_t* sel_off, const uint64_t* sel_id, uint32_t n_seg,
                            const uint64_t* seg_base, const uint64_t* const* seg_row, const char* const* seg_ts,
                            size_t stride, const uint64_t* const* seg_coff, const uint8_t* const* seg_content,
                            const char* json, const uint64_t* json_off, uint8_t* out, uint64_t* out_off);

/* ------------------------------------------------------- wire codec, device
 * The same codecs over bodies resident in DEVICE memory (evm_wire_dev.hip):
 * a server round's SyncRequests decoded where they lie in HBM, their client
 * trees parsed and the SyncResponses built there (index.ts:112-116, :121-136,
 * :233-241).  Same grammar and results as the host calls above (one device
 * thread runs the host's walk per body / tree).  All array arguments are
 * device pointers unless marked host.  The kernels read the bodies / texts
 * in whole 16-B chunks: the chunks holding the arena's bytes must be
 * readable (any device allocation is; torch's are 512-B granular).
 *
 * scan: per body (arena[off[k] .. off[k + 1])) its evm_pb_sync and status, as
 * evm_pb_scan_batch.  split: as evm_pb_split_batch (ts rows, content_off of
 * N + 1 entries, contents concatenated) plus owner[i] = owner_of[k] for body
 * k's rows (owner_of / owner may be NULL); rows of stride % 16 == 0, >= 48
 * (16-B aligned ts); ts_len / ts_off are not produced
 * (the device path takes only bodies whose timestamps are all 46 bytes).
 * gather: n byte spans of src packed into dst (dst_off from the caller). */
int evm_pb_scan_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n, evm_pb_sync* info,
                    int32_t* status);
int evm_pb_split_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n,
                     const int32_t* status, const uint64_t* msg_base, const uint64_t* content_base,
                     const uint32_t* owner_of, char* ts, size_t stride, uint64_t* content_off, uint8_t* content,
                     uint32_t* owner);
/* The same two steps sharing the scan's walk: scan_index also records where
 * each message's field starts, body k's i-th message at slots[off[k] / 50 + i]
 * (slots: off[n] / 50 + 1 entries; a message whose timestamp is 46 bytes takes
 * >= 50, so the bodies' ranges do not overlap), and split_index reads them
 * instead of walking the bodies again (a body whose messages do not fit its
 * range -- a shorter timestamp -- fails the split with EVM_EINVAL: the caller
 * takes only bodies whose evm_pb_sync.nonstd_ts is 0). */
int evm_pb_scan_index_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n,
                          evm_pb_sync* info, int32_t* status, uint64_t* slots);
int evm_pb_split_index_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n,
                           const int32_t* status, const uint64_t* msg_base, const uint64_t* content_base,
                           const uint32_t* owner_of, char* ts, size_t stride, uint64_t* content_off, uint8_t* content,
                           uint32_t* owner, const uint64_t* slots);
int evm_gather_spans_dev(evm_ctx* ctx, const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                         const uint64_t* dst_off, uint32_t n, uint8_t* dst);
/* evm_tree_from_json for n_owners texts json[at[o] .. at[o] + len[o]) (len 0:
 * the owner sent no tree -> the empty tree).  status[o] (device int32): 0,
 * EVM_ETREE (the host parser rejects the text: merkleTreeFromString throws),
 * or EVM_TREE_UNSORTED (children keys out of ascending order -- valid JSON
 * that JSON.stringify never writes: parse it on the host).  The tree is
 * returned whatever the statuses (an owner with a nonzero status is empty in
 * it); the call fails only on a bad argument or an allocation. */
#define EVM_TREE_UNSORTED 1000
int evm_tree_from_json_dev(evm_ctx* ctx, uint32_t n_owners, const uint8_t* json, const uint64_t* at,
                           const uint64_t* len, int32_t* status, evm_tree** out);
/* evm_pb_encode_responses with the selection, the log and the output on the
 * device: response r answers owner owners[r] -- its messages are the ids
 * sel_id[sel_off[o] .. sel_off[o + 1]) of that owner in an
 * evm_server_select result (sel_off: tree's n_owners + 1 entries), none when
 * skip[r] (uint8, may be NULL; a RangeError request), its merkleTree the
 * JSON of that owner of `tree`, emitted straight into the response.  seg_base (host, ascending)
 * and the host arrays of device pointers seg_row / seg_ts / seg_coff /
 * seg_content describe the log as in evm_pb_encode_responses.  out NULL:
 * out_off (n + 1) and *total (host) only; else cap >= *total bytes. */
int evm_pb_encode_responses_dev(evm_ctx* ctx, uint32_t n, const evm_tree* tree, const uint32_t* owners,
                                const uint64_t* sel_off, const uint64_t* sel_id, const uint8_t* skip, uint32_t n_seg,
                                const uint64_t* seg_base, const uint64_t* const* seg_row, const char* const* seg_ts,
                                size_t stride, const uint64_t* const* seg_coff, const uint8_t* const* seg_content,
                                uint8_t* out, size_t cap, uint64_t* out_off, uint64_t* total);

/* ------------------------------------------------------------ sync server
 * The server's request handler, apps/server/src/index.ts:204-251 (parseBody
 * :108-116, getMerkleTree :118-134, addMessages :136-171, getMessages
 * :173-202, SyncResponse.toBinary :233-241), for n SyncRequest bodies in one
 * call, run on the device end to end: the bodies decoded where they lie, the
 * userId -> owner slot directory a device hash table (new users take slots in
 * request order), one addMessages over every request (the reference's
 * per-request transactions: a request with a row outside the native domain
 * commits nothing), the client trees parsed, one getMessages, the responses
 * built in device memory.  The server owns the directory and the message log
 * (the rows and contents getMessages answers with); the store is the
 * caller's (evm_store_new with n_owners = the user capacity).
 *
 * A userId with a byte >= 0x80 is the caller's too (EVM_EHANDOVER: protobuf-ts
 * decodes it as UTF-8, and an invalid sequence decodes lossily).
 *
 * evm_sync_round: bodies arena[off[k] .. off[k + 1]) (off: HOST, n + 1
 * entries); where = EVM_SYNC_HOST (arena in host memory: staged through
 * pinned buffers to the device) or EVM_SYNC_DEVICE (arena in device memory,
 * readable in whole 16-B chunks).  Call status: EVM_OK, EVM_EROUNDS (a userId
 * in two requests: nothing applied -- the caller splits the call into rounds
 * of one request per user, in order), EVM_ECAPACITY (more users than the
 * store's owners: nothing applied), or an error.  Per request (host
 * result[n]): EVM_OK (response bytes [resp_off[k], resp_off[k + 1]) of the
 * round's response arena), EVM_EINVAL (SyncRequest.fromBinary threw -> 500),
 * EVM_ETREE (merkleTreeFromString threw -> 500; its rows are committed, as
 * the reference's addMessages ran first), EVM_ERANGE (diffMerkleTrees threw
 * RangeError -> 500; rows committed), EVM_ENONCANON (a timestamp outside
 * the native domain: nothing of the request stored -- the caller's reference
 * path decides: RangeError of toISOString, or a lenient spelling V8
 * accepts), EVM_EHANDOVER (see the status).  resp_off: host n + 1;
 * *resp_bytes: the arena's size.  evm_sync_fetch copies the arena to host
 * memory; evm_sync_responses_dev returns it in device memory (valid until
 * the next round).
 *
 * The rest serves a caller that runs some requests on its own path (the
 * reference's, for EVM_ENONCANON / EVM_EHANDOVER) against the same store:
 * evm_sync_users looks up (insert != 0: and adds, in order) users given in
 * host memory -> slots; evm_sync_user_flag hands a user over (1: every later
 * request of it answers EVM_EHANDOVER) or takes it back (0); evm_sync_log_add
 * appends rows ingested outside a round to the message log (host arrays:
 * ts rows of `stride` bytes, content_off n + 1 from 0, contents) and returns
 * their first message id (ids are consecutive, shared with the rounds);
 * evm_sync_log_read reads messages back by id (host: ts 46 B each,
 * content_off n + 1, contents; content NULL: sizes only). */
#define EVM_SYNC_HOST 0
#define EVM_SYNC_DEVICE 1
typedef struct evm_sync_server evm_sync_server;
int evm_sync_create(evm_ctx* ctx, evm_store* store, evm_sync_server** out);
int evm_sync_destroy(evm_sync_server* s);
int evm_sync_round(evm_sync_server* s, const uint8_t* arena, const uint64_t* off, uint32_t n, int where,
                   int32_t* result, uint64_t* resp_off, uint64_t* resp_bytes);
int evm_sync_fetch(evm_sync_server* s, uint8_t* out);
const uint8_t* evm_sync_responses_dev(const evm_sync_server* s);
int evm_sync_users(evm_sync_server* s, const uint8_t* ids, const uint64_t* id_off, uint32_t n, int insert,
                   uint32_t* slots);
int evm_sync_user_flag(evm_sync_server* s, uint32_t slot, int flag);
int evm_sync_user_count(const evm_sync_server* s, uint32_t* n_users, uint64_t* key_bytes);
int evm_sync_user_keys(evm_sync_server* s, uint8_t* keys, uint64_t* key_off);
int evm_sync_log_add(evm_sync_server* s, const char* ts, size_t stride, uint64_t n, const uint64_t* content_off,
                     const uint8_t* content, uint64_t* first_id);
int evm_sync_log_read(evm_sync_server* s, const uint64_t* ids, uint64_t n, char* ts, uint64_t* content_off,
                      uint8_t* content);
uint64_t evm_sync_next_id(const evm_sync_server* s);
/* the last round's wall time by part, ms[8]: staging in (host rounds), decode,
 * users, addMessages, client trees, getMessages, encode, staging out (fetch) */
int evm_sync_timing(const evm_sync_server* s, double* ms);

/* ------------------------------------------------------------------------
 * Multi-GPU owner sharding (evm_dist.hip).  One process per
 * GPU and one evm_dist per context; every call below is collective (all
 * ranks call it, in the same order) except evm_dist_take and
 * evm_dist_directory.  Owners are independent in the whole path, so every
 * owner lives on one rank: by default rank owner % world as local owner
 * owner / world (dense owner ids the caller assigns); after
 * evm_dist_directory, rank murmur3(userId) mod world with
 * dense local ids.  Replaces nothing in the reference (one process there);
 * it is what lets the N-API caller run one addon per GPU of a node.
 *
 * Failure: a rank that fails locally (bad argument, allocation) still joins
 * every collective of the call, flagged, and then EVERY rank returns an
 * error (the failing rank its own code, the others EVM_EDIST) -- no rank is
 * left waiting in a receive.  Only a NULL ctx / d / n_recv returns at once.
 *
 * Transports: RCCL (librccl.so.1, opened at run time; evm_dist_init), or an
 * in-process loopback hub (evm_dist_init_loopback): `world` contexts, one
 * host thread each, device-to-device copies instead of xGMI -- the same
 * partitions, count exchange, grouping and gathers, testable on one GPU.
 * ------------------------------------------------------------------------ */
#define EVM_DIST_ID_BYTES 128
typedef struct evm_dist evm_dist;
typedef struct evm_dist_hub evm_dist_hub;
/* a new communicator id (rank 0 makes it and hands it to the others) */
int evm_dist_unique_id(uint8_t* id);
/* collective: the communicator of `world` ranks (world <= 64) on ctx's device */
int evm_dist_init(evm_ctx* ctx, const uint8_t* id, int rank, int world, evm_dist** out);
/* loopback: a hub for `world` in-process ranks; each rank's thread calls
 * evm_dist_init_loopback with its own context.  Free the hub after every
 * evm_dist on it. */
int evm_dist_hub_new(int world, evm_dist_hub** out);
void evm_dist_hub_free(evm_dist_hub* hub);
/* a rank's thread failed outside the library: every pending and later
 * collective on the hub returns EVM_EDIST instead of waiting for it */
void evm_dist_hub_abort(evm_dist_hub* hub);
int evm_dist_init_loopback(evm_ctx* ctx, evm_dist_hub* hub, int rank, evm_dist** out);
void evm_dist_free(evm_ctx* ctx, evm_dist* d);
int evm_dist_info(const evm_dist* d, int* rank, int* world);
/* local (every rank computes the same): the owner directory.  ids: device,
 * n_owners userId strings of id_len bytes at `stride` (index = global owner
 * id).  Owner g goes to rank murmur3(userId_g) mod world (MurmurHash3_x86_32,
 * seed 0, the murmurhash@2.0.1 of timestamp.ts:87-88) as local id = its rank
 * among that rank's owners in global order.  Afterwards evm_dist_route sends
 * row i to the directory's rank of owner[i], evm_dist_take writes local ids,
 * and evm_dist_gather_roots maps local roots back to global owners.
 * Optional outputs (device): dest[n_owners], local[n_owners]; *n_local (host)
 * = owners this rank serves.  n_owners == 0 removes the directory. */
int evm_dist_directory(evm_ctx* ctx, evm_dist* d, const char* ids, size_t stride, size_t id_len, uint32_t n_owners,
                       uint8_t* dest, uint32_t* local, uint32_t* n_local);
/* collective: every row (device ts[n * stride], stride % 8 == 0; owner[n]
 * global owner ids; optional aux[n], e.g. the cell) goes to rank dest[i]
 * (dest given), the directory's rank of owner[i], or owner[i] % world.  The
 * received rows stay in the context's staging buffer in (source rank,
 * source order) -- the global batch order when each rank's input is its
 * slice of the batch in rank order; *n_recv = their count (host).  48-B rows
 * travel as 32-B packed records (bytes 46-47, padding, arrive as zero)
 * unless some row anywhere in the job is outside the native domain or some
 * rank's rows are not 48-B rows at a 16-B aligned address: then every rank
 * sends raw records and every byte arrives (the ranks agree on the format
 * through the count words; raw records need one stride on every rank, else
 * every rank returns EVM_EINVAL before any data moves).  A row whose
 * destination is out of range is dropped and EVM_EINVAL returned on its
 * rank after the exchange completed. */
int evm_dist_route(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                   const uint32_t* aux, const uint8_t* dest, uint64_t* n_recv);
/* evm_dist_route with flags.  EVM_ROUTE_NO_SRC: the caller will not ask
 * evm_dist_take for source indexes nor call evm_dist_return /
 * evm_dist_split_winners after this route -- with aux == NULL the rows then
 * travel as 24 B instead of 32, when every rank routes so (the ranks agree
 * through the count words): three arrays -- (tc, node), case mask, and the
 * owner as the receiver will use it (its local id when a directory or split
 * is set, else the global id), so evm_dist_ingest reads the owner column as
 * it arrives. */
#define EVM_ROUTE_NO_SRC 1u
/* EVM_ROUTE_KEEP_INPUT (with EVM_ROUTE_NO_SRC): the caller keeps `ts` and
 * `owner` valid and unchanged until the route's last evm_dist_take /
 * evm_dist_ingest.  On a 24-B route this rank's own rows are then neither
 * parsed nor copied by the route (at world 1 without a split: nothing moves at
 * all -- the received rows and owner ids are the caller's as they lie): take
 * copies them from `ts`, ingest parses them there.  A row of them outside the native domain is then found by the
 * ingest (EVM_ENONCANON, flagged), not by the route's format vote. */
#define EVM_ROUTE_KEEP_INPUT 2u
int evm_dist_route_ex(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                      const uint32_t* aux, const uint8_t* dest, uint32_t flags, uint64_t* n_recv);
/* local: the last route's rows into caller buffers (device): out_ts rows of
 * out_stride bytes (out_stride % 8 == 0, out_ts 8-B aligned), out_owner (global ids; local ids with a directory),
 * optional out_aux and out_src (source rank << 32 | index in that rank's
 * input).  group == 0: in receive order; 0 < group <= 64: grouped by local
 * owner (owner / world, or the directory's local id, < group), receive order
 * inside each group, group_off (host, group + 1) the bounds.
 * cap < n_recv: EVM_ECAPACITY (the rows stay staged; take again). */
int evm_dist_take(evm_ctx* ctx, evm_dist* d, uint32_t group, char* out_ts, size_t out_stride, uint32_t* out_owner,
                  uint32_t* out_aux, uint64_t* out_src, uint64_t cap, uint64_t* group_off);
/* local: addMessages of the last route's rows into `store` (its owners =
 * this rank's local owners: the directory's local ids, a split's hot slots)
 * -- exactly evm_server_ingest over what evm_dist_take(group 0) would return
 * (row i of the receive order: id id_base + i, flags[i]; n_recv flags), but
 * packed records are read where they arrived: no 48-B rows are rebuilt and
 * parsed again.  Needs evm_dist_directory (or evm_dist_split).  The route's
 * rows stay staged (evm_dist_take still works after it). */
int evm_dist_ingest(evm_ctx* ctx, evm_dist* d, evm_store* store, uint64_t id_base, uint8_t* flags);
/* rows the last route delivered to this rank (0 before any route / NULL d) */
uint64_t evm_dist_received(const evm_dist* d);
/* collective: every owner's root over all ranks.  This rank's local owners
 * are the owners of trees[0..n_trees) in order (one tree set for all of
 * them, or one single-owner tree per owner): local owner j = global owner
 * j * world + rank, at most ceil(n_global / world) of them -- or, with a
 * directory (n_owners_global == its size), the directory's local ids.
 * root/present: device [n_owners_global]. */
int evm_dist_gather_roots(evm_ctx* ctx, evm_dist* d, const evm_tree* const* trees, uint32_t n_trees,
                          uint32_t n_owners_global, int32_t* root, uint8_t* present);

/* ---- hot owners split over every rank (BASELINE config 5) ----
 * A skewed owner distribution (Zipf 1.2: the top owner ~18 % of all rows)
 * would pin one rank.  A split owner lives on EVERY rank, as local id
 * hot_base + h (h: its index in the hot list), and each of its rows goes to
 * the rank murmur3(its 46 timestamp bytes) mod world picks -- every copy of
 * one (owner, timestamp) meets on one rank, so INSERT OR IGNORE (index.ts:154)
 * and the per-rank Merkle XOR stay exact, and the owner's tree is the XOR
 * merge of its per-rank partial trees (insertIntoMerkleTree is
 * order-independent, merkleTree.test.ts:30-42).  getMessages of a split
 * owner (index.ts:173-202): diff its FULL tree (evm_dist_merge_trees) against
 * the client's, each rank selects its share after that bound
 * (evm_store_select_after with sel_key), evm_dist_merge_select merges the
 * shares in timestamp order.
 *
 * collective: owners with more than `share` x (all rows / world) rows over
 * all ranks -> hot (host, sorted ascending), *n_hot (EVM_ECAPACITY if > cap).
 * owner: device [n] global ids < n_owners_global. */
int evm_dist_hot_owners(evm_ctx* ctx, evm_dist* d, const uint32_t* owner, size_t n, uint32_t n_owners_global,
                        double share, uint32_t* hot, uint32_t cap, uint32_t* n_hot);
/* local (every rank passes the same list): split the listed global owners
 * (host, distinct, < n_owners_global; after evm_dist_directory when there is
 * one, n_owners_global = its size).  Afterwards evm_dist_route sends a split
 * owner's rows by timestamp hash, evm_dist_take writes local ids for every
 * row (hot_base + h for a split owner), and evm_dist_gather_roots XORs the
 * split owners' partial roots (its trees then cover hot_base + n_hot local
 * owners).  *hot_base (host, may be NULL) = the cold local slots per rank.
 * n_hot == 0 removes the split. */
int evm_dist_split(evm_ctx* ctx, evm_dist* d, const uint32_t* hot, uint32_t n_hot, uint32_t n_owners_global,
                   uint32_t* hot_base);
/* collective: the full trees of owners [owner_lo, owner_lo + count) of t:
 * every rank's leaves of them all-gathered on the device and XOR-merged
 * (evm_tree_merge semantics), rebased to owners 0..count-1 -- the same tree
 * on every rank.  (count: the same on every rank.) */
int evm_dist_merge_trees(evm_ctx* ctx, evm_dist* d, const evm_tree* t, uint32_t owner_lo, uint32_t count,
                         evm_tree** out);
/* collective: n_groups selections split over ranks -> one per group, every
 * rank's rows merged in timestamp order (ORDER BY "timestamp", index.ts:101;
 * equal keys: lower rank first).  off: device [n_groups + 1] row bounds into
 * id / key (key: 3 x u64 per row, evm_store_select_after's sel_key; off[0]
 * need not be 0).  Outputs (device, the same on every rank): out_off
 * [n_groups + 1] from 0, out_id[cap]; *n_out = rows (EVM_ECAPACITY if > cap,
 * out_off still written). */
int evm_dist_merge_select(evm_ctx* ctx, evm_dist* d, uint32_t n_groups, const uint64_t* off, const uint64_t* id,
                          const uint64_t* key, uint64_t* out_off, uint64_t* out_id, uint64_t cap, uint64_t* n_out);

/* ---- one owner's applyMessages batch split over the ranks by cell ----------
 * (the client side of config 5).  The LWW decisions of applyMessages.ts:26-131
 * are per cell: route every row with dest = evm_dist_cell_dest (its cell's
 * rank) and the cell as aux, take in receive order (the global batch order),
 * apply on this rank's cells; the global __message PK check (one timestamp in
 * two cells) runs on the rank evm_dist_ts_dest picks (route by it, then
 * evm_cross_cell_check); evm_dist_agree_status combines the statuses;
 * evm_dist_return sends the flags back to the rows' source positions,
 * evm_dist_split_winners maps the winners to global batch indexes, and
 * evm_dist_merge_trees XOR-merges the per-rank partial trees.
 * local: dest[i] = murmur3(row i's 46 timestamp bytes) mod world (device) */
int evm_dist_ts_dest(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, uint8_t* dest);
/* local: dest[i] = the rank of cell[i] (a fixed mix of the id, mod world) */
int evm_dist_cell_dest(evm_ctx* ctx, evm_dist* d, const uint32_t* cell, size_t n, uint8_t* dest);
/* collective: val (device, the last route's received rows in receive order,
 * elem = 1/2/4/8 bytes each) back to the rows' source ranks: out[source
 * index] (device, n_out elements) on every rank. */
int evm_dist_return(evm_ctx* ctx, evm_dist* d, const void* val, uint32_t elem, void* out, size_t n_out);
/* collective: win (device [n_cells]: an index into the last route's receive
 * order, or -1) -> out (device int64 [n_cells], every rank): the global batch
 * index of the winner (the ranks' inputs in rank order) or -1; a cell's
 * winner comes from the one rank that holds the cell. */
int evm_dist_split_winners(evm_ctx* ctx, evm_dist* d, const int32_t* win, uint32_t n_cells, int64_t* out);
/* collective: *max_status = the largest `local` over the ranks */
int evm_dist_agree_status(evm_ctx* ctx, evm_dist* d, int32_t local, int32_t* max_status);

#ifdef __cplusplus
}
#endif
#endif /* EVM_H */
