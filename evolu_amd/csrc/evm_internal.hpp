// Host-side internals shared by the engine's translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/evm.h"
#include "evm_device.hpp"

namespace evm {
struct Info;
}

struct evm_pending;
namespace evm {
struct HostStage;
}

struct evm_ctx {
  int device;
  hipStream_t own;
  hipStream_t stream;
  // kernel timing (evm_prof_*): HIP event pairs per kernel name, on `stream`
  bool prof = false;
  evm::Info* hinfo = nullptr;  // pinned host copy of a call's status record (read_info)
  uint32_t* hland = nullptr;   // pinned landing words (evm::land_words)
  std::string prof_only;  // evm_prof_only: time just this kernel ("" = all)
  int client_path = 0;  // EVM_OPT_CLIENT_PATH
  int server_path = 0;  // EVM_OPT_SERVER_PATH
  int overlap = 1;      // EVM_OPT_OVERLAP: independent checks on a second stream
  int test_fail = 0;       // evm_test_fault (include/evm_test.h; tests only)
  int radix_onesweep = 1;  // EVM_OPT_RADIX: 1 one-sweep radix passes (look-back), 0 histogram + scan + scatter
  int diff_grid = 0;       // EVM_OPT_DIFF_GRID: k_diff workgroups per CU (0: one lane group per owner)
  int select_path = 0;     // EVM_OPT_SELECT_PATH: 0 one-pass keep + rank + emit, 1 keep / scan / emit passes
  int n_cu = 256;          // compute units of the device
  hipStream_t side = nullptr;  // second stream (forked from / joined to `stream` inside a call)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> prof_events;
  std::map<std::string, std::pair<double, uint64_t>> prof_total;  // ms, launches (drained)
  std::vector<hipEvent_t> prof_pool;  // recycled events: no hipEventCreate inside a timed loop
  // persistent hash set for the cross-cell timestamp check (epoch-tagged slots)
  unsigned long long* xtab = nullptr;
  int xtab_lg = 0;
  unsigned xepoch = 0;
  // persistent workspace (Scratch arena)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  size_t ws_top = 0;   // arena bytes in use
  size_t ws_vtop = 0;  // bytes the current call would use (arena + pool overflow)
  size_t ws_need = 0;  // largest ws_vtop seen
  evm_stats stats{};   // allocation counters (evm_get_stats)
  // freed tree / store blocks kept for reuse (stream-ordered on `stream`):
  // a steady-state loop of ingests / applies makes no allocation calls
  std::vector<std::pair<void*, size_t>> blocks;
  std::vector<evm_pending*> pend_pool;  // finished evm_apply_batch_async handles (pinned slot + event kept)
  evm::HostStage* stage = nullptr;  // pinned chunks + copy stream for host <-> device staging (evm_sync.hip)
};

// One MerkleTree per owner, as sorted unique leaves keyed by
// ck = owner << 40 | code (code: 20 base-4 digits, see evm_device.hpp).
//
// Owner o's leaves are [off[o], end[o]).  A compact tree has end = off + 1
// (the owners' ranges back to back, pfx one exclusive prefix XOR over all of
// them).  A GAPPED tree -- what an ingest into an empty store leaves, K5
// having written each owner's leaves where its messages sat in the batch --
// has owner ranges with room between them and pfx exclusive per owner
// (pfx[off[o]] = 0, pfx[end[o]] = the owner's root).  Either way the hash of
// a node is pfx[hi] ^ pfx[lo] over its owner-local range, which is all the
// diff and the roots read; every other reader first calls tree_compact.
struct evm_tree {
  size_t bytes;  // size of the one device block holding the arrays (base = off)
  uint32_t n_owners;
  uint64_t n_leaves;  // leaves (a gapped tree: the sum of its owners' ranges)
  unsigned long long* off;  // [n_owners + 1] leaf range of each owner: [off[o], end[o])
  unsigned long long* end;  // off + 1, or (gapped) its own [n_owners] array
  unsigned long long* ck;   // [n_leaves] (gapped: [cap])
  int32_t* xr;    // [n_leaves] XOR of the hashes whose key ends at the leaf
  int32_t* pfx;   // [n_leaves + 1] exclusive prefix XOR of xr (node hash = range XOR)
  uint64_t cap = 0;     // gapped: leaf slots allocated
  bool gapped = false;
};

namespace evm {

typedef unsigned long long u64;
typedef uint32_t u32;

// Per-call device status block.
struct Info {
  u32 bad;        // some record lacks EVM_META_VALID
  u32 collision;  // cross-cell duplicate timestamp
  u32 minute_min;
  u32 minute_max;
  u64 ck_min;
  u64 ck_max;
  u32 maxlen;  // longest base-3 key
  u32 bad_aux; // an aux id out of range
  u32 fold_overflow;  // dense minute fold not applicable (range too wide / mixed key lengths)
  u32 n_leaves;       // leaves produced by the dense fold
  u32 xc_oversize;    // a hash bucket of the cross-cell check overflowed LDS
  u32 ties;           // tc path: a message's tc equals its cell's running max (node ranks decide)
  u32 xf_redo;        // tc path: the fused check + fold cannot finish (minute span, full bucket, fingerprint match)
};

inline Info info_init() {
  Info h;
  h.bad = 0;
  h.collision = 0;
  h.minute_min = 0xffffffffu;
  h.minute_max = 0;
  h.ck_min = ~0ull;
  h.ck_max = 0;
  h.maxlen = 0;
  h.bad_aux = 0;
  h.fold_overflow = 0;
  h.n_leaves = 0;
  h.xc_oversize = 0;
  h.ties = 0;
  h.xf_redo = 0;
  return h;
}

inline int hip_ok(hipError_t e) {
  if (e == hipSuccess) return EVM_OK;
  return e == hipErrorOutOfMemory ? EVM_ENOMEM : EVM_EDEVICE;
}
#define HIPR(expr)                          \
  do {                                      \
    hipError_t e_ = (expr);                 \
    if (e_ != hipSuccess) return evm::hip_ok(e_); \
  } while (0)

// Per-call scratch: a bump arena in the context's persistent workspace,
// stream-ordered on ctx->stream (calls on one context never overlap on the
// device).  When the arena is short the pool backs the call and the
// outermost Scratch of the next call grows the arena to the size seen, so a
// repeated workload makes no allocation calls at all.
class Scratch {
 public:
  explicit Scratch(evm_ctx* c) : ctx_(c), mark_(c->ws_top), vmark_(c->ws_vtop) {
    if (mark_ == 0 && vmark_ == 0 && ctx_->ws_need > ctx_->ws_bytes) {
      (void)hipStreamSynchronize(ctx_->stream);
      if (ctx_->ws) (void)hipFree(ctx_->ws);
      ctx_->ws = nullptr;
      ctx_->ws_bytes = 0;
      const size_t want = ctx_->ws_need + ctx_->ws_need / 8;
      if (hipMalloc(&ctx_->ws, want) == hipSuccess) ctx_->ws_bytes = want;
      ++ctx_->stats.workspace_regrows;
    }
  }
  ~Scratch() {
    ctx_->ws_top = mark_;
    ctx_->ws_vtop = vmark_;
    for (void* p : ptrs_) (void)hipFreeAsync(p, ctx_->stream);
  }
  template <typename T>
  T* alloc(size_t n) {
    const size_t bytes = (sizeof(T) * (n ? n : 1) + 255) & ~(size_t)255;
    ctx_->ws_vtop += bytes;
    if (ctx_->ws_vtop > ctx_->ws_need) ctx_->ws_need = ctx_->ws_vtop;
    if (ctx_->ws && ctx_->ws_top + bytes <= ctx_->ws_bytes && ctx_->ws_top + bytes == ctx_->ws_vtop) {
      void* p = static_cast<char*>(ctx_->ws) + ctx_->ws_top;
      ctx_->ws_top += bytes;
      return static_cast<T*>(p);
    }
    void* p = nullptr;
    if (hipMallocAsync(&p, bytes, ctx_->stream) != hipSuccess) return nullptr;
    ++ctx_->stats.scratch_pool_allocs;
    ctx_->stats.scratch_pool_bytes += bytes;
    ptrs_.push_back(p);
    return static_cast<T*>(p);
  }

 private:
  evm_ctx* ctx_;
  size_t mark_, vmark_;
  std::vector<void*> ptrs_;
};

// Records a start/stop event pair around one launch when profiling is on.
class ProfScope {
 public:
  ProfScope(evm_ctx* c, const char* name, hipStream_t s = nullptr) : ctx_(c), name_(name), s_(s ? s : c->stream) {
    if (!ctx_->prof || (!ctx_->prof_only.empty() && ctx_->prof_only != name_)) return;
    a_ = take();
    b_ = take();
    if (a_ && b_) {
      (void)hipEventRecord(a_, s_);
    } else {
      if (a_) ctx_->prof_pool.push_back(a_);
      if (b_) ctx_->prof_pool.push_back(b_);
      a_ = b_ = nullptr;
    }
  }
  ~ProfScope() {
    if (a_ && b_) {
      (void)hipEventRecord(b_, s_);
      ctx_->prof_events[name_].push_back({a_, b_});
    }
  }

 private:
  hipEvent_t take() {
    if (!ctx_->prof_pool.empty()) {
      hipEvent_t e = ctx_->prof_pool.back();
      ctx_->prof_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
  }
  evm_ctx* ctx_;
  const char* name_;
  hipStream_t s_;
  hipEvent_t a_ = nullptr, b_ = nullptr;
};

// Work forked onto ctx->side after everything queued on ctx->stream so far;
// the destructor joins it back (ctx->stream waits for it) on every path out.
class SideFork {
 public:
  explicit SideFork(evm_ctx* c) : ctx_(c) {
    on_ = ctx_->overlap && ctx_->side && hipEventRecord(ctx_->ev_fork, ctx_->stream) == hipSuccess &&
          hipStreamWaitEvent(ctx_->side, ctx_->ev_fork, 0) == hipSuccess;
  }
  hipStream_t stream() const { return on_ ? ctx_->side : ctx_->stream; }
  void join() {
    if (on_) {
      (void)hipEventRecord(ctx_->ev_join, ctx_->side);
      (void)hipStreamWaitEvent(ctx_->stream, ctx_->ev_join, 0);
      on_ = false;
    }
  }
  // the side work stays unjoined (the caller ordered what depends on it itself)
  void detach() { on_ = false; }
  ~SideFork() { join(); }

 private:
  evm_ctx* ctx_;
  bool on_ = false;
};

// Every kernel launch goes through KLAUNCH (needs `ctx` in scope).
#define KLAUNCH(kern, grid, block, ...)                                  \
  do {                                                                   \
    evm::ProfScope ps_(ctx, #kern);                                      \
    hipLaunchKernelGGL(kern, grid, block, 0, ctx->stream, __VA_ARGS__); \
  } while (0)

// Same, with dynamic LDS bytes.
#define KLAUNCH_LDS(kern, grid, block, lds, ...)                            \
  do {                                                                     \
    evm::ProfScope ps_(ctx, #kern);                                        \
    hipLaunchKernelGGL(kern, grid, block, lds, ctx->stream, __VA_ARGS__); \
  } while (0)

enum OwnerMode { OWNER_ZERO = 0, OWNER_AUX = 1, OWNER_CELL = 2 };

inline int grid_for(size_t n, int threads, int cap = 8192) {
  size_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > (size_t)cap) g = cap;
  return (int)g;
}

inline int ceil_log2(size_t x) {
  int k = 0;
  while (((size_t)1 << k) < x) ++k;
  return k;
}

// Small device values to the host in ONE launch and one synchronisation: a
// kernel stores the 4-B words into pinned host memory (no copy-engine blit
// per value, no pageable staging); up to LAND_MAX words per call.
constexpr int LAND_MAX = 32;
struct LandList {
  const uint32_t* src[LAND_MAX];
  void* dst[LAND_MAX];
  int n = 0;
  // `bytes` (a multiple of 4) at dev -> host
  void add(const void* dev, void* host, size_t bytes) {
    for (size_t k = 0; k < bytes / 4 && n < LAND_MAX; ++k, ++n) {
      src[n] = static_cast<const uint32_t*>(dev) + k;
      dst[n] = static_cast<uint32_t*>(host) + k;
    }
  }
};
int land_words(evm_ctx* ctx, const LandList& l);
// Zero up to ZERO_MAX small device buffers (a multiple of 4 bytes each) in one launch.
constexpr int ZERO_MAX = 8;
struct ZeroList {
  uint32_t* p[ZERO_MAX];
  uint32_t words[ZERO_MAX];
  uint32_t fill[ZERO_MAX];
  int n = 0;
  void add(void* dev, size_t bytes, uint32_t value = 0) {
    p[n] = static_cast<uint32_t*>(dev);
    words[n] = (uint32_t)(bytes / 4);
    fill[n] = value;
    ++n;
  }
};
int zero_small(evm_ctx* ctx, const ZeroList& z);

inline int read_info(evm_ctx* ctx, const Info* dev, Info* host) {
  static_assert(sizeof(Info) % 4 == 0 && sizeof(Info) / 4 <= LAND_MAX, "Info lands as words");
  LandList l;
  l.add(dev, host, sizeof(Info));
  return land_words(ctx, l);
}

// the initial record is written by a one-thread kernel (launch argument), not
// copied from pageable host memory
int launch_info_set(evm_ctx* ctx, Info* d, const Info& h);

inline int new_info(evm_ctx* ctx, Scratch& S, Info** out) {
  Info* d = S.alloc<Info>(1);
  if (!d) return EVM_ENOMEM;
  int st = launch_info_set(ctx, d, info_init());
  if (st) return st;
  *out = d;
  return EVM_OK;
}

// Device blocks for trees and stores, recycled through ctx->blocks (best fit,
// at most BLOCK_CACHE kept); *bytes is updated to the block's real size.
void* block_alloc(evm_ctx* ctx, size_t* bytes);
void block_free(evm_ctx* ctx, void* p, size_t bytes);
void block_cache_clear(evm_ctx* ctx);
}  // namespace evm
void evm_pending_pool_clear(evm_ctx* ctx);  // evm_client.hip
void evm_host_stage_free(evm_ctx* ctx);     // evm_sync.hip
namespace evm {

// shared launchers (evm_engine.hip)
int launch_iota(evm_ctx* ctx, u32* v, size_t n);
int launch_sel(evm_ctx* ctx, const uint8_t* flags, uint8_t mask, size_t n, u32* sel);
int launch_fold_prep(evm_ctx* ctx, const evm_rec* rec, const uint8_t* flags, uint8_t sel_mask, const u32* pos,
                     int owner_mode, const u32* cell_owner, size_t n, u64* ck, u32* h, Info* info);
int launch_diff(evm_ctx* ctx, const evm_tree* a, const evm_tree* b, int64_t* millis);
void tree_destroy(evm_ctx* ctx, evm_tree* t);  // stream-ordered release

int launch_pack(evm_ctx* ctx, const char* ts, size_t stride, size_t n, const u32* aux, u32 aux_limit, evm_rec* out,
                Info* info, u32* minute_out = nullptr);
// 48-B rows (16-B aligned): the minutes and the pack's checks, no records
int launch_minutes(evm_ctx* ctx, const char* ts, size_t n, const u32* aux, u32 aux_limit, Info* info,
                   u32* minute_out);
template <typename T, template <typename> class Op>
int scan_exclusive(evm_ctx* ctx, Scratch& S, const T* in, size_t n, T* out, T* total_dev);
// k <= 3 exclusive add-scans of one length n (one launch when n is small)
int scan_exclusive_cols(evm_ctx* ctx, Scratch& S, int k, const uint32_t* const* ins, size_t n, uint32_t* const* outs,
                        uint32_t* const* tots);
template <typename K>
int radix_sort_pairs(evm_ctx* ctx, Scratch& S, K*& keys, u32*& vals, size_t n, int lo_bit, int hi_bit);
int reduce_runs(evm_ctx* ctx, Scratch& S, const u64* ck, const int32_t* h, size_t m, u64* out_ck, int32_t* out_xr,
                uint64_t* out_count);
int tree_finalize(evm_ctx* ctx, Scratch& S, u32 n_owners, const u64* ck, const int32_t* xr, uint64_t L, evm_tree** out);
// An uninitialised tree with room for `cap` leaves (n_leaves = cap until the
// caller sets it); the caller's kernels fill off, ck, xr and pfx.
int tree_alloc_cap(evm_ctx* ctx, u32 n_owners, uint64_t cap, evm_tree** out);
// Same, with the leaf count still on the device (*d_count <= cap): the tree is
// built without a host round trip; the caller sets (*out)->n_leaves after its
// one synchronisation.
int tree_finalize_dev(evm_ctx* ctx, Scratch& S, u32 n_owners, const u64* ck, const int32_t* xr, const u32* d_count,
                      uint64_t cap, evm_tree** out);
int merge_into_tree(evm_ctx* ctx, Scratch& S, const evm_tree* in, u32 n_owners, const u64* nck, const int32_t* nxr,
                    uint64_t L1, evm_tree** out);
// A gapped tree with room for `cap` leaves (off, end, ck, xr, pfx all filled by
// the caller's kernels; n_leaves set by the caller).
int tree_alloc_gapped(evm_ctx* ctx, u32 n_owners, uint64_t cap, evm_tree** out);
// A gapped tree made compact in place (same object; nothing to do for a
// compact one).  Every reader but the diff and the roots calls it first.
int tree_compact(evm_ctx* ctx, const evm_tree* t);
// evm_json_dev.hip: per requested owner its tree JSON's length (device len[n];
// *bad |= 1 for an owner out of range) and the plan the emit follows (arrays
// in S); the texts written at out + off[j]
// A client tree text of len bytes has at most len / 14 nodes (`"0":{"hash":0}`
// is the shortest non-root node): its leaf slots in a parsed tree, with the
// owner's prefix slot.
constexpr u32 JP_MIN_NODE = 14;
__host__ __device__ inline u64 json_slot_bound(u64 len) { return len / JP_MIN_NODE + 2; }
int json_tree_slots(evm_ctx* ctx, Scratch& S, u32 n_owners, const u64* len, u64** slots);
int json_tree_parse(evm_ctx* ctx, u32 n_owners, const uint8_t* json, const u64* at, const u64* len, const u64* slots,
                    int32_t* status, evm_tree* t, u64* nl);

struct JsonPlan {
  uint32_t n = 0;             // (the texts are placed by the caller from the lengths)
  uint16_t* plen = nullptr;   // each leaf's piece length, by leaf slot (in the caller's Scratch)
};
int json_plan(evm_ctx* ctx, Scratch& S, const evm_tree* t, const uint32_t* owners, uint32_t n, uint64_t* len,
              uint32_t* bad, JsonPlan* plan);
int json_emit(evm_ctx* ctx, const evm_tree* t, const uint32_t* owners, uint32_t n, const JsonPlan& plan,
              const uint64_t* off, char* out);
int fold_into_tree(evm_ctx* ctx, Scratch& S, const evm_tree* in, u32 n_owners, u64* ck, u32* h, size_t m,
                   const Info& host_info, evm_tree** out);
// evm_pb_encode_responses_dev in one pass: out_for(total) gives the output
// buffer (null: sizes only) once the sizes are known (evm_wire_dev.hip).
// pre: the tree texts' plan made by the caller (json_plan over the same
// owners: lengths pre_jlen[n], its out-of-range flag pre_bad), already on or
// joined to the context's stream
int encode_responses_dev(evm_ctx* ctx, uint32_t n, const evm_tree* tree, const uint32_t* owners,
                         const uint64_t* osel_off, const uint64_t* osel_id, const uint8_t* skip, uint32_t n_seg,
                         const uint64_t* seg_base, const uint64_t* const* seg_row, const char* const* seg_ts,
                         size_t stride, const uint64_t* const* seg_coff, const uint8_t* const* seg_content,
                         const std::function<uint8_t*(uint64_t)>& out_for, uint64_t* out_off, uint64_t* total,
                         const JsonPlan* pre = nullptr, const uint64_t* pre_jlen = nullptr,
                         const uint32_t* pre_bad = nullptr);

// A route's received packed records, read where they lie (evm_dist_ingest):
// the parsed form of each 46-B timestamp -- tc, node, case mask |
// EVM_META_VALID -- from which format_ts46 rebuilds the string exactly.
// Record i is in the receive buffer, except this rank's own rows
// [self_lo, self_hi), which never left the send buffer.  32-B records (rec,
// self non-null): tc u64 at 0, node u64 at 8, the mask word at moff.  Narrow
// routes (tn non-null): (tc, node) 16 B per row in one array, the mask words
// in another.
struct WireSrc {
  const char* rec;
  const char* self;
  u64 self_lo, self_hi;
  u32 rb, moff;
  const char* tn;
  const char* self_tn;
  const u32* cm;
  const u32* self_cm;
  // EVM_ROUTE_KEEP_INPUT: this rank's own rows never left the caller's rows
  // -- received row i in [self_lo, self_hi) is ts row self_idx[i - self_lo]
  const uint8_t* self_ts = nullptr;
  u32 self_stride = 0;
  const u32* self_idx = nullptr;
};
__device__ __forceinline__ bool wire_self_row(const WireSrc& w, size_t i) {
  return w.self_ts && i >= w.self_lo && i < w.self_hi;
}
// an own row of a keep-input route, as its 12 little-endian words (bytes 46-47 zero)
__device__ __forceinline__ void wire_self_words(const WireSrc& w, size_t i, u32 (&x)[12]) {
  const size_t k = w.self_idx ? (size_t)w.self_idx[i - w.self_lo] : i - w.self_lo;  // (null: the rows as they lie)
  const uint4* row = reinterpret_cast<const uint4*>(w.self_ts + k * w.self_stride);
  const uint4 a = row[0], b = row[1], c = row[2];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w & 0xffffu;
}
__device__ __forceinline__ void wire_load(const WireSrc& w, size_t i, u64* tc, u64* node, u32* cm) {
  const bool mine = i >= w.self_lo && i < w.self_hi;
  if (w.self_ts && mine) {  // (parsed here: the same words the route would have sent)
    u32 x[12];
    wire_self_words(w, i, x);
    const Parsed p = parse_ts46(x);
    *tc = p.tc;
    *node = p.node;
    *cm = p.meta & (EVM_META_CASEMASK | EVM_META_VALID);
    return;
  }
  if (w.tn) {
    const uint4 v = *reinterpret_cast<const uint4*>(mine ? w.self_tn + (i - w.self_lo) * 16 : w.tn + i * 16);
    *tc = (u64)v.x | ((u64)v.y << 32);
    *node = (u64)v.z | ((u64)v.w << 32);
    *cm = mine ? w.self_cm[i - w.self_lo] : w.cm[i];
    return;
  }
  const char* p = mine ? w.self + (i - w.self_lo) * w.rb : w.rec + i * w.rb;
  const uint2* q = reinterpret_cast<const uint2*>(p);
  const uint2 a = q[0], b = q[1];
  *tc = (u64)a.x | ((u64)a.y << 32);
  *node = (u64)b.x | ((u64)b.y << 32);
  *cm = *reinterpret_cast<const u32*>(p + w.moff);
}
// addMessages over received records (evm_server.hip): owner[i] = the local
// owner of record i; ids id_base + i, flags[i] -- as evm_server_ingest over
// the rows evm_dist_take would rebuild, without rebuilding them
int server_ingest_wire(evm_ctx* ctx, evm_store* s, const WireSrc& w, size_t n, const u32* owner, uint64_t id_base,
                       uint8_t* flags);

}  // namespace evm
