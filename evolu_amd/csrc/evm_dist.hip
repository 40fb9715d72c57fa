// Owner sharding across GPUs: the evm_dist_* C ABI.
//
// One process per GPU.  Owners are independent in the whole hot path (each is
// its own client database for applyMessages.ts:26-131; the server keys rows
// and trees by userId, apps/server/src/index.ts:64-75), so every owner lives
// on one rank and the only exchanges are
//
//   * evm_dist_route: messages to their owner's rank.  A stable partition by
//     destination packs wire records into one send buffer; one all-to-all of
//     the G per-destination counts, then one group of sends/receives moves
//     the records -- each peer's records contiguous, so the receive buffer is
//     in (source rank, source order) = global batch order, which the
//     reference's first-occurrence rules depend on.
//   * evm_dist_take: the received rows out of the staging buffer into the
//     caller's arrays, optionally grouped by local owner (a second stable
//     partition on the device) so each owner's rows are one contiguous
//     applyMessages batch.
//   * evm_dist_gather_roots: an all-gather of the per-owner roots (no XOR
//     reduction is needed: every unsplit owner lives on one rank).
//
// Which rank serves an owner: owner % world by default, or -- once
// evm_dist_directory has hashed the owners' userId strings -- murmur3(userId)
// mod world, with dense local ids per rank.
//
// Collectives agree on failure: a rank that fails locally (bad arguments,
// allocation) still joins every collective of the call with zero counts and
// an error bit in its count words, so no peer waits forever in a receive;
// every rank then returns an error.
//
// Transports: RCCL (opened at run time with dlopen: inside a process that
// already has it -- PyTorch's copy -- the same instance is used), or an
// in-process loopback hub: `world` contexts driven by `world` host threads,
// device-to-device copies instead of xGMI.  The loopback runs the same
// partition, count exchange, grouping and gather code as RCCL, so a world-2
// exchange is testable on one GPU.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

namespace {

// ------------------------------------------------------------------ RCCL (dlopen)
struct Rccl {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllToAll) all_to_all = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
};

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    Rccl t;
    t.h = h;
    bool ok = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      ok = ok && f;
    };
    sym(t.get_unique_id, "ncclGetUniqueId");
    sym(t.comm_init_rank, "ncclCommInitRank");
    sym(t.comm_destroy, "ncclCommDestroy");
    sym(t.all_to_all, "ncclAllToAll");
    sym(t.all_gather, "ncclAllGather");
    sym(t.send, "ncclSend");
    sym(t.recv, "ncclRecv");
    sym(t.group_start, "ncclGroupStart");
    sym(t.group_end, "ncclGroupEnd");
    if (ok) r = t;
  });
  return r.h ? &r : nullptr;
}

static_assert(sizeof(ncclUniqueId) == EVM_DIST_ID_BYTES, "unique id size");

constexpr u32 MAX_BUCKETS = 64;

// ------------------------------------------------------------------ transports
// The three collectives the exchange needs, stream ordered on the caller's
// stream.  Counts and offsets are host arrays (RCCL's point-to-point calls
// take host counts).
struct Transport {
  virtual ~Transport() = default;
  // every rank sends word p of `send` to rank p and receives rank p's word
  // `rank` into recv[p] (G words each way, device)
  virtual int all_to_all_u64(const u64* send, u64* recv, hipStream_t s) = 0;
  // bytes [soff[p], soff[p] + slen[p]) of sbase to rank p; rank p's bytes
  // for this rank into rbase + roff[p] (rlen[p] of them)
  virtual int exchange(const char* sbase, const uint64_t* soff, const uint64_t* slen, char* rbase,
                       const uint64_t* roff, const uint64_t* rlen, hipStream_t s) = 0;
  // rank p's `per` words into all + p * per
  virtual int all_gather_u64(const u64* mine, u64* all, size_t per, hipStream_t s) = 0;
};

struct RcclTransport final : Transport {
  const Rccl* r = nullptr;
  ncclComm_t comm = nullptr;
  int world = 1;
  ~RcclTransport() override {
    if (comm) r->comm_destroy(comm);
  }
  int all_to_all_u64(const u64* send, u64* recv, hipStream_t s) override {
    return r->all_to_all(send, recv, 1, ncclUint64, comm, s) == ncclSuccess ? EVM_OK : EVM_EDIST;
  }
  int exchange(const char* sbase, const uint64_t* soff, const uint64_t* slen, char* rbase, const uint64_t* roff,
               const uint64_t* rlen, hipStream_t s) override {
    // transfers in pieces of at most CHUNK bytes (a 4 GiB self-send arrived
    // corrupted in one call); both sides cut a peer's bytes alike, and
    // point-to-point calls to one peer match in issue order
    constexpr uint64_t CHUNK = 1ull << 29;
    if (r->group_start() != ncclSuccess) return EVM_EDIST;
    int st = EVM_OK;
    // (a zero-length transfer is skipped on both sides alike: the counts agree)
    for (int p = 0; p < world; ++p) {
      for (uint64_t o = 0; o < slen[p];) {
        const uint64_t k = std::min<uint64_t>(CHUNK, slen[p] - o);
        if (r->send(sbase + soff[p] + o, k, ncclUint8, p, comm, s) != ncclSuccess) st = EVM_EDIST;
        o += k;
      }
      for (uint64_t o = 0; o < rlen[p];) {
        const uint64_t k = std::min<uint64_t>(CHUNK, rlen[p] - o);
        if (r->recv(rbase + roff[p] + o, k, ncclUint8, p, comm, s) != ncclSuccess) st = EVM_EDIST;
        o += k;
      }
    }
    if (r->group_end() != ncclSuccess) st = EVM_EDIST;  // always closed, whatever failed inside
    return st;
  }
  int all_gather_u64(const u64* mine, u64* all, size_t per, hipStream_t s) override {
    return r->all_gather(mine, all, per, ncclUint64, comm, s) == ncclSuccess ? EVM_OK : EVM_EDIST;
  }
};

}  // namespace

// In-process rendezvous of `world` contexts (one host thread each).
struct evm_dist_hub {
  int world = 1;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  struct Post {
    const char* p = nullptr;
    const uint64_t* off = nullptr;
    const uint64_t* len = nullptr;
  };
  Post post[MAX_BUCKETS];
  bool aborted = false;
  // false once the hub is aborted (a rank's thread died): nobody waits for it
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
    }
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

namespace {

// Each collective: the rank's inputs are complete (stream synchronised), it
// posts them, all ranks meet, each copies what it receives from the peers'
// posted buffers on its own stream, synchronises, and all meet again before
// anyone may reuse a buffer.
struct LoopTransport final : Transport {
  evm_dist_hub* hub = nullptr;
  int rank = 0, world = 1;
  // post -> meet -> copy (copy(p) for every peer p) -> synchronise -> meet
  template <typename F>
  int collective(const char* p, const uint64_t* off, const uint64_t* len, hipStream_t s, F copy) {
    int st = hip_ok(hipStreamSynchronize(s));
    hub->post[rank] = {p, off, len};
    if (!hub->barrier()) return EVM_EDIST;
    for (int q = 0; q < world && !st; ++q) st = copy(q);
    const int st2 = hip_ok(hipStreamSynchronize(s));
    if (!hub->barrier()) return EVM_EDIST;
    return st ? st : st2;
  }
  int all_to_all_u64(const u64* send, u64* recv, hipStream_t s) override {
    return collective(reinterpret_cast<const char*>(send), nullptr, nullptr, s, [&](int p) {
      return hip_ok(hipMemcpyAsync(recv + p, reinterpret_cast<const u64*>(hub->post[p].p) + rank, sizeof(u64),
                                   hipMemcpyDeviceToDevice, s));
    });
  }
  int exchange(const char* sbase, const uint64_t* soff, const uint64_t* slen, char* rbase, const uint64_t* roff,
               const uint64_t* rlen, hipStream_t s) override {
    return collective(sbase, soff, slen, s, [&](int p) {
      const evm_dist_hub::Post& q = hub->post[p];
      if (q.len[rank] != rlen[p]) return (int)EVM_EDIST;  // the peer sends another size than the counts said
      if (!rlen[p]) return (int)EVM_OK;
      return hip_ok(hipMemcpyAsync(rbase + roff[p], q.p + q.off[rank], rlen[p], hipMemcpyDeviceToDevice, s));
    });
  }
  int all_gather_u64(const u64* mine, u64* all, size_t per, hipStream_t s) override {
    return collective(reinterpret_cast<const char*>(mine), nullptr, nullptr, s, [&](int p) {
      return hip_ok(
          hipMemcpyAsync(all + (size_t)p * per, hub->post[p].p, per * sizeof(u64), hipMemcpyDeviceToDevice, s));
    });
  }
};

// ------------------------------------------------------------------ kernels
constexpr int DT = 256;               // threads per partition block
constexpr int DROUNDS = 16;           // rows per thread per block
constexpr u32 DTILE = DT * DROUNDS;   // rows per block
constexpr size_t META = 16;           // raw records: owner u32, aux u32, source index u32, pad
constexpr size_t PACKED = 32;         // packed records (48-B timestamp rows): tc, node, owner, aux, index, case|valid
constexpr size_t NARROW = 24;         // bytes per row without aux / source index (EVM_ROUTE_NO_SRC), as three
                                      // arrays: (tc, node) 16 B, case|valid 4 B, the receiver's owner id 4 B
enum { FMT_RAW = 0, FMT_PACKED = 1, FMT_NARROW = 2, FMT_ST8 = 4 /* RECV: rebuilt rows with 8-B stores */ };
constexpr u32 PK_VALID = 1u << 16;
// count words exchanged per route: the row count in the low bits, flags on top
constexpr u64 CNT_ERR = 1ull << 63;      // the sending rank failed locally (nothing is exchanged)
constexpr u64 CNT_INVALID = 1ull << 62;  // the sending rank holds a row outside the native domain
constexpr u64 CNT_RAW = 1ull << 61;      // the sending rank cannot send packed records (its stride / alignment)
constexpr u64 CNT_WIDE = 1ull << 60;     // the sending rank needs aux / source indexes: no narrow records
constexpr u64 CNT_MASK = (1ull << 48) - 1;
constexpr int CNT_STRIDE_SHIFT = 48;       // stride / 8 in bits 48..57: raw records need one stride on every rank
constexpr u64 CNT_STRIDE_MAX = 1023;
// d->cnt layout (u64 words, mirrored in pinned host memory)
constexpr u32 W_SEND = 0;                      // [64] send counts
constexpr u32 W_RECV = MAX_BUCKETS;            // [64] receive counts
constexpr u32 W_ROFF = 2 * MAX_BUCKETS;        // [65] receive offsets (rows)
constexpr u32 W_AGREE_S = 3 * MAX_BUCKETS + 8; // [64] agreement words sent
constexpr u32 W_AGREE_R = 4 * MAX_BUCKETS + 8; // [64] agreement words received
constexpr u32 W_BAD = 5 * MAX_BUCKETS + 8;     // the local flags: [0] bad destination, [1] invalid row
constexpr u32 W_GS = 5 * MAX_BUCKETS + 16;     // [2] (status, value) gathered
constexpr u32 W_GR = 5 * MAX_BUCKETS + 18;     // [2 * 64] every rank's (status, value)
constexpr u32 CNT_WORDS = 7 * MAX_BUCKETS + 24;

// Routing of row i.  SEND: the destination rank -- the caller's dest, a hash
// of the row's timestamp for a split (hot) owner, the directory's rank of the
// owner, or owner % world.  RECV (wire records, owner at byte `ooff`): the
// local owner -- hot_base + hot index for a split owner, the directory's local
// id, or owner / world.  >= B: out of range (reported, not routed).
constexpr u32 HOT_NONE = 0xffffffffu;
struct Route {
  const u32* owner;
  const uint8_t* dest;
  const uint8_t* dir_dest;   // directory: rank of every global owner
  const u32* dir_local;      // directory: local id of every global owner on its rank
  u32 n_dir;
  u32 world;
  const u32* hot;            // split: hot index of every global owner (HOT_NONE: not split)
  u32 n_hot_tab;             // global owners the table covers
  u32 hot_base;              // local id of hot owner 0 on every rank
  const char* ts;            // SEND: the rows (a split owner's rows go by timestamp hash)
  size_t stride;
  // RECV: this rank's rows to itself never travel -- received rows
  // [self_lo, self_hi) are read from the send buffer at self_rec
  const char* self_rec;
  u64 self_lo, self_hi;
  // narrow routes travel as three arrays (SoA): (tc, node) 16 B, case mask |
  // valid 4 B, and the owner 4 B -- the receiver's local id when a directory
  // or split is set (so the received owner column is the store's owner array
  // as it arrives), else the global id.  RECV: the received arrays (the owner
  // one contiguous, this rank's own part copied in) and this rank's own rows'
  // (tc, node) and masks in the send buffer.
  const char* soa_a;
  const u32* soa_b;
  const u32* soa_c;
  const char* self_a;
  const u32* self_b;
  // EVM_ROUTE_KEEP_INPUT on a narrow route.  SEND: rows of bucket keep_me
  // are not parsed or copied; their input index goes to self_idx (from the
  // bucket's first slot).  RECV: own row i is ts row self_idx[i - self_lo].
  u32 keep_me;
  u32* self_idx;
  const char* self_ts;
  size_t self_stride;
};
constexpr u32 NO_KEEP = 0xffffffffu;

// received record i: the staging buffer, or this rank's own rows in the send buffer
__device__ __forceinline__ const char* recv_rec(const Route& R, const char* rec, size_t rb, size_t i) {
  return (i >= R.self_lo && i < R.self_hi) ? R.self_rec + (i - R.self_lo) * rb : rec + i * rb;
}
__device__ __forceinline__ bool is_self(const Route& R, size_t i) { return i >= R.self_lo && i < R.self_hi; }
// a narrow route's received row i: (tc, node) and the case mask | valid word
__device__ __forceinline__ uint4 narrow_tn(const Route& R, size_t i) {
  return *reinterpret_cast<const uint4*>(is_self(R, i) ? R.self_a + (i - R.self_lo) * 16 : R.soa_a + i * 16);
}
__device__ __forceinline__ u32 narrow_cm(const Route& R, size_t i) {
  return is_self(R, i) ? R.self_b[i - R.self_lo] : R.soa_b[i];
}

// The timestamp-hash rank of a row (murmur3 of its 46 bytes: equal strings,
// equal ranks -- every copy of one (owner, timestamp) meets on one rank, so
// INSERT OR IGNORE and the Merkle XOR stay exact per rank).  stride % 8 == 0.
__device__ __forceinline__ u32 ts_rank(const char* row, u32 world) {
  const uint2* q = reinterpret_cast<const uint2*>(row);
  u32 w[12];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint2 v = q[k];
    w[2 * k] = v.x;
    w[2 * k + 1] = v.y;
  }
  w[11] &= 0xffffu;
  return murmur3_46(w) % world;
}

__device__ __forceinline__ bool is_hot(const Route& R, u32 o) {
  return R.hot && o < R.n_hot_tab && R.hot[o] != HOT_NONE;
}

__device__ __forceinline__ u32 local_of(const Route& R, u32 o) {
  if (is_hot(R, o)) return R.hot_base + R.hot[o];
  if (R.dir_local) return o < R.n_dir ? R.dir_local[o] : 0xffffffffu;
  return o / R.world;
}

template <int MODE>
__device__ __forceinline__ u32 bucket_of(size_t i, const Route& R, const char* rec, size_t rb, size_t ooff) {
  if (MODE == 0) {
    if (R.dest) return R.dest[i];
    const u32 o = R.owner[i];
    if (is_hot(R, o)) return ts_rank(R.ts + i * R.stride, R.world);
    if (R.dir_dest) return o < R.n_dir ? (u32)R.dir_dest[o] : 0xffffffffu;
    return o % R.world;
  }
  if (R.soa_c) {  // narrow: the owner column arrived as the sender wrote it
    const u32 c = R.soa_c[i];
    return (R.dir_local || R.hot) ? c : c / R.world;
  }
  const u32 o = *reinterpret_cast<const u32*>(recv_rec(R, rec, rb, i) + ooff);
  return local_of(R, o);
}
enum { SEND = 0, RECV = 1 };

// Packed wire form of a 48-B timestamp row: the parsed (tc, node, case mask)
// -- 16 B instead of 46 -- from which the receiver rebuilds the identical
// string with format_ts46 (a canonical timestamp is a function of them,
// timestamp.ts:43-55).  Only a route whose rows are ALL in the native domain
// travels packed; one row outside it anywhere in the job sends every rank's
// rows raw.

// lanes holding the same bucket id (bits = ceil(log2 B) ballots)
__device__ __forceinline__ u64 match_bucket(u32 b, bool active, int bits) {
  u64 peers = __ballot(active);
  for (int k = 0; k < bits; ++k) {
    const bool bit = (b >> k) & 1u;
    const u64 bal = __ballot(bit);
    peers &= bit ? bal : ~bal;
  }
  return active ? peers : 0ull;
}

// per-block bucket counts, bucket-major ([b * nblocks + block]): their
// exclusive scan is every (bucket, block)'s first output slot, stable.  The
// lanes of one bucket add once per wave (few buckets: a per-row LDS atomic
// would serialise on one address -- at world 1 every row is bucket 0)
template <int MODE>
__global__ __launch_bounds__(DT) void k_dist_count(Route R, const char* __restrict__ rec, size_t rb, size_t ooff,
                                                   size_t n, u32 B, int bits, u32 nblocks, u32* __restrict__ counts,
                                                   u32* __restrict__ bad) {
  __shared__ u32 c[MAX_BUCKETS];
  if (threadIdx.x < MAX_BUCKETS) c[threadIdx.x] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * DTILE;
  const u64 lt = lanemask_lt();
  bool oob = false;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    const u32 b = i < n ? bucket_of<MODE>(i, R, rec, rb, ooff) : 0u;
    const bool act = i < n && b < B;
    oob |= i < n && b >= B;
    const u64 peers = match_bucket(b, act, bits);
    if (act && (peers & lt) == 0) atomicAdd(&c[b], (u32)__popcll(peers));
  }
  __syncthreads();
  if (threadIdx.x < B) counts[(size_t)threadIdx.x * nblocks + blockIdx.x] = c[threadIdx.x];
  if (__ballot(oob) && __lane_id() == 0) atomicOr(bad, 1u);
}


// Stable slot of this thread's row among the rows of its bucket: rows of a
// block in order, ranked within the block with wave ballots + a 4-wave prefix
// in LDS, placed after the (bucket, block) slot the scan gave.  Every thread
// of the block calls it once per round.
struct Ranker {
  u32 run[MAX_BUCKETS];
  u32 wcnt[2][DT / 64][MAX_BUCKETS];  // by round parity: a wave clears its row of round r + 1
                                      // while wave 0 may still sum round r's
};
__device__ __forceinline__ u32 rank_slot(Ranker& L, int r, u32 b, bool act, u32 B, int bits) {
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  u32(*wc)[MAX_BUCKETS] = L.wcnt[r & 1];
  wc[wv][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  const u64 peers = match_bucket(b, act, bits);
  const u64 lt = lanemask_lt();
  if (act && (peers & lt) == 0) wc[wv][b] = (u32)__popcll(peers);
  __syncthreads();
  u32 p = 0;
  if (act) {
    p = L.run[b] + (u32)__popcll(peers & lt);
    for (int w = 0; w < wv; ++w) p += wc[w][b];
  }
  __syncthreads();
  if (threadIdx.x < B) {
    u32 t = 0;
    for (int w = 0; w < DT / 64; ++w) t += wc[w][threadIdx.x];
    L.run[threadIdx.x] += t;
  }
  return p;
}

__device__ __forceinline__ void copy_row(char* __restrict__ dst, const char* __restrict__ src, size_t bytes) {
  // stride % 8 == 0 (checked on the host); 16-B accesses when both ends allow
  if (bytes == 48 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4 a = s[0], b = s[1], c = s[2];
    d[0] = a;
    d[1] = b;
    d[2] = c;
    return;
  }
  const u64* s = reinterpret_cast<const u64*>(src);
  u64* d = reinterpret_cast<u64*>(dst);
  for (size_t k = 0; k < bytes / 8; ++k) d[k] = s[k];
}

// Stable scatter.  offs == nullptr: no partition (row i -> slot i).
//   SEND: caller rows -> wire records (packed, or ts | owner, aux, index);
//         a row outside the native domain sets *invalid (packed only)
//   RECV: wire records -> caller arrays (+ source rank from the receive offsets)
// (SEND, narrow: out_rec holds the three arrays of soa_n rows each)
template <int MODE>
__global__ __launch_bounds__(DT) void k_dist_scatter(
    Route R, const char* __restrict__ ts, size_t stride, const u32* __restrict__ aux, const char* __restrict__ rec,
    size_t rb, int fmt, size_t n, u32 B, int bits, u32 nblocks, const u32* __restrict__ offs,
    char* __restrict__ out_rec, char* __restrict__ out_ts, size_t out_stride, u32* __restrict__ out_owner,
    u32* __restrict__ out_aux, u64* __restrict__ out_src, const u64* __restrict__ roff, u32 n_src,
    u32* __restrict__ invalid, size_t soa_n) {
  __shared__ Ranker L;
  if (offs && threadIdx.x < B) L.run[threadIdx.x] = offs[(size_t)threadIdx.x * nblocks + blockIdx.x];
  const size_t base = (size_t)blockIdx.x * DTILE;
  // (keep-input: the first slot of this rank's own bucket)
  const u32 keep_first = (MODE == SEND && fmt == FMT_NARROW && R.keep_me != NO_KEEP) ? offs[(size_t)R.keep_me * nblocks]
                                                                                     : 0u;
  bool inv = false;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    const bool ok = i < n;
    size_t pos = i;
    u32 bk = 0;
    if (offs) {
      const u32 b = ok ? bucket_of<MODE>(i, R, rec, rb, (fmt & 3) ? 16 : stride) : 0u;
      const bool act = ok && b < B;
      const u32 p = rank_slot(L, r, b, act, B, bits);
      if (!act) continue;  // (a row with an out-of-range bucket is reported by k_dist_count)
      pos = p;
      bk = b;
    } else if (!ok) {
      continue;
    }
    if (MODE == SEND && fmt == FMT_NARROW && offs && bk == R.keep_me) {
      // this rank's own row stays in the caller's rows: its index, and the
      // owner column (the receiver's id) -- not parsed, not copied
      const u32 o = R.owner[i];
      R.self_idx[pos - keep_first] = (u32)i;
      reinterpret_cast<u32*>(out_rec + soa_n * 20)[pos] = (R.dir_local || R.hot) ? local_of(R, o) : o;
      continue;
    }
    if (MODE == SEND && fmt != FMT_RAW) {
      const uint4* row = reinterpret_cast<const uint4*>(ts + i * stride);
      const uint4 x = row[0], y = row[1], z = row[2];
      const u32 w[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w & 0xffffu};
      const Parsed p = parse_ts46(w);
      inv |= (p.meta & EVM_META_VALID) == 0;
      const u32 cm = (p.meta & EVM_META_CASEMASK) | ((p.meta & EVM_META_VALID) ? PK_VALID : 0u);
      if (fmt == FMT_NARROW) {  // three arrays: (tc, node), mask, the receiver's owner id
        const u32 o = R.owner[i];
        reinterpret_cast<uint4*>(out_rec)[pos] = make_uint4((u32)p.tc, (u32)(p.tc >> 32), (u32)p.node,
                                                            (u32)(p.node >> 32));
        reinterpret_cast<u32*>(out_rec + soa_n * 16)[pos] = cm;
        reinterpret_cast<u32*>(out_rec + soa_n * 20)[pos] = (R.dir_local || R.hot) ? local_of(R, o) : o;
      } else {
        uint4* dst = reinterpret_cast<uint4*>(out_rec + pos * rb);
        dst[0] = make_uint4((u32)p.tc, (u32)(p.tc >> 32), (u32)p.node, (u32)(p.node >> 32));
        dst[1] = make_uint4(R.owner[i], aux ? aux[i] : 0u, (u32)i, cm);
      }
    } else if (MODE == SEND) {
      char* dst = out_rec + pos * rb;
      copy_row(dst, ts + i * stride, stride);
      uint4 m;
      m.x = R.owner[i];
      m.y = aux ? aux[i] : 0u;
      m.z = (u32)i;
      m.w = 0u;
      *reinterpret_cast<uint4*>(dst + stride) = m;
    } else {
      const bool nar = (fmt & 3) == FMT_NARROW;
      const char* src = nar ? nullptr : recv_rec(R, rec, rb, i);
      uint4 m;
      if (fmt & 3) {
        uint4 a;
        u32 w[12];
        if (nar && R.self_ts && is_self(R, i)) {  // (keep-input: the caller's own row, byte for byte)
          const size_t k = R.self_idx ? (size_t)R.self_idx[i - R.self_lo] : i - R.self_lo;
          const uint4* row = reinterpret_cast<const uint4*>(R.self_ts + k * R.self_stride);
          const uint4 x = row[0], y = row[1], z = row[2];
          w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
          w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
          w[8] = z.x; w[9] = z.y; w[10] = z.z; w[11] = z.w & 0xffffu;
          m = make_uint4(R.soa_c[i], 0u, 0u, 0u);
        } else {
          if (nar) {
            a = narrow_tn(R, i);
            m = make_uint4(R.soa_c[i], 0u, 0u, narrow_cm(R, i));
          } else {
            a = reinterpret_cast<const uint4*>(src)[0];
            m = reinterpret_cast<const uint4*>(src)[1];
          }
          format_ts46((u64)a.x | ((u64)a.y << 32), (u64)a.z | ((u64)a.w << 32), m.w & 0xffffu, w);
        }
        if (!(fmt & FMT_ST8)) {
          uint4* dst = reinterpret_cast<uint4*>(out_ts + pos * out_stride);
          dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
          dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
          dst[2] = make_uint4(w[8], w[9], w[10], w[11]);
        } else {  // an output row only 8-B aligned
          uint2* dst = reinterpret_cast<uint2*>(out_ts + pos * out_stride);
#pragma unroll
          for (int k = 0; k < 6; ++k) dst[k] = make_uint2(w[2 * k], w[2 * k + 1]);
        }
      } else {
        copy_row(out_ts + pos * out_stride, src, stride);
        m = *reinterpret_cast<const uint4*>(src + stride);
      }
      // (a narrow route's owner column is already the receiver's id)
      out_owner[pos] = (!nar && (R.dir_local || R.hot)) ? local_of(R, m.x) : m.x;
      if (out_aux) out_aux[pos] = m.y;
      if (out_src) {
        // source rank: the last r with roff[r] <= i
        u32 lo = 0, hi = n_src;
        while (hi - lo > 1) {
          const u32 mid = (lo + hi) >> 1;
          if (roff[mid] <= i) lo = mid;
          else hi = mid;
        }
        out_src[pos] = ((u64)lo << 32) | m.z;
      }
    }
  }
  if (MODE == SEND && fmt != FMT_RAW && invalid && __ballot(inv) && __lane_id() == 0) atomicOr(invalid, 1u);
}

__global__ void k_owner_over(const u32* __restrict__ owner, size_t n, u32 limit, u32* __restrict__ bad) {
  // (16-B loads where the column is 16-B aligned; the head and tail one by one)
  const size_t head = std::min<size_t>(n, ((16 - ((uintptr_t)owner & 15)) & 15) / 4);
  const size_t nq = (n - head) / 4;
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u* q = reinterpret_cast<const v4u*>(owner + head);
  bool b = false;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < nq; i += nt) {
    const v4u v = __builtin_nontemporal_load(q + i);
    b |= (v.x >= limit) | (v.y >= limit) | (v.z >= limit) | (v.w >= limit);
  }
  for (size_t i = tid; i < head; i += nt) b |= owner[i] >= limit;
  for (size_t i = head + nq * 4 + tid; i < n; i += nt) b |= owner[i] >= limit;
  if (__ballot(b) && __lane_id() == 0) atomicOr(bad, 1u);
}

// the local owner of every received packed record (evm_dist_ingest): the
// records stay where they are, only the owner column is written
__global__ void k_dist_owner(Route R, const char* __restrict__ rec, size_t rb, size_t n, u32* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = local_of(R, *reinterpret_cast<const u32*>(recv_rec(R, rec, rb, i) + 16));
}

// bucket totals from the scanned count matrix
__global__ void k_dist_totals(const u32* __restrict__ offs, const u32* __restrict__ total, u32 B, u32 nblocks,
                              u64* __restrict__ out) {
  const u32 b = threadIdx.x;
  if (b >= B) return;
  const u32 a = offs[(size_t)b * nblocks];
  const u32 e = b + 1 < B ? offs[(size_t)(b + 1) * nblocks] : *total;
  out[b] = (u64)(e - a);
}

// the count words this rank sends: counts (or zeros) plus the flag bits
__global__ void k_dist_mark(u64* __restrict__ cnt, u32 G, int zero, int err, const u32* __restrict__ flags, u64 bits) {
  const u32 p = threadIdx.x;
  if (p >= G) return;
  u64 v = (zero ? 0ull : cnt[p]) | bits;
  if (err) v |= CNT_ERR;
  if (flags && flags[1]) v |= CNT_INVALID;
  cnt[p] = v;
}

__global__ void k_dist_root_pack(const u64* __restrict__ off, const u64* __restrict__ end, const int32_t* __restrict__ pfx,
                                 u32 n_owners, u32 per, u64* __restrict__ out) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < per; o += gridDim.x * blockDim.x) {
    u64 v = 0;
    if (o < n_owners) {
      const u64 a = off[o], b = end[o];
      v = (u64)(uint32_t)(pfx[b] ^ pfx[a]) | ((u64)(b > a) << 32);
    }
    out[o] = v;
  }
}

// gathered [rank][per + 1] -> global owner g: local g / world of rank g % world,
// or the directory's (rank, local) of g; a split owner: the XOR of every
// rank's partial root at its hot slot (present if any part is)
__global__ void k_dist_root_unpack(const u64* __restrict__ all, u32 world, u32 stride, u32 n_global,
                                   const uint8_t* __restrict__ dir_dest, const u32* __restrict__ dir_local,
                                   const u32* __restrict__ hot, u32 n_hot_tab, u32 hot_base,
                                   int32_t* __restrict__ root, uint8_t* __restrict__ present) {
  for (u32 g = blockIdx.x * blockDim.x + threadIdx.x; g < n_global; g += gridDim.x * blockDim.x) {
    u64 v;
    if (hot && g < n_hot_tab && hot[g] != HOT_NONE) {
      u32 x = 0, p = 0;
      for (u32 r = 0; r < world; ++r) {
        const u64 w = all[(size_t)r * stride + hot_base + hot[g]];
        x ^= (u32)w;
        p |= (u32)(w >> 32);
      }
      v = (u64)x | ((u64)(p != 0) << 32);
    } else {
      v = dir_dest ? all[(size_t)dir_dest[g] * stride + dir_local[g]] : all[(size_t)(g % world) * stride + g / world];
    }
    root[g] = (int32_t)(uint32_t)v;
    present[g] = (uint8_t)(v >> 32);
  }
}

// MurmurHash3_x86_32, seed 0, of `len` bytes (murmurhash@2.0.1 over an ASCII
// userId; SURVEY 8(e) shards owners by murmur3(ownerId) mod G)
__device__ u32 murmur3_bytes(const uint8_t* p, u32 len) {
  const u32 c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  u32 h = 0u;
  const u32 nb = len >> 2;
  for (u32 i = 0; i < nb; ++i) {
    u32 k = (u32)p[4 * i] | ((u32)p[4 * i + 1] << 8) | ((u32)p[4 * i + 2] << 16) | ((u32)p[4 * i + 3] << 24);
    k *= c1;
    k = rotl32(k, 15) * c2;
    h ^= k;
    h = rotl32(h, 13) * 5u + 0xe6546b64u;
  }
  const u32 t = len & 3u;
  u32 k = 0;
  if (t >= 3) k ^= (u32)p[4 * nb + 2] << 16;
  if (t >= 2) k ^= (u32)p[4 * nb + 1] << 8;
  if (t >= 1) {
    k ^= (u32)p[4 * nb];
    k *= c1;
    k = rotl32(k, 15) * c2;
    h ^= k;
  }
  h ^= len;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__global__ void k_dir_hash(const uint8_t* __restrict__ ids, size_t stride, u32 len, u32 n, u32 world,
                           uint8_t* __restrict__ dest, u32* __restrict__ hash_out) {
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const u32 h = murmur3_bytes(ids + (size_t)i * stride, len);
    dest[i] = (uint8_t)(h % world);
    if (hash_out) hash_out[i] = h;
  }
}

// local id of owner i = its stable slot among the owners of its rank
__global__ __launch_bounds__(DT) void k_dir_local(const uint8_t* __restrict__ dest, u32 n, u32 B, int bits,
                                                  u32 nblocks, const u32* __restrict__ offs, u32* __restrict__ local) {
  __shared__ Ranker L;
  if (threadIdx.x < B) L.run[threadIdx.x] = offs[(size_t)threadIdx.x * nblocks + blockIdx.x];
  const size_t base = (size_t)blockIdx.x * DTILE;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    const bool ok = i < n;
    const u32 b = ok ? dest[i] : 0u;
    const u32 p = rank_slot(L, r, b, ok, B, bits);
    if (ok) local[i] = p - offs[(size_t)b * nblocks];
  }
}


// ------------------------------------------------------------------ split kernels
// Rows per global owner (hot-owner detection).
__global__ void k_split_hist(const u32* __restrict__ owner, size_t n, u32 n_global, u64* __restrict__ counts,
                             u32* __restrict__ bad) {
  bool oob = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32 o = owner[i];
    if (o < n_global) atomicAdd(&counts[o], 1ull);
    else oob = true;
  }
  if (__ballot(oob) && __lane_id() == 0) atomicOr(bad, 1u);
}

// Owners whose row count over all ranks exceeds thr (gathered [rank][per]).
__global__ void k_split_select(const u64* __restrict__ all, u32 world, size_t per, u32 n_global, u64 thr,
                               u32* __restrict__ list, u32* __restrict__ n_list, u32 cap) {
  for (u32 g = blockIdx.x * blockDim.x + threadIdx.x; g < n_global; g += gridDim.x * blockDim.x) {
    u64 t = 0;
    for (u32 r = 0; r < world; ++r) t += all[(size_t)r * per + g];
    if (t > thr) {
      const u32 k = atomicAdd(n_list, 1u);
      if (k < cap) list[k] = g;
    }
  }
}

__global__ void k_ts_dest(const char* __restrict__ ts, size_t stride, size_t n, u32 world, uint8_t* __restrict__ dest) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dest[i] = (uint8_t)ts_rank(ts + i * stride, world);
}

// a fixed mix of the cell id (dist.py cell_dest)
__global__ void k_cell_dest(const u32* __restrict__ cell, size_t n, u32 world, uint8_t* __restrict__ dest) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dest[i] = (uint8_t)(((cell[i] * 0x9E3779B1u) >> 8) % world);
}

// Leaves of owners [lo, lo + count) rebased to owner 0: [L][ck x L][xr, two per word]
__global__ void k_merge_pack(const u64* __restrict__ ck, const int32_t* __restrict__ xr, u64 a, u64 L, u32 lo,
                             u64* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = L;
  u64* oc = out + 1;
  int32_t* ox = reinterpret_cast<int32_t*>(out + 1 + L);
  for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < L; k += (u64)gridDim.x * blockDim.x) {
    oc[k] = ck[a + k] - ((u64)lo << 40);
    ox[k] = xr[a + k];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (L & 1)) ox[L] = 0;
}

// selection payload: [n + 1 offsets from 0][m ids][3m keys]
__global__ void k_sel_pack(const uint64_t* __restrict__ off, const uint64_t* __restrict__ id,
                           const uint64_t* __restrict__ key, u32 n, u64 m, u64* __restrict__ out) {
  const u64 a = off[0];
  for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < (u64)n + 1 + 4 * m; k += (u64)gridDim.x * blockDim.x) {
    u64 v;
    if (k <= n) v = off[k] - a;
    else if (k <= n + m) v = id[a + (k - n - 1)];
    else v = key[3 * a + (k - n - 1 - m)];
    out[k] = v;
  }
}

__device__ __forceinline__ bool key_lt3(const u64* a, const u64* b) {
  return a[0] != b[0] ? a[0] < b[0] : (a[1] != b[1] ? a[1] < b[1] : a[2] < b[2]);
}

// out_off[g] = sum over ranks of their group offsets
__global__ void k_sel_off(const u64* __restrict__ all, u32 world, size_t per, u32 n, uint64_t* __restrict__ out_off) {
  for (u32 g = blockIdx.x * blockDim.x + threadIdx.x; g <= n; g += gridDim.x * blockDim.x) {
    u64 t = 0;
    for (u32 r = 0; r < world; ++r) t += all[(size_t)r * per + g];
    out_off[g] = t;
  }
}

// Every gathered row to its place: its group's start + its rank inside its
// own part + the rows of the other ranks' parts of the group that sort before
// it (equal keys: the lower rank first).  rbase: [world + 1] row prefix.
__global__ void k_sel_merge(const u64* __restrict__ all, u32 world, size_t per, u32 n, const u64* __restrict__ rbase,
                            const uint64_t* __restrict__ out_off, uint64_t* __restrict__ out_id) {
  const u64 M = rbase[world];
  for (u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x; t < M; t += (u64)gridDim.x * blockDim.x) {
    u32 p = 0;
    while (rbase[p + 1] <= t) ++p;
    const u64 j = t - rbase[p];
    const u64* A = all + (size_t)p * per;
    const u64 mp = A[n];
    // group of row j: the last g with off[g] <= j
    u32 lo = 0, hi = n;
    while (hi - lo > 1) {
      const u32 mid = (lo + hi) >> 1;
      if (A[mid] <= j) lo = mid;
      else hi = mid;
    }
    const u32 g = lo;
    const u64* key = A + n + 1 + mp + 3 * j;
    u64 pos = out_off[g] + (j - A[g]);
    for (u32 q = 0; q < world; ++q) {
      if (q == p) continue;
      const u64* B = all + (size_t)q * per;
      const u64 mq = B[n];
      const u64* kq = B + n + 1 + mq;
      u64 a = B[g], b = B[g + 1];
      // rows of q's group g before this key: < key (q > p) or <= key (q < p)
      while (a < b) {
        const u64 mid = (a + b) >> 1;
        const bool before = q < p ? !key_lt3(key, kq + 3 * mid) : key_lt3(kq + 3 * mid, key);
        if (before) a = mid + 1;
        else b = mid;
      }
      pos += a - B[g];
    }
    out_id[pos] = A[n + 1 + j];
  }
}

// return path: (source index, value) of every received row, in receive order
__global__ void k_ret_pack(Route R, const char* __restrict__ rec, size_t rb, size_t ooff, size_t n,
                           const uint8_t* __restrict__ val, u32 elem, u64* __restrict__ out) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    const u32 idx = *reinterpret_cast<const u32*>(recv_rec(R, rec, rb, k) + ooff + 8);
    u64 v = 0;
    for (u32 b = 0; b < elem; ++b) v |= (u64)val[k * elem + b] << (8 * b);
    out[2 * k] = idx;
    out[2 * k + 1] = v;
  }
}

__global__ void k_ret_scatter(const u64* __restrict__ in, size_t n, uint8_t* __restrict__ out, size_t n_out, u32 elem,
                              u32* __restrict__ bad) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    const u64 idx = in[2 * k], v = in[2 * k + 1];
    if (idx >= n_out) {
      atomicOr(bad, 1u);
      continue;
    }
    for (u32 b = 0; b < elem; ++b) out[idx * elem + b] = (uint8_t)(v >> (8 * b));
  }
}

// winners: index into the receive order -> global batch index + 1 (0: none)
__global__ void k_win_map(Route R, const int32_t* __restrict__ win, u32 n_cells, const char* __restrict__ rec, size_t rb,
                          size_t ooff, u64 n_recv, const u64* __restrict__ roff, u32 world,
                          const u64* __restrict__ base, u64* __restrict__ out, u32* __restrict__ bad) {
  for (u32 c = blockIdx.x * blockDim.x + threadIdx.x; c < n_cells; c += gridDim.x * blockDim.x) {
    const int32_t w = win[c];
    u64 v = 0;
    if (w >= 0) {
      if ((u64)w >= n_recv) {
        atomicOr(bad, 1u);
      } else {
        u32 s = 0;
        while (s + 1 < world && roff[s + 1] <= (u64)w) ++s;
        const u32 idx = *reinterpret_cast<const u32*>(recv_rec(R, rec, rb, (size_t)w) + ooff + 8);
        v = base[s] + idx + 1;
      }
    }
    out[c] = v;
  }
}

__global__ void k_win_reduce(const u64* __restrict__ all, u32 world, size_t per, u32 n_cells, int64_t* __restrict__ out) {
  for (u32 c = blockIdx.x * blockDim.x + threadIdx.x; c < n_cells; c += gridDim.x * blockDim.x) {
    u64 m = 0;
    for (u32 r = 0; r < world; ++r) m = max(m, all[(size_t)r * per + c]);
    out[c] = (int64_t)m - 1;
  }
}

}  // namespace

struct evm_dist {
  Transport* tx = nullptr;
  int rank = 0, world = 1;
  size_t stride = 48, rb = 64;
  int packed = 0;  // the last route's records: packed (48-B rows) or raw
  int narrow = 0;  // ... packed without aux / source index (24 B)
  // the last route's rows from this rank to itself stay in the send buffer:
  // received rows [self_lo, self_hi) at send + self_off
  uint64_t self_lo = 0, self_hi = 0;
  size_t self_off = 0;
  uint64_t self_row = 0;  // (narrow: the first of them among the send buffer's rows)
  // INVARIANT: `send` belongs to the last route until the next one -- take,
  // ingest, return and split_winners read this rank's own rows from it.  Any
  // other writer of `send` must set send_gen = 0 first; the readers check
  // send_gen == route_gen (self_rows_intact) and refuse the call otherwise.
  // EVM_ROUTE_KEEP_INPUT: the last route left this rank's own rows in the
  // caller's rows (self_ts; received row self_lo + k is row self_idx[k])
  const char* self_ts = nullptr;
  size_t self_stride = 0;
  u32* self_idx = nullptr;  // (null with self_identity: row k is ts row k)
  size_t self_idx_cap = 0;  // bytes
  // world 1, keep-input, no split: the route IS the caller's rows (owner
  // column included: at world 1 every owner's local id is itself)
  bool self_identity = false;
  const u32* self_owner = nullptr;
  uint64_t route_gen = 0;  // routes finished by this rank
  uint64_t send_gen = 0;   // the route whose records `send` holds (0: none)
  char* send = nullptr;  // wire records (send side), device
  size_t send_cap = 0;   // bytes
  char* recv = nullptr;  // received records (staging for evm_dist_take)
  size_t recv_cap = 0;
  uint64_t n_recv = 0;
  u64* cnt = nullptr;   // device count / offset / agreement words (CNT_WORDS)
  u64* hcnt = nullptr;  // pinned host mirror
  uint64_t recv_off[MAX_BUCKETS + 1] = {};
  // owner directory (evm_dist_directory): global owner -> (rank, local id)
  uint8_t* dir_dest = nullptr;
  u32* dir_local = nullptr;
  u32 n_dir = 0;
  u32 dir_per = 0;      // the most owners any rank serves
  u32 dir_n_local = 0;  // owners this rank serves
  // hot-owner split (evm_dist_split): global owner -> hot index on every rank
  u32* hot = nullptr;
  u32 n_hot_tab = 0, n_hot = 0, hot_base = 0;
  // the last route: rows this rank sent to / received from every peer, and
  // its input size (evm_dist_return, evm_dist_split_winners)
  uint64_t sent[MAX_BUCKETS] = {}, recvd[MAX_BUCKETS] = {};
  uint64_t n_in = 0;
};

namespace {

// the last route's own rows are still where it left them (see evm_dist)
bool self_rows_intact(const evm_dist* d) { return d->self_hi == d->self_lo || d->send_gen == d->route_gen; }

int grow(char** p, size_t* cap, size_t want) {
  if (want <= *cap) return EVM_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t bytes = want + want / 8 + 4096;
  HIPR(hipMalloc(p, bytes));
  *cap = bytes;
  return EVM_OK;
}

Route route_of(const evm_dist* d, const u32* owner, const uint8_t* dest) {
  Route R;
  R.owner = owner;
  R.dest = dest;
  R.dir_dest = d->dir_dest;
  R.dir_local = d->dir_local;
  R.n_dir = d->n_dir;
  R.world = (u32)d->world;
  R.hot = d->hot;
  R.n_hot_tab = d->n_hot_tab;
  R.hot_base = d->hot_base;
  R.ts = nullptr;
  R.stride = 0;
  R.self_rec = d->send + d->self_off;
  R.self_lo = d->self_lo;
  R.self_hi = d->self_hi;
  R.soa_a = nullptr;
  R.soa_b = nullptr;
  R.soa_c = nullptr;
  R.self_a = nullptr;
  R.self_b = nullptr;
  R.keep_me = NO_KEEP;
  R.self_idx = d->self_idx;
  R.self_ts = d->self_ts;
  R.self_stride = d->self_stride;
  if (d->self_identity) {  // (the caller's rows as they lie: owner column included)
    R.soa_c = d->self_owner;
    R.self_idx = nullptr;
  } else if (d->narrow && d->packed) {  // the last route's three arrays (receive side) and this rank's own rows
    R.soa_a = d->recv;
    R.soa_b = reinterpret_cast<const u32*>(d->recv + d->n_recv * 16);
    R.soa_c = reinterpret_cast<const u32*>(d->recv + d->n_recv * 20);
    R.self_a = d->send + d->self_row * 16;
    R.self_b = reinterpret_cast<const u32*>(d->send + d->n_in * 16) + d->self_row;
  }
  return R;
}

// stable partition of n rows into B buckets: counts -> scan -> totals.
// Returns the scanned slot matrix (offs) and the bucket totals (device).
template <int MODE>
int partition_offsets(evm_ctx* ctx, Scratch& S, const Route& R, const char* rec, size_t rb, size_t ooff, size_t n,
                      u32 B, u32** offs_out, u32* nblocks_out, u64* totals, u32* bad) {
  const u32 nblocks = (u32)std::max<size_t>(1, (n + DTILE - 1) / DTILE);
  u32* counts = S.alloc<u32>((size_t)B * nblocks);
  u32* offs = S.alloc<u32>((size_t)B * nblocks + 1);
  if (!counts || !offs) return EVM_ENOMEM;
  KLAUNCH((k_dist_count<MODE>), dim3(nblocks), dim3(DT), R, rec, rb, ooff, n, B, ceil_log2(B), nblocks, counts, bad);
  int st = scan_exclusive<u32, OpAdd>(ctx, S, counts, (size_t)B * nblocks, offs, offs + (size_t)B * nblocks);
  if (st) return st;
  KLAUNCH(k_dist_totals, dim3(1), dim3(MAX_BUCKETS), offs, offs + (size_t)B * nblocks, B, nblocks, totals);
  *offs_out = offs;
  *nblocks_out = nblocks;
  return hip_ok(hipGetLastError());
}

// One agreement round: every rank's status word to every rank; returns the
// first failure of any rank (EVM_OK when all succeeded).
int agree(evm_ctx* ctx, evm_dist* d, int local) {
  const u32 G = (u32)d->world;
  for (u32 p = 0; p < G; ++p) d->hcnt[W_AGREE_S + p] = (u64)(u32)local;
  HIPR(hipMemcpyAsync(d->cnt + W_AGREE_S, d->hcnt + W_AGREE_S, G * sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  int st = d->tx->all_to_all_u64(d->cnt + W_AGREE_S, d->cnt + W_AGREE_R, ctx->stream);
  if (st) return st;
  HIPR(hipMemcpyAsync(d->hcnt + W_AGREE_R, d->cnt + W_AGREE_R, G * sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (local) return local;
  for (u32 p = 0; p < G; ++p)
    if (d->hcnt[W_AGREE_R + p]) return EVM_EDIST;
  return EVM_OK;
}

int dist_alloc(evm_ctx* ctx, evm_dist* d) {
  if (hipMalloc(&d->cnt, CNT_WORDS * sizeof(u64)) != hipSuccess ||
      hipHostMalloc(&d->hcnt, CNT_WORDS * sizeof(u64), hipHostMallocDefault) != hipSuccess)
    return EVM_ENOMEM;
  memset(d->hcnt, 0, CNT_WORDS * sizeof(u64));
  return hip_ok(hipMemsetAsync(d->cnt, 0, CNT_WORDS * sizeof(u64), ctx->stream));
}


// One all-gather of (status, value) per rank: the peers' values into vals
// (host, world words); any rank's status set -> every rank fails.
int gather_status(evm_ctx* ctx, evm_dist* d, int local, u64 value, uint64_t* vals) {
  const u32 G = (u32)d->world;
  d->hcnt[W_GS] = (u64)(u32)local;
  d->hcnt[W_GS + 1] = value;
  HIPR(hipMemcpyAsync(d->cnt + W_GS, d->hcnt + W_GS, 2 * sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  int st = d->tx->all_gather_u64(d->cnt + W_GS, d->cnt + W_GR, 2, ctx->stream);
  if (st) return st;
  HIPR(hipMemcpyAsync(d->hcnt + W_GR, d->cnt + W_GR, 2 * G * sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (local) return local;
  for (u32 p = 0; p < G; ++p) {
    if (d->hcnt[W_GR + 2 * p]) return EVM_EDIST;
    if (vals) vals[p] = d->hcnt[W_GR + 2 * p + 1];
  }
  return EVM_OK;
}

}  // namespace

extern "C" {

int evm_dist_unique_id(uint8_t* id) {
  if (!id) return EVM_EINVAL;
  const Rccl* r = rccl();
  if (!r) return EVM_EDIST;
  ncclUniqueId u;
  if (r->get_unique_id(&u) != ncclSuccess) return EVM_EDIST;
  memcpy(id, &u, sizeof(u));
  return EVM_OK;
}

int evm_dist_init(evm_ctx* ctx, const uint8_t* id, int rank, int world, evm_dist** out) {
  if (!ctx || !id || !out || world < 1 || world > (int)MAX_BUCKETS || rank < 0 || rank >= world) return EVM_EINVAL;
  *out = nullptr;
  const Rccl* r = rccl();
  if (!r) return EVM_EDIST;
  HIPR(hipSetDevice(ctx->device));
  evm_dist* d = new evm_dist;
  d->rank = rank;
  d->world = world;
  RcclTransport* t = new RcclTransport;
  t->r = r;
  t->world = world;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  if (r->comm_init_rank(&t->comm, world, u, rank) != ncclSuccess) {
    t->comm = nullptr;
    delete t;
    delete d;
    return EVM_EDIST;
  }
  d->tx = t;
  const int st = dist_alloc(ctx, d);
  if (st) {
    evm_dist_free(ctx, d);
    return st;
  }
  *out = d;
  return EVM_OK;
}

int evm_dist_hub_new(int world, evm_dist_hub** out) {
  if (!out || world < 1 || world > (int)MAX_BUCKETS) return EVM_EINVAL;
  evm_dist_hub* h = new evm_dist_hub;
  h->world = world;
  *out = h;
  return EVM_OK;
}

void evm_dist_hub_free(evm_dist_hub* hub) { delete hub; }

void evm_dist_hub_abort(evm_dist_hub* hub) {
  if (hub) hub->abort();
}

int evm_dist_init_loopback(evm_ctx* ctx, evm_dist_hub* hub, int rank, evm_dist** out) {
  if (!ctx || !hub || !out || rank < 0 || rank >= hub->world) return EVM_EINVAL;
  *out = nullptr;
  HIPR(hipSetDevice(ctx->device));
  evm_dist* d = new evm_dist;
  d->rank = rank;
  d->world = hub->world;
  LoopTransport* t = new LoopTransport;
  t->hub = hub;
  t->rank = rank;
  t->world = hub->world;
  d->tx = t;
  const int st = dist_alloc(ctx, d);
  if (st) {
    evm_dist_free(ctx, d);
    return st;
  }
  *out = d;
  return EVM_OK;
}

void evm_dist_free(evm_ctx* ctx, evm_dist* d) {
  if (!d) return;
  if (ctx) (void)hipStreamSynchronize(ctx->stream);
  delete d->tx;
  if (d->send) (void)hipFree(d->send);
  if (d->self_idx) (void)hipFree(d->self_idx);
  if (d->recv) (void)hipFree(d->recv);
  if (d->cnt) (void)hipFree(d->cnt);
  if (d->hcnt) (void)hipHostFree(d->hcnt);
  if (d->dir_dest) (void)hipFree(d->dir_dest);
  if (d->dir_local) (void)hipFree(d->dir_local);
  if (d->hot) (void)hipFree(d->hot);
  delete d;
}

int evm_dist_info(const evm_dist* d, int* rank, int* world) {
  if (!d) return EVM_EINVAL;
  if (rank) *rank = d->rank;
  if (world) *world = d->world;
  return EVM_OK;
}

int evm_dist_directory(evm_ctx* ctx, evm_dist* d, const char* ids, size_t stride, size_t id_len, uint32_t n_owners,
                       uint8_t* dest_out, uint32_t* local_out, uint32_t* n_local) {
  if (!ctx || !d || (n_owners && (!ids || id_len == 0 || id_len > stride || id_len > 4096))) return EVM_EINVAL;
  if (d->dir_dest) (void)hipFree(d->dir_dest);
  if (d->dir_local) (void)hipFree(d->dir_local);
  if (d->hot) (void)hipFree(d->hot);  // (a split's hot slots follow the directory's: set it again)
  d->dir_dest = nullptr;
  d->dir_local = nullptr;
  d->hot = nullptr;
  d->n_hot_tab = d->n_hot = d->hot_base = 0;
  d->n_dir = d->dir_per = d->dir_n_local = 0;
  if (n_local) *n_local = 0;
  if (!n_owners) return EVM_OK;
  const u32 G = (u32)d->world;
  HIPR(hipMalloc(&d->dir_dest, n_owners));
  HIPR(hipMalloc(&d->dir_local, (size_t)n_owners * sizeof(u32)));
  Scratch S(ctx);
  u32* bad = S.alloc<u32>(1);
  u64* tot = S.alloc<u64>(MAX_BUCKETS);
  if (!bad || !tot) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  KLAUNCH(k_dir_hash, dim3(grid_for(n_owners, 256)), dim3(256), reinterpret_cast<const uint8_t*>(ids), stride,
          (u32)id_len, n_owners, G, d->dir_dest, (u32*)nullptr);
  Route R = route_of(d, nullptr, d->dir_dest);
  R.dir_dest = nullptr;
  R.dir_local = nullptr;
  u32* offs = nullptr;
  u32 nblocks = 0;
  int st = partition_offsets<SEND>(ctx, S, R, nullptr, 0, 0, n_owners, G, &offs, &nblocks, tot, bad);
  if (st) return st;
  KLAUNCH(k_dir_local, dim3(nblocks), dim3(DT), d->dir_dest, n_owners, G, ceil_log2(G), nblocks, offs, d->dir_local);
  uint64_t h[MAX_BUCKETS];
  HIPR(hipMemcpyAsync(h, tot, G * sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  if (dest_out) HIPR(hipMemcpyAsync(dest_out, d->dir_dest, n_owners, hipMemcpyDeviceToDevice, ctx->stream));
  if (local_out)
    HIPR(hipMemcpyAsync(local_out, d->dir_local, (size_t)n_owners * sizeof(u32), hipMemcpyDeviceToDevice, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  u64 mx = 0;
  for (u32 p = 0; p < G; ++p) mx = std::max<u64>(mx, h[p]);
  d->n_dir = n_owners;
  d->dir_per = (u32)mx;
  d->dir_n_local = (u32)h[d->rank];
  if (n_local) *n_local = d->dir_n_local;
  return EVM_OK;
}

int evm_dist_route(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                   const uint32_t* aux, const uint8_t* dest, uint64_t* n_recv) {
  return evm_dist_route_ex(ctx, d, ts, stride, n, owner, aux, dest, 0u, n_recv);
}

int evm_dist_route_ex(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                      const uint32_t* aux, const uint8_t* dest, uint32_t flags_in, uint64_t* n_recv) {
  if (!ctx || !d || !n_recv) return EVM_EINVAL;  // nothing to join the collective with
  *n_recv = 0;
  d->n_recv = 0;
  const u32 G = (u32)d->world;
  int lerr = EVM_OK;  // a local failure: the rank still joins the count exchange, flagged
  if (stride < 46 || stride % 8 || stride / 8 > CNT_STRIDE_MAX || (n && (!ts || !owner)) || n >= 0xffffffffull)
    lerr = EVM_EINVAL;
  // 48-B rows, 16-B aligned: packed 32-B records (a third of the xGMI bytes of
  // raw ones).  Every rank must use one record format: a rank that cannot
  // pack says so in its count words (CNT_RAW) and then every rank sends raw.
  // (a rank with no rows sends nothing: it votes for no format and no stride)
  const bool packed0 = !lerr && (n == 0 || (stride == 48 && ((uintptr_t)ts & 15) == 0));
  // no aux and no source indexes wanted: 24-B records (a quarter fewer xGMI
  // and HBM bytes), when every rank asks for them (CNT_WIDE otherwise)
  const bool narrow0 = packed0 && !aux && (flags_in & EVM_ROUTE_NO_SRC);
  // own rows left in the caller's rows (read there by take / ingest)
  const bool keep0 = narrow0 && (flags_in & EVM_ROUTE_KEEP_INPUT) && n > 0;
  size_t rb = packed0 ? (narrow0 ? NARROW : PACKED) : stride + META;
  d->self_identity = false;
  if (G == 1 && keep0 && !lerr && !dest && !d->hot) {
    // one rank and the caller keeps its rows: there is nothing to move --
    // the received rows are the caller's rows as they lie (at world 1 the
    // directory's local id of every owner is itself); only the owners' range
    // is checked, as the partition would
    bool ok = true;
    if (d->dir_dest) {
      Scratch S1(ctx);
      u32* bad = S1.alloc<u32>(1);
      if (!bad) return EVM_ENOMEM;
      HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
      KLAUNCH(k_owner_over, dim3(grid_for(n / 4, 256, 8192)), dim3(256), owner, n, d->n_dir, bad);
      u32 hb = 0;
      HIPR(hipMemcpyAsync(&hb, bad, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
      HIPR(hipStreamSynchronize(ctx->stream));
      ok = hb == 0;
    }
    if (ok) {
      d->self_off = d->self_row = 0;
      d->self_lo = 0;
      d->self_hi = n;
      d->recv_off[0] = 0;
      d->recv_off[1] = n;
      d->stride = stride;
      d->rb = NARROW;
      d->packed = d->narrow = 1;
      d->n_recv = n;
      d->n_in = n;
      d->sent[0] = d->recvd[0] = n;
      d->send_gen = ++d->route_gen;
      d->self_ts = ts;
      d->self_stride = stride;
      d->self_owner = owner;
      d->self_identity = true;
      *n_recv = n;
      return EVM_OK;
    }
  }
  Scratch S(ctx);
  u32* flags = S.alloc<u32>(2);  // [0] a destination out of range, [1] a row outside the native domain
  u64* scnt = d->cnt + W_SEND;
  u64* rcnt = d->cnt + W_RECV;
  d->self_lo = d->self_hi = 0;  // (a failed route leaves no rows to take)
  d->self_off = 0;
  d->self_row = 0;
  d->packed = d->narrow = 0;
  d->send_gen = 0;  // (rewritten below)
  d->self_ts = nullptr;
  Route R = route_of(d, owner, dest);
  R.ts = ts;
  R.stride = stride;
  if (keep0 && !lerr) {
    lerr = grow(reinterpret_cast<char**>(&d->self_idx), &d->self_idx_cap, n * sizeof(u32));
    R.keep_me = (u32)d->rank;
    R.self_idx = d->self_idx;
  }
  u32* offs = nullptr;
  u32 nblocks = 0;
  d->n_in = 0;
  if (!flags) lerr = lerr ? lerr : EVM_ENOMEM;
  if (!lerr) lerr = hip_ok(hipMemsetAsync(flags, 0, 2 * sizeof(u32), ctx->stream));
  if (!lerr) lerr = grow(&d->send, &d->send_cap, std::max<size_t>(n, 1) * rb);
  if (!lerr && n) {
    lerr = partition_offsets<SEND>(ctx, S, R, nullptr, rb, stride, n, G, &offs, &nblocks, scnt, flags);
    if (!lerr) {
      KLAUNCH((k_dist_scatter<SEND>), dim3(nblocks), dim3(DT), R, ts, stride, aux, (const char*)nullptr, rb,
              packed0 ? (narrow0 ? (int)FMT_NARROW : (int)FMT_PACKED) : (int)FMT_RAW, n, G, ceil_log2(G), nblocks,
              offs, d->send, (char*)nullptr, (size_t)0, (u32*)nullptr, (u32*)nullptr, (u64*)nullptr,
              (const u64*)nullptr, 0u, flags + 1, n);
      lerr = hip_ok(hipGetLastError());
    }
  }
  // the counts: one all-to-all of G words (flag bits on top), one read back
  const u64 fmt = (packed0 ? 0ull : CNT_RAW) | (narrow0 ? 0ull : CNT_WIDE) |
                  ((u64)(lerr || !n ? 0 : stride / 8) << CNT_STRIDE_SHIFT);
  KLAUNCH(k_dist_mark, dim3(1), dim3(MAX_BUCKETS), scnt, G, (lerr || !n) ? 1 : 0, lerr ? 1 : 0,
          (const u32*)(lerr ? nullptr : flags), fmt);
  int st = d->tx->all_to_all_u64(scnt, rcnt, ctx->stream);
  if (st) return st;
  if (!lerr) {
    HIPR(hipMemsetAsync(d->cnt + W_BAD, 0, 2 * sizeof(u64), ctx->stream));
    HIPR(hipMemcpy2DAsync(d->cnt + W_BAD, sizeof(u64), flags, sizeof(u32), sizeof(u32), 2, hipMemcpyDeviceToDevice,
                          ctx->stream));
  }
  HIPR(hipMemcpyAsync(d->hcnt, d->cnt, CNT_WORDS * sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  const u64* hs = d->hcnt + W_SEND;
  const u64* hr = d->hcnt + W_RECV;
  bool any_err = lerr != EVM_OK, any_inv = false, any_raw = false, any_wide = false, mixed_stride = false;
  u64 agreed = 0;  // the stride of the ranks that hold rows (0: a rank without rows -- a wildcard)
  for (u32 p = 0; p < G; ++p) {
    any_err |= (hr[p] & CNT_ERR) != 0;
    any_inv |= (hr[p] & CNT_INVALID) != 0;
    any_raw |= (hr[p] & CNT_RAW) != 0;
    any_wide |= (hr[p] & CNT_WIDE) != 0;
    const u64 sw = (hr[p] >> CNT_STRIDE_SHIFT) & CNT_STRIDE_MAX;
    if (sw && agreed && sw != agreed) mixed_stride = true;
    if (sw) agreed = sw;
  }
  if (any_err) return lerr ? lerr : EVM_EDIST;  // every rank saw the flag: nobody exchanges
  const bool bad_dest = d->hcnt[W_BAD] != 0;
  // a row outside the native domain anywhere, or a rank that cannot pack:
  // every rank sends raw records (the packed form cannot carry the original
  // bytes); same slots, wider records.  Every rank sees the same count words,
  // so every rank takes the same decision.
  const bool packed = !any_raw && !any_inv;
  // raw records carry the row bytes at the sender's stride: one stride on
  // every rank, or nobody exchanges (every rank sees the mismatch)
  if (!packed && mixed_stride) return EVM_EINVAL;
  // a rank without rows receives raw records at the senders' stride
  if (!packed && !n && agreed) stride = (size_t)agreed * 8;
  const bool narrow = packed && !any_wide;
  const int fmt_final = packed ? (narrow ? (int)FMT_NARROW : (int)FMT_PACKED) : (int)FMT_RAW;
  const size_t rb_final = packed ? (narrow ? NARROW : PACKED) : stride + META;
  if (rb_final != rb) {  // another rank's rows decide the format: scatter again in it
    rb = rb_final;
    lerr = grow(&d->send, &d->send_cap, std::max<size_t>(n, 1) * rb);
    if (!lerr && n) {
      KLAUNCH((k_dist_scatter<SEND>), dim3(nblocks), dim3(DT), R, ts, stride, aux, (const char*)nullptr, rb,
              fmt_final, n, G, ceil_log2(G), nblocks, offs, d->send, (char*)nullptr, (size_t)0, (u32*)nullptr,
              (u32*)nullptr, (u64*)nullptr, (const u64*)nullptr, 0u, (u32*)nullptr, n);
      lerr = hip_ok(hipGetLastError());
    }
  }
  uint64_t soff[MAX_BUCKETS + 1], slen[MAX_BUCKETS], roff[MAX_BUCKETS + 1], rlen[MAX_BUCKETS];
  soff[0] = 0;
  d->recv_off[0] = 0;
  for (u32 p = 0; p < G; ++p) {
    const u64 a = hs[p] & CNT_MASK, b = hr[p] & CNT_MASK;
    soff[p + 1] = soff[p] + a;
    d->recv_off[p + 1] = d->recv_off[p] + b;
  }
  const uint64_t total = d->recv_off[G];
  if (!lerr) lerr = grow(&d->recv, &d->recv_cap, std::max<uint64_t>(total, 1) * rb);
  // every rank can receive (and send) before anyone starts: agree
  if ((st = agree(ctx, d, lerr))) return st;
  for (u32 p = 0; p < G; ++p) {
    slen[p] = (hs[p] & CNT_MASK) * rb;
    rlen[p] = (hr[p] & CNT_MASK) * rb;
    soff[p] *= rb;
    roff[p] = d->recv_off[p] * rb;
  }
  // this rank's rows to itself stay where the scatter put them (take reads
  // them there): at world 1 the whole batch, at world G a G-th of it, is not
  // copied through the transport
  const u32 me = (u32)d->rank;
  const size_t self_off = soff[me];
  const uint64_t self_row = self_off / rb;
  slen[me] = rlen[me] = 0;
  if (narrow) {
    // three arrays, each exchanged per peer at its own element size; the
    // owner column of this rank's own rows is copied into place, so the
    // received owner column is contiguous
    const size_t esz[3] = {16, 4, 4}, sb0[3] = {0, n * 16, n * 20}, rb0[3] = {0, total * 16, total * 20};
    for (int k = 0; k < 3; ++k) {
      uint64_t so[MAX_BUCKETS], sl[MAX_BUCKETS], ro[MAX_BUCKETS], rl[MAX_BUCKETS];
      for (u32 p = 0; p < G; ++p) {
        so[p] = soff[p] / rb * esz[k];
        sl[p] = slen[p] / rb * esz[k];
        ro[p] = roff[p] / rb * esz[k];
        rl[p] = rlen[p] / rb * esz[k];
      }
      if ((st = d->tx->exchange(d->send + sb0[k], so, sl, d->recv + rb0[k], ro, rl, ctx->stream))) return st;
    }
    const uint64_t mine = d->recv_off[me + 1] - d->recv_off[me];
    if (mine)
      HIPR(hipMemcpyAsync(d->recv + total * 20 + d->recv_off[me] * 4, d->send + n * 20 + self_row * 4, mine * 4,
                          hipMemcpyDeviceToDevice, ctx->stream));
  } else if ((st = d->tx->exchange(d->send, soff, slen, d->recv, roff, rlen, ctx->stream))) {
    return st;
  }
  d->self_off = self_off;
  d->self_row = self_row;
  d->self_lo = d->recv_off[me];
  d->self_hi = d->recv_off[me + 1];
  // receive offsets on the device (source rank of every row in evm_dist_take)
  u64* droff = d->cnt + W_ROFF;
  for (u32 p = 0; p <= G; ++p) d->hcnt[W_ROFF + p] = d->recv_off[p];
  HIPR(hipMemcpyAsync(droff, d->hcnt + W_ROFF, (G + 1) * sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  d->stride = stride;
  d->rb = rb;
  d->packed = packed ? 1 : 0;
  d->narrow = narrow ? 1 : 0;
  d->n_recv = total;
  d->n_in = n;
  d->send_gen = ++d->route_gen;
  if (keep0 && narrow) {
    d->self_ts = ts;
    d->self_stride = stride;
  }
  for (u32 p = 0; p < G; ++p) {
    d->sent[p] = hs[p] & CNT_MASK;
    d->recvd[p] = hr[p] & CNT_MASK;
  }
  *n_recv = total;
  return bad_dest ? EVM_EINVAL : hip_ok(hipGetLastError());
}

int evm_dist_take(evm_ctx* ctx, evm_dist* d, uint32_t group, char* out_ts, size_t out_stride, uint32_t* out_owner,
                  uint32_t* out_aux, uint64_t* out_src, uint64_t cap, uint64_t* group_off) {
  if (!ctx || !d || (group && !group_off) || group > MAX_BUCKETS) return EVM_EINVAL;
  const size_t n = d->n_recv;
  if (n && (!out_ts || !out_owner || out_stride < d->stride || out_stride % 8)) return EVM_EINVAL;
  if (n && d->narrow && out_src) return EVM_EINVAL;  // (a EVM_ROUTE_NO_SRC route carried no source indexes)
  // record format + rebuilt rows: 16-B stores, or 8-B stores into an output that is only 8-B aligned
  const int packed = d->packed ? ((d->narrow ? (int)FMT_NARROW : (int)FMT_PACKED) |
                                  ((out_stride % 16 || ((uintptr_t)out_ts & 15)) ? (int)FMT_ST8 : 0))
                               : (int)FMT_RAW;
  if (n > cap) return EVM_ECAPACITY;
  if (!self_rows_intact(d)) return EVM_EINVAL;
  const u32 G = (u32)d->world;
  const u64* droff = d->cnt + W_ROFF;
  const Route R = route_of(d, nullptr, nullptr);
  const size_t ooff = d->packed ? 16 : d->stride;
  if (!group) {
    if (n)
      KLAUNCH((k_dist_scatter<RECV>), dim3((u32)((n + DTILE - 1) / DTILE)), dim3(DT), R, (const char*)nullptr,
              d->stride, (const u32*)nullptr, d->recv, d->rb, packed, n, 1u, 0, 1u, (const u32*)nullptr,
              (char*)nullptr, out_ts, out_stride, out_owner, out_aux, (u64*)out_src, droff, G + 1, (u32*)nullptr,
              (size_t)0);
    return hip_ok(hipGetLastError());
  }
  Scratch S(ctx);
  u32* bad = S.alloc<u32>(1);
  u64* tot = S.alloc<u64>(MAX_BUCKETS + 1);
  if (!bad || !tot) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  HIPR(hipMemsetAsync(tot, 0, (MAX_BUCKETS + 1) * sizeof(u64), ctx->stream));
  if (n) {
    u32* offs = nullptr;
    u32 nblocks = 0;
    int st = partition_offsets<RECV>(ctx, S, R, d->recv, d->rb, ooff, n, group, &offs, &nblocks, tot, bad);
    if (st) return st;
    KLAUNCH((k_dist_scatter<RECV>), dim3(nblocks), dim3(DT), R, (const char*)nullptr, d->stride, (const u32*)nullptr,
            d->recv, d->rb, packed, n, group, ceil_log2(group), nblocks, offs, (char*)nullptr, out_ts, out_stride,
            out_owner, out_aux, (u64*)out_src, droff, G + 1, (u32*)nullptr, (size_t)0);
  }
  HIPR(hipMemcpyAsync(tot + MAX_BUCKETS, bad, sizeof(u32), hipMemcpyDeviceToDevice, ctx->stream));
  uint64_t h[MAX_BUCKETS + 1];
  HIPR(hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if ((uint32_t)h[MAX_BUCKETS]) return EVM_EINVAL;  // a local owner >= group
  group_off[0] = 0;
  for (u32 b = 0; b < group; ++b) group_off[b + 1] = group_off[b] + h[b];
  return EVM_OK;
}

uint64_t evm_dist_received(const evm_dist* d) { return d ? d->n_recv : 0; }

int evm_dist_ingest(evm_ctx* ctx, evm_dist* d, evm_store* store, uint64_t id_base, uint8_t* flags) {
  if (!ctx || !d || !store) return EVM_EINVAL;
  const size_t n = d->n_recv;
  if (n == 0) return EVM_OK;
  if (!flags || !(d->dir_local || d->hot)) return EVM_EINVAL;  // local ids come from the directory / split
  if (!self_rows_intact(d)) return EVM_EINVAL;
  if (d->self_identity)  // (world 1: the caller's rows and owners, as they lie)
    return evm_server_ingest(ctx, store, d->self_ts, d->self_stride, n, d->self_owner, id_base, flags);
  const Route R = route_of(d, nullptr, nullptr);
  if (d->packed && d->narrow) {  // the owner column arrived as the store's owner ids
    const WireSrc w{nullptr,  nullptr,  R.self_lo,  R.self_hi,          0u,         0u,
                    R.soa_a,  R.self_a, R.soa_b,    R.self_b,           (const uint8_t*)d->self_ts,
                    (u32)d->self_stride, d->self_idx};
    return server_ingest_wire(ctx, store, w, n, R.soa_c, id_base, flags);
  }
  Scratch S(ctx);
  u32* owner = S.alloc<u32>(n);
  if (!owner) return EVM_ENOMEM;
  if (!d->packed) {
    // raw records (some rank's rows are outside the native domain): the rows
    // themselves, then the ingest that flags the culprits
    const size_t os = (d->stride + 15) & ~(size_t)15;
    char* rows = S.alloc<char>(n * os);
    if (!rows) return EVM_ENOMEM;
    int st = evm_dist_take(ctx, d, 0, rows, os, owner, nullptr, nullptr, n, nullptr);
    if (st) return st;
    return evm_server_ingest(ctx, store, rows, os, n, owner, id_base, flags);
  }
  KLAUNCH(k_dist_owner, dim3(grid_for(n, 256, 16384)), dim3(256), R, (const char*)d->recv, d->rb, n, owner);
  const WireSrc w{d->recv, R.self_rec, R.self_lo, R.self_hi, (u32)d->rb, 28u, nullptr, nullptr, nullptr, nullptr};
  return server_ingest_wire(ctx, store, w, n, owner, id_base, flags);
}

int evm_dist_gather_roots(evm_ctx* ctx, evm_dist* d, const evm_tree* const* trees, uint32_t n_trees,
                          uint32_t n_owners_global, int32_t* root, uint8_t* present) {
  if (!ctx || !d) return EVM_EINVAL;  // nothing to join the collective with
  const u32 G = (u32)d->world;
  // every rank sizes the gather alike: from the directory, or ceil(n / world)
  // (a split adds its hot slots after every rank's cold ones)
  const u32 per = (d->hot ? d->hot_base + d->n_hot : d->dir_dest ? d->dir_per : (n_owners_global + G - 1) / G);
  const u32 stride = per + 1;  // + one status word per rank
  int lerr = EVM_OK;
  if ((n_trees && !trees) || (n_owners_global && (!root || !present))) lerr = EVM_EINVAL;
  if (d->dir_dest && n_owners_global != d->n_dir) lerr = EVM_EINVAL;
  if (d->hot && n_owners_global != d->n_hot_tab) lerr = EVM_EINVAL;
  size_t local = 0;
  for (u32 k = 0; k < n_trees && !lerr; ++k) {
    if (!trees[k]) lerr = EVM_EINVAL;
    else local += trees[k]->n_owners;
  }
  if (!lerr && local > per) lerr = EVM_EINVAL;
  Scratch S(ctx);
  u64* mine = S.alloc<u64>(stride);
  u64* all = S.alloc<u64>((size_t)stride * G);
  if (!mine || !all) return EVM_ENOMEM;  // (a scratch pool failure leaves nothing to send from)
  HIPR(hipMemsetAsync(mine, 0, sizeof(u64) * stride, ctx->stream));
  if (!lerr) {
    // this rank's local owners: the trees' owners in order, then zeros up to `per`
    u32 at = 0;
    for (u32 k = 0; k < n_trees; ++k) {
      const evm_tree* t = trees[k];
      if (t->n_owners)
        KLAUNCH(k_dist_root_pack, dim3(grid_for(t->n_owners, 256)), dim3(256), t->off, t->end, t->pfx, t->n_owners,
                t->n_owners, mine + at);
      at += t->n_owners;
    }
  }
  d->hcnt[W_AGREE_S] = (u64)(u32)lerr;
  HIPR(hipMemcpyAsync(mine + per, d->hcnt + W_AGREE_S, sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  int st = d->tx->all_gather_u64(mine, all, stride, ctx->stream);
  if (st) return st;
  // any rank's status word set: every rank fails
  u64* hs = d->hcnt + W_AGREE_R;
  HIPR(hipMemcpy2DAsync(hs, sizeof(u64), all + per, stride * sizeof(u64), sizeof(u64), G, hipMemcpyDeviceToHost,
                        ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (lerr) return lerr;
  for (u32 p = 0; p < G; ++p)
    if (hs[p]) return EVM_EDIST;
  if (!n_owners_global) return EVM_OK;
  KLAUNCH(k_dist_root_unpack, dim3(grid_for(n_owners_global, 256)), dim3(256), all, G, stride, n_owners_global,
          d->dir_dest, d->dir_local, (const u32*)d->hot, d->n_hot_tab, d->hot_base, root, present);
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

// ------------------------------------------------------------------ hot-owner split
int evm_dist_hot_owners(evm_ctx* ctx, evm_dist* d, const uint32_t* owner, size_t n, uint32_t n_owners_global,
                        double share, uint32_t* hot, uint32_t cap, uint32_t* n_hot) {
  if (!ctx || !d || !n_hot) return EVM_EINVAL;
  *n_hot = 0;
  const u32 G = (u32)d->world;
  int lerr = EVM_OK;
  if ((n && !owner) || (cap && !hot) || !(share > 0.0)) lerr = EVM_EINVAL;
  // the owner count and the total rows must agree before the count gather
  uint64_t vals[MAX_BUCKETS];
  int st = gather_status(ctx, d, lerr, n_owners_global, vals);
  if (st) return st;
  for (u32 p = 0; p < G; ++p)
    if (vals[p] != n_owners_global) lerr = EVM_EINVAL;
  if ((st = gather_status(ctx, d, lerr, n, vals))) return st;
  uint64_t total = 0;
  for (u32 p = 0; p < G; ++p) total += vals[p];
  if (G == 1 || n_owners_global == 0) return EVM_OK;
  Scratch S(ctx);
  u64* counts = S.alloc<u64>(n_owners_global);
  u64* all = S.alloc<u64>((size_t)n_owners_global * G);
  u32* list = S.alloc<u32>((size_t)std::max<u32>(cap, 1) + 2);
  lerr = (!counts || !all || !list) ? EVM_ENOMEM : EVM_OK;
  if (!lerr) {
    lerr = hip_ok(hipMemsetAsync(counts, 0, sizeof(u64) * n_owners_global, ctx->stream));
    if (!lerr) lerr = hip_ok(hipMemsetAsync(list, 0, sizeof(u32) * 2, ctx->stream));
    if (!lerr && n)
      KLAUNCH(k_split_hist, dim3(grid_for(n, 256)), dim3(256), owner, n, n_owners_global, counts, list + 1);
  }
  if ((st = gather_status(ctx, d, lerr, 0, nullptr))) return st;
  if ((st = d->tx->all_gather_u64(counts, all, n_owners_global, ctx->stream))) return st;
  // hot: more than `share` of one rank's fair share of all rows
  const double fair = (double)total / G;
  const u64 thr = (u64)(share * fair);
  KLAUNCH(k_split_select, dim3(grid_for(n_owners_global, 256)), dim3(256), (const u64*)all, G,
          (size_t)n_owners_global, n_owners_global, thr, list + 2, list, cap);
  u32 h[2];
  HIPR(hipMemcpyAsync(h, list, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (h[1]) return EVM_EINVAL;  // an owner id >= n_owners_global (after the collectives: nobody waits)
  *n_hot = h[0];
  if (h[0] > cap) return EVM_ECAPACITY;
  if (h[0]) {
    HIPR(hipMemcpyAsync(hot, list + 2, sizeof(u32) * h[0], hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    std::sort(hot, hot + h[0]);  // (the device list is in arrival order)
  }
  return EVM_OK;
}

int evm_dist_split(evm_ctx* ctx, evm_dist* d, const uint32_t* hot, uint32_t n_hot, uint32_t n_owners_global,
                   uint32_t* hot_base) {
  if (!ctx || !d || (n_hot && !hot) || n_hot > n_owners_global) return EVM_EINVAL;
  if (d->dir_dest && n_owners_global != d->n_dir) return EVM_EINVAL;
  std::vector<u32> tab;
  if (n_hot) {
    tab.assign(n_owners_global, HOT_NONE);
    for (u32 h = 0; h < n_hot; ++h) {
      if (hot[h] >= n_owners_global || tab[hot[h]] != HOT_NONE) return EVM_EINVAL;  // in range, no repeats
      tab[hot[h]] = h;
    }
  }
  if (d->hot) (void)hipFree(d->hot);
  d->hot = nullptr;
  d->n_hot_tab = d->n_hot = d->hot_base = 0;
  const u32 G = (u32)d->world;
  const u32 base = d->dir_dest ? d->dir_per : (n_owners_global + G - 1) / G;
  if (hot_base) *hot_base = base;
  if (!n_hot) return EVM_OK;
  HIPR(hipMalloc(&d->hot, sizeof(u32) * n_owners_global));
  HIPR(hipMemcpyAsync(d->hot, tab.data(), sizeof(u32) * n_owners_global, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  d->n_hot_tab = n_owners_global;
  d->n_hot = n_hot;
  d->hot_base = base;
  return EVM_OK;
}

int evm_dist_ts_dest(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, uint8_t* dest) {
  if (!ctx || !d || stride < 48 || stride % 8 || (n && (!ts || !dest))) return EVM_EINVAL;
  if (n) KLAUNCH(k_ts_dest, dim3(grid_for(n, 256)), dim3(256), ts, stride, n, (u32)d->world, dest);
  return hip_ok(hipGetLastError());
}

int evm_dist_cell_dest(evm_ctx* ctx, evm_dist* d, const uint32_t* cell, size_t n, uint8_t* dest) {
  if (!ctx || !d || (n && (!cell || !dest))) return EVM_EINVAL;
  if (n) KLAUNCH(k_cell_dest, dim3(grid_for(n, 256)), dim3(256), cell, n, (u32)d->world, dest);
  return hip_ok(hipGetLastError());
}

int evm_dist_merge_trees(evm_ctx* ctx, evm_dist* d, const evm_tree* t, uint32_t owner_lo, uint32_t count,
                         evm_tree** out) {
  if (!ctx || !d || !out) return EVM_EINVAL;
  *out = nullptr;
  const u32 G = (u32)d->world;
  int lerr = EVM_OK;
  if (!t || owner_lo + (uint64_t)count > t->n_owners) lerr = EVM_EINVAL;
  if (!lerr) lerr = tree_compact(ctx, t);  // (a rank that fails still joins the gathers, flagged)
  u64 ab[2] = {0, 0};
  if (!lerr && count) {
    HIPR(hipMemcpyAsync(&ab[0], t->off + owner_lo, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipMemcpyAsync(&ab[1], t->off + owner_lo + count, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
  }
  const u64 L = ab[1] - ab[0];
  const u64 words = 1 + L + (L + 1) / 2;
  uint64_t sizes[MAX_BUCKETS];
  // (count must match too: every rank's parts are trees of `count` owners)
  int st = gather_status(ctx, d, lerr, ((u64)count << 40) | words, sizes);
  if (st) return st;
  u64 per = 0;
  for (u32 p = 0; p < G; ++p) {
    if ((sizes[p] >> 40) != count) lerr = EVM_EINVAL;
    per = std::max<u64>(per, sizes[p] & ((1ull << 40) - 1));
  }
  Scratch S(ctx);
  u64* mine = S.alloc<u64>(per);
  u64* all = S.alloc<u64>(per * G);
  if (!lerr && (!mine || !all)) lerr = EVM_ENOMEM;
  if (!lerr)
    KLAUNCH(k_merge_pack, dim3(grid_for(std::max<u64>(L, 1), 256)), dim3(256), (const u64*)t->ck, t->xr, ab[0], L,
            owner_lo, mine);
  if ((st = gather_status(ctx, d, lerr, 0, nullptr))) return st;
  if ((st = d->tx->all_gather_u64(mine, all, per, ctx->stream))) return st;
  // XOR-merge the parts in rank order (the same tree on every rank)
  evm_tree* acc = nullptr;
  for (u32 p = 0; p < G; ++p) {
    const u64* A = all + (size_t)p * per;
    u64 lp = 0;  // (the part's leaf count: its first word)
    HIPR(hipMemcpyAsync(&lp, A, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    const u64* ckp = A + 1;
    const int32_t* xrp = reinterpret_cast<const int32_t*>(A + 1 + lp);
    evm_tree* next = nullptr;
    st = acc ? merge_into_tree(ctx, S, acc, count, ckp, xrp, lp, &next) : tree_finalize(ctx, S, count, ckp, xrp, lp, &next);
    if (acc) tree_destroy(ctx, acc);
    if (st) {
      if (next) tree_destroy(ctx, next);
      return st;
    }
    acc = next;
  }
  *out = acc;
  return evm_sync(ctx);
}

int evm_dist_merge_select(evm_ctx* ctx, evm_dist* d, uint32_t n_groups, const uint64_t* off, const uint64_t* id,
                          const uint64_t* key, uint64_t* out_off, uint64_t* out_id, uint64_t cap, uint64_t* n_out) {
  if (!ctx || !d || !n_out) return EVM_EINVAL;
  *n_out = 0;
  const u32 G = (u32)d->world;
  int lerr = EVM_OK;
  if (!off || !out_off) lerr = EVM_EINVAL;
  u64 ab[2] = {0, 0};
  if (!lerr) {
    HIPR(hipMemcpyAsync(&ab[0], off, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipMemcpyAsync(&ab[1], off + n_groups, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    if (ab[1] < ab[0] || (ab[1] > ab[0] && (!id || !key))) lerr = EVM_EINVAL;
  }
  const u64 m = lerr ? 0 : ab[1] - ab[0];
  uint64_t sizes[MAX_BUCKETS];
  int st = gather_status(ctx, d, lerr, ((u64)n_groups << 40) | m, sizes);
  if (st) return st;
  u64 rb[MAX_BUCKETS + 1];
  rb[0] = 0;
  u64 mx = 0;
  for (u32 p = 0; p < G; ++p) {
    if ((sizes[p] >> 40) != n_groups) lerr = EVM_EINVAL;
    const u64 mp = sizes[p] & ((1ull << 40) - 1);
    rb[p + 1] = rb[p] + mp;
    mx = std::max<u64>(mx, mp);
  }
  const u64 per = (u64)n_groups + 1 + 4 * mx;
  Scratch S(ctx);
  u64* mine = S.alloc<u64>(per);
  u64* all = S.alloc<u64>(per * G);
  u64* drb = S.alloc<u64>(G + 1);
  if (!lerr && (!mine || !all || !drb)) lerr = EVM_ENOMEM;
  if (!lerr) {
    KLAUNCH(k_sel_pack, dim3(grid_for(n_groups + 1 + 4 * m, 256)), dim3(256), off, id, key, n_groups, m, mine);
    // every rank's row count sits at its word n_groups (its last offset)
    lerr = hip_ok(hipMemcpyAsync(drb, rb, sizeof(u64) * (G + 1), hipMemcpyHostToDevice, ctx->stream));
  }
  if ((st = gather_status(ctx, d, lerr, 0, nullptr))) return st;
  if ((st = d->tx->all_gather_u64(mine, all, per, ctx->stream))) return st;
  const u64 M = rb[G];
  *n_out = M;
  KLAUNCH(k_sel_off, dim3(grid_for(n_groups + 1, 256)), dim3(256), (const u64*)all, G, (size_t)per, n_groups, out_off);
  if (M > cap) {
    HIPR(hipStreamSynchronize(ctx->stream));
    return EVM_ECAPACITY;
  }
  if (M) {
    if (!out_id) return EVM_EINVAL;
    KLAUNCH(k_sel_merge, dim3(grid_for(M, 256)), dim3(256), (const u64*)all, G, (size_t)per, n_groups,
            (const u64*)drb, out_off, out_id);
  }
  return evm_sync(ctx);
}

int evm_dist_return(evm_ctx* ctx, evm_dist* d, const void* val, uint32_t elem, void* out, size_t n_out) {
  if (!ctx || !d) return EVM_EINVAL;
  const u32 G = (u32)d->world;
  const size_t n = d->n_recv;
  int lerr = EVM_OK;
  if ((elem != 1 && elem != 2 && elem != 4 && elem != 8) || (n && !val) || (n_out && !out)) lerr = EVM_EINVAL;
  if (d->narrow) lerr = EVM_EINVAL;  // the last route carried no source indexes (EVM_ROUTE_NO_SRC)
  if (!self_rows_intact(d)) lerr = EVM_EINVAL;
  const size_t ooff = d->packed ? 16 : d->stride;
  Scratch S(ctx);
  u32* bad = S.alloc<u32>(1);
  u64 back = 0;
  for (u32 p = 0; p < G; ++p) back += d->sent[p];
  if (!bad) lerr = lerr ? lerr : EVM_ENOMEM;
  // (the packed pairs go to scratch: the send buffer still holds this rank's own rows)
  u64* sbuf = S.alloc<u64>(2 * std::max<size_t>(n, 1));
  u64* rbuf = S.alloc<u64>(2 * std::max<u64>(back, 1));
  if (!lerr && (!rbuf || !sbuf)) lerr = EVM_ENOMEM;
  if (!lerr) {
    lerr = hip_ok(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
    if (!lerr && n)
      KLAUNCH(k_ret_pack, dim3(grid_for(n, 256)), dim3(256), route_of(d, nullptr, nullptr), (const char*)d->recv,
              d->rb, ooff, n, (const uint8_t*)val, elem, sbuf);
  }
  if (int st = agree(ctx, d, lerr)) return st;
  // rows go back to the rank they came from: the route's counts reversed
  uint64_t soff[MAX_BUCKETS], slen[MAX_BUCKETS], roff[MAX_BUCKETS], rlen[MAX_BUCKETS];
  uint64_t so = 0, ro = 0;
  for (u32 p = 0; p < G; ++p) {
    soff[p] = so * 16;
    slen[p] = d->recvd[p] * 16;
    roff[p] = ro * 16;
    rlen[p] = d->sent[p] * 16;
    so += d->recvd[p];
    ro += d->sent[p];
  }
  int st = d->tx->exchange(reinterpret_cast<const char*>(sbuf), soff, slen, reinterpret_cast<char*>(rbuf), roff, rlen,
                           ctx->stream);
  if (st) return st;
  if (back)
    KLAUNCH(k_ret_scatter, dim3(grid_for(back, 256)), dim3(256), (const u64*)rbuf, (size_t)back, (uint8_t*)out, n_out,
            elem, bad);
  u32 hb = 0;
  HIPR(hipMemcpyAsync(&hb, bad, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  return hb ? EVM_EINVAL : EVM_OK;  // a source index >= n_out
}

int evm_dist_split_winners(evm_ctx* ctx, evm_dist* d, const int32_t* win, uint32_t n_cells, int64_t* out) {
  if (!ctx || !d) return EVM_EINVAL;
  const u32 G = (u32)d->world;
  int lerr = EVM_OK;
  if (n_cells && (!win || !out)) lerr = EVM_EINVAL;
  if (d->narrow) lerr = EVM_EINVAL;  // (no source indexes)
  if (!self_rows_intact(d)) lerr = EVM_EINVAL;
  uint64_t nin[MAX_BUCKETS];
  int st = gather_status(ctx, d, lerr, ((u64)n_cells << 40) | d->n_in, nin);
  if (st) return st;
  u64 base[MAX_BUCKETS + 1];
  base[0] = 0;
  for (u32 p = 0; p < G; ++p) {
    if ((nin[p] >> 40) != n_cells) lerr = EVM_EINVAL;
    base[p + 1] = base[p] + (nin[p] & ((1ull << 40) - 1));
  }
  Scratch S(ctx);
  u64* mine = S.alloc<u64>(std::max<u32>(n_cells, 1));
  u64* all = S.alloc<u64>((size_t)std::max<u32>(n_cells, 1) * G);
  u64* dbase = S.alloc<u64>(G + 1);
  u32* bad = S.alloc<u32>(1);
  if (!lerr && (!mine || !all || !dbase || !bad)) lerr = EVM_ENOMEM;
  if (!lerr) {
    lerr = hip_ok(hipMemcpyAsync(dbase, base, sizeof(u64) * (G + 1), hipMemcpyHostToDevice, ctx->stream));
    if (!lerr) lerr = hip_ok(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
    if (!lerr && n_cells)
      KLAUNCH(k_win_map, dim3(grid_for(n_cells, 256)), dim3(256), route_of(d, nullptr, nullptr), win, n_cells,
              (const char*)d->recv, d->rb,
              d->packed ? (size_t)16 : d->stride, (u64)d->n_recv, (const u64*)(d->cnt + W_ROFF), G,
              (const u64*)dbase, mine, bad);
    if (!lerr) {
      u32 hb = 0;
      lerr = hip_ok(hipMemcpyAsync(&hb, bad, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
      if (!lerr) lerr = hip_ok(hipStreamSynchronize(ctx->stream));
      if (!lerr && hb) lerr = EVM_EINVAL;  // a winner past the received rows
    }
  }
  if ((st = gather_status(ctx, d, lerr, 0, nullptr))) return st;
  if (!n_cells) return EVM_OK;
  if ((st = d->tx->all_gather_u64(mine, all, n_cells, ctx->stream))) return st;
  KLAUNCH(k_win_reduce, dim3(grid_for(n_cells, 256)), dim3(256), (const u64*)all, G, (size_t)n_cells, n_cells, out);
  return evm_sync(ctx);
}

int evm_dist_agree_status(evm_ctx* ctx, evm_dist* d, int32_t local, int32_t* max_status) {
  if (!ctx || !d || !max_status) return EVM_EINVAL;
  const u32 G = (u32)d->world;
  uint64_t v[MAX_BUCKETS];
  const int st = gather_status(ctx, d, EVM_OK, (u64)(u32)local, v);
  if (st) return st;
  int32_t m = 0;
  for (u32 p = 0; p < G; ++p) m = std::max<int32_t>(m, (int32_t)(u32)v[p]);
  *max_status = m;
  return EVM_OK;
}

}  // extern "C"
