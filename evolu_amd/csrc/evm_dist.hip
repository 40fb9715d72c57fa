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
    for (int p = 0; p < world; ++p) {
      uint64_t o = 0;
      do {
        const uint64_t k = std::min<uint64_t>(CHUNK, slen[p] - o);
        if (r->send(sbase + soff[p] + o, k, ncclUint8, p, comm, s) != ncclSuccess) st = EVM_EDIST;
        o += k;
      } while (o < slen[p]);
      o = 0;
      do {
        const uint64_t k = std::min<uint64_t>(CHUNK, rlen[p] - o);
        if (r->recv(rbase + roff[p] + o, k, ncclUint8, p, comm, s) != ncclSuccess) st = EVM_EDIST;
        o += k;
      } while (o < rlen[p]);
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
constexpr u32 PK_VALID = 1u << 16;
// count words exchanged per route: the row count in the low bits, flags on top
constexpr u64 CNT_ERR = 1ull << 63;      // the sending rank failed locally (nothing is exchanged)
constexpr u64 CNT_INVALID = 1ull << 62;  // the sending rank holds a row outside the native domain
constexpr u64 CNT_MASK = (1ull << 48) - 1;
// d->cnt layout (u64 words, mirrored in pinned host memory)
constexpr u32 W_SEND = 0;                      // [64] send counts
constexpr u32 W_RECV = MAX_BUCKETS;            // [64] receive counts
constexpr u32 W_ROFF = 2 * MAX_BUCKETS;        // [65] receive offsets (rows)
constexpr u32 W_AGREE_S = 3 * MAX_BUCKETS + 8; // [64] agreement words sent
constexpr u32 W_AGREE_R = 4 * MAX_BUCKETS + 8; // [64] agreement words received
constexpr u32 W_BAD = 5 * MAX_BUCKETS + 8;     // the local flags: [0] bad destination, [1] invalid row
constexpr u32 CNT_WORDS = 5 * MAX_BUCKETS + 16;

// Routing of row i.  SEND: the destination rank -- the caller's dest, the
// directory's rank of the owner, or owner % world.  RECV (wire records, owner
// at byte `ooff`): the local owner -- the directory's local id, or owner /
// world.  >= B: out of range (reported, not routed).
struct Route {
  const u32* owner;
  const uint8_t* dest;
  const uint8_t* dir_dest;   // directory: rank of every global owner
  const u32* dir_local;      // directory: local id of every global owner on its rank
  u32 n_dir;
  u32 world;
};

template <int MODE>
__device__ __forceinline__ u32 bucket_of(size_t i, const Route& R, const char* rec, size_t rb, size_t ooff) {
  if (MODE == 0) {
    if (R.dest) return R.dest[i];
    const u32 o = R.owner[i];
    if (R.dir_dest) return o < R.n_dir ? (u32)R.dir_dest[o] : 0xffffffffu;
    return o % R.world;
  }
  const u32 o = *reinterpret_cast<const u32*>(rec + i * rb + ooff);
  if (R.dir_local) return o < R.n_dir ? R.dir_local[o] : 0xffffffffu;
  return o / R.world;
}
enum { SEND = 0, RECV = 1 };

// Packed wire form of a 48-B timestamp row: the parsed (tc, node, case mask)
// -- 16 B instead of 46 -- from which the receiver rebuilds the identical
// string with format_ts46 (a canonical timestamp is a function of them,
// timestamp.ts:43-55).  Only a route whose rows are ALL in the native domain
// travels packed; one row outside it anywhere in the job sends every rank's
// rows raw.

// per-block bucket counts, bucket-major ([b * nblocks + block]): their
// exclusive scan is every (bucket, block)'s first output slot, stable
template <int MODE>
__global__ __launch_bounds__(DT) void k_dist_count(Route R, const char* __restrict__ rec, size_t rb, size_t ooff,
                                                   size_t n, u32 B, u32 nblocks, u32* __restrict__ counts,
                                                   u32* __restrict__ bad) {
  __shared__ u32 c[MAX_BUCKETS];
  if (threadIdx.x < MAX_BUCKETS) c[threadIdx.x] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * DTILE;
  bool oob = false;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    if (i < n) {
      const u32 b = bucket_of<MODE>(i, R, rec, rb, ooff);
      if (b < B) atomicAdd(&c[b], 1u);
      else oob = true;
    }
  }
  __syncthreads();
  if (threadIdx.x < B) counts[(size_t)threadIdx.x * nblocks + blockIdx.x] = c[threadIdx.x];
  if (__ballot(oob) && __lane_id() == 0) atomicOr(bad, 1u);
}

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
template <int MODE>
__global__ __launch_bounds__(DT) void k_dist_scatter(
    Route R, const char* __restrict__ ts, size_t stride, const u32* __restrict__ aux, const char* __restrict__ rec,
    size_t rb, int packed, size_t n, u32 B, int bits, u32 nblocks, const u32* __restrict__ offs,
    char* __restrict__ out_rec, char* __restrict__ out_ts, size_t out_stride, u32* __restrict__ out_owner,
    u32* __restrict__ out_aux, u64* __restrict__ out_src, const u64* __restrict__ roff, u32 n_src,
    u32* __restrict__ invalid) {
  __shared__ Ranker L;
  if (offs && threadIdx.x < B) L.run[threadIdx.x] = offs[(size_t)threadIdx.x * nblocks + blockIdx.x];
  const size_t base = (size_t)blockIdx.x * DTILE;
  bool inv = false;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    const bool ok = i < n;
    size_t pos = i;
    if (offs) {
      const u32 b = ok ? bucket_of<MODE>(i, R, rec, rb, packed ? 16 : stride) : 0u;
      const bool act = ok && b < B;
      const u32 p = rank_slot(L, r, b, act, B, bits);
      if (!act) continue;  // (a row with an out-of-range bucket is reported by k_dist_count)
      pos = p;
    } else if (!ok) {
      continue;
    }
    if (MODE == SEND && packed) {
      const uint4* row = reinterpret_cast<const uint4*>(ts + i * stride);
      const uint4 x = row[0], y = row[1], z = row[2];
      const u32 w[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w & 0xffffu};
      const Parsed p = parse_ts46(w);
      inv |= (p.meta & EVM_META_VALID) == 0;
      uint4* dst = reinterpret_cast<uint4*>(out_rec + pos * rb);
      dst[0] = make_uint4((u32)p.tc, (u32)(p.tc >> 32), (u32)p.node, (u32)(p.node >> 32));
      dst[1] = make_uint4(R.owner[i], aux ? aux[i] : 0u, (u32)i,
                          (p.meta & EVM_META_CASEMASK) | ((p.meta & EVM_META_VALID) ? PK_VALID : 0u));
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
      const char* src = rec + i * rb;
      uint4 m;
      if (packed) {
        const uint4 a = reinterpret_cast<const uint4*>(src)[0];
        m = reinterpret_cast<const uint4*>(src)[1];
        u32 w[12];
        format_ts46((u64)a.x | ((u64)a.y << 32), (u64)a.z | ((u64)a.w << 32), m.w & 0xffffu, w);
        uint4* dst = reinterpret_cast<uint4*>(out_ts + pos * out_stride);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
        dst[2] = make_uint4(w[8], w[9], w[10], w[11]);
      } else {
        copy_row(out_ts + pos * out_stride, src, stride);
        m = *reinterpret_cast<const uint4*>(src + stride);
      }
      out_owner[pos] = R.dir_local ? (m.x < R.n_dir ? R.dir_local[m.x] : 0xffffffffu) : m.x;
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
  if (MODE == SEND && packed && invalid && __ballot(inv) && __lane_id() == 0) atomicOr(invalid, 1u);
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
__global__ void k_dist_mark(u64* __restrict__ cnt, u32 G, int zero, int err, const u32* __restrict__ flags) {
  const u32 p = threadIdx.x;
  if (p >= G) return;
  u64 v = zero ? 0ull : cnt[p];
  if (err) v |= CNT_ERR;
  if (flags && flags[1]) v |= CNT_INVALID;
  cnt[p] = v;
}

__global__ void k_dist_root_pack(const u64* __restrict__ off, const int32_t* __restrict__ pfx, u32 n_owners, u32 per,
                                 u64* __restrict__ out) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < per; o += gridDim.x * blockDim.x) {
    u64 v = 0;
    if (o < n_owners) {
      const u64 a = off[o], b = off[o + 1];
      v = (u64)(uint32_t)(pfx[b] ^ pfx[a]) | ((u64)(b > a) << 32);
    }
    out[o] = v;
  }
}

// gathered [rank][per + 1] -> global owner g: local g / world of rank g % world,
// or the directory's (rank, local) of g
__global__ void k_dist_root_unpack(const u64* __restrict__ all, u32 world, u32 stride, u32 n_global,
                                   const uint8_t* __restrict__ dir_dest, const u32* __restrict__ dir_local,
                                   int32_t* __restrict__ root, uint8_t* __restrict__ present) {
  for (u32 g = blockIdx.x * blockDim.x + threadIdx.x; g < n_global; g += gridDim.x * blockDim.x) {
    const u64 v = dir_dest ? all[(size_t)dir_dest[g] * stride + dir_local[g]] : all[(size_t)(g % world) * stride + g / world];
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

}  // namespace

struct evm_dist {
  Transport* tx = nullptr;
  int rank = 0, world = 1;
  size_t stride = 48, rb = 64;
  int packed = 0;  // the last route's records: packed (48-B rows) or raw
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
};

namespace {

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
  KLAUNCH((k_dist_count<MODE>), dim3(nblocks), dim3(DT), R, rec, rb, ooff, n, B, nblocks, counts, bad);
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
  if (d->recv) (void)hipFree(d->recv);
  if (d->cnt) (void)hipFree(d->cnt);
  if (d->hcnt) (void)hipHostFree(d->hcnt);
  if (d->dir_dest) (void)hipFree(d->dir_dest);
  if (d->dir_local) (void)hipFree(d->dir_local);
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
  d->dir_dest = nullptr;
  d->dir_local = nullptr;
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
  if (!ctx || !d || !n_recv) return EVM_EINVAL;  // nothing to join the collective with
  *n_recv = 0;
  d->n_recv = 0;
  const u32 G = (u32)d->world;
  int lerr = EVM_OK;  // a local failure: the rank still joins the count exchange, flagged
  if (stride < 46 || stride % 8 || (n && (!ts || !owner)) || n >= 0xffffffffull) lerr = EVM_EINVAL;
  // 48-B rows, 16-B aligned: packed 32-B records (a third of the xGMI bytes of raw ones)
  const bool packed0 = !lerr && stride == 48 && ((uintptr_t)ts & 15) == 0;
  size_t rb = packed0 ? PACKED : stride + META;
  Scratch S(ctx);
  u32* flags = S.alloc<u32>(2);  // [0] a destination out of range, [1] a row outside the native domain
  u64* scnt = d->cnt + W_SEND;
  u64* rcnt = d->cnt + W_RECV;
  const Route R = route_of(d, owner, dest);
  u32* offs = nullptr;
  u32 nblocks = 0;
  if (!flags) lerr = lerr ? lerr : EVM_ENOMEM;
  if (!lerr) lerr = hip_ok(hipMemsetAsync(flags, 0, 2 * sizeof(u32), ctx->stream));
  if (!lerr) lerr = grow(&d->send, &d->send_cap, std::max<size_t>(n, 1) * rb);
  if (!lerr && n) {
    lerr = partition_offsets<SEND>(ctx, S, R, nullptr, rb, stride, n, G, &offs, &nblocks, scnt, flags);
    if (!lerr) {
      KLAUNCH((k_dist_scatter<SEND>), dim3(nblocks), dim3(DT), R, ts, stride, aux, (const char*)nullptr, rb,
              packed0 ? 1 : 0, n, G, ceil_log2(G), nblocks, offs, d->send, (char*)nullptr, (size_t)0, (u32*)nullptr,
              (u32*)nullptr, (u64*)nullptr, (const u64*)nullptr, 0u, flags + 1);
      lerr = hip_ok(hipGetLastError());
    }
  }
  // the counts: one all-to-all of G words (flag bits on top), one read back
  KLAUNCH(k_dist_mark, dim3(1), dim3(MAX_BUCKETS), scnt, G, (lerr || !n) ? 1 : 0, lerr ? 1 : 0,
          (const u32*)(lerr ? nullptr : flags));
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
  bool any_err = lerr != EVM_OK, any_inv = false;
  for (u32 p = 0; p < G; ++p) {
    any_err |= (hr[p] & CNT_ERR) != 0;
    any_inv |= (hr[p] & CNT_INVALID) != 0;
  }
  if (any_err) return lerr ? lerr : EVM_EDIST;  // every rank saw the flag: nobody exchanges
  const bool bad_dest = d->hcnt[W_BAD] != 0;
  // a row outside the native domain anywhere: every rank sends raw records
  // (the packed form cannot carry the original bytes); same slots, wider records
  const bool packed = packed0 && !any_inv;
  if (packed0 && !packed) {
    rb = stride + META;
    lerr = grow(&d->send, &d->send_cap, std::max<size_t>(n, 1) * rb);
    if (!lerr && n) {
      KLAUNCH((k_dist_scatter<SEND>), dim3(nblocks), dim3(DT), R, ts, stride, aux, (const char*)nullptr, rb, 0, n, G,
              ceil_log2(G), nblocks, offs, d->send, (char*)nullptr, (size_t)0, (u32*)nullptr, (u32*)nullptr,
              (u64*)nullptr, (const u64*)nullptr, 0u, (u32*)nullptr);
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
  if ((st = d->tx->exchange(d->send, soff, slen, d->recv, roff, rlen, ctx->stream))) return st;
  // receive offsets on the device (source rank of every row in evm_dist_take)
  u64* droff = d->cnt + W_ROFF;
  for (u32 p = 0; p <= G; ++p) d->hcnt[W_ROFF + p] = d->recv_off[p];
  HIPR(hipMemcpyAsync(droff, d->hcnt + W_ROFF, (G + 1) * sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  d->stride = stride;
  d->rb = rb;
  d->packed = packed ? 1 : 0;
  d->n_recv = total;
  *n_recv = total;
  return bad_dest ? EVM_EINVAL : hip_ok(hipGetLastError());
}

int evm_dist_take(evm_ctx* ctx, evm_dist* d, uint32_t group, char* out_ts, size_t out_stride, uint32_t* out_owner,
                  uint32_t* out_aux, uint64_t* out_src, uint64_t cap, uint64_t* group_off) {
  if (!ctx || !d || (group && !group_off) || group > MAX_BUCKETS) return EVM_EINVAL;
  const size_t n = d->n_recv;
  if (n && (!out_ts || !out_owner || out_stride < d->stride || out_stride % 8)) return EVM_EINVAL;
  if (n && d->packed && (out_stride % 16 || ((uintptr_t)out_ts & 15))) return EVM_EINVAL;  // rebuilt rows: 16-B stores
  if (n > cap) return EVM_ECAPACITY;
  const u32 G = (u32)d->world;
  const u64* droff = d->cnt + W_ROFF;
  const Route R = route_of(d, nullptr, nullptr);
  const size_t ooff = d->packed ? 16 : d->stride;
  if (!group) {
    if (n)
      KLAUNCH((k_dist_scatter<RECV>), dim3((u32)((n + DTILE - 1) / DTILE)), dim3(DT), R, (const char*)nullptr,
              d->stride, (const u32*)nullptr, d->recv, d->rb, d->packed, n, 1u, 0, 1u, (const u32*)nullptr,
              (char*)nullptr, out_ts, out_stride, out_owner, out_aux, (u64*)out_src, droff, G + 1, (u32*)nullptr);
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
            d->recv, d->rb, d->packed, n, group, ceil_log2(group), nblocks, offs, (char*)nullptr, out_ts, out_stride,
            out_owner, out_aux, (u64*)out_src, droff, G + 1, (u32*)nullptr);
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

int evm_dist_gather_roots(evm_ctx* ctx, evm_dist* d, const evm_tree* const* trees, uint32_t n_trees,
                          uint32_t n_owners_global, int32_t* root, uint8_t* present) {
  if (!ctx || !d) return EVM_EINVAL;  // nothing to join the collective with
  const u32 G = (u32)d->world;
  // every rank sizes the gather alike: from the directory, or ceil(n / world)
  const u32 per = d->dir_dest ? d->dir_per : (n_owners_global + G - 1) / G;
  const u32 stride = per + 1;  // + one status word per rank
  int lerr = EVM_OK;
  if ((n_trees && !trees) || (n_owners_global && (!root || !present))) lerr = EVM_EINVAL;
  if (d->dir_dest && n_owners_global != d->n_dir) lerr = EVM_EINVAL;
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
        KLAUNCH(k_dist_root_pack, dim3(grid_for(t->n_owners, 256)), dim3(256), t->off, t->pfx, t->n_owners,
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
          d->dir_dest, d->dir_local, root, present);
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

}  // extern "C"
