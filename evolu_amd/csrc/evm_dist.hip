// Owner sharding over RCCL: the evm_dist_* C ABI.
//
// One process per GPU.  Owners are independent in the whole hot path (each is
// its own client database for applyMessages.ts:26-131; the server keys rows
// and trees by userId, apps/server/src/index.ts:64-75), so rank r serves the
// owners with owner % world == r and the only exchanges are
//
//   * evm_dist_route: messages to their owner's rank.  A stable partition by
//     destination packs 64-byte wire records (timestamp row + owner, aux,
//     source index) into one send buffer; one RCCL all-to-all of the G
//     per-destination counts, then one group of ncclSend/ncclRecv moves the
//     records -- each peer's records contiguous, so the receive buffer is in
//     (source rank, source order) = global batch order, which the
//     reference's first-occurrence rules depend on.  One G-entry count read
//     back to the host per call: RCCL's point-to-point calls take host counts.
//   * evm_dist_take: the received rows out of the staging buffer into the
//     caller's arrays, optionally grouped by local owner (a second stable
//     partition on the device) so each owner's rows are one contiguous
//     applyMessages batch.
//   * evm_dist_gather_roots: ncclAllGather of the per-owner roots (RCCL has
//     no XOR reduction and none is needed: every cold owner lives on one rank).
//
// RCCL is opened at run time (dlopen librccl.so.1): inside a process that
// already has it (PyTorch's copy) the same instance is used.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
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

#define NCCLR(expr)                                   \
  do {                                                \
    if ((expr) != ncclSuccess) return EVM_EDIST;      \
  } while (0)

static_assert(sizeof(ncclUniqueId) == EVM_DIST_ID_BYTES, "unique id size");

// ------------------------------------------------------------------ kernels
constexpr int DT = 256;               // threads per partition block
constexpr int DROUNDS = 16;           // rows per thread per block
constexpr u32 DTILE = DT * DROUNDS;   // rows per block
constexpr u32 MAX_BUCKETS = 64;
constexpr size_t META = 16;           // raw records: owner u32, aux u32, source index u32, pad
constexpr size_t PACKED = 32;         // packed records (48-B timestamp rows): tc, node, owner, aux, index, case|valid
constexpr u32 PK_VALID = 1u << 16;
constexpr u32 CNT_WORDS = 4 * MAX_BUCKETS;
constexpr u32 CNT_BAD = CNT_WORDS - 1;

// bucket of row i: SEND (caller arrays) -> destination rank; RECV (wire
// records, owner at byte `ooff`) -> local owner (owner / world)
enum { SEND = 0, RECV = 1 };

template <int MODE>
__device__ __forceinline__ u32 bucket_of(size_t i, const u32* owner, const uint8_t* dest, const char* rec, size_t rb,
                                         size_t ooff, u32 world) {
  if (MODE == SEND) return dest ? (u32)dest[i] : owner[i] % world;
  const u32 o = *reinterpret_cast<const u32*>(rec + i * rb + ooff);
  return o / world;
}

// Packed wire form of a 48-B timestamp row: the parsed (tc, node, case mask)
// -- 16 B instead of 46 -- from which the receiver rebuilds the identical
// string (a canonical timestamp is a function of them, timestamp.ts:43-55).
// A row outside the native domain travels as "invalid" and is rebuilt as
// 0xFF bytes, which the engine rejects exactly like the original.
__device__ __forceinline__ void put_byte(u32 (&w)[12], int i, u32 c) { w[i >> 2] |= (c & 0xffu) << (8 * (i & 3)); }
__device__ __forceinline__ void put_dec(u32 (&w)[12], int at, u32 v, int digits) {
  for (int k = digits - 1; k >= 0; --k) {
    put_byte(w, at + k, 0x30u + v % 10u);
    v /= 10u;
  }
}
__device__ __forceinline__ void format_ts46(u64 tc, u64 node, u32 cmask, bool valid, u32 (&w)[12]) {
  for (int k = 0; k < 12; ++k) w[k] = 0;
  if (!valid) {
    for (int k = 0; k < 11; ++k) w[k] = 0xffffffffu;
    w[11] = 0xffffu;
    return;
  }
  const u64 ms = tc >> 16;
  const u32 ctr = (u32)(tc & 0xffffu);
  const u64 days = ms / 86400000ull;
  const u32 rem = (u32)(ms - days * 86400000ull);
  // civil date of a day count (proleptic Gregorian, days since 1970-01-01)
  const u64 z = days + 719468ull;
  const u64 era = z / 146097ull;
  const u32 doe = (u32)(z - era * 146097ull);
  const u32 yoe = (doe - doe / 1460u + doe / 36524u - doe / 146096u) / 365u;
  const u32 doy = doe - (365u * yoe + yoe / 4u - yoe / 100u);
  const u32 mp = (5u * doy + 2u) / 153u;
  const u32 d = doy - (153u * mp + 2u) / 5u + 1u;
  const u32 m = mp < 10u ? mp + 3u : mp - 9u;
  const u32 y = (u32)(yoe + era * 400ull) + (m <= 2u ? 1u : 0u);
  put_dec(w, 0, y, 4);
  put_byte(w, 4, '-');
  put_dec(w, 5, m, 2);
  put_byte(w, 7, '-');
  put_dec(w, 8, d, 2);
  put_byte(w, 10, 'T');
  put_dec(w, 11, rem / 3600000u, 2);
  put_byte(w, 13, ':');
  put_dec(w, 14, rem / 60000u % 60u, 2);
  put_byte(w, 16, ':');
  put_dec(w, 17, rem / 1000u % 60u, 2);
  put_byte(w, 19, '.');
  put_dec(w, 20, rem % 1000u, 3);
  put_byte(w, 23, 'Z');
  put_byte(w, 24, '-');
  for (int k = 0; k < 4; ++k) {
    const u32 v = (ctr >> (12 - 4 * k)) & 15u;
    put_byte(w, 25 + k, v < 10u ? 0x30u + v : 0x37u + v);  // upper-case hex counter
  }
  put_byte(w, 29, '-');
  for (int k = 0; k < 16; ++k) {
    const u32 v = (u32)(node >> (60 - 4 * k)) & 15u;
    put_byte(w, 30 + k, v < 10u ? 0x30u + v : (((cmask >> k) & 1u) ? 0x37u : 0x57u) + v);
  }
}

// per-block bucket counts, bucket-major ([b * nblocks + block]): their
// exclusive scan is every (bucket, block)'s first output slot, stable
template <int MODE>
__global__ __launch_bounds__(DT) void k_dist_count(const u32* __restrict__ owner, const uint8_t* __restrict__ dest,
                                                   const char* __restrict__ rec, size_t rb, size_t ooff, size_t n,
                                                   u32 world, u32 B, u32 nblocks, u32* __restrict__ counts,
                                                   u32* __restrict__ bad) {
  __shared__ u32 c[MAX_BUCKETS];
  if (threadIdx.x < MAX_BUCKETS) c[threadIdx.x] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * DTILE;
  bool oob = false;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    if (i < n) {
      const u32 b = bucket_of<MODE>(i, owner, dest, rec, rb, ooff, world);
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

// Stable scatter: rows of a block in order, ranked within the block with
// wave ballots + a 4-wave prefix in LDS, placed after the (bucket, block)
// slot the scan gave.  offs == nullptr: no partition (row i -> slot i).
//   SEND: caller rows -> wire records (ts | owner, aux, index)
//   RECV: wire records -> caller arrays (+ source rank from the receive offsets)
template <int MODE>
__global__ __launch_bounds__(DT) void k_dist_scatter(
    const char* __restrict__ ts, size_t stride, const u32* __restrict__ owner, const u32* __restrict__ aux,
    const uint8_t* __restrict__ dest, const char* __restrict__ rec, size_t rb, int packed, size_t n, u32 world, u32 B,
    int bits,
    u32 nblocks, const u32* __restrict__ offs, char* __restrict__ out_rec, char* __restrict__ out_ts,
    size_t out_stride, u32* __restrict__ out_owner, u32* __restrict__ out_aux, u64* __restrict__ out_src,
    const u64* __restrict__ roff, u32 n_src) {
  __shared__ u32 run[MAX_BUCKETS];
  __shared__ u32 wcnt[2][DT / 64][MAX_BUCKETS];  // by round parity: a wave clears its row of round r + 1
                                                 // while wave 0 may still sum round r's
  const int lane = __lane_id(), wv = threadIdx.x >> 6;
  if (offs && threadIdx.x < B) run[threadIdx.x] = offs[(size_t)threadIdx.x * nblocks + blockIdx.x];
  const u64 lt = lanemask_lt();
  const size_t base = (size_t)blockIdx.x * DTILE;
  for (int r = 0; r < DROUNDS; ++r) {
    const size_t i = base + (size_t)r * DT + threadIdx.x;
    const bool ok = i < n;
    size_t pos = i;
    if (offs) {
      const u32 b = ok ? bucket_of<MODE>(i, owner, dest, rec, rb, packed ? 16 : stride, world) : 0u;
      const bool act = ok && b < B;
      u32(*wc)[MAX_BUCKETS] = wcnt[r & 1];
      wc[wv][lane] = 0;
      __builtin_amdgcn_wave_barrier();
      const u64 peers = match_bucket(b, act, bits);
      if (act && (peers & lt) == 0) wc[wv][b] = (u32)__popcll(peers);
      __syncthreads();
      if (act) {
        u32 p = run[b] + (u32)__popcll(peers & lt);
        for (int w = 0; w < wv; ++w) p += wc[w][b];
        pos = p;
      }
      __syncthreads();
      if (threadIdx.x < B) {
        u32 t = 0;
        for (int w = 0; w < DT / 64; ++w) t += wc[w][threadIdx.x];
        run[threadIdx.x] += t;
      }
      if (!act) continue;  // (a row with an out-of-range bucket is reported by k_dist_count)
    } else if (!ok) {
      continue;
    }
    if (MODE == SEND && packed) {
      const uint4* row = reinterpret_cast<const uint4*>(ts + i * stride);
      const uint4 x = row[0], y = row[1], z = row[2];
      const u32 w[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w & 0xffffu};
      const Parsed p = parse_ts46(w);
      uint4* dst = reinterpret_cast<uint4*>(out_rec + pos * rb);
      dst[0] = make_uint4((u32)p.tc, (u32)(p.tc >> 32), (u32)p.node, (u32)(p.node >> 32));
      dst[1] = make_uint4(owner[i], aux ? aux[i] : 0u, (u32)i,
                          (p.meta & EVM_META_CASEMASK) | ((p.meta & EVM_META_VALID) ? PK_VALID : 0u));
    } else if (MODE == SEND) {
      char* dst = out_rec + pos * rb;
      copy_row(dst, ts + i * stride, stride);
      uint4 m;
      m.x = owner[i];
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
        format_ts46((u64)a.x | ((u64)a.y << 32), (u64)a.z | ((u64)a.w << 32), m.w & 0xffffu, (m.w & PK_VALID) != 0,
                    w);
        uint4* dst = reinterpret_cast<uint4*>(out_ts + pos * out_stride);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
        dst[2] = make_uint4(w[8], w[9], w[10], w[11]);
      } else {
        copy_row(out_ts + pos * out_stride, src, stride);
        m = *reinterpret_cast<const uint4*>(src + stride);
      }
      out_owner[pos] = m.x;
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

// gathered [rank][local owner] -> global owner g = local * world + rank
__global__ void k_dist_root_unpack(const u64* __restrict__ all, u32 world, u32 per, u32 n_global,
                                   int32_t* __restrict__ root, uint8_t* __restrict__ present) {
  for (u32 g = blockIdx.x * blockDim.x + threadIdx.x; g < n_global; g += gridDim.x * blockDim.x) {
    const u64 v = all[(size_t)(g % world) * per + g / world];
    root[g] = (int32_t)(uint32_t)v;
    present[g] = (uint8_t)(v >> 32);
  }
}

}  // namespace

struct evm_dist {
  const Rccl* r = nullptr;
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  size_t stride = 48, rb = 64;
  int packed = 0;  // the last route's records: packed (48-B rows) or raw
  char* send = nullptr;  // wire records (send side), device
  size_t send_cap = 0;   // bytes
  char* recv = nullptr;  // received records (staging for evm_dist_take)
  size_t recv_cap = 0;
  uint64_t n_recv = 0;
  // device: [0, 64) send counts, [64, 128) receive counts, [128, 193) receive
  // offsets, [CNT_BAD] the bad-row flag; hcnt: its pinned host mirror
  u64* cnt = nullptr;
  u64* hcnt = nullptr;
  uint64_t recv_off[MAX_BUCKETS + 1] = {};
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

// stable partition of n rows into B buckets: counts -> scan -> scatter.
// Returns the scanned slot matrix (offs) and the bucket totals (device).
template <int MODE>
int partition_offsets(evm_ctx* ctx, Scratch& S, const u32* owner, const uint8_t* dest, const char* rec, size_t rb,
                      size_t ooff, size_t n, u32 world, u32 B, u32** offs_out, u32* nblocks_out, u64* totals,
                      u32* bad) {
  const u32 nblocks = (u32)std::max<size_t>(1, (n + DTILE - 1) / DTILE);
  u32* counts = S.alloc<u32>((size_t)B * nblocks);
  u32* offs = S.alloc<u32>((size_t)B * nblocks + 1);
  if (!counts || !offs) return EVM_ENOMEM;
  KLAUNCH((k_dist_count<MODE>), dim3(nblocks), dim3(DT), owner, dest, rec, rb, ooff, n, world, B, nblocks, counts,
          bad);
  int st = scan_exclusive<u32, OpAdd>(ctx, S, counts, (size_t)B * nblocks, offs, offs + (size_t)B * nblocks);
  if (st) return st;
  KLAUNCH(k_dist_totals, dim3(1), dim3(MAX_BUCKETS), offs, offs + (size_t)B * nblocks, B, nblocks, totals);
  *offs_out = offs;
  *nblocks_out = nblocks;
  return hip_ok(hipGetLastError());
}

}  // namespace

extern "C" {

int evm_dist_unique_id(uint8_t* id) {
  if (!id) return EVM_EINVAL;
  const Rccl* r = rccl();
  if (!r) return EVM_EDIST;
  ncclUniqueId u;
  NCCLR(r->get_unique_id(&u));
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
  d->r = r;
  d->rank = rank;
  d->world = world;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  if (r->comm_init_rank(&d->comm, world, u, rank) != ncclSuccess) {
    delete d;
    return EVM_EDIST;
  }
  const size_t words = CNT_WORDS;
  if (hipMalloc(&d->cnt, words * sizeof(u64)) != hipSuccess ||
      hipHostMalloc(&d->hcnt, words * sizeof(u64), hipHostMallocDefault) != hipSuccess) {
    evm_dist_free(ctx, d);
    return EVM_ENOMEM;
  }
  *out = d;
  return EVM_OK;
}

void evm_dist_free(evm_ctx* ctx, evm_dist* d) {
  if (!d) return;
  if (ctx) (void)hipStreamSynchronize(ctx->stream);
  if (d->comm) d->r->comm_destroy(d->comm);
  if (d->send) (void)hipFree(d->send);
  if (d->recv) (void)hipFree(d->recv);
  if (d->cnt) (void)hipFree(d->cnt);
  if (d->hcnt) (void)hipHostFree(d->hcnt);
  delete d;
}

int evm_dist_info(const evm_dist* d, int* rank, int* world) {
  if (!d) return EVM_EINVAL;
  if (rank) *rank = d->rank;
  if (world) *world = d->world;
  return EVM_OK;
}

int evm_dist_route(evm_ctx* ctx, evm_dist* d, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                   const uint32_t* aux, const uint8_t* dest, uint64_t* n_recv) {
  if (!ctx || !d || !n_recv || stride < 46 || stride % 8 || (n && (!ts || !owner))) return EVM_EINVAL;
  if (n >= 0xffffffffull) return EVM_EINVAL;
  const u32 G = (u32)d->world;
  // 48-B rows, 16-B aligned: packed 32-B records (half the xGMI bytes); other strides travel raw
  const int packed = stride == 48 && ((uintptr_t)ts & 15) == 0 ? 1 : 0;
  const size_t rb = packed ? PACKED : stride + META;
  d->stride = stride;
  d->rb = rb;
  d->packed = packed;
  Scratch S(ctx);
  u32* bad = S.alloc<u32>(1);
  if (!bad) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  int st = grow(&d->send, &d->send_cap, std::max<size_t>(n, 1) * rb);
  if (st) return st;
  u32* offs = nullptr;
  u32 nblocks = 0;
  u64* scnt = d->cnt;
  u64* rcnt = d->cnt + MAX_BUCKETS;
  if (n) {
    if ((st = partition_offsets<SEND>(ctx, S, owner, dest, nullptr, rb, stride, n, G, G, &offs, &nblocks, scnt, bad)))
      return st;
    KLAUNCH((k_dist_scatter<SEND>), dim3(nblocks), dim3(DT), ts, stride, owner, aux, dest, (const char*)nullptr, rb,
            packed, n, G, G, ceil_log2(G), nblocks, offs, d->send, (char*)nullptr, (size_t)0, (u32*)nullptr,
            (u32*)nullptr, (u64*)nullptr, (const u64*)nullptr, 0u);
  } else {
    HIPR(hipMemsetAsync(scnt, 0, G * sizeof(u64), ctx->stream));
  }
  // the counts: one all-to-all of G words, one read back (with the bad-row flag)
  NCCLR(d->r->all_to_all(scnt, rcnt, 1, ncclUint64, d->comm, ctx->stream));
  HIPR(hipMemsetAsync(d->cnt + CNT_BAD, 0, sizeof(u64), ctx->stream));
  HIPR(hipMemcpyAsync(d->cnt + CNT_BAD, bad, sizeof(u32), hipMemcpyDeviceToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(d->hcnt, d->cnt, CNT_WORDS * sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  const u64* hs = d->hcnt;
  const u64* hr = d->hcnt + MAX_BUCKETS;
  const bool any_bad = d->hcnt[CNT_BAD] != 0;
  uint64_t soff[MAX_BUCKETS + 1];
  soff[0] = 0;
  d->recv_off[0] = 0;
  for (u32 p = 0; p < G; ++p) {
    soff[p + 1] = soff[p] + hs[p];
    d->recv_off[p + 1] = d->recv_off[p] + hr[p];
  }
  const uint64_t total = d->recv_off[G];
  if ((st = grow(&d->recv, &d->recv_cap, std::max<uint64_t>(total, 1) * rb))) return st;
  // every rank takes part in the exchange even when its own input was bad
  // (a peer waiting in ncclRecv would hang otherwise); the bad rows were
  // not packed, so such a rank sends fewer rows than it counted -> its
  // counts above exclude them (k_dist_totals counts only in-range buckets)
  NCCLR(d->r->group_start());
  for (u32 p = 0; p < G; ++p) {
    NCCLR(d->r->send(d->send + soff[p] * rb, hs[p] * rb, ncclUint8, (int)p, d->comm, ctx->stream));
    NCCLR(d->r->recv(d->recv + d->recv_off[p] * rb, hr[p] * rb, ncclUint8, (int)p, d->comm, ctx->stream));
  }
  NCCLR(d->r->group_end());
  // receive offsets on the device (source rank of every row in evm_dist_take)
  u64* droff = d->cnt + 2 * MAX_BUCKETS;
  for (u32 p = 0; p <= G; ++p) d->hcnt[2 * MAX_BUCKETS + p] = d->recv_off[p];
  HIPR(hipMemcpyAsync(droff, d->hcnt + 2 * MAX_BUCKETS, (G + 1) * sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  d->n_recv = total;
  *n_recv = total;
  return any_bad ? EVM_EINVAL : hip_ok(hipGetLastError());
}

int evm_dist_take(evm_ctx* ctx, evm_dist* d, uint32_t group, char* out_ts, size_t out_stride, uint32_t* out_owner,
                  uint32_t* out_aux, uint64_t* out_src, uint64_t cap, uint64_t* group_off) {
  if (!ctx || !d || group > MAX_BUCKETS || (group && !group_off)) return EVM_EINVAL;
  const size_t n = d->n_recv;
  if (n && (!out_ts || !out_owner || out_stride < d->stride || out_stride % 8)) return EVM_EINVAL;
  if (n && d->packed && (out_stride % 16 || ((uintptr_t)out_ts & 15))) return EVM_EINVAL;  // rebuilt rows: 16-B stores
  if (n > cap) return EVM_ECAPACITY;
  const u32 G = (u32)d->world;
  const u64* droff = d->cnt + 2 * MAX_BUCKETS;
  Scratch S(ctx);
  if (!group) {
    if (n)
      KLAUNCH((k_dist_scatter<RECV>), dim3((u32)((n + DTILE - 1) / DTILE)), dim3(DT), (const char*)nullptr, d->stride,
              (const u32*)nullptr, (const u32*)nullptr, (const uint8_t*)nullptr, d->recv, d->rb, d->packed, n, G, 1u, 0,
              1u,
              (const u32*)nullptr, (char*)nullptr, out_ts, out_stride, out_owner, out_aux, (u64*)out_src, droff, G + 1);
    return hip_ok(hipGetLastError());
  }
  u32* bad = S.alloc<u32>(1);
  u64* tot = S.alloc<u64>(MAX_BUCKETS + 1);
  if (!bad || !tot) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  HIPR(hipMemsetAsync(tot, 0, (MAX_BUCKETS + 1) * sizeof(u64), ctx->stream));
  if (n) {
    u32* offs = nullptr;
    u32 nblocks = 0;
    int st = partition_offsets<RECV>(ctx, S, nullptr, nullptr, d->recv, d->rb, d->packed ? 16 : d->stride, n, G,
                                     group, &offs, &nblocks, tot, bad);
    if (st) return st;
    KLAUNCH((k_dist_scatter<RECV>), dim3(nblocks), dim3(DT), (const char*)nullptr, d->stride, (const u32*)nullptr,
            (const u32*)nullptr, (const uint8_t*)nullptr, d->recv, d->rb, d->packed, n, G, group, ceil_log2(group),
            nblocks, offs,
            (char*)nullptr, out_ts, out_stride, out_owner, out_aux, (u64*)out_src, droff, G + 1);
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
  if (!ctx || !d || (n_trees && !trees) || (n_owners_global && (!root || !present))) return EVM_EINVAL;
  const u32 G = (u32)d->world;
  const u32 per = (n_owners_global + G - 1) / G;
  size_t local = 0;
  for (u32 k = 0; k < n_trees; ++k) {
    if (!trees[k]) return EVM_EINVAL;
    local += trees[k]->n_owners;
  }
  if (local > per) return EVM_EINVAL;
  if (!n_owners_global) return EVM_OK;
  Scratch S(ctx);
  u64* mine = S.alloc<u64>(per);
  u64* all = S.alloc<u64>((size_t)per * G);
  if (!mine || !all) return EVM_ENOMEM;
  // this rank's local owners: the trees' owners in order, then zeros up to `per`
  u32 at = 0;
  for (u32 k = 0; k < n_trees; ++k) {
    const evm_tree* t = trees[k];
    const u32 cnt = k + 1 < n_trees ? t->n_owners : per - at;  // the last launch also zero-fills the tail
    if (cnt)
      KLAUNCH(k_dist_root_pack, dim3(grid_for(cnt, 256)), dim3(256), t->off, t->pfx, t->n_owners, cnt, mine + at);
    at += t->n_owners;
  }
  if (!n_trees) HIPR(hipMemsetAsync(mine, 0, sizeof(u64) * per, ctx->stream));
  NCCLR(d->r->all_gather(mine, all, per, ncclUint64, d->comm, ctx->stream));
  KLAUNCH(k_dist_root_unpack, dim3(grid_for(n_owners_global, 256)), dim3(256), all, G, per, n_owners_global, root,
          present);
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

}  // extern "C"
