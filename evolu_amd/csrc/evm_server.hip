// Sync server hot path (apps/server/src/index.ts) on MI355X.
//
//   addMessages (index.ts:138-171): per message, INSERT OR IGNORE into
//     message(timestamp, userId) -- PRIMARY KEY(timestamp, userId) -- and
//     XOR into the owner's tree iff the row was inserted (changes === 1).
//   getMessages (index.ts:173-202): diff the owner's tree with the client's;
//     on Some(d) select the owner's rows with timestamp > ISO(d)-0000-0000..0
//     and timestamp NOT LIKE '%' || nodeId, ORDER BY timestamp.
//
// Store layout (device, sorted by (owner, timestamp string order)):
//   owner u32 | tc u64 = millis << 16 | counter | rk_hi u64, rk_lo u32 = the
//   node's 16 chars as 5-bit ASCII-order ranks (chars 0-11 / 12-15) | id u64.
// (tc, rk_hi, rk_lo) is injective and ordered exactly like the strings.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

struct evm_store {
  size_t bytes;  // the one device block holding the arrays (base = off)
  uint32_t n_owners;
  uint64_t n;
  unsigned long long* off;  // [n_owners + 1]
  u32* owner;               // [n]
  unsigned long long* tc;   // [n]
  unsigned long long* hi;   // [n]
  u32* lo;                  // [n]
  unsigned long long* id;   // [n]
  evm_tree* tree;
};

namespace {

struct SKey {
  u32 owner;
  u64 tc;
  u64 hi;
  u32 lo;
};

__device__ __forceinline__ int skey_cmp(const SKey& a, const SKey& b) {
  if (a.owner != b.owner) return a.owner < b.owner ? -1 : 1;
  if (a.tc != b.tc) return a.tc < b.tc ? -1 : 1;
  if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
  if (a.lo != b.lo) return a.lo < b.lo ? -1 : 1;
  return 0;
}

// node (hex value, case mask) -> 5-bit ranks, chars 0..11 in hi, 12..15 in lo
__device__ __forceinline__ void node_ranks(u64 node, u32 mask, u64* hi, u32* lo) {
  u64 h = 0;
  u32 l = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const u32 v = (u32)(node >> (60 - 4 * i)) & 15u;
    const u32 r = node_char_rank(v, (mask >> i) & 1u);
    if (i < 12) h = (h << 5) | r;
    else l = (l << 5) | r;
  }
  *hi = h;
  *lo = l;
}

__device__ __forceinline__ SKey skey_of(const evm_rec& r) {
  SKey k;
  k.owner = r.aux;
  k.tc = r.tc;
  node_ranks(r.node, r.meta & EVM_META_CASEMASK, &k.hi, &k.lo);
  return k;
}

// A record read once (non-temporal: shorter issue-to-land latency).
__device__ __forceinline__ evm_rec load_rec_nt(const evm_rec* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u* q = reinterpret_cast<const v4u*>(p);
  const v4u a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
  evm_rec r;
  r.tc = (u64)a.x | ((u64)a.y << 32);
  r.node = (u64)a.z | ((u64)a.w << 32);
  r.meta = b.x;
  r.hash = b.y;
  r.minute = b.z;
  r.aux = b.w;
  return r;
}

struct StoreView {
  const u64* off;
  const u32* owner;
  const u64* tc;
  const u64* hi;
  const u32* lo;
};

__device__ __forceinline__ SKey skey_at(const StoreView& s, size_t k) { return SKey{s.owner[k], s.tc[k], s.hi[k], s.lo[k]}; }

// first k in [a, b) with s[k] >= x
__device__ __forceinline__ size_t store_lower(const StoreView& s, size_t a, size_t b, const SKey& x) {
  while (a < b) {
    const size_t m = (a + b) >> 1;
    if (skey_cmp(skey_at(s, m), x) < 0) a = m + 1;
    else b = m;
  }
  return a;
}

// ---------------------------------------------------------------- sort fields
enum Field { F_LO = 0, F_HI = 1, F_TC = 2, F_OWNER = 3, F_MS = 4, F_CTR = 5, N_FIELDS = 6 };

__device__ __forceinline__ u64 field_of(const SKey& k, int f) {
  return f == F_LO ? (u64)k.lo : f == F_HI ? k.hi : f == F_TC ? k.tc : f == F_OWNER ? (u64)k.owner
         : f == F_MS ? k.tc >> 16 : k.tc & 0xffffu;
}

__global__ void k_sv_field(const evm_rec* __restrict__ rec, const u32* __restrict__ perm, size_t n, int field,
                           u64* __restrict__ out) {
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    out[p] = field_of(skey_of(rec[perm[p]]), field);
}

// min / max of every field over the batch (decides the radix bits per field)
struct FieldRange {
  u64 mn[N_FIELDS];
  u64 mx[N_FIELDS];
};

// (idx: message i's record is rec[idx[i]], else rec[i])
__global__ void k_sv_ranges(const evm_rec* __restrict__ rec, const u32* __restrict__ idx, size_t n,
                            FieldRange* __restrict__ fr) {
  u64 mn[N_FIELDS], mx[N_FIELDS];
#pragma unroll
  for (int f = 0; f < N_FIELDS; ++f) {
    mn[f] = ~0ull;
    mx[f] = 0;
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const SKey k = skey_of(rec[idx ? idx[i] : i]);
#pragma unroll
    for (int f = 0; f < N_FIELDS; ++f) {
      const u64 v = field_of(k, f);
      mn[f] = min(mn[f], v);
      mx[f] = max(mx[f], v);
    }
  }
#pragma unroll
  for (int f = 0; f < N_FIELDS; ++f) {
    mn[f] = wave_min(mn[f]);
    mx[f] = wave_max(mx[f]);
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int f = 0; f < N_FIELDS; ++f) {
      atomic_min_if(&fr->mn[f], mn[f]);
      atomic_max_if(&fr->mx[f], mx[f]);
    }
  }
}

// Compound sort key (owner - omin : ob | millis - mmin : mb | counter : cb),
// when ob + mb + cb <= 64: one radix sort orders the batch by (owner, tc);
// equal compound keys (same owner and tc, different node) are then ordered
// by the node ranks in k_sv_ties.
struct CKey {
  u64 omin, mmin;
  int mb, cb;
};
// perm values: the batch index, or the caller's index orig[i] of a sub-batch
// (idx: message i's record is rec[idx[i]], else rec[i])
__global__ void k_sv_ckey(const evm_rec* __restrict__ rec, const u32* __restrict__ idx, size_t n, CKey ck,
                          u64* __restrict__ key, u32* __restrict__ perm, const u32* __restrict__ orig) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const evm_rec r = rec[idx ? idx[i] : i];
    key[i] = (((u64)r.aux - ck.omin) << (ck.mb + ck.cb)) | (((r.tc >> 16) - ck.mmin) << ck.cb) | (r.tc & 0xffffu);
    perm[i] = orig ? orig[i] : (u32)i;
  }
}

constexpr int TIE_MAX = 64;

// The batch's records in sorted order (one gather; the kernels after it read
// sequentially).
__global__ void k_sv_gather(const evm_rec* __restrict__ rec, const u32* __restrict__ perm, size_t n,
                            evm_rec* __restrict__ srec) {
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    srec[p] = rec[perm[p]];  // (a non-temporal gather measured slower here: 3.1 vs 2.8 ms)
}

__device__ __forceinline__ bool same_node(const evm_rec& a, const evm_rec& b) {
  return a.node == b.node && ((a.meta ^ b.meta) & EVM_META_CASEMASK) == 0;
}

// Runs of equal compound keys (one owner and tc, several nodes): every member
// counts the members that sort before it by (node ranks, position) -- the
// positions inside a run are in batch order (the radix sort is stable) -- and
// records itself as the source of sorted position run start + rank.  A run
// longer than TIE_MAX flags the slow (full-field) sort.
__global__ void k_sv_ties(const u64* __restrict__ key, const evm_rec* __restrict__ srec, size_t n,
                          u32* __restrict__ src, u32* __restrict__ too_long) {
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x) {
    const u64 k = key[p];
    const bool left = p > 0 && key[p - 1] == k, right = p + 1 < n && key[p + 1] == k;
    if (!left && !right) {
      src[p] = (u32)p;
      continue;
    }
    size_t s = p, e = p + 1;
    while (s > 0 && key[s - 1] == k && p - s < TIE_MAX) --s;
    while (e < n && key[e] == k && e - s <= TIE_MAX) ++e;
    if (e - s > TIE_MAX || (s > 0 && key[s - 1] == k)) {
      atomicOr(too_long, 1u);
      continue;
    }
    const evm_rec r = srec[p];
    const u32 cp = r.meta & EVM_META_CASEMASK;
    u64 hp = 0;
    u32 lp = 0;
    node_ranks(r.node, cp, &hp, &lp);
    u32 rank = 0;
    for (size_t q = s; q < e; ++q) {
      if (q == p) continue;
      const evm_rec x = srec[q];
      const u32 cq = x.meta & EVM_META_CASEMASK;
      bool before;
      if (!(cp | cq)) {
        // no upper-case hex on either side: the ranks order like the hex values
        before = x.node < r.node || (x.node == r.node && q < p);
      } else {
        u64 hq;
        u32 lq;
        node_ranks(x.node, cq, &hq, &lq);
        before = hq < hp || (hq == hp && (lq < lp || (lq == lp && q < p)));
      }
      rank += before ? 1u : 0u;
    }
    src[s + rank] = (u32)p;
  }
}

// ------------------------------------------------------------ dedup + marks
// Sorted order d (record srec[src[d]], or srec[d] without a tie permutation):
// first occurrence of (owner, timestamp) in batch order (equal timestamps sit
// in batch order) that the store does not hold yet.
__global__ void k_sv_mark(const evm_rec* __restrict__ srec, const u32* __restrict__ src, const u32* __restrict__ perm,
                          const u64* __restrict__ skeys, size_t n, StoreView st, uint8_t* __restrict__ flags,
                          u32* __restrict__ sel, const u32* __restrict__ orig) {
  for (size_t d = (size_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (size_t)gridDim.x * blockDim.x) {
    const size_t p = src ? src[d] : d;
    const evm_rec r = srec[p];
    bool first = true;
    if (d > 0) {
      // sorted compound keys differ => the timestamps differ; equal => same owner and tc
      if (!skeys) {
        first = skey_cmp(skey_of(srec[d - 1]), skey_of(r)) != 0;
      } else if (skeys[d] == skeys[d - 1]) {
        first = !same_node(srec[src[d - 1]], r);
      }
    }
    bool ins = first;
    if (ins) {
      const u32 owner = r.aux;
      const size_t a = st.off[owner], b = st.off[owner + 1];
      if (a < b) {
        const SKey k = skey_of(r);
        const size_t q = store_lower(st, a, b, k);
        ins = !(q < b && skey_cmp(skey_at(st, q), k) == 0);
      }
    }
    const u32 i = perm[p];
    flags[orig ? orig[i] : i] = ins ? (uint8_t)EVM_MSG_INS : (uint8_t)0;
    sel[d] = ins ? 1u : 0u;
  }
}

__global__ void k_sv_compact(const evm_rec* __restrict__ srec, const u32* __restrict__ src,
                             const u32* __restrict__ perm, const u32* __restrict__ sel, const u32* __restrict__ pos,
                             size_t n, u64 id_base, u32* __restrict__ o_owner, u64* __restrict__ o_tc,
                             u64* __restrict__ o_hi, u32* __restrict__ o_lo, u64* __restrict__ o_id,
                             u64* __restrict__ l_ck, u32* __restrict__ l_h, const u32* __restrict__ orig) {
  for (size_t d = (size_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (size_t)gridDim.x * blockDim.x) {
    if (!sel[d]) continue;
    const size_t p = src ? src[d] : d;
    const evm_rec r = srec[p];
    const SKey k = skey_of(r);
    const u32 q = pos[d];
    const u32 i = perm[p];
    o_owner[q] = k.owner;
    o_tc[q] = k.tc;
    o_hi[q] = k.hi;
    o_lo[q] = k.lo;
    o_id[q] = id_base + (orig ? orig[i] : i);
    // leaves come out sorted by (owner, minute); the codes follow that order
    // when the owner's key lengths agree (k_sv_sorted_check tells)
    l_ck[q] = ((u64)k.owner << 40) | minute_code(r.minute);
    l_h[q] = r.hash;
  }
}

__global__ void k_sv_bad(const evm_rec* __restrict__ rec, size_t n, uint8_t* __restrict__ flags,
                         const u32* __restrict__ orig) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    flags[orig ? orig[i] : i] = (rec[i].meta & EVM_META_VALID) ? 0u : EVM_MSG_BAD;
}

// nothing inserted (a call that commits nothing after K5 wrote its flags)
__global__ void k_flags_clear(size_t n, uint8_t* __restrict__ flags, const u32* __restrict__ orig) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    flags[orig ? orig[i] : i] = 0;
}

__global__ void k_sv_sorted_check(const u64* __restrict__ ck, size_t m, u32* __restrict__ unsorted) {
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x + 1; q < m; q += (size_t)gridDim.x * blockDim.x)
    if (ck[q] < ck[q - 1]) *unsorted = 1u;
}

// ------------------------------------------------------------------ merge
struct StoreOut {
  u32* owner;
  u64* tc;
  u64* hi;
  u32* lo;
  u64* id;
};

// Both sides are sorted by (owner, key) and carry per-owner offsets (b.off /
// a.off): a row's merged position = its index + the other side's rows of
// lower owners + a search inside the other side's segment of its owner.
__global__ void k_sv_merge_old(StoreView a, const u64* __restrict__ a_id, size_t na, StoreView b, size_t nb,
                               StoreOut o) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += (size_t)gridDim.x * blockDim.x) {
    const SKey k = skey_at(a, i);
    const size_t j = store_lower(b, b.off[k.owner], b.off[k.owner + 1], k);
    const size_t q = i + j;
    o.owner[q] = k.owner;
    o.tc[q] = k.tc;
    o.hi[q] = k.hi;
    o.lo[q] = k.lo;
    o.id[q] = a_id[i];
  }
}

__global__ void k_sv_merge_new(StoreView b, const u64* __restrict__ b_id, size_t nb, StoreView a, size_t na,
                               StoreOut o) {
  for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += (size_t)gridDim.x * blockDim.x) {
    const SKey k = skey_at(b, j);
    const size_t i = store_lower(a, a.off[k.owner], a.off[k.owner + 1], k);  // keys are disjoint
    const size_t q = i + j;
    o.owner[q] = k.owner;
    o.tc[q] = k.tc;
    o.hi[q] = k.hi;
    o.lo[q] = k.lo;
    o.id[q] = b_id[j];
  }
}

__global__ void k_add_u64(const u64* __restrict__ a, const u64* __restrict__ b, size_t n, u64* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = a[i] + b[i];
}

__global__ void k_sv_owner_off(const u32* __restrict__ owner, size_t n, u32 n_owners, u64* __restrict__ off) {
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o <= n_owners; o += (size_t)gridDim.x * blockDim.x) {
    size_t a = 0, b = n;
    while (a < b) {
      const size_t m = (a + b) >> 1;
      if (owner[m] < (u32)o) a = m + 1;
      else b = m;
    }
    off[o] = a;
  }
}

// ------------------------------------------------ owner runs (requests)
// Run heads (owner[i] != owner[i-1]) compacted in two reads of the owner
// column: a wave owns a tile of RUN_TILE messages, counts its heads
// (k_run_count), and after a scan of the tile counts writes each head at
// its rank (k_run_emit).  (Was: a u32 head flag per message and a scan over
// n -- 32 B/msg of traffic instead of 8.)
constexpr int RUN_ITEMS = 64;
constexpr size_t RUN_TILE = 64 * RUN_ITEMS;
constexpr int RUN_THREADS = 256;

__device__ __forceinline__ bool run_head(const u32* __restrict__ owner, size_t n, size_t i) {
  return i < n && (i == 0 || owner[i] != owner[i - 1]);
}

// Full tiles of a 16-B aligned column: a lane reads 4 consecutive owners per
// step (a wave step = 1 KiB), the owner before its first one comes from the
// lane below (lane 0: the previous step's last, or the owner before the tile).
// Returns the lane's 4 head bits (bit j: message 4 * (step * 64 + lane) + j).
__device__ __forceinline__ u32 run_heads4(const uint4 v, u32& carry, int lane) {
  u32 prev = __shfl_up(v.w, 1, 64);
  if (lane == 0) prev = carry;
  carry = __shfl(v.w, 63, 64);
  return (v.x != prev ? 1u : 0u) | (v.y != v.x ? 2u : 0u) | (v.z != v.y ? 4u : 0u) | (v.w != v.z ? 8u : 0u);
}
__device__ __forceinline__ bool run_vec_tile(const u32* __restrict__ owner, size_t n, size_t base) {
  return base + RUN_TILE <= n && ((uintptr_t)owner & 15) == 0;
}
__device__ __forceinline__ u32 run_carry0(const u32* __restrict__ owner, size_t base) {
  return base ? owner[base - 1] : ~owner[0];  // message 0 always starts a run
}

__global__ __launch_bounds__(RUN_THREADS) void k_run_count(const u32* __restrict__ owner, size_t n,
                                                           u32* __restrict__ tcnt) {
  const size_t t = (size_t)blockIdx.x * (RUN_THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t base = t * RUN_TILE;
  if (base >= n) return;  // uniform per wave
  u32 c = 0;
  if (run_vec_tile(owner, n, base)) {
    const uint4* o4 = reinterpret_cast<const uint4*>(owner + base);
    u32 carry = run_carry0(owner, base);
    uint4 v[RUN_TILE / 256];
#pragma unroll
    for (int s = 0; s < (int)(RUN_TILE / 256); ++s) v[s] = o4[s * 64 + lane];
#pragma unroll
    for (int s = 0; s < (int)(RUN_TILE / 256); ++s) c += (u32)__popc(run_heads4(v[s], carry, lane));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  } else {
#pragma unroll 16
    for (int it = 0; it < RUN_ITEMS; ++it)
      c += (u32)__popcll(__ballot(run_head(owner, n, base + (size_t)it * 64 + lane)));
  }
  if (lane == 0) tcnt[t] = c;
}

__global__ __launch_bounds__(RUN_THREADS) void k_run_emit(const u32* __restrict__ owner, size_t n,
                                                          const u32* __restrict__ toff, u32* __restrict__ run_start,
                                                          u32* __restrict__ run_owner) {
  const size_t t = (size_t)blockIdx.x * (RUN_THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t base = t * RUN_TILE;
  if (base >= n) return;
  const u64 lt = lanemask_lt();
  u32 r = toff[t];
  if (run_vec_tile(owner, n, base)) {
    const uint4* o4 = reinterpret_cast<const uint4*>(owner + base);
    u32 carry = run_carry0(owner, base);
    uint4 v[RUN_TILE / 256];
#pragma unroll
    for (int s = 0; s < (int)(RUN_TILE / 256); ++s) v[s] = o4[s * 64 + lane];
#pragma unroll
    for (int s = 0; s < (int)(RUN_TILE / 256); ++s) {
      const u32 hm = run_heads4(v[s], carry, lane);
      const u32 c = (u32)__popc(hm);  // 0..4: its wave prefix from three ballots
      const u64 b0 = __ballot(c & 1u), b1 = __ballot(c & 2u), b2 = __ballot(c & 4u);
      u32 k = r + (u32)__popcll(b0 & lt) + 2u * (u32)__popcll(b1 & lt) + 4u * (u32)__popcll(b2 & lt);
      const u32 i0 = (u32)(base + ((size_t)s * 64 + lane) * 4);
      const u32 ov[4] = {v[s].x, v[s].y, v[s].z, v[s].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (hm & (1u << j)) {
          run_start[k] = i0 + j;
          run_owner[k] = ov[j];
          ++k;
        }
      r += (u32)__popcll(b0) + 2u * (u32)__popcll(b1) + 4u * (u32)__popcll(b2);
    }
    return;
  }
#pragma unroll 16
  for (int it = 0; it < RUN_ITEMS; ++it) {
    const size_t i = base + (size_t)it * 64 + lane;
    const bool h = run_head(owner, n, i);
    const u64 bal = __ballot(h);
    if (h) {
      const u32 k = r + (u32)__popcll(bal & lt);
      run_start[k] = (u32)i;
      run_owner[k] = owner[i];
    }
    r += (u32)__popcll(bal);
  }
}

constexpr u32 SEG_NOBASE = 0xffffffffu;  // SegView::cbase: the segment is not one run

// lengths of the runs in (owner, batch) order
__global__ void k_run_len(const u32* __restrict__ run_start, const u32* __restrict__ order, u32 R, size_t n,
                          u32* __restrict__ len) {
  for (u32 j = blockIdx.x * blockDim.x + threadIdx.x; j < R; j += gridDim.x * blockDim.x) {
    const u32 r = order[j];
    len[j] = (u32)((r + 1 < R ? (size_t)run_start[r + 1] : n) - run_start[r]);
  }
}

// first message position of every owner: the position of its first run
// (and cbase[o]: the batch start of an owner whose share is one run -- a
// whole SyncRequest, the common case -- so K5 reads no perm for it)
__global__ void k_run_seg(const u32* __restrict__ run_owner_sorted, u32 R, const u32* __restrict__ run_pos, u32 O,
                          u64* __restrict__ seg, Info* __restrict__ info, const u32* __restrict__ run_start,
                          const u32* __restrict__ order, u32* __restrict__ cbase, u32* __restrict__ multi) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && R && run_owner_sorted[R - 1] >= O) atomicOr(&info->bad_aux, 1u);
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o <= O; o += gridDim.x * blockDim.x) {
    u32 a = 0, b = R;
    while (a < b) {
      const u32 m = (a + b) >> 1;
      if (run_owner_sorted[m] < o) a = m + 1;
      else b = m;
    }
    seg[o] = run_pos[a];  // run_pos[R] = n
    if (o < O && cbase) {
      const bool has = a < R && run_owner_sorted[a] == o;
      const bool one = has && (a + 1 == R || run_owner_sorted[a + 1] != o);
      cbase[o] = one ? run_start[order[a]] : SEG_NOBASE;
      if (has && !one) atomic_or_if(multi, 1u);  // an owner of several runs: K5 reads its share through perm
    }
  }
}

// perm over owner-major positions.  Runs j0 .. j0+RF_RUNS-1 (in owner order)
// fill one contiguous range of perm, so a wave takes RF_RUNS of them: lanes
// fetch one run's (position, start) each, then the wave writes the whole
// range coalesced, each element finding its run among the RF_RUNS bounds.
constexpr int RF_RUNS = 8;
__global__ __launch_bounds__(256) void k_run_fill(const u32* __restrict__ run_pos, const u32* __restrict__ run_start,
                                                  const u32* __restrict__ order, u32 R, u32* __restrict__ perm) {
  const u32 lane = threadIdx.x & 63;
  const size_t waves = (size_t)gridDim.x * 4;
  for (size_t j0 = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RF_RUNS; j0 < R; j0 += waves * RF_RUNS) {
    u32 p = 0, st = 0;
    if (lane <= (u32)RF_RUNS) {
      const size_t j = min(j0 + lane, (size_t)R);  // past the last run: its end
      p = run_pos[j];
      if (lane < (u32)RF_RUNS && j < R) st = run_start[order[j]];
    }
    u32 pr[RF_RUNS], sr[RF_RUNS];
#pragma unroll
    for (int r = 0; r < RF_RUNS; ++r) {
      pr[r] = __shfl(p, r, 64);
      sr[r] = __shfl(st, r, 64);
    }
    const u32 end = __shfl(p, RF_RUNS, 64);
    for (u32 q = pr[0] + lane; q < end; q += 64) {
      u32 v = sr[0] + (q - pr[0]);
#pragma unroll
      for (int r = 1; r < RF_RUNS; ++r)
        if (q >= pr[r]) v = sr[r] + (q - pr[r]);
      perm[q] = v;
    }
  }
}

// --------------------------------------------- sub-batches (hybrid ingest)
// messages whose owner's share exceeds the LDS capacity
__global__ void k_big_mask(const u32* __restrict__ owner, size_t n, const uint8_t* __restrict__ ownbig,
                           uint8_t* __restrict__ mask) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    mask[i] = ownbig[owner[i]];
}

__global__ void k_mask_u32(const uint8_t* __restrict__ mask, size_t n, u32* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = mask[i];
}

// the masked indices in order: pos = exclusive count of masked before i
__global__ void k_pick(const uint8_t* __restrict__ mask, const u32* __restrict__ pos, size_t n, u32* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (mask[i]) out[pos[i]] = (u32)i;
}

// per-owner isolation (evm_server_ingest_ex): an owner with a culprit row
__global__ void k_owner_bad(const uint8_t* __restrict__ flags, const u32* __restrict__ owner, size_t n, u32 O,
                            uint8_t* __restrict__ obad) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if ((flags[i] & EVM_MSG_BAD) && owner[i] < O) obad[owner[i]] = 1;
}
// rows of owners without one (mask) and their count (keep as u32 for the scan)
__global__ void k_owner_keep(const u32* __restrict__ owner, size_t n, const uint8_t* __restrict__ obad,
                             uint8_t* __restrict__ mask, u32* __restrict__ keep) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint8_t k = obad[owner[i]] ? 0 : 1;
    mask[i] = k;
    keep[i] = k;
  }
}

// records of a sub-batch from the caller's packed records
__global__ void k_sv_rec_sel(const evm_rec* __restrict__ prec, const u32* __restrict__ orig, size_t n,
                             evm_rec* __restrict__ out, u32* __restrict__ owner_out) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    const evm_rec r = prec[orig[k]];
    out[k] = r;
    owner_out[k] = r.aux;
  }
}

// ------------------------------------------------------ K5: owner ingest
// When every owner's share of the batch fits SVO_CAP rows (the common case:
// a request carries one owner's messages, index.ts:224-248), one workgroup
// per owner runs that owner's addMessages in LDS, with no global sort by
// timestamp:
//   A  gather the owner's records in batch order (the stable owner sort),
//      bitonic sort by (order key, batch position); the first occurrence of
//      each timestamp that the store does not hold gets EVM_MSG_INS
//      (index.ts:154 changes === 1); the inserted rows (sorted) and their
//      per-minute XOR leaves go to the owner's slice of batch-sized
//      temporaries; per-owner counts.
//   B  (after the counts are scanned) merge the owner's stored rows with the
//      new rows, and its tree leaves with the new leaves -- equal minutes
//      XOR-combine, as repeated insertIntoMerkleTree calls do -- straight into
//      the new store and tree.
constexpr int SVO_THREADS = 256;
constexpr u32 SVO_CAP = 4096;  // largest share of one owner handled in LDS
constexpr int SVO_TIE_MAX = 32;  // longest run of one (millis, counter) with distinct nodes
constexpr u32 SVO_BUCKET_MAX = 16;  // counting-sort bucket size finished by insertion sort
constexpr u64 SVO_SCAN_STORED = 16;  // stored rows read once per segment while <= 16 x its new rows
// The new leaves' tree searches run over the segment's tree codes staged in LDS
// (measured: reingest K5 4.00 -> 3.26-3.30 ms, but the LDS search takes 81
// VGPRs -- five waves per SIMD instead of six, the empty store's K5 2.60 ->
// 2.72 ms; forcing six spills 28 B per lane.  So the 1,024 class takes the
// LDS search only into a store that has a tree: K5 is instantiated both ways)
constexpr int SVO_SB = 4;  // stored rows per thread whose loads are issued together

struct SvoStatus {
  u32 big;       // an owner's share exceeds the launch's capacity
  u32 fallback;  // a share spans > 2^37 ms, a tie run is longer than SVO_TIE_MAX, or new leaves mix key lengths
  u32 lens;      // bit L: some segment's first or last new leaf has a base-3 key of length L
};

// first k in [lo, hi) with a[k] >= x
__device__ __forceinline__ u64 lb_u64(const u64* a, u64 lo, u64 hi, u64 x) {
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// A segment: a contiguous piece of one owner's share of the batch and the
// key range it covers.  Normally one segment per owner (the identity view:
// owner = s, bounds from the owner offsets).  An owner whose share exceeds
// SVO_CAP is cut into key-range segments at minute splitters (sampled from
// its messages): every copy of a timestamp lands in one segment, so the
// per-segment dedup is the owner's; each segment also owns the owner's
// stored rows [sa, sb) and tree leaves [la, lb) of its minute range (the
// first segment from -inf, the last to +inf), so the merge writes every
// stored row and leaf exactly once.
struct SegView {
  const u32* owner;  // [NS] (null: identity)
  const u64* start;  // [NS + 1] offsets into perm
  const u64* sa;     // stored rows [sa[s], sb[s])
  const u64* sb;
  const u64* la;     // tree leaves [la[s], lb[s])
  const u64* lb;
  // [NS] (or null): a segment whose messages are ONE request run -- batch
  // positions cbase[s] + t, no perm read (SEG_NOBASE: read perm)
  const u32* cbase = nullptr;
};
__device__ __forceinline__ u32 seg_owner(const SegView& v, u32 s) { return v.owner ? v.owner[s] : s; }

template <u32 CAP>
struct SvoLog2 {
  static constexpr int v = CAP == 128 ? 7 : CAP == 256 ? 8 : CAP == 512 ? 9 : CAP == 1024 ? 10 : CAP == 2048 ? 11 : 12;
};

// Phase A for owners whose share is <= CAP.  LDS by batch position t (the
// owner's share in batch order): node ranks, batch index, hash; sort keys
// (tc - tc_min) << PB | t, sorted by a bitonic network (8-B elements only);
// runs of one tc (distinct nodes) are then put in node order.
// where K5 reads a message: packed records (evm_rec), the 48-B timestamp
// rows (parsed in the workgroup), or a route's received records in place
enum { SRC_REC = 0, SRC_ROWS = 1, SRC_WIRE = 2 };
// (compiled for six waves per SIMD instead of the five its registers allow
// -- the LDS fits six 1,024-capacity workgroups per CU -- it ran no faster:
// config 3 2.60 vs 2.58 ms, config 4 3.31 vs 3.24)
template <u32 CAP, int SRC, int THREADS = SVO_THREADS, bool LEAF = false>
__global__ __launch_bounds__(THREADS) void k_svo_a(
    const evm_rec* __restrict__ rec, const uint8_t* __restrict__ ts, size_t stride, Info* __restrict__ info,
    const u32* __restrict__ perm, SegView sv, StoreView st,
    const u64* __restrict__ t_ck, u64 id_base, uint8_t* __restrict__ flags,
    u64* __restrict__ n_tc, u64* __restrict__ n_hi, u32* __restrict__ n_lo, u64* __restrict__ n_id,
    u64* __restrict__ l_ck, int32_t* __restrict__ l_xr, uint8_t* __restrict__ l_dup, u32* __restrict__ cnt_rows,
    u32* __restrict__ cnt_new, u32* __restrict__ cnt_leaves, u32* __restrict__ cnt_xor, SvoStatus* __restrict__ status,
    const u32* __restrict__ orig, const u32* __restrict__ list, u32* __restrict__ mid_list, u32* __restrict__ mid1,
    uint8_t* __restrict__ ownbig, u32* __restrict__ n_owner, int flags_preset, u32* __restrict__ mid512,
    WireSrc wsrc, int skip_stored, int32_t* __restrict__ l_pfx, u64* __restrict__ g_off, u64* __restrict__ g_end) {
  constexpr int PER = CAP / THREADS;
  constexpr int PB = SvoLog2<CAP>::v;
  constexpr u64 PMASK = CAP - 1;
  __shared__ u64 s_k[CAP];   // sort keys; later: minute / hash of the inserted rows
  __shared__ u64 s_rh[CAP];  // by position: node ranks 0..11; later: per-leaf XOR / minute
  __shared__ u32 s_rl[CAP];  //              node ranks 12..15
  __shared__ u32 s_h[CAP];   //              hash
  // (the batch index of position t is perm[a + t], re-read from L2 in the
  // dedup phase: without it the 1,024 kernel's LDS fits five workgroups per CU)
  // counting sort: bucket counts, then starts; then the candidate flags.  Up
  // to 2,048 they ride in the top 12 bits of s_rl (20 bits of ranks): 4 KiB
  // less LDS, six 1,024 workgroups per CU instead of five
  constexpr bool PACK = CAP <= 2048;
  constexpr u32 RLM = (1u << 20) - 1u;
  __shared__ u32 s_cnt[PACK ? 1 : CAP];
  auto cnt_get = [&](u32 i) -> u32 { return PACK ? s_rl[i] >> 20 : s_cnt[i]; };
  auto cnt_set = [&](u32 i, u32 v) {
    if (PACK) s_rl[i] = (s_rl[i] & RLM) | (v << 20);
    else s_cnt[i] = v;
  };
  auto rl_get = [&](u32 i) -> u32 { return s_rl[i] & RLM; };
  __shared__ u64 s_red[2 * (THREADS / 64)];
  __shared__ u32 tmp[THREADS / 64 + 1];
  __shared__ u64 tmp64[THREADS / 64 + 1];
  __shared__ uint16_t s_b3[243];  // base-3 digits of 0..242 (the leaves' key codes)
  const u32 s = list ? list[blockIdx.x] : blockIdx.x;  // pass 2: only the segments pass 1 deferred
  const u32 o = seg_owner(sv, s);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u64 a = sv.start[s];
  const u64 m = sv.start[s + 1] - a;  // an unsorted owner column (bad ids) may underflow: "big"
  const u64 la = sv.la[s], lb = sv.lb[s];
  // the segment's new leaves: slots [a + s, a + s + m] (one more than its
  // messages: room for a gapped tree's owner-local prefix end, l_pfx)
  const u64 lb0 = a + s;
  // the batch index of share position t (the set is what matters, not its order)
  const u32 cb = sv.cbase ? sv.cbase[s] : SEG_NOBASE;
  auto pidx = [&](u32 t) -> u32 { return cb != SEG_NOBASE ? cb + t : perm[a + t]; };
  if (m > CAP || m == 0) {
    if (threadIdx.x == 0) {
      if (m <= 512 && mid512) {
        mid512[1 + atomicAdd(&mid512[0], 1u)] = s;  // for the 512 pass (after the one-wave pass)
      } else if (m <= 1024 && mid1) {
        mid1[1 + atomicAdd(&mid1[0], 1u)] = s;  // for the 1,024 pass
      } else if (m <= SVO_CAP && mid_list) {
        mid_list[1 + atomicAdd(&mid_list[0], 1u)] = s;  // for the SVO_CAP pass
      } else if (m) {
        atomicOr(&status->big, 1u);
        ownbig[o] = 1;  // the owner's messages go to the sort path (k_seg_fix drops its other segments)
      }
      cnt_rows[s] = 0;
      cnt_new[s] = 0;
      cnt_leaves[s] = (u32)(lb - la);
      cnt_xor[s] = 0;
      if (g_off) {  // (a deferred segment's pass writes these again)
        g_off[o] = g_end[o] = lb0;
        l_pfx[lb0] = 0;
      }
    }
    return;
  }
  for (u32 t = threadIdx.x; t < 243; t += THREADS) s_b3[t] = (uint16_t)b3_raw5(t);  // (read after many barriers)
  u32 P = 1;
  while (P < m) P <<= 1;
  // gather: all batch indices, then all records (independent loads in flight)
  u32 bi[PER];
  u64 tc[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 t = threadIdx.x + k * THREADS;
    bi[k] = t < m ? pidx(t) : 0u;
  }
  u64 tmin = ~0ull, tmax = 0;
  if (SRC == SRC_ROWS) {
    // the timestamp rows themselves (no packed records): parse + murmur3 here
    u32 bad = 0;
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    // double-buffered: row k + 1's loads in flight while row k is parsed
    // (config 3 K5 2.55 -> 2.50 ms, into a 100M-row store 3.21 -> 2.87 ms)
    v4u nx{}, ny{}, nz{};
    auto load_row = [&](int k) {
      const u32 t = threadIdx.x + k * THREADS;
      if (t < m) {
        const v4u* row = reinterpret_cast<const v4u*>(ts + (size_t)bi[k] * stride);
        nx = __builtin_nontemporal_load(row);
        ny = __builtin_nontemporal_load(row + 1);
        nz = __builtin_nontemporal_load(row + 2);
      }
    };
    load_row(0);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const v4u x = nx, y = ny, z = nz;
      if (k + 1 < PER) load_row(k + 1);
      const u32 t = threadIdx.x + k * THREADS;
      if (t < m) {
        const u32 w[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w & 0xffffu};
        const Parsed p = parse_ts46(w);
        bad |= (p.meta & EVM_META_VALID) ? 0u : 1u;
        s_rh[t] = p.rh;  // (== node_ranks(p.node, case mask): the parse's SWAR ranks)
        s_rl[t] = p.rl;
        s_h[t] = p.hash;
        tc[k] = p.tc;
        tmin = min(tmin, p.tc);
        tmax = max(tmax, p.tc);
      }
    }
    if (__ballot(bad) && lane == 0) atomicOr(&info->bad, 1u);  // nothing is applied: the host re-packs to flag them
  } else if (SRC == SRC_WIRE) {
    // received (tc, node, case mask): the string is rebuilt in registers for
    // murmur3 (a canonical timestamp is a function of them)
    u32 bad = 0;
    // received records double-buffered: record k + 1's loads in flight while
    // record k's string is rebuilt and hashed
    u64 ntc = 0, nnode = 0;
    u32 ncm = 0;
    auto load_w = [&](int k) {
      const u32 t = threadIdx.x + k * THREADS;
      if (t < m && !wire_self_row(wsrc, bi[k])) wire_load(wsrc, bi[k], &ntc, &nnode, &ncm);
    };
    load_w(0);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u64 wtc = ntc, wnode = nnode;
      const u32 cm = ncm;
      if (k + 1 < PER) load_w(k + 1);
      const u32 t = threadIdx.x + k * THREADS;
      if (t < m && wire_self_row(wsrc, bi[k])) {
        // a keep-input route's own row: the caller's string, parsed here
        u32 x[12];
        wire_self_words(wsrc, bi[k], x);
        const Parsed p = parse_ts46(x);
        bad |= (p.meta & EVM_META_VALID) ? 0u : 1u;
        s_rh[t] = p.rh;
        s_rl[t] = p.rl;
        s_h[t] = p.hash;
        tc[k] = p.tc;
        tmin = min(tmin, p.tc);
        tmax = max(tmax, p.tc);
      } else if (t < m) {  // (all PER loads up front instead: 86 -> more VGPRs, 15 % slower)
        u32 w[12];
        format_ts46(wtc, wnode, cm & EVM_META_CASEMASK, w);
        bad |= (cm & EVM_META_VALID) ? 0u : 1u;
        u64 hi;
        u32 lo;
        node_ranks(wnode, cm & EVM_META_CASEMASK, &hi, &lo);
        s_rh[t] = hi;
        s_rl[t] = lo;
        s_h[t] = murmur3_46(w);
        tc[k] = wtc;
        tmin = min(tmin, wtc);
        tmax = max(tmax, wtc);
      }
    }
    if (__ballot(bad) && lane == 0) atomicOr(&info->bad, 1u);
  } else {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 t = threadIdx.x + k * THREADS;
      if (t < m) {
        const evm_rec r = load_rec_nt(rec + bi[k]);
        u64 hi;
        u32 lo;
        node_ranks(r.node, r.meta & EVM_META_CASEMASK, &hi, &lo);
        s_rh[t] = hi;
        s_rl[t] = lo;
        s_h[t] = r.hash;
        tc[k] = r.tc;
        tmin = min(tmin, r.tc);
        tmax = max(tmax, r.tc);
      }
    }
  }
  tmin = wave_min(tmin);
  tmax = wave_max(tmax);
  if (lane == 0) {
    s_red[wv] = tmin;
    s_red[THREADS / 64 + wv] = tmax;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < THREADS / 64; ++w) {
    tmin = min(tmin, s_red[w]);
    tmax = max(tmax, s_red[THREADS / 64 + w]);
  }
  if ((tmax - tmin) >> (64 - PB)) {  // span too wide for the 64-bit sort key
    if (threadIdx.x == 0) atomicOr(&status->fallback, 1u);
    return;
  }
  // order by (tc, position): a counting sort over CAP buckets of the tc span
  // (shares spread over time land ~1 per bucket), each bucket finished by an
  // insertion sort; a share with a crowded bucket (bursts) takes the bitonic
  // network instead.
  const int sbits = (tmax - tmin) ? 64 - __builtin_clzll(tmax - tmin) : 0;
  const int shift = sbits > PB ? sbits - PB : 0;
  for (u32 t = threadIdx.x; t < CAP; t += THREADS) {
    if (PACK) s_rl[t] &= RLM;
    else s_cnt[t] = 0;
  }
  __syncthreads();
  u32 bk[PER], rk[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 t = threadIdx.x + k * THREADS;
    bk[k] = rk[k] = 0;
    if (t < m) {
      bk[k] = (u32)((tc[k] - tmin) >> shift);
      rk[k] = PACK ? atomicAdd(&s_rl[bk[k]], 1u << 20) >> 20 : atomicAdd(&s_cnt[bk[k]], 1u);
    }
  }
  __syncthreads();
  {
    u32 loc[PER], sum = 0, mx = 0;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      loc[r] = cnt_get(threadIdx.x * PER + r);
      sum += loc[r];
      mx = max(mx, loc[r]);
    }
    u32 run = block_inclusive_scan<u32>(sum, tmp, OpAdd<u32>(), (u32*)nullptr) - sum;
    block_inclusive_scan<u32>(mx, tmp, OpMax<u32>(), &mx);
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      cnt_set(threadIdx.x * PER + r, run);
      run += loc[r];
    }
    __syncthreads();
    if (mx <= SVO_BUCKET_MAX) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const u32 t = threadIdx.x + k * THREADS;
        if (t < m) s_k[cnt_get(bk[k]) + rk[k]] = ((tc[k] - tmin) << PB) | t;
      }
      __syncthreads();
      // each key's place in its bucket = the bucket's keys below it (keys are
      // distinct: they carry the position); every key counts in parallel
      // instead of one thread insertion-sorting a bucket
      u32 dst[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const u32 t = threadIdx.x + k * THREADS;
        dst[k] = 0;
        if (t < m) {
          const u32 b0 = cnt_get(bk[k]), b1 = bk[k] + 1 < CAP ? cnt_get(bk[k] + 1) : (u32)m;
          const u64 key = ((tc[k] - tmin) << PB) | t;
          u32 r = 0;
          for (u32 x = b0; x < b1; ++x) r += s_k[x] < key ? 1u : 0u;
          dst[k] = b0 + r;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const u32 t = threadIdx.x + k * THREADS;
        if (t < m) s_k[dst[k]] = ((tc[k] - tmin) << PB) | t;
      }
    } else {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const u32 t = threadIdx.x + k * THREADS;
        if (t < P) s_k[t] = t < m ? ((tc[k] - tmin) << PB) | t : ~0ull;
      }
      __syncthreads();
      for (u32 k = 2; k <= P; k <<= 1) {
        for (u32 j = k >> 1; j > 0; j >>= 1) {
          for (u32 t = threadIdx.x; t < P / 2; t += THREADS) {
            const u32 i = 2 * t - (t & (j - 1)), l = i + j;
            const u64 x = s_k[i], y = s_k[l];
            if ((y < x) == ((i & k) == 0)) {
              s_k[i] = y;
              s_k[l] = x;
            }
          }
          __syncthreads();
        }
      }
    }
  }
  __syncthreads();
  // runs of one tc: order by the node ranks (then position).  Each member
  // finds its run's bounds and counts the members below it, all in parallel
  // (runs are short: distinct nodes at one (millis, counter))
  {
    constexpr int PT = (CAP + THREADS - 1) / THREADS;
    u64 kk[PT];
    u32 kd[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const u32 p = threadIdx.x + k * THREADS;
      kd[k] = p;
      kk[k] = 0;
      if (p >= m) continue;
      const u64 kp = s_k[p];
      kk[k] = kp;
      const u64 tp = kp >> PB;
      const bool lo_eq = p > 0 && s_k[p - 1] >> PB == tp, hi_eq = p + 1 < m && s_k[p + 1] >> PB == tp;
      if (!lo_eq && !hi_eq) continue;
      u32 b0 = p, b1 = p + 1;
      while (b0 > 0 && s_k[b0 - 1] >> PB == tp && p - b0 < SVO_TIE_MAX) --b0;
      while (b1 < m && s_k[b1] >> PB == tp && b1 - b0 <= SVO_TIE_MAX) ++b1;
      if (b1 - b0 > SVO_TIE_MAX || (b0 > 0 && s_k[b0 - 1] >> PB == tp)) {
        atomicOr(&status->fallback, 1u);
        continue;
      }
      const u32 px = (u32)(kp & PMASK);
      const u64 hx = s_rh[px];
      const u32 lx = rl_get(px);
      u32 r = 0;
      for (u32 q = b0; q < b1; ++q) {
        const u32 pq = (u32)(s_k[q] & PMASK);
        const u64 hq = s_rh[pq];
        const u32 lq = rl_get(pq);
        r += (hq < hx || (hq == hx && (lq < lx || (lq == lx && pq < px)))) ? 1u : 0u;
      }
      kd[k] = b0 + r;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const u32 p = threadIdx.x + k * THREADS;
      if (p < m && kd[k] != p) s_k[kd[k]] = kk[k];
    }
  }
  __syncthreads();
  // among equal timestamps the one first in the batch (smallest batch index)
  // is the candidate insert -- independent of the order the segment's
  // messages were listed in (key-range segments are gathered unordered).
  // s_cnt[p] = 1: p is its timestamp's candidate.  A run's first position
  // decides the whole run (O(run) per run).
  for (u32 p = threadIdx.x; p < m; p += THREADS) {
    const u64 kp = s_k[p];
    const u32 pp = (u32)(kp & PMASK);
    auto same = [&](u32 x, u32 y) {
      const u32 px = (u32)(s_k[x] & PMASK), py = (u32)(s_k[y] & PMASK);
      return (s_k[x] >> PB) == (s_k[y] >> PB) && s_rh[px] == s_rh[py] && rl_get(px) == rl_get(py);
    };
    if (p > 0 && same(p - 1, p)) continue;  // not a run start: the start decides
    u32 e = p + 1;
    if (e < m && same(p, e)) {
      u32 best = p, bb = pidx(pp);
      for (; e < m && same(e - 1, e); ++e) {
        const u32 be = pidx((u32)(s_k[e] & PMASK));
        if (be < bb) {
          bb = be;
          best = e;
        }
      }
      for (u32 q = p; q < e; ++q) cnt_set(q, q == best ? 1u : 0u);
    } else {
      cnt_set(p, 1u);
    }
  }
  __syncthreads();
  // INSERT OR IGNORE against the stored rows (index.ts:154): a timestamp the
  // store already holds inserts nothing.  The segment's stored rows are read
  // once, coalesced, and each looked up among the sorted new keys in LDS
  // (the run of its timestamp loses its candidate) -- instead of a binary
  // search of the stored rows per candidate (four scattered global loads a
  // step, ~10 steps: the steady-state ingest's cost before).  A segment with
  // far more stored rows than new ones keeps the per-candidate searches.
  const u64 sa = sv.sa[s], sb = sv.sb[s];
  // (skip_stored: EVM_OPT_TEST_FAIL 2 -- the check left out, so that a
  // stored timestamp reaches the merge as a new row: its guard's test)
  const bool scan_stored = !skip_stored && sb > sa && sb - sa <= SVO_SCAN_STORED * m;
  if (scan_stored) {
    // (SVO_SB stored rows per thread per round: their tc loads, then the
    // ranks of those in the new keys' span, each batch issued together)
    constexpr int SB = SVO_SB;
    for (u64 k0 = sa + threadIdx.x; k0 < sb; k0 += (u64)SB * THREADS) {
      u64 btc[SB], bhi[SB];
      u32 blo[SB];
#pragma unroll
      for (int r = 0; r < SB; ++r) {
        const u64 k = k0 + (u64)r * THREADS;
        btc[r] = k < sb ? st.tc[k] : ~0ull;
      }
#pragma unroll
      for (int r = 0; r < SB; ++r) {
        const u64 k = k0 + (u64)r * THREADS;
        const bool in = k < sb && btc[r] >= tmin && btc[r] <= tmax;
        bhi[r] = in ? st.hi[k] : 0ull;
        blo[r] = in ? st.lo[k] : 0u;
      }
#pragma unroll
      for (int r = 0; r < SB; ++r) {
        const u64 ktc = btc[r];
        if (k0 + (u64)r * THREADS >= sb || ktc < tmin || ktc > tmax) continue;
        const u64 kd = ktc - tmin, khi = bhi[r];
        const u32 klo = blo[r];
        u32 lo = 0, hi = (u32)m;
        while (lo < hi) {  // first sorted position >= (tc, ranks)
          const u32 mid = (lo + hi) >> 1;
          const u64 kp = s_k[mid];
          const u64 td = kp >> PB;
          const u32 px = (u32)(kp & PMASK);
          const bool below = td != kd ? td < kd : s_rh[px] != khi ? s_rh[px] < khi : rl_get(px) < klo;
          if (below) lo = mid + 1;
          else hi = mid;
        }
        for (u32 p = lo; p < m; ++p) {  // the timestamp's run: its candidate is already stored
          const u64 kp = s_k[p];
          const u32 px = (u32)(kp & PMASK);
          if ((kp >> PB) != kd || s_rh[px] != khi || rl_get(px) != klo) break;
          cnt_set(p, 0u);
        }
      }
    }
    __syncthreads();
  }
  // first occurrences not yet stored; thread t owns sorted positions t, t +
  // THREADS, ... (row r = the positions r * THREADS ..): each row's stores
  // below are one coalesced run per wave, and the LDS reads are conflict-free
  // (ownership of t * PER .. made every store instruction a 32-B-strided
  // partial-line write: the row stores cost K5 a quarter of its time)
  u64 mt[PER], mh[PER];
  u32 ml[PER], mb[PER], mhash[PER];
  u32 insm = 0;
  constexpr int NPK = (PER + 3) / 4;  // per-row counts packed 4 to a u64 (16 bits each: <= THREADS)
  u64 cpk[NPK];
#pragma unroll
  for (int j = 0; j < NPK; ++j) cpk[j] = 0;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const u32 p = threadIdx.x + r * THREADS;
    mt[r] = mh[r] = 0;
    ml[r] = mb[r] = mhash[r] = 0;
    if (p < m) {
      const u64 kp = s_k[p];
      const u32 pos = (u32)(kp & PMASK);
      mt[r] = tmin + (kp >> PB);
      mh[r] = s_rh[pos];
      ml[r] = rl_get(pos);
      mb[r] = pidx(pos);
      mhash[r] = s_h[pos];
      bool ins = cnt_get(p) != 0;
      if (ins && sb > sa && !scan_stored && !skip_stored) {
        const SKey k{o, mt[r], mh[r], ml[r]};
        const size_t q = store_lower(st, sa, sb, k);
        ins = !(q < sb && skey_cmp(skey_at(st, q), k) == 0);
      }
      if (ins) {
        insm |= 1u << r;
        cpk[r >> 2] += 1ull << (16 * (r & 3));
      }
    }
  }
  // minute = millis / 60000: one 64-bit division per segment, then 32-bit
  // divisions of the offsets from a whole-minute base (spans < 2^32 ms)
  const u64 base_min = (tmin >> 16) / 60000ull, base_ms = base_min * 60000ull;
  const bool narrow = ((tmax >> 16) - base_ms) >> 32 == 0;
  // each row's inserted rows before this thread's (packed block scans; their
  // barriers free the LDS arrays), then the rows' bases from the totals
  u32 qr[PER];
  u32 M = 0;
#pragma unroll
  for (int j = 0; j < NPK; ++j) {
    u64 tot;
    const u64 ex = block_inclusive_scan<u64>(cpk[j], tmp64, OpAdd<u64>(), &tot) - cpk[j];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      if (4 * j + f < PER) {
        qr[4 * j + f] = M + (u32)((ex >> (16 * f)) & 0xFFFFull);
        M += (u32)((tot >> (16 * f)) & 0xFFFFull);
      }
    }
  }
  u32* s_min = reinterpret_cast<u32*>(s_k);  // inserted rows, sorted: minute
  u32* s_hq = s_min + CAP;                   //                        hash
  u32* s_lx = reinterpret_cast<u32*>(s_rh);  // per leaf: XOR
  u32* s_lm = s_lx + CAP;                    //           minute
  for (u32 t = threadIdx.x; t < CAP; t += THREADS) s_lx[t] = 0;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const u32 p = threadIdx.x + r * THREADS;
    if (p < m) {
      const bool ins = (insm >> r) & 1u;
      const u32 ob = orig ? orig[mb[r]] : mb[r];  // the message's index in the caller's batch
      // flags_preset: the batch's flags were set to INS by a coalesced fill;
      // only the duplicates (the minority) need a random 1-B store
      if (!ins || !flags_preset) flags[ob] = ins ? (uint8_t)EVM_MSG_INS : (uint8_t)0;
      if (ins) {
        const u32 q = qr[r];
        const u64 w = a + q;
        n_tc[w] = mt[r];
        n_hi[w] = mh[r];
        n_lo[w] = ml[r];
        n_id[w] = id_base + ob;
        if (n_owner) n_owner[w] = o;  // (the rows are written into an empty store's own arrays)
        s_min[q] = narrow ? (u32)base_min + (u32)((mt[r] >> 16) - base_ms) / 60000u
                          : (u32)((mt[r] >> 16) / 60000ull);  // == rec.minute on the native domain
        s_hq[q] = mhash[r];
      }
    }
  }
  __syncthreads();
  // leaves: runs of one minute among the inserted rows (sorted by millis);
  // every row's leaf = the run heads at or before it (packed scans again)
  u32 hm = 0;
  u64 hpk[NPK];
#pragma unroll
  for (int j = 0; j < NPK; ++j) hpk[j] = 0;
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const u32 p = threadIdx.x + r * THREADS;
    if (p < M && (p == 0 || s_min[p] != s_min[p - 1])) {
      hm |= 1u << r;
      hpk[r >> 2] += 1ull << (16 * (r & 3));
    }
  }
  u32 lidr[PER];
  u32 NL = 0;
#pragma unroll
  for (int j = 0; j < NPK; ++j) {
    u64 tot;
    const u64 inc = block_inclusive_scan<u64>(hpk[j], tmp64, OpAdd<u64>(), &tot);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      if (4 * j + f < PER) {
        lidr[4 * j + f] = NL + (u32)((inc >> (16 * f)) & 0xFFFFull) - 1u;  // (the row's head count at or before it)
        NL += (u32)((tot >> (16 * f)) & 0xFFFFull);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const u32 p = threadIdx.x + r * THREADS;
    if (p < M) {
      // (a row's leaf: the last head at or before it -- in an earlier row of
      // positions when no head in this row precedes it)
      u32 lid = lidr[r];
      if ((hm >> r) & 1u) s_lm[lid] = s_min[p];
      atomicXor(&s_lx[lid], s_hq[p]);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && NL) {
    const int l0 = base3_len(s_lm[0]), l1 = base3_len(s_lm[NL - 1]);
    if (l0 != l1) atomicOr(&status->fallback, 1u);
    // (one key length over the batch: code order = minute order; a same-address
    // atomic from every workgroup would serialise -- only new bits are written)
    atomic_or_if(&status->lens, (1u << l0) | (1u << l1));
  }
  u32 dups = 0, lx = 0;
  // LEAF (a store with a tree): the segment's tree codes staged in the dead
  // rank / hash arrays, so the new leaves' searches stay in LDS
  const u64 tl = lb - la;
  const bool leaf_lds = LEAF && tl <= CAP;
  if constexpr (LEAF) {
    if (leaf_lds)
      for (u32 i = threadIdx.x; i < (u32)tl; i += THREADS) {
        const u64 c = t_ck[la + i];
        s_rl[i] = (u32)(c >> 32);
        s_h[i] = (u32)c;
      }
    __syncthreads();
  }
  for (u32 l = threadIdx.x; l < NL; l += THREADS) {
    const u64 code = ((u64)o << 40) | minute_code_from(s_lm[l], [&](u32 x) { return (u32)s_b3[x]; });
    u64 k;
    bool dup;
    if (leaf_lds) {
      u32 lo = 0, hi = (u32)tl;
      while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if ((((u64)s_rl[mid] << 32) | s_h[mid]) < code) lo = mid + 1;
        else hi = mid;
      }
      k = la + lo;
      dup = lo < (u32)tl && (((u64)s_rl[lo] << 32) | s_h[lo]) == code;
    } else {
      k = lb_u64(t_ck, la, lb, code);
      dup = k < lb && t_ck[k] == code;
    }
    l_ck[lb0 + l] = code;
    l_xr[lb0 + l] = (int32_t)s_lx[l];
    // (a gapped tree -- the empty store's, g_off -- is final here: no merge or
    // copy reads the marks, and no leaf of an empty tree is a duplicate)
    if (!g_off) l_dup[lb0 + l] = dup ? 1 : 0;
    dups += dup ? 1u : 0u;
    lx ^= s_lx[l];
  }
  if (g_off) {
    // a gapped tree (the empty store, one segment per owner): the owner's
    // leaves stay where they are, with their owner-local exclusive prefix XOR
    // -- each wave scans one contiguous quarter of the leaves 64 at a time
    // (coalesced stores), carried in from the quarters before it
    constexpr u32 NW = THREADS / 64;
    const u32 ch = ((NL + NW - 1) / NW + 63) & ~63u;
    const u32 l0 = min(NL, wv * ch), l1 = min(NL, l0 + ch);
    u32 x = 0;
    for (u32 l = l0 + lane; l < l1; l += 64) x ^= s_lx[l];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x ^= __shfl_xor(x, d, 64);
    __syncthreads();  // (tmp: free after the scans above)
    if (lane == 0) tmp[wv] = x;
    __syncthreads();
    u32 carry = 0;
    for (u32 w = 0; w < wv; ++w) carry ^= tmp[w];
    for (u32 b = l0; b < l1; b += 64) {  // (wave-uniform bounds: every lane takes part in the shuffles)
      const u32 l = b + lane;
      const u32 v = l < l1 ? s_lx[l] : 0u;
      u32 inc = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(inc, d, 64);
        if (lane >= (u32)d) inc ^= y;
      }
      if (l < l1) l_pfx[lb0 + l] = (int32_t)(carry ^ inc ^ v);
      carry ^= __shfl(inc, 63, 64);
    }
    if (wv == NW - 1 && lane == 0) {  // (the last wave's carry: every leaf)
      l_pfx[lb0 + NL] = (int32_t)carry;
      g_off[o] = lb0;
      g_end[o] = lb0 + NL;
    }
    __syncthreads();  // (tmp is read again below)
  }
  u32 dtot;
  block_inclusive_scan<u32>(dups, tmp, OpAdd<u32>(), &dtot);
  // the XOR of the segment's new leaves (the empty store's copy writes the
  // tree's prefix XOR from these: no scan over the leaves)
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) lx ^= __shfl_xor(lx, d, 64);
  if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = lx;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 x = 0;
    for (int w = 0; w < THREADS / 64; ++w) x ^= tmp[w];
    cnt_rows[s] = M;
    cnt_new[s] = NL;
    cnt_leaves[s] = (u32)(lb - la) + NL - dtot;
    cnt_xor[s] = x;
  }
}

// Segments by share size, listed per K5 capacity (<= 128, <= 512, <= 1,024,
// the rest): each K5 pass then launches exactly its segments -- a workgroup
// per segment that would only defer itself costs a dispatch all the same.
// lists[c * (NS + 1)] = count of class c, its segments after it.
constexpr int SEG_CLASSES = 6;
__global__ void k_seg_classes(SegView sv, u32 NS, u32* __restrict__ lists) {
  const int lane = threadIdx.x & 63;
  const u64 lt = lanemask_lt();
  for (u32 s0 = blockIdx.x * blockDim.x; s0 < NS; s0 += gridDim.x * blockDim.x) {  // uniform per wave
    const u32 s = s0 + threadIdx.x;
    int cls = -1;
    if (s < NS) {
      const u64 m = sv.start[s + 1] - sv.start[s];
      cls = m <= 128 ? 0 : m <= 256 ? 1 : m <= 512 ? 2 : m <= 1024 ? 3 : m <= 2048 ? 4 : 5;
    }
#pragma unroll
    for (int c = 0; c < SEG_CLASSES; ++c) {
      const u64 b = __ballot(cls == c);
      if (!b) continue;
      u32* L = lists + (size_t)c * (NS + 1);
      const int leader = __builtin_ctzll(b);
      u32 base = 0;
      if (lane == leader) base = atomicAdd(&L[0], (u32)__popcll(b));
      base = __shfl(base, leader, 64);
      if (cls == c) L[1 + base + (u32)__popcll(b & lt)] = s;
    }
  }
}

// segments of an owner sent to the sort path contribute nothing here (its
// stored rows and leaves are still copied)
__global__ void k_seg_fix(SegView sv, u32 NS, const uint8_t* __restrict__ ownbig, u32* __restrict__ cnt_rows,
                          u32* __restrict__ cnt_new, u32* __restrict__ cnt_leaves, u32* __restrict__ cnt_xor) {
  for (u32 s = blockIdx.x * blockDim.x + threadIdx.x; s < NS; s += gridDim.x * blockDim.x) {
    if (!ownbig[seg_owner(sv, s)]) continue;
    cnt_rows[s] = 0;
    cnt_new[s] = 0;
    cnt_leaves[s] = (u32)(sv.lb[s] - sv.la[s]);
    cnt_xor[s] = 0;
  }
}

// The merge of a segment's stored rows / tree leaves with its new ones.  With
// at most SVB_LDS new keys (nearly every segment) they sit in LDS: a stored
// row finds its place by a binary search there (#new keys below it), and a
// new row's place comes from the same searches -- a histogram of those counts,
// whose inclusive prefix at j is the number of stored rows below new row j
// (keys are disjoint) -- so no search touches global memory.  Larger
// segments search the global arrays as before.  Leaves the same way (an equal
// tree leaf counts one bin higher: it is not below the new code).
constexpr u32 SVB_LDS = 1024;
constexpr int SVB_B = 4;  // stored rows / leaves per thread whose loads are issued together
// Rows of a segment with <= SVB_SRC output rows (stored + new) are written
// once, in output order: the searches fill a source map in LDS (output
// position -> stored row or new row) and a third pass copies each output row
// from its source, consecutive lanes on consecutive rows.  (Writing stored
// rows at their places and the new ones into the gaps afterwards touched
// every output line twice: 16.4 GB written per reingest merge vs ~8.7 GB.)
constexpr u32 SVB_SRC = 4096;
constexpr uint16_t SVB_NEW = 0x8000, SVB_EQ = 0x4000;
static_assert(SVB_LDS <= SVB_EQ && SVB_SRC <= SVB_NEW, "source map fields");


__device__ __forceinline__ void svb_inclusive_prefix(u32* h, u32 m, u32* tmp) {
  // h[0..m) -> inclusive prefix sums in place (m <= SVB_LDS + 1)
  constexpr u32 PER = (SVB_LDS + 1 + SVO_THREADS - 1) / SVO_THREADS;
  const u32 b0 = min(m, threadIdx.x * PER), b1 = min(m, b0 + PER);
  u32 sum = 0;
  for (u32 q = b0; q < b1; ++q) sum += h[q];
  u32 run = block_inclusive_scan<u32>(sum, tmp, OpAdd<u32>(), (u32*)nullptr) - sum;
  for (u32 q = b0; q < b1; ++q) {
    run += h[q];
    h[q] = run;
  }
  __syncthreads();
}

// MERGE = false: the store is empty (no stored rows, no tree leaves): no LDS
// staging (its 24 KiB would cost occupancy for nothing).
template <bool MERGE>
__global__ __launch_bounds__(SVO_THREADS) void k_svo_b(
    SegView sv, u32 NS, u32 n_owners, StoreView st, const u64* __restrict__ st_id, const u64* __restrict__ n_tc,
    const u64* __restrict__ n_hi, const u32* __restrict__ n_lo, const u64* __restrict__ n_id,
    const u32* __restrict__ cnt_rows, const u32* __restrict__ row_pos,
    const u64* __restrict__ t_ck, const int32_t* __restrict__ t_xr, const u64* __restrict__ l_ck,
    const int32_t* __restrict__ l_xr, const uint8_t* __restrict__ l_dup, const u32* __restrict__ cnt_new,
    const u32* __restrict__ leaf_pos, StoreOut so, u64* __restrict__ so_off, u64* __restrict__ to_ck,
    int32_t* __restrict__ to_xr, u64* __restrict__ to_off, int rows_in_place, u32* __restrict__ merr) {
  __shared__ u32 s_dp[SVO_CAP + 1];  // exclusive prefix count of the new leaves already in the tree
  // The merge places rows by assuming the segment's stored and new keys are
  // disjoint (K5 dropped every stored timestamp) and that K5's l_dup marks
  // exactly the new leaves equal to a tree leaf.  Both are checked here: a
  // stored row equal to a new one, a hole left in a source map, or a count of
  // equal leaves other than K5's sets *merr (the host then discards the new
  // store and returns EVM_ESTATE) and the segment writes nothing past that
  // point; the writes before it stay inside the segment's output range.
  __shared__ u32 s_bad, s_eq;
  __shared__ u32 tmp[SVO_THREADS / 64 + 1];
  constexpr u32 LN = MERGE ? SVB_LDS : 1;
  __shared__ u64 k_tc[LN], k_hi[LN];  // new row keys (then new leaf codes in k_tc)
  __shared__ u32 k_lo[LN];
  __shared__ u32 hist[LN + 1];
  __shared__ uint16_t src[MERGE ? SVB_SRC : 1];  // output row -> source (SVB_NEW | new j, or stored k - sa)
  const u32 s = blockIdx.x;
  const u32 o = seg_owner(sv, s);
  const u64 a = sv.start[s];
  const u32 M = cnt_rows[s], NL = cnt_new[s];
  const u64 sa = sv.sa[s], sb = sv.sb[s];
  const u64 base = sa + row_pos[s];  // rows of the earlier segments: old + new
  // rows: the owner's stored and new keys are disjoint sorted lists
  // rows_in_place: an empty store whose every message was inserted -- the
  // K5 rows already sit at their final places (position = batch position)
  const bool lds_rows = MERGE && !rows_in_place && M <= SVB_LDS;
  const bool by_src = lds_rows && (sb - sa) + M <= SVB_SRC;
  constexpr uint16_t SRC_HOLE = 0xffff;  // (no valid entry: row / leaf indexes stay below SVB_EQ)
  if (threadIdx.x == 0) s_bad = s_eq = 0;
  if (lds_rows) {
    for (u32 j = threadIdx.x; j < M; j += SVO_THREADS) {
      k_tc[j] = n_tc[a + j];
      k_hi[j] = n_hi[a + j];
      k_lo[j] = n_lo[a + j];
    }
    for (u32 j = threadIdx.x; j <= M; j += SVO_THREADS) hist[j] = 0;
    if (by_src)
      for (u32 p = threadIdx.x; p < (u32)(sb - sa) + M; p += SVO_THREADS) src[p] = SRC_HOLE;
  }
  __syncthreads();
  // (assembling each output column of a segment in LDS and writing it once,
  // coalesced, measured slower: reingest merge 5.77 vs 4.91 ms in one run)
  // (SVB_B rows per thread per round, all their loads issued before any is
  // used: one memory latency per round instead of one per row)
  for (u64 k0 = sa + threadIdx.x; !rows_in_place && k0 < sb; k0 += (u64)SVB_B * SVO_THREADS) {
    u64 rtc[SVB_B], rhi[SVB_B], rid[SVB_B];
    u32 rlo[SVB_B];
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u64 k = k0 + (u64)r * SVO_THREADS;
      rtc[r] = rhi[r] = rid[r] = 0;
      rlo[r] = 0;
      if (k < sb) {
        rtc[r] = st.tc[k];
        rhi[r] = st.hi[k];
        rlo[r] = st.lo[k];
        if (!by_src) rid[r] = st_id[k];
      }
    }
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u64 k = k0 + (u64)r * SVO_THREADS;
      if (k >= sb) break;
      const SKey key{o, rtc[r], rhi[r], rlo[r]};  // (the segment's stored rows are all owner o's)
      u32 lo = 0, hi = M;
      if (lds_rows) {
        while (lo < hi) {  // (one owner: compare (tc, hi, lo))
          const u32 mid = (lo + hi) >> 1;
          const bool below = k_tc[mid] != key.tc ? k_tc[mid] < key.tc
                             : k_hi[mid] != key.hi ? k_hi[mid] < key.hi : k_lo[mid] < key.lo;
          if (below) lo = mid + 1;
          else hi = mid;
        }
        if (lo < M && k_tc[lo] == key.tc && k_hi[lo] == key.hi && k_lo[lo] == key.lo) s_bad = 1;  // not disjoint
        atomicAdd(&hist[lo], 1u);
      } else {
        while (lo < hi) {
          const u32 mid = (lo + hi) >> 1;
          if (skey_cmp(SKey{o, n_tc[a + mid], n_hi[a + mid], n_lo[a + mid]}, key) < 0) lo = mid + 1;
          else hi = mid;
        }
        if (lo < M && skey_cmp(SKey{o, n_tc[a + lo], n_hi[a + lo], n_lo[a + lo]}, key) == 0) s_bad = 1;
      }
      if (by_src) {
        src[(k - sa) + lo] = (uint16_t)(k - sa);
        continue;
      }
      const u64 w = base + (k - sa) + lo;
      so.owner[w] = o;
      so.tc[w] = key.tc;
      so.hi[w] = key.hi;
      so.lo[w] = key.lo;
      so.id[w] = rid[r];
    }
  }
  __syncthreads();
  if (lds_rows) svb_inclusive_prefix(hist, M + 1, tmp);  // hist[j] = stored rows below new row j
  if (by_src) {
    for (u32 j = threadIdx.x; j < M; j += SVO_THREADS) src[j + hist[j]] = (uint16_t)(SVB_NEW | j);
    __syncthreads();
    for (u32 p = threadIdx.x; p < (u32)(sb - sa) + M; p += SVO_THREADS)
      if (src[p] == SRC_HOLE) s_bad = 1;  // (two rows placed at one output position)
    __syncthreads();
  }
  if (s_bad) {  // (uniform: read after a barrier)
    if (threadIdx.x == 0) atomicOr(merr, 1u);
    return;
  }
  if (by_src) {
    const u32 T = (u32)(sb - sa) + M;
    for (u32 p0 = threadIdx.x; p0 < T; p0 += SVB_B * SVO_THREADS) {
      u64 vtc[SVB_B], vhi[SVB_B], vid[SVB_B];
      u32 vlo[SVB_B];
#pragma unroll
      for (int r = 0; r < SVB_B; ++r) {
        const u32 p = p0 + r * SVO_THREADS;
        vtc[r] = vhi[r] = vid[r] = 0;
        vlo[r] = 0;
        if (p < T) {
          const u32 e = src[p];
          if (e & SVB_NEW) {
            const u32 j = e & (SVB_NEW - 1u);
            vtc[r] = k_tc[j];
            vhi[r] = k_hi[j];
            vlo[r] = k_lo[j];
            vid[r] = n_id[a + j];
          } else {
            const u64 k = sa + e;
            vtc[r] = st.tc[k];
            vhi[r] = st.hi[k];
            vlo[r] = st.lo[k];
            vid[r] = st_id[k];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < SVB_B; ++r) {
        const u32 p = p0 + r * SVO_THREADS;
        if (p >= T) break;
        const u64 w = base + p;
        so.owner[w] = o;
        so.tc[w] = vtc[r];
        so.hi[w] = vhi[r];
        so.lo[w] = vlo[r];
        so.id[w] = vid[r];
      }
    }
  }
  for (u32 j0 = threadIdx.x; !rows_in_place && !by_src && j0 < M; j0 += SVB_B * SVO_THREADS) {
    u64 nid[SVB_B];
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u32 j = j0 + r * SVO_THREADS;
      nid[r] = j < M ? n_id[a + j] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u32 j = j0 + r * SVO_THREADS;
      if (j >= M) break;
      SKey key;
      u64 below;
      if (lds_rows) {
        key = SKey{o, k_tc[j], k_hi[j], k_lo[j]};
        below = hist[j];
      } else {
        key = SKey{o, n_tc[a + j], n_hi[a + j], n_lo[a + j]};
        below = store_lower(st, sa, sb, key) - sa;
      }
      const u64 w = base + j + below;
      so.owner[w] = o;
      so.tc[w] = key.tc;
      so.hi[w] = key.hi;
      so.lo[w] = key.lo;
      so.id[w] = nid[r];
    }
  }
  // leaves: union of the tree's and the new ones by code, equal codes XOR-combined
  // (K5 wrote the segment's new leaves at slots a + s ..)
  const u64 la = sv.la[s], lb = sv.lb[s];
  const u64 an = a + s;
  const u64 lbase = leaf_pos[s];
  constexpr int PERB = SVO_CAP / SVO_THREADS;
  u32 d[PERB], c = 0;
#pragma unroll
  for (int r = 0; r < PERB; ++r) {
    const u32 j = threadIdx.x * PERB + r;
    d[r] = j < NL ? (u32)l_dup[an + j] : 0u;
    c += d[r];
  }
  u32 dtot;
  u32 run = block_inclusive_scan<u32>(c, tmp, OpAdd<u32>(), &dtot) - c;
#pragma unroll
  for (int r = 0; r < PERB; ++r) {
    const u32 j = threadIdx.x * PERB + r;
    if (j < NL) s_dp[j] = run;
    run += d[r];
  }
  if (threadIdx.x == 0) s_dp[NL] = dtot;
  const bool lds_leaves = MERGE && NL <= SVB_LDS;
  // leaves written once through the source map too: a tree leaf's entry is
  // its index, a new leaf's SVB_NEW | j, a tree leaf equal to new leaf j
  // SVB_NEW | SVB_EQ | j with the combined XOR parked in eqx[j] (k_hi is free)
  const u64 TL = (lb - la) + NL - dtot;
  const bool leaves_src = lds_leaves && TL <= SVB_SRC;
  u32* eqx = reinterpret_cast<u32*>(k_hi);
  __syncthreads();  // (the rows' LDS keys are dead: the leaf codes take k_tc)
  if (lds_leaves) {
    for (u32 j = threadIdx.x; j < NL; j += SVO_THREADS) k_tc[j] = l_ck[an + j];
    for (u32 j = threadIdx.x; j <= NL; j += SVO_THREADS) hist[j] = 0;
    if (leaves_src)
      for (u32 q = threadIdx.x; q < (u32)TL; q += SVO_THREADS) src[q] = SRC_HOLE;
  }
  __syncthreads();
  for (u64 k0 = la + threadIdx.x; k0 < lb; k0 += (u64)SVB_B * SVO_THREADS) {
    u64 tcode[SVB_B];
    int32_t txr[SVB_B];
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u64 k = k0 + (u64)r * SVO_THREADS;
      tcode[r] = k < lb ? t_ck[k] : 0ull;
      txr[r] = k < lb ? t_xr[k] : 0;
    }
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u64 k = k0 + (u64)r * SVO_THREADS;
      if (k >= lb) break;
      const u64 code = tcode[r];
      u32 j;
      bool eq;
      if (lds_leaves) {
        u32 lo = 0, hi = NL;
        while (lo < hi) {
          const u32 mid = (lo + hi) >> 1;
          if (k_tc[mid] < code) lo = mid + 1;
          else hi = mid;
        }
        j = lo;
        eq = j < NL && k_tc[j] == code;
        if (eq) atomicAdd(&s_eq, 1u);
        atomicAdd(&hist[j + (eq ? 1u : 0u)], 1u);  // (an equal tree leaf is not below new leaf j)
        if (leaves_src) {
          const u32 q = (u32)(k - la) + j - s_dp[j];
          if (eq) {
            eqx[j] = (u32)(txr[r] ^ l_xr[an + j]);
            src[q] = (uint16_t)(SVB_NEW | SVB_EQ | j);
          } else {
            src[q] = (uint16_t)(k - la);
          }
          continue;
        }
      } else {
        j = (u32)(lb_u64(l_ck, an, an + NL, code) - an);  // new leaves below this code
        eq = j < NL && l_ck[an + j] == code;
        if (eq) atomicAdd(&s_eq, 1u);
      }
      const u64 w = lbase + (k - la) + j - s_dp[j];
      if (w >= lbase + TL) continue;  // (only when l_dup and the tree disagree: flagged below)
      to_ck[w] = code;
      to_xr[w] = txr[r] ^ (eq ? l_xr[an + j] : 0);
    }
  }
  __syncthreads();
  if (lds_leaves) svb_inclusive_prefix(hist, NL + 1, tmp);  // hist[j] = tree leaves below new leaf j
  if (s_eq != dtot) {  // (uniform: read after a barrier) K5's equal leaves are not the tree's
    if (threadIdx.x == 0) atomicOr(merr, 2u);
    return;
  }
  if (leaves_src) {
    for (u32 j = threadIdx.x; j < NL; j += SVO_THREADS)
      if (!l_dup[an + j]) src[(j - s_dp[j]) + hist[j]] = (uint16_t)(SVB_NEW | j);
    __syncthreads();
    for (u32 q = threadIdx.x; q < (u32)TL; q += SVO_THREADS)
      if (src[q] == SRC_HOLE) s_bad = 1;
    __syncthreads();
    if (s_bad) {
      if (threadIdx.x == 0) atomicOr(merr, 4u);
      return;
    }
    for (u32 q0 = threadIdx.x; q0 < (u32)TL; q0 += SVB_B * SVO_THREADS) {
      u64 vck[SVB_B];
      int32_t vxr[SVB_B];
#pragma unroll
      for (int r = 0; r < SVB_B; ++r) {
        const u32 q = q0 + r * SVO_THREADS;
        vck[r] = 0;
        vxr[r] = 0;
        if (q < (u32)TL) {
          const u32 e = src[q];
          if (e & SVB_NEW) {
            const u32 j = e & (SVB_EQ - 1u);
            vck[r] = k_tc[j];
            vxr[r] = (e & SVB_EQ) ? (int32_t)eqx[j] : l_xr[an + j];
          } else {
            vck[r] = t_ck[la + e];
            vxr[r] = t_xr[la + e];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < SVB_B; ++r) {
        const u32 q = q0 + r * SVO_THREADS;
        if (q >= (u32)TL) break;
        to_ck[lbase + q] = vck[r];
        to_xr[lbase + q] = vxr[r];
      }
    }
  }
  for (u32 j = threadIdx.x; !leaves_src && j < NL; j += SVO_THREADS) {
    if (l_dup[an + j]) continue;
    const u64 code = lds_leaves ? k_tc[j] : l_ck[an + j];
    const u64 below = lds_leaves ? (u64)hist[j] : lb_u64(t_ck, la, lb, code) - la;
    const u64 w = lbase + (j - s_dp[j]) + below;
    if (w >= lbase + TL) continue;
    to_ck[w] = code;
    to_xr[w] = l_xr[an + j];
  }
  if (threadIdx.x == 0) {
    if (s == 0 || seg_owner(sv, s - 1) != o) {  // the owner's first segment starts its rows and leaves
      so_off[o] = base;
      to_off[o] = lbase;
    }
    if (s == NS - 1) {
      so_off[n_owners] = base + (sb - sa) + M;
      to_off[n_owners] = lbase + (lb - la) + NL - dtot;
    }
  }
}

// The empty store's commit (no stored rows, no tree leaves: k_svo_b<false>'s
// case): each segment's rows -- unless K5 already placed them -- and its new
// leaves copied to their places, one wave per segment and SVB_B items per lane
// in flight.  Nothing merges, so none of the merge's block scans and barriers
// (~100k segments of ~1,000 rows: the merge's per-workgroup fixed work was
// most of its time).
constexpr int SVC_WAVES = 4;
__global__ __launch_bounds__(64 * SVC_WAVES) void k_svo_copy(
    SegView sv, u32 NS, u32 n_owners, const u64* __restrict__ n_tc, const u64* __restrict__ n_hi,
    const u32* __restrict__ n_lo, const u64* __restrict__ n_id, const u32* __restrict__ cnt_rows,
    const u32* __restrict__ row_pos, const u64* __restrict__ l_ck, const int32_t* __restrict__ l_xr,
    const u32* __restrict__ cnt_new, const u32* __restrict__ leaf_pos, StoreOut so, u64* __restrict__ so_off,
    u64* __restrict__ to_ck, int32_t* __restrict__ to_xr, u64* __restrict__ to_off, int rows_in_place,
    const int32_t* __restrict__ xpos, int32_t* __restrict__ to_pfx) {
  const u32 s = blockIdx.x * SVC_WAVES + (threadIdx.x >> 6);
  if (s >= NS) return;  // (a whole wave: the kernel has no block barrier)
  const u32 lane = threadIdx.x & 63;
  const u32 o = seg_owner(sv, s);
  const u64 a = sv.start[s];
  const u32 M = cnt_rows[s], NL = cnt_new[s];
  const u64 base = sv.sa[s] + row_pos[s];
  const u64 lbase = leaf_pos[s];
  for (u32 j0 = lane; !rows_in_place && j0 < M; j0 += SVB_B * 64) {
    u64 vtc[SVB_B], vhi[SVB_B], vid[SVB_B];
    u32 vlo[SVB_B];
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u32 j = j0 + r * 64;
      const bool in = j < M;
      vtc[r] = in ? n_tc[a + j] : 0ull;
      vhi[r] = in ? n_hi[a + j] : 0ull;
      vlo[r] = in ? n_lo[a + j] : 0u;
      vid[r] = in ? n_id[a + j] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u32 j = j0 + r * 64;
      if (j >= M) break;
      const u64 w = base + j;
      so.owner[w] = o;
      so.tc[w] = vtc[r];
      so.hi[w] = vhi[r];
      so.lo[w] = vlo[r];
      so.id[w] = vid[r];
    }
  }
  // the tree's exclusive prefix XOR over the copied leaves, carried from the
  // segments before (xpos: a scan of K5's per-segment XORs)
  u32 carry = (u32)xpos[s];
  for (u32 k0 = 0; k0 < NL; k0 += SVB_B * 64) {  // (wave-uniform bounds: every lane takes part in the shuffles)
    const u32 j0 = k0 + lane;
    u64 vck[SVB_B];
    int32_t vxr[SVB_B];
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u32 j = j0 + r * 64;
      vck[r] = j < NL ? l_ck[a + s + j] : 0ull;  // (K5's slots for the segment's new leaves)
      vxr[r] = j < NL ? l_xr[a + s + j] : 0;
    }
#pragma unroll
    for (int r = 0; r < SVB_B; ++r) {
      const u32 j = j0 + r * 64;
      u32 inc = (u32)vxr[r];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(inc, d, 64);
        if (lane >= (u32)d) inc ^= y;
      }
      if (j < NL) {
        to_ck[lbase + j] = vck[r];
        to_xr[lbase + j] = vxr[r];
        to_pfx[lbase + j] = (int32_t)(carry ^ inc ^ (u32)vxr[r]);
      }
      carry ^= __shfl(inc, 63, 64);
    }
  }
  if (lane == 0 && s == NS - 1) to_pfx[lbase + NL] = (int32_t)carry;  // the tree's total
  if (lane == 0) {
    if (s == 0 || seg_owner(sv, s - 1) != o) {  // the owner's first segment starts its rows and leaves
      so_off[o] = base;
      to_off[o] = lbase;
    }
    if (s == NS - 1) {
      so_off[n_owners] = base + M;
      to_off[n_owners] = lbase + NL;
    }
  }
}

// ------------------------------------------------------------------ select
// rank -> hex value (case folded)
__device__ __forceinline__ u32 rank_hex(u32 r) { return r >= 16u ? r - 6u : r; }

__device__ __forceinline__ u64 node_hex_of(u64 hi, u32 lo) {
  u64 v = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) v = (v << 4) | rank_hex((u32)(hi >> (55 - 5 * i)) & 31u);
#pragma unroll
  for (int i = 0; i < 4; ++i) v = (v << 4) | rank_hex((lo >> (15 - 5 * i)) & 31u);
  return v;
}

// the requester's nodeId: 16 hex chars, either case -> folded value (or -1)
__device__ __forceinline__ bool parse_node16(const uint8_t* s, u64* v) {
  u64 x = 0;
  for (int i = 0; i < 16; ++i) {
    const u32 c = s[i];
    u32 d;
    if (c - 0x30u < 10u) d = c - 0x30u;
    else if (c - 0x41u < 6u) d = c - 0x37u;
    else if (c - 0x61u < 6u) d = c - 0x57u;
    else return false;
    x = (x << 4) | d;
  }
  *v = x;
  return true;
}

// getMessages selection, load-balanced over the candidate rows (an owner's
// rows after its bound) rather than over owners: one Zipf-hot owner's tens of
// millions of rows spread over the whole chip instead of one thread.
// Pass 1 (per owner): the first row after the bound and the candidate count.
__global__ void k_sv_sel_first(StoreView st, u32 n_owners, const int64_t* __restrict__ diff,
                               const uint8_t* __restrict__ node, const uint8_t* __restrict__ active,
                               u64* __restrict__ first, u32* __restrict__ cand, u64* __restrict__ req,
                               u32* __restrict__ bad) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < n_owners; o += gridDim.x * blockDim.x) {
    cand[o] = 0;
    first[o] = 0;
    if (active && !active[o]) continue;
    const int64_t d = diff[o];
    if (d < 0) continue;  // none or RangeError
    if (node) {
      u64 r = 0;
      if (!parse_node16(node + 16 * (size_t)o, &r)) {
        atomicOr(bad, 1u);
        continue;
      }
      req[o] = r;
    }
    const size_t a = st.off[o], b = st.off[o + 1];
    // timestamp > "ISO(d)-0000-0000000000000000": smallest key with tc = d << 16
    const SKey since{o, (u64)d << 16, 0ull, 0u};
    size_t q = store_lower(st, a, b, since);
    if (q < b && skey_cmp(skey_at(st, q), since) == 0) ++q;  // strictly greater
    first[o] = q;
    cand[o] = (u32)(b - q);
  }
}

constexpr int SEL_THREADS = 256;

// Owner of candidate j: the last owner whose candidate offset is <= j (owners
// with no candidates share their successor's offset and are skipped).
__device__ __forceinline__ u32 cand_owner(const u32* __restrict__ cpos, u32 lo, u32 hi, u32 j) {
  while (lo + 1 < hi) {  // invariant: cpos[lo] <= j < cpos[hi] (cpos[n_owners] = C)
    const u32 mid = (lo + hi) >> 1;
    if (cpos[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Pass 2 (per candidate): keep unless the row's node is the requester's
// (`NOT LIKE '%' || nodeId`).  Each block narrows the owner search to its
// own tile of candidates.  cpos has n_owners + 1 entries.
__global__ __launch_bounds__(SEL_THREADS) void k_sv_sel_keep(StoreView st, u32 n_owners, u32 C,
                                                             const u32* __restrict__ cpos, const u64* __restrict__ first,
                                                             const u64* __restrict__ req, u32* __restrict__ keep) {
  __shared__ u32 range[2];
  for (u32 j0 = blockIdx.x * SEL_THREADS; j0 < C; j0 += gridDim.x * SEL_THREADS) {
    const u32 j1 = min(C, j0 + SEL_THREADS) - 1;
    __syncthreads();
    if (threadIdx.x == 0) range[0] = cand_owner(cpos, 0, n_owners, j0);
    if (threadIdx.x == 1) range[1] = cand_owner(cpos, 0, n_owners, j1) + 1;
    __syncthreads();
    const u32 j = j0 + threadIdx.x;
    if (j > j1) continue;
    const u32 o = cand_owner(cpos, range[0], range[1], j);
    const size_t k = first[o] + (j - cpos[o]);
    keep[j] = node_hex_of(st.hi[k], st.lo[k]) != req[o];
  }
}

// Pass 3 (per candidate): write the kept ids at their selection positions
// (kpos = exclusive scan of keep, or null when every candidate is kept).
__global__ __launch_bounds__(SEL_THREADS) void k_sv_sel_emit(u32 n_owners, u32 C, const u32* __restrict__ cpos,
                                                             const u64* __restrict__ first, const u32* __restrict__ keep,
                                                             const u32* __restrict__ kpos, const u64* __restrict__ id,
                                                             u64* __restrict__ sel_id, StoreView st,
                                                             u64* __restrict__ sel_key) {
  __shared__ u32 range[2];
  for (u32 j0 = blockIdx.x * SEL_THREADS; j0 < C; j0 += gridDim.x * SEL_THREADS) {
    const u32 j1 = min(C, j0 + SEL_THREADS) - 1;
    __syncthreads();
    if (threadIdx.x == 0) range[0] = cand_owner(cpos, 0, n_owners, j0);
    if (threadIdx.x == 1) range[1] = cand_owner(cpos, 0, n_owners, j1) + 1;
    __syncthreads();
    const u32 j = j0 + threadIdx.x;
    if (j > j1) continue;
    if (keep && !keep[j]) continue;
    const u32 o = cand_owner(cpos, range[0], range[1], j);
    const size_t k = first[o] + (j - cpos[o]);
    const u32 q = kpos ? kpos[j] : j;
    sel_id[q] = id[k];
    if (sel_key) {  // the row's order key: merges selections of one owner split over ranks
      sel_key[3 * (size_t)q] = st.tc[k];
      sel_key[3 * (size_t)q + 1] = st.hi[k];
      sel_key[3 * (size_t)q + 2] = st.lo[k];
    }
  }
}

// Passes 2 + 3 in one launch (a requester to exclude): each tile of
// SEL_TILE candidates decides keep (the row's node is not the requester's),
// ranks its kept rows in candidate order with wave ballots, finds the kept
// rows of every tile before it by decoupled look-back (tiles taken in launch
// order from a counter, so every tile waited for is already running), and
// writes the kept ids at their selection positions (< cap; *total = all
// kept, written by the last tile).  kst[j] = kept rows before candidate j,
// for j an owner's first candidate (the owner offsets, k_sv_sel_off).
constexpr int SEL_ITEMS = 8;
constexpr u32 SEL_TILE = SEL_THREADS * SEL_ITEMS;
constexpr u32 SEL_SPIN_MAX = 1u << 24;
__global__ __launch_bounds__(SEL_THREADS) void k_sv_sel_scan(StoreView st, u32 n_owners, u32 C,
                                                             const u32* __restrict__ cpos, const u64* __restrict__ first,
                                                             const u64* __restrict__ req, const u64* __restrict__ id,
                                                             u64 cap, u64* __restrict__ sel_id, u64* __restrict__ sel_key,
                                                             u32* __restrict__ kst, u64* __restrict__ status,
                                                             u32* __restrict__ tile_ctr, u32* __restrict__ total,
                                                             u32* __restrict__ err) {
  constexpr int NW = SEL_THREADS / 64;
  __shared__ u32 range[2];
  __shared__ u32 tile_s;
  __shared__ u32 wc[SEL_ITEMS][NW];
  __shared__ u64 excl_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) tile_s = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const u32 tile = tile_s;
  const u32 j0 = tile * SEL_TILE;
  const u32 j1 = min(C, j0 + SEL_TILE) - 1;
  if (threadIdx.x == 0) range[0] = cand_owner(cpos, 0, n_owners, j0);
  if (threadIdx.x == 1) range[1] = cand_owner(cpos, 0, n_owners, j1) + 1;
  __syncthreads();
  // the tile's owners' candidate starts staged in LDS: each candidate's owner
  // search runs there instead of as a chain of dependent global loads (a
  // tile spanning more owners than it has candidates searches in place)
  __shared__ u32 s_cpos[SEL_TILE + 1];
  const u32 r0 = range[0], nr = range[1] - range[0];
  const bool staged = nr <= SEL_TILE;
  if (staged)
    for (u32 x = threadIdx.x; x <= nr; x += SEL_THREADS) s_cpos[x] = cpos[r0 + x];
  __syncthreads();
  auto owner_of = [&](u32 j) -> u32 {
    if (!staged) return cand_owner(cpos, r0, range[1], j);
    u32 lo = 0, hi = nr;  // invariant: s_cpos[lo] <= j < s_cpos[hi]
    while (lo + 1 < hi) {
      const u32 mid = (lo + hi) >> 1;
      if (s_cpos[mid] <= j) lo = mid;
      else hi = mid;
    }
    return r0 + lo;
  };
  auto start_of = [&](u32 o) -> u32 { return staged ? s_cpos[o - r0] : cpos[o]; };
  const u64 lt = lanemask_lt();
  u32 own[SEL_ITEMS], rk[SEL_ITEMS];
  u64 kk[SEL_ITEMS];
  u32 keepm = 0;
#pragma unroll
  for (int r = 0; r < SEL_ITEMS; ++r) {
    const u32 j = j0 + r * SEL_THREADS + threadIdx.x;
    bool keep = false;
    own[r] = 0;
    kk[r] = 0;
    if (j <= j1) {
      const u32 o = owner_of(j);
      const size_t k = first[o] + (j - start_of(o));
      own[r] = o;
      kk[r] = k;
      keep = node_hex_of(st.hi[k], st.lo[k]) != req[o];
    }
    const u64 b = __ballot(keep);
    rk[r] = (u32)__popcll(b & lt);
    if (lane == 0) wc[r][w] = (u32)__popcll(b);
    keepm |= keep ? 1u << r : 0u;
  }
  __syncthreads();
  u32 before[SEL_ITEMS], tsum = 0;  // kept rows of this tile before (round r, wave w)
#pragma unroll
  for (int r = 0; r < SEL_ITEMS; ++r) {
    u32 b = tsum;
    for (int x = 0; x < NW; ++x) {
      if (x < w) b += wc[r][x];
      tsum += wc[r][x];
    }
    before[r] = b;
  }
  if (threadIdx.x < 64) {  // wave 0: publish, look back 64 tiles per step, publish the prefix
    u64* my = status + tile;
    if (threadIdx.x == 0)
      __hip_atomic_store(my, (tile == 0 ? LB_PRE : LB_AGG) | (u64)tsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u64 excl = tile ? lookback_wave(status, tile, LbAdd<u64>(), SEL_SPIN_MAX, err) : 0ull;
    if (threadIdx.x == 0) {
      if (tile) __hip_atomic_store(my, LB_PRE | (excl + tsum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      excl_s = excl;
      if (j1 == C - 1) *total = (u32)(excl + tsum);
    }
  }
  __syncthreads();
  const u64 excl = excl_s;
#pragma unroll
  for (int r = 0; r < SEL_ITEMS; ++r) {
    const u32 j = j0 + r * SEL_THREADS + threadIdx.x;
    if (j > j1) continue;
    const u64 q = excl + before[r] + rk[r];
    if (j == start_of(own[r])) kst[j] = (u32)q;  // the owner's first candidate: its selection offset
    if (!((keepm >> r) & 1u) || q >= cap) continue;
    const size_t k = kk[r];
    sel_id[q] = id[k];
    if (sel_key) {
      sel_key[3 * q] = st.tc[k];
      sel_key[3 * q + 1] = st.hi[k];
      sel_key[3 * q + 2] = st.lo[k];
    }
  }
}

// Per-owner selection offsets: sel_off[o] = kept candidates before owner o.
__global__ void k_sv_sel_off(u32 n_owners, u32 C, const u32* __restrict__ cpos, const u32* __restrict__ kpos,
                             const u32* __restrict__ ktot, u64* __restrict__ sel_off) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o <= n_owners; o += gridDim.x * blockDim.x) {
    const u32 c = cpos[o];
    sel_off[o] = kpos ? (c < C ? kpos[c] : *ktot) : c;
  }
}

StoreView view_of(const evm_store* s) { return StoreView{s->off, s->owner, s->tc, s->hi, s->lo}; }

int store_alloc(evm_ctx* ctx, evm_store* s, u32 n_owners, uint64_t n) {
  s->n_owners = n_owners;
  s->n = n;
  const size_t m = std::max<uint64_t>(n, 1);
  // one stream-ordered allocation per store (arrays 256-B aligned inside it;
  // s->off is its base)
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_off = up(sizeof(u64) * (n_owners + 1)), b4 = up(sizeof(u32) * m), b8 = up(sizeof(u64) * m);
  size_t bytes = b_off + 2 * b4 + 3 * b8;
  char* base = static_cast<char*>(block_alloc(ctx, &bytes));
  if (!base) return EVM_ENOMEM;
  s->bytes = bytes;
  s->off = reinterpret_cast<unsigned long long*>(base);
  s->owner = reinterpret_cast<u32*>(base + b_off);
  s->lo = reinterpret_cast<u32*>(base + b_off + b4);
  s->tc = reinterpret_cast<unsigned long long*>(base + b_off + 2 * b4);
  s->hi = reinterpret_cast<unsigned long long*>(base + b_off + 2 * b4 + b8);
  s->id = reinterpret_cast<unsigned long long*>(base + b_off + 2 * b4 + 2 * b8);
  return EVM_OK;
}

void store_release_arrays(evm_ctx* ctx, evm_store* s) {
  if (s->off) block_free(ctx, s->off, s->bytes);  // the base of the store's one block
  s->off = nullptr;
  s->owner = nullptr;
  s->tc = s->hi = s->id = nullptr;
  s->lo = nullptr;
}

// ------------------------------------------- key-range segments (big owners)
constexpr u32 SEG_TARGET = 560;  // messages per segment of a cut owner: minute-granular splitters and
                                            // sampling noise keep nearly all below 1,024 (the fast kernel)
static_assert(SEG_TARGET >= 64 && SEG_TARGET <= 4096, "segment target");
constexpr u32 SEG_SPLIT_MIN = 1024; // shares above this are cut (the 1,024 kernel is the fast one)
static u32 seg_target() { return SEG_TARGET; }
constexpr u32 SAMPLE_STRIDE = 16;   // one sampled minute per 16 messages of a cut owner
constexpr u32 SEG_TABLE_RATIO = 64; // minute -> segment table when the splitters span <= 64 minutes per segment

__device__ __forceinline__ u32 upper_u32(const u32* a, u32 n, u32 x) {  // first k with a[k] > x
  u32 lo = 0, hi = n;
  while (lo < hi) {
    const u32 mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// per owner: segments (1 unless the share exceeds SVO_CAP), samples, splitters
__global__ void k_seg_plan(const u64* __restrict__ seg, u32 O, u32 target, u32* __restrict__ nb, u32* __restrict__ ns,
                           u32* __restrict__ nsp) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < O; o += gridDim.x * blockDim.x) {
    const u64 m = seg[o + 1] - seg[o];
    const bool big = m > SEG_SPLIT_MIN;
    const u32 b = big ? (u32)((m + target - 1) / target) : 1u;
    nb[o] = b;
    ns[o] = big ? (u32)((m + SAMPLE_STRIDE - 1) / SAMPLE_STRIDE) : 0u;
    nsp[o] = b - 1;
  }
}

// sample q of owner o: the minute of its share's message at j * SAMPLE_STRIDE
// (share in batch order: a spread-out sample); key (owner, minute - gmin)
__device__ __forceinline__ u32 minute_of(const evm_rec* rec, const u32* minute, size_t i) {
  return minute ? minute[i] : rec[i].minute;
}

__global__ void k_seg_sample(const evm_rec* __restrict__ rec, const u32* __restrict__ minute,
                             const u32* __restrict__ perm, const u64* __restrict__ seg,
                             const u32* __restrict__ soff, u32 O, u32 nsamp, u32 gmin, int mb,
                             u64* __restrict__ key, u32* __restrict__ val) {
  for (u32 q = blockIdx.x * blockDim.x + threadIdx.x; q < nsamp; q += gridDim.x * blockDim.x) {
    const u32 o = upper_u32(soff, O + 1, q) - 1;
    const u64 p = seg[o] + (u64)(q - soff[o]) * SAMPLE_STRIDE;
    const u32 mnt = minute_of(rec, minute, perm[p]);
    key[q] = ((u64)o << mb) | (u64)(mnt - gmin);
    val[q] = q;
  }
}

// splitter k (1 .. nb-1) of owner o: the sorted sample at rank k * ns / nb
__global__ void k_seg_split(const u64* __restrict__ skey, const u32* __restrict__ soff, const u32* __restrict__ spoff,
                            const u32* __restrict__ bbase, u32 O, u32 nsp, u32 gmin, int mb, u32* __restrict__ sp) {
  const u64 mask = (1ull << mb) - 1;
  for (u32 q = blockIdx.x * blockDim.x + threadIdx.x; q < nsp; q += gridDim.x * blockDim.x) {
    const u32 o = upper_u32(spoff, O + 1, q) - 1;
    const u32 k = q - spoff[o] + 1;
    const u64 nso = soff[o + 1] - soff[o], nbo = bbase[o + 1] - bbase[o];
    if (!nso) {  // no sample: one segment takes everything (if it overflows, the owner takes the sort path)
      sp[q] = 0xffffffffu;
      continue;
    }
    const u64 r = soff[o] + (u64)k * nso / nbo;
    sp[q] = (u32)(skey[r] & mask) + gmin;
  }
}

// per cut owner: the length of its minute -> segment table (the minutes from
// its first to its last splitter), 0 when that span is too wide (search)
__global__ void k_seg_tlen(const u32* __restrict__ spoff, const u32* __restrict__ sp, u32 O, u32* __restrict__ tlen) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < O; o += gridDim.x * blockDim.x) {
    const u32 a = spoff[o], k = spoff[o + 1] - a;
    u32 len = 0;
    if (k) {
      const u64 span = (u64)sp[a + k - 1] - sp[a] + 1;
      len = span <= (u64)SEG_TABLE_RATIO * (k + 1) ? (u32)span : 0u;
    }
    tlen[o] = len;
  }
}

// table entry q of owner o: the segment (splitters <= minute) of minute sp_first + j
__global__ void k_seg_table(const u32* __restrict__ spoff, const u32* __restrict__ sp, const u32* __restrict__ toff,
                            u32 O, u32 ntab, u32* __restrict__ tab) {
  for (u32 q = blockIdx.x * blockDim.x + threadIdx.x; q < ntab; q += gridDim.x * blockDim.x) {
    const u32 o = upper_u32(toff, O + 1, q) - 1;
    const u32 a = spoff[o], k = spoff[o + 1] - a;
    tab[q] = upper_u32(sp + a, k, sp[a] + (q - toff[o]));
  }
}

// Per owner, everything a message's segment lookup needs in one 32-B record
// (first segment, segment count, splitter offset, table offset and length,
// first splitter): one dependent load instead of six.
struct alignas(16) SegOwn {
  u32 b0, nbo, a, t0, tl, first, pad0, pad1;
};
__global__ void k_seg_own(const u32* __restrict__ bbase, const u32* __restrict__ spoff, const u32* __restrict__ sp,
                          const u32* __restrict__ toff, u32 O, SegOwn* __restrict__ own) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < O; o += gridDim.x * blockDim.x) {
    SegOwn r;
    r.b0 = bbase[o];
    r.nbo = bbase[o + 1] - r.b0;
    r.a = spoff[o];
    r.t0 = toff[o];
    r.tl = toff[o + 1] - r.t0;
    r.first = r.nbo > 1 ? sp[r.a] : 0u;
    r.pad0 = r.pad1 = 0;
    own[o] = r;
  }
}

// every message's segment: the owner's first, plus the splitters <= its minute.
// Four messages per thread, their lookups (owner record -> table) interleaved
// so the L2 round trips overlap; the batch index is not written (the segment
// sort's first pass makes the identity values).
constexpr int SK_ITEMS = 4;  // (8: 1.43 ms, 2: 1.50, 4: 1.45 on the config-5 shape -- the lookups are not the limit)
// Where a message's minute comes from: the compact minutes / packed records,
// the timestamp row's first 16 bytes (minute16), or a received record's tc.
struct MinuteSrc {
  const evm_rec* rec;
  const u32* minute;
  const uint8_t* ts;  // rows (16-B aligned, stride % 16 == 0), or null
  size_t stride;
  WireSrc wire;               // wire.rec != null: received records
};
__device__ __forceinline__ u32 minute_at(const MinuteSrc& m, size_t i) {
  if (m.ts) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(m.ts + i * m.stride));
    return minute16(v.x, v.y, v.z, v.w);
  }
  if (m.wire.rec || m.wire.tn) {
    u64 tc, node;
    u32 cm;
    wire_load(m.wire, i, &tc, &node, &cm);
    return (u32)((tc >> 16) / 60000ull);
  }
  return minute_of(m.rec, m.minute, i);
}
// (an owner >= O -- the batch is refused -- gets key NS, after every segment)
__global__ __launch_bounds__(256) void k_seg_key(MinuteSrc msrc, const u32* __restrict__ owner, size_t n, u32 O,
                                                 u32 NS, const SegOwn* __restrict__ own, const u32* __restrict__ sp,
                                                 const u32* __restrict__ tab, u32* __restrict__ key,
                                                 Info* __restrict__ info) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * SK_ITEMS;
  bool bad = false;
  for (size_t i0 = (size_t)blockIdx.x * blockDim.x * SK_ITEMS + threadIdx.x; i0 < n; i0 += stride) {
    u32 o[SK_ITEMS], mnt[SK_ITEMS], k[SK_ITEMS];
    SegOwn r[SK_ITEMS];
#pragma unroll
    for (int j = 0; j < SK_ITEMS; ++j) {
      const size_t i = i0 + (size_t)j * blockDim.x;
      o[j] = i < n ? owner[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < SK_ITEMS; ++j) {
      const bool ok = o[j] < O;
      bad |= !ok;
      r[j] = own[ok ? o[j] : 0u];
      if (!ok) r[j].b0 = NS, r[j].nbo = 1;
    }
    // only a message of a cut owner needs its minute: the rows of the rest
    // (an owner of one segment -- most owners of a Zipf stream) are not read
#pragma unroll
    for (int j = 0; j < SK_ITEMS; ++j) {
      const size_t i = i0 + (size_t)j * blockDim.x;
      mnt[j] = i < n && r[j].nbo > 1 ? minute_at(msrc, i) : 0u;
    }
#pragma unroll
    for (int j = 0; j < SK_ITEMS; ++j) {
      k[j] = r[j].b0;
      if (r[j].nbo > 1) {
        if (r[j].tl) {
          const u32 d = mnt[j] - r[j].first;
          k[j] += mnt[j] < r[j].first ? 0u : d >= r[j].tl ? r[j].nbo - 1 : tab[r[j].t0 + d];
        } else {
          k[j] += upper_u32(sp + r[j].a, r[j].nbo - 1, mnt[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < SK_ITEMS; ++j) {
      const size_t i = i0 + (size_t)j * blockDim.x;
      if (i < n) key[i] = k[j];
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomic_or_if(&info->bad_aux, 1u);
}

// The fused plan's samples (no minutes pass): every 16th message's minute
// straight from its row / record, the sampled minute range, and the owner
// check of the sampled rows.  mm = {min, max} (k_seg_key checks every owner).
__global__ __launch_bounds__(256) void k_seg_smin(MinuteSrc msrc, const u32* __restrict__ owner, size_t n, u32 O, u32* __restrict__ smin,
                           u32* __restrict__ mm, Info* __restrict__ info) {
  const size_t nq = (n + SAMPLE_STRIDE - 1) / SAMPLE_STRIDE;
  u32 mn = 0xffffffffu, mx = 0u, bad = 0u;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (size_t)gridDim.x * blockDim.x) {
    const size_t i = q * SAMPLE_STRIDE;
    const u32 m = minute_at(msrc, i);
    smin[q] = m;
    mn = min(mn, m);
    mx = max(mx, m);
    bad |= owner[i] >= O ? 1u : 0u;
  }
  // (one conditional global update per workgroup: same-address atomics from
  // every wave serialise at the memory side)
  block_fold_bounds<u32, 256>(mn, mx, bad, &mm[0], &mm[1], &info->bad_aux);
}

__global__ void k_seg_start(const u32* __restrict__ skey, size_t n, u32 NS, u64* __restrict__ start) {
  for (u32 b = blockIdx.x * blockDim.x + threadIdx.x; b <= NS; b += gridDim.x * blockDim.x) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
      const size_t mid = (lo + hi) >> 1;
      if (skey[mid] < b) lo = mid + 1;
      else hi = mid;
    }
    start[b] = lo;
  }
}

// every 16th batch position: (owner, minute - gmin) (mb = 0: owner only)
// (smin: the samples' minutes by sample index, from k_seg_smin)
__global__ void k_seg_sample_all(const evm_rec* __restrict__ rec, const u32* __restrict__ minute,
                                 const u32* __restrict__ owner, size_t n, u32 gmin, int mb, u64* __restrict__ key,
                                 u32* __restrict__ val, const u32* __restrict__ smin) {
  const size_t nq = (n + SAMPLE_STRIDE - 1) / SAMPLE_STRIDE;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (size_t)gridDim.x * blockDim.x) {
    const size_t i = q * SAMPLE_STRIDE;
    u64 k = (u64)owner[i] << mb;
    if (mb) k |= (u64)((smin ? smin[q] : minute_of(rec, minute, i)) - gmin);
    key[q] = k;
    val[q] = (u32)q;
  }
}

// segments per owner from its sample count (share ~ 16 x samples)
__global__ void k_seg_plan_est(const u32* __restrict__ soff, u32 O, int cut, u32 target, u32* __restrict__ nb,
                               u32* __restrict__ nsp) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < O; o += gridDim.x * blockDim.x) {
    const u64 est = (u64)(soff[o + 1] - soff[o]) * SAMPLE_STRIDE;
    // (estimates above 3/4 of the split size are cut too: a share estimated low
    // would otherwise exceed 1,024 and take the slower SVO_CAP kernel)
    const u32 b = cut && est > SEG_SPLIT_MIN * 3 / 4 ? (u32)((est + target - 1) / target) : 1u;
    nb[o] = b;
    nsp[o] = b - 1;
  }
}

// per owner: its samples' range in the sorted sample keys
__global__ void k_seg_soff(const u64* __restrict__ skey, u32 nsamp, u32 O, int mb, u32* __restrict__ soff) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o <= O; o += gridDim.x * blockDim.x) {
    const u64 x = (u64)o << mb;
    u32 lo = 0, hi = nsamp;
    while (lo < hi) {
      const u32 mid = (lo + hi) >> 1;
      if (skey[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    soff[o] = lo;
  }
}

__global__ void k_widen(const u32* __restrict__ a, size_t n, u64* __restrict__ b) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// segment b's owner and the first stored row / tree leaf of its minute range
__global__ void k_seg_ranges(const u32* __restrict__ bbase, const u32* __restrict__ spoff, const u32* __restrict__ sp,
                             u32 O, u32 NS, StoreView st, const u64* __restrict__ t_off, const u64* __restrict__ t_end,
                             const u64* __restrict__ t_ck, u32* __restrict__ sowner, u64* __restrict__ sa,
                             u64* __restrict__ la) {
  for (u32 b = blockIdx.x * blockDim.x + threadIdx.x; b < NS; b += gridDim.x * blockDim.x) {
    const u32 o = upper_u32(bbase, O + 1, b) - 1;
    const u32 k = b - bbase[o];
    sowner[b] = o;
    u64 r0 = st.off[o], l0 = t_off[o];
    if (k) {
      const u32 mlo = sp[spoff[o] + k - 1];
      const u64 tc0 = ((u64)mlo * 60000ull) << 16;  // rows with minute >= mlo: tc >= this
      u64 hi = st.off[o + 1];
      while (r0 < hi) {
        const u64 mid = (r0 + hi) >> 1;
        if (st.tc[mid] < tc0) r0 = mid + 1;
        else hi = mid;
      }
      l0 = lb_u64(t_ck, l0, t_end[o], ((u64)o << 40) | minute_code(mlo));
    }
    sa[b] = r0;
    la[b] = l0;
  }
}

__global__ void k_seg_ends(const u32* __restrict__ sowner, u32 NS, StoreView st, const u64* __restrict__ t_end,
                           const u64* __restrict__ sa, const u64* __restrict__ la, u64* __restrict__ sb,
                           u64* __restrict__ lb) {
  for (u32 b = blockIdx.x * blockDim.x + threadIdx.x; b < NS; b += gridDim.x * blockDim.x) {
    const u32 o = sowner[b];
    const bool next = b + 1 < NS && sowner[b + 1] == o;
    sb[b] = next ? sa[b + 1] : st.off[o + 1];
    lb[b] = next ? la[b + 1] : t_end[o];
  }
}

static int base3_len_host(uint32_t m) {
  int L = 1;
  uint64_t p = 3;
  while (L < CODE_DIGITS && (uint64_t)m >= p) {
    p *= 3;
    ++L;
  }
  return L;
}

// K5 driver.  On success *done = true and (*ns, *new_tree) hold the new store
// arrays and tree; *done = false (status OK) when some owner's share exceeds
// SVO_CAP or mixes key lengths: the caller takes the global sort path with
// the same packed records.  Validity of the batch is checked here (one host
// round trip for the whole ingest).
// Received route records -> packed records (REC) and / or the compact
// minutes, with the pack's checks: the local owner in range (bad_aux), the
// native domain (bad), the minute range.  aux = the local owner.
template <bool REC>
__global__ __launch_bounds__(256) void k_wire_pack(WireSrc w, size_t n, const u32* __restrict__ owner, u32 limit,
                                                   evm_rec* __restrict__ out, Info* __restrict__ info,
                                                   u32* __restrict__ minute_out) {
  u32 bad = 0, bad_aux = 0, mn = 0xffffffffu, mx = 0u;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    u64 tc, node;
    u32 cm;
    wire_load(w, i, &tc, &node, &cm);
    const u32 o = owner[i];
    const u32 minute = (u32)((tc >> 16) / 60000ull);
    bad_aux |= o >= limit ? 1u : 0u;
    if (REC) {
      u32 ww[12];
      format_ts46(tc, node, cm & EVM_META_CASEMASK, ww);
      evm_rec r;
      r.tc = tc;
      r.node = node;
      r.meta = cm;
      r.hash = (cm & EVM_META_VALID) ? murmur3_46(ww) : 0u;
      r.minute = minute;
      r.aux = o;
      out[i] = r;
    }
    if (minute_out) minute_out[i] = minute;
    if (cm & EVM_META_VALID) {
      mn = min(mn, minute);
      mx = max(mx, minute);
    } else {
      bad = 1;
    }
  }
  bad = wave_max(bad);
  bad_aux = wave_max(bad_aux);
  mn = wave_min(mn);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) {
    if (bad) atomic_or_if(&info->bad, 1u);
    if (bad_aux) atomic_or_if(&info->bad_aux, 1u);
    if (mn != 0xffffffffu) {
      atomic_min_if(&info->minute_min, mn);
      atomic_max_if(&info->minute_max, mx);
    }
  }
}

int launch_wire_pack(evm_ctx* ctx, const WireSrc& w, size_t n, const u32* owner, u32 limit, evm_rec* out, Info* info,
                     u32* minute_out) {
  if (n == 0) return EVM_OK;
  if (out)
    KLAUNCH(k_wire_pack<true>, dim3(grid_for(n, 256, 8192)), dim3(256), w, n, owner, limit, out, info, minute_out);
  else
    KLAUNCH(k_wire_pack<false>, dim3(grid_for(n, 256, 8192)), dim3(256), w, n, owner, limit, out, info, minute_out);
  return hip_ok(hipGetLastError());
}

int ingest_by_owner(evm_ctx* ctx, Scratch& S, const evm_store* s, const evm_rec* rec, const u32* minute,
                    const u32* owner, size_t n, const u32* orig, uint64_t id_base, uint8_t* flags, Info* info, u32* perm,
                    evm_store* ns, evm_tree** new_tree, bool* done, uint8_t* bigmask, bool* big_only, const char* ts,
                    size_t stride, const std::function<int()>& pack_now, const WireSrc* wire) {
  // fused: the records are not packed yet; K5 parses the timestamp rows itself
  // unless a step needs records or minutes (then pack_now() packs them)
  bool fused = (bool)pack_now;
  auto unfuse = [&]() -> int {
    if (!fused) return EVM_OK;
    fused = false;
    return pack_now();
  };
  // the segment keys need only the minutes: 48-B rows get them (and the
  // pack's checks) without the 32-B records, which K5 then does not read
  bool have_min = false;
  auto minutes = [&]() -> int {
    if (!fused || have_min) return EVM_OK;
    if (wire) {
      have_min = true;
      return launch_wire_pack(ctx, *wire, n, owner, s->n_owners, nullptr, info, const_cast<u32*>(minute));
    }
    if (stride != 48) return unfuse();
    have_min = true;
    return launch_minutes(ctx, ts, n, owner, s->n_owners, info, const_cast<u32*>(minute));
  };
  *done = false;
  *big_only = false;
  const u32 O = s->n_owners;
  int st;
  // stable sort of the batch index by owner: each owner's share in batch order
  u64* seg = S.alloc<u64>((size_t)O + 1);
  SvoStatus* status = S.alloc<SvoStatus>(1);
  u64* n_tc = S.alloc<u64>(n);
  u64* n_hi = S.alloc<u64>(n);
  u32* n_lo = S.alloc<u32>(n);
  u64* n_id = S.alloc<u64>(n);
  u32* tot = S.alloc<u32>(2);
  uint8_t* ownbig = S.alloc<uint8_t>(O);
  if (!seg || !status || !n_tc || !n_hi || !n_lo || !n_id || !tot || !ownbig) return EVM_ENOMEM;
  const int obits = O > 1 ? 32 - __builtin_clz(O - 1) : 0;
  // requests arrive as runs of one owner (index.ts:224-248): sort the runs,
  // not the messages, when they are long enough
  const size_t n_rt = (n + RUN_TILE - 1) / RUN_TILE;
  const dim3 rgrid((unsigned)((n_rt + RUN_THREADS / 64 - 1) / (RUN_THREADS / 64)));
  u32* tcnt = S.alloc<u32>(n_rt);
  u32* toff = S.alloc<u32>(n_rt);
  u32* nrun = S.alloc<u32>(1);
  if (!tcnt || !toff || !nrun) return EVM_ENOMEM;
  KLAUNCH(k_run_count, rgrid, dim3(RUN_THREADS), owner, n, tcnt);
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, tcnt, n_rt, toff, nrun))) return st;
  u32 R = 0;
  {
    LandList l;
    l.add(nrun, &R, sizeof(u32));
    if ((st = land_words(ctx, l))) return st;
  }
  u32* ov = perm;
  const bool runs = (size_t)R * 8 <= n;
  const evm_tree* t = s->tree;
  Info hi;
  auto check_landed = [&]() -> int {  // (hi already read)
    int e;
    if (hi.bad_aux) return EVM_EINVAL;
    if (hi.bad) {
      if ((e = unfuse())) return e;  // the culprits are flagged from packed records
      KLAUNCH(k_sv_bad, dim3(grid_for(n, 256)), dim3(256), rec, n, flags, orig);
      (void)evm_sync(ctx);
      return EVM_ENONCANON;
    }
    return EVM_OK;
  };
  auto check_info = [&]() -> int {
    int e = read_info(ctx, info, &hi);
    if (e) return e;
    if (hi.bad_aux) return EVM_EINVAL;
    if (hi.bad) {
      if ((e = unfuse())) return e;  // the culprits are flagged from packed records
      KLAUNCH(k_sv_bad, dim3(grid_for(n, 256)), dim3(256), rec, n, flags, orig);
      (void)evm_sync(ctx);
      return EVM_ENONCANON;
    }
    return EVM_OK;
  };
  // a batch's minutes all have one base-3 key length: code order = minute
  // order, so an owner can be cut at minutes (else no owner is cut)
  auto cuttable = [&]() {
    return ctx->server_path != 3 && hi.minute_min <= hi.minute_max &&
           base3_len_host(hi.minute_min) == base3_len_host(hi.minute_max);
  };
  u32* nb = S.alloc<u32>((size_t)O + 1);
  u32* nsm = S.alloc<u32>((size_t)O + 1);
  u32* nsp = S.alloc<u32>((size_t)O + 1);
  u32* bbase = S.alloc<u32>((size_t)O + 1);
  u32* soff = S.alloc<u32>((size_t)O + 1);
  u32* spoff = S.alloc<u32>((size_t)O + 1);
  if (!nb || !nsm || !nsp || !bbase || !soff || !spoff) return EVM_ENOMEM;
  SegView sv{nullptr, seg, s->off, s->off + 1, t->off, t->end};  // (a gapped tree: its owners' ranges as they lie)
  u32 NS = O;
  const u32* kperm = ov;  // batch indices, segment by segment
  bool split = false;
  u64* skey = nullptr;   // sorted samples: owner << mb | minute - gmin
  // interleaved owners with K5 parsing the rows / records itself: the plan
  // reads the minutes from them directly (no minutes pass)
  const bool seg_fused = fused && (wire || (stride % 16 == 0 && ((uintptr_t)ts & 15) == 0));
  u32* smin = nullptr;   // the samples' minutes (seg_fused)
  MinuteSrc msrc{rec, minute, nullptr, 0, WireSrc{nullptr, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr}};
  if (seg_fused) {
    if (wire) msrc.wire = *wire;
    else {
      msrc.ts = reinterpret_cast<const uint8_t*>(ts);
      msrc.stride = stride;
    }
  }
  u32 gmin = 0;
  int mb = 1;
  u32 nspl = 0;
  if (runs) {
    // requests arrive as runs of one owner (index.ts:224-248): sort the runs, not the messages
    u32* run_start = S.alloc<u32>(R);
    u32* run_owner = S.alloc<u32>(R);
    u32* order = S.alloc<u32>(R);
    u32* len = S.alloc<u32>(R);
    u32* run_pos = S.alloc<u32>((size_t)R + 1);
    if (!run_start || !run_owner || !order || !len || !run_pos) return EVM_ENOMEM;
    KLAUNCH(k_run_emit, rgrid, dim3(RUN_THREADS), owner, n, toff, run_start, run_owner);
    if ((st = launch_iota(ctx, order, R))) return st;
    u32* rk = run_owner;
    u32* rv = order;
    if ((st = radix_sort_pairs<u32>(ctx, S, rk, rv, R, 0, obits))) return st;
    KLAUNCH(k_run_len, dim3(grid_for(R, 256)), dim3(256), run_start, rv, R, n, len);
    if ((st = scan_exclusive<u32, OpAdd>(ctx, S, len, R, run_pos, run_pos + R))) return st;
    u32* cbase = S.alloc<u32>(std::max<u32>(O, 1));
    u32* multi = S.alloc<u32>(1);
    if (!cbase || !multi) return EVM_ENOMEM;
    HIPR(hipMemsetAsync(multi, 0, sizeof(u32), ctx->stream));
    KLAUNCH(k_run_seg, dim3(grid_for((size_t)O + 1, 256)), dim3(256), rk, R, run_pos, O, seg, info,
            (const u32*)run_start, (const u32*)rv, cbase, multi);
    sv.cbase = cbase;
    // owners above SEG_SPLIT_MIN: key-range segments, splitters from every
    // 16th message of their share
    KLAUNCH(k_seg_plan, dim3(grid_for(O, 256)), dim3(256), seg, O, seg_target(), nb, nsm, nsp);
    {
      const u32* ins[3] = {nb, nsm, nsp};
      u32* outs[3] = {bbase, soff, spoff};
      u32* tots[3] = {bbase + O, soff + O, spoff + O};
      if ((st = scan_exclusive_cols(ctx, S, 3, ins, O, outs, tots))) return st;
    }
    u32 plan[4] = {0, 0, 0, 0};  // segments, samples, splitters, an owner of several runs
    {
      LandList l;
      l.add(bbase + O, &plan[0], sizeof(u32));
      l.add(soff + O, &plan[1], sizeof(u32));
      l.add(spoff + O, &plan[2], sizeof(u32));
      l.add(multi, &plan[3], sizeof(u32));
      l.add(info, &hi, sizeof(Info));  // (the status record too: no cut owner, no minutes pass)
      if ((st = land_words(ctx, l))) return st;
    }
    if (plan[1] > 0 && (st = minutes())) return st;  // cut owners: the splitters need the minutes
    if ((st = plan[1] > 0 ? check_info() : check_landed())) return st;
    split = plan[1] > 0 && cuttable();
    // the batch indices in owner order: read by the cut owners' sampling and
    // by K5 for owners of several runs; when every owner is one run (one
    // SyncRequest per owner, config 3) K5 indexes from the run starts and the
    // 4-B-per-message permutation is not written at all
    if (plan[3] || split)
      KLAUNCH(k_run_fill, dim3(grid_for(R, 4 * RF_RUNS, 1 << 16)), dim3(256), run_pos, run_start, rv, R, perm);
    if (split) {
      gmin = hi.minute_min;
      mb = std::max(1, ceil_log2((size_t)(hi.minute_max - gmin) + 1));
      NS = plan[0];
      nspl = plan[2];
      const u32 nsamp = plan[1];
      skey = S.alloc<u64>(nsamp);
      u32* sval = S.alloc<u32>(nsamp);
      if (!skey || !sval) return EVM_ENOMEM;
      KLAUNCH(k_seg_sample, dim3(grid_for(nsamp, 256)), dim3(256), rec, minute, ov, seg, soff, O, nsamp, gmin, mb, skey,
              sval);
      if ((st = radix_sort_pairs<u64>(ctx, S, skey, sval, nsamp, 0, mb + obits))) return st;
    }
  } else {
    // messages of many owners interleaved: plan from a sample of every 16th
    // batch position (each owner's share estimated as 16 x its samples; a
    // wrong estimate costs speed only -- an overfull segment sends its owner
    // to the sort path); then ONE sort of the batch by segment, which also
    // groups the owners (no separate owner sort)
    const u32 nq = (u32)((n + SAMPLE_STRIDE - 1) / SAMPLE_STRIDE);
    if (seg_fused) {
      // no minutes pass: the sampled rows' minutes give the range (the
      // segments' first / last splitters are open-ended, so a minute outside
      // it still lands in a segment; K5 reports the key lengths it saw)
      smin = S.alloc<u32>(nq);
      u32* mm = S.alloc<u32>(2);
      if (!smin || !mm) return EVM_ENOMEM;
      {
        ZeroList z;
        z.add(mm, sizeof(u32), 0xffffffffu);
        z.add(mm + 1, sizeof(u32));
        if ((st = zero_small(ctx, z))) return st;
      }
      KLAUNCH(k_seg_smin, dim3(grid_for(nq, 256)), dim3(256), msrc, owner, n, O, smin, mm, info);
      u32 hmm[2];
      HIPR(hipMemcpyAsync(hmm, mm, sizeof(hmm), hipMemcpyDeviceToHost, ctx->stream));
      if ((st = read_info(ctx, info, &hi))) return st;
      if (hi.bad_aux) return EVM_EINVAL;
      hi.minute_min = hmm[0];
      hi.minute_max = hmm[1];
    } else {
      if ((st = minutes())) return st;
      if ((st = check_info())) return st;
    }
    if (cuttable()) {
      gmin = hi.minute_min;
      mb = std::max(1, ceil_log2((size_t)(hi.minute_max - gmin) + 1));
    } else {
      gmin = 0;
      mb = 0;  // no minutes in the key: one segment per owner
    }
    skey = S.alloc<u64>(nq);
    u32* sval = S.alloc<u32>(nq);
    if (!skey || !sval) return EVM_ENOMEM;
    KLAUNCH(k_seg_sample_all, dim3(grid_for(nq, 256)), dim3(256), rec, minute, owner, n, gmin, mb, skey, sval,
            (const u32*)smin);
    if ((st = radix_sort_pairs<u64>(ctx, S, skey, sval, nq, 0, mb + obits))) return st;
    KLAUNCH(k_seg_soff, dim3(grid_for((size_t)O + 1, 256)), dim3(256), skey, nq, O, mb, soff);
    KLAUNCH(k_seg_plan_est, dim3(grid_for(O, 256)), dim3(256), soff, O, mb > 0 ? 1 : 0, seg_target(), nb, nsp);
    {
      const u32* ins[2] = {nb, nsp};
      u32* outs[2] = {bbase, spoff};
      u32* tots[2] = {bbase + O, spoff + O};
      if ((st = scan_exclusive_cols(ctx, S, 2, ins, O, outs, tots))) return st;
    }
    u32 plan[2] = {0, 0};
    {
      LandList l;
      l.add(bbase + O, &plan[0], sizeof(u32));
      l.add(spoff + O, &plan[1], sizeof(u32));
      if ((st = land_words(ctx, l))) return st;
    }
    split = true;  // (possibly one segment per owner)
    NS = plan[0];
    nspl = plan[1];
  }
  if (split) {
    u32* sp = S.alloc<u32>(std::max<u32>(nspl, 1));
    u32* bkey = S.alloc<u32>(n);
    u64* sstart = S.alloc<u64>((size_t)NS + 1);
    u32* sown = S.alloc<u32>(NS);
    u64* ssa = S.alloc<u64>(NS);
    u64* ssb = S.alloc<u64>(NS);
    u64* sla = S.alloc<u64>(NS);
    u64* slb = S.alloc<u64>(NS);
    if (!sp || !bkey || !sstart || !sown || !ssa || !ssb || !sla || !slb) return EVM_ENOMEM;
    if (nspl)
      KLAUNCH(k_seg_split, dim3(grid_for(nspl, 256)), dim3(256), skey, soff, spoff, bbase, O, nspl, gmin, mb, sp);
    // minute -> segment tables of the cut owners (a lookup per message instead of a search)
    u32* tlen = S.alloc<u32>((size_t)O + 1);
    u32* tboff = S.alloc<u32>((size_t)O + 1);
    if (!tlen || !tboff) return EVM_ENOMEM;
    KLAUNCH(k_seg_tlen, dim3(grid_for(O, 256)), dim3(256), spoff, sp, O, tlen);
    if ((st = scan_exclusive<u32, OpAdd>(ctx, S, tlen, O, tboff, tboff + O))) return st;
    u32 ntab = 0;
    {
      LandList l;
      l.add(tboff + O, &ntab, sizeof(u32));
      if ((st = land_words(ctx, l))) return st;
    }
    u32* tab = S.alloc<u32>(std::max<u32>(ntab, 1));
    if (!tab) return EVM_ENOMEM;
    if (ntab) KLAUNCH(k_seg_table, dim3(grid_for(ntab, 256)), dim3(256), spoff, sp, tboff, O, ntab, tab);
    SegOwn* sown_rec = S.alloc<SegOwn>(std::max<u32>(O, 1));
    if (!sown_rec) return EVM_ENOMEM;
    KLAUNCH(k_seg_own, dim3(grid_for(O, 256)), dim3(256), bbase, spoff, sp, tboff, O, sown_rec);
    // (the minutes from the rows / records when the plan read them so, else the minutes array)
    MinuteSrc kms = msrc;
    if (!(seg_fused && !runs))
      kms = MinuteSrc{rec, minute, nullptr, 0, WireSrc{nullptr, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr}};
    KLAUNCH(k_seg_key, dim3(grid_for((n + SK_ITEMS - 1) / SK_ITEMS, 256)), dim3(256), kms, owner, n, O, NS,
            (const SegOwn*)sown_rec, sp, tab, bkey, info);
    u32* bk = bkey;
    u32* bv = nullptr;  // the batch index: the identity, made by the sort's first pass
    if ((st = radix_sort_pairs<u32>(ctx, S, bk, bv, n, 0, std::max(1, ceil_log2((size_t)NS + 1))))) return st;
    KLAUNCH(k_seg_start, dim3(grid_for((size_t)NS + 1, 256)), dim3(256), bk, n, NS, sstart);
    KLAUNCH(k_seg_ranges, dim3(grid_for(NS, 256)), dim3(256), bbase, spoff, sp, O, NS, view_of(s), (const u64*)t->off,
            (const u64*)t->end, (const u64*)t->ck, sown, ssa, sla);
    KLAUNCH(k_seg_ends, dim3(grid_for(NS, 256)), dim3(256), sown, NS, view_of(s), (const u64*)t->end, ssa, sla, ssb,
            slb);
    sv = SegView{sown, sstart, ssa, ssb, sla, slb};
    kperm = bv;
  }
  // K5's new leaves: segment s's at slots [start + s, start + s + m] (n + NS + 1 in all).
  // Into an empty store with one segment per owner they are the new tree
  // itself, gapped (evm_tree): each owner's leaves where K5 wrote them, with
  // its owner-local prefix XOR -- no copy pass (adopted below when every
  // message was inserted; otherwise k_svo_copy compacts them as before).
  const size_t n_slots = n + (size_t)NS + 1;
  evm_tree* gt = nullptr;
  struct GapGuard {
    evm_ctx* ctx;
    evm_tree*& t;
    ~GapGuard() {
      if (t) tree_destroy(ctx, t);
    }
  } gap_guard{ctx, gt};
  if (s->n == 0 && t->n_leaves == 0 && !split && (st = tree_alloc_gapped(ctx, O, n_slots, &gt))) return st;
  u64* l_ck = gt ? (u64*)gt->ck : S.alloc<u64>(n_slots);
  int32_t* l_xr = gt ? gt->xr : S.alloc<int32_t>(n_slots);
  uint8_t* l_dup = S.alloc<uint8_t>(n_slots);
  if (!l_ck || !l_xr || !l_dup) return EVM_ENOMEM;
  int32_t* l_pfx = gt ? gt->pfx : nullptr;
  u64* g_off = gt ? (u64*)gt->off : nullptr;
  u64* g_end = gt ? (u64*)gt->end : nullptr;
  u32* cnt = S.alloc<u32>(4 * (size_t)NS + 1);  // rows, new leaves, merged leaves, new leaves' XOR (per segment)
  u32* pos = S.alloc<u32>(2 * (size_t)NS);  // row / leaf offsets
  u32* mid = S.alloc<u32>((size_t)NS + 1);  // [count, segments whose share is in (1024, SVO_CAP]]
  if (!cnt || !pos || !mid) return EVM_ENOMEM;
  u32 *c_rows = cnt, *c_new = cnt + NS, *c_leaves = cnt + 2 * (size_t)NS, *c_xor = cnt + 3 * (size_t)NS;
  // an empty store (a new server, config 3): K5 writes its rows straight into
  // the new store's arrays at their batch positions -- if every message is
  // inserted that is the final layout and k_svo_b copies no row
  u32* n_owner = nullptr;
  evm_store pre{};
  if (s->n == 0) {
    if ((st = store_alloc(ctx, &pre, O, n))) {
      store_release_arrays(ctx, &pre);
      return st;
    }
    n_tc = pre.tc;
    n_hi = pre.hi;
    n_lo = pre.lo;
    n_id = pre.id;
    n_owner = pre.owner;
  }
  struct PreGuard {  // released on every path that does not adopt it
    evm_ctx* ctx;
    evm_store* p;
    ~PreGuard() { store_release_arrays(ctx, p); }
  } pre_guard{ctx, &pre};
  SvoStatus hs;
  u32 ht[2], hmid = 0;
  const int preset = orig ? 0 : 1;
  if (preset) HIPR(hipMemsetAsync(flags, EVM_MSG_INS, n, ctx->stream));
  {
    ZeroList z;
    z.add(status, sizeof(SvoStatus));
    z.add(mid, sizeof(u32));
    if ((st = zero_small(ctx, z))) return st;
  }
  HIPR(hipMemsetAsync(ownbig, 0, O, ctx->stream));
  // the common share size over every segment (more workgroups per CU); larger
  // shares are listed and take the SVO_CAP kernel over just those segments
  const uint8_t* tsb = reinterpret_cast<const uint8_t*>(ts);
  const WireSrc wsrc = wire ? *wire : WireSrc{nullptr, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr};
  // pass A over every segment with the capacity that fits the typical share
  // (small segments -- Zipf tails, cut owners -- take the 512 kernel: half the
  // per-workgroup fixed work, twice the occupancy); larger shares are listed
  // for the 1,024 and SVO_CAP passes
  const bool small = NS && n / NS < 400;
  const bool leaf = t->n_leaves > 0;
  const int skip_stored = ctx->test_fail == 2 ? 1 : 0;
  auto pass = [&](u32 cap, dim3 grid, const u32* list, u32* l1, u32* l2, u32* l512) {
#define SVO_ARGS                                                                                                      \
  rec, tsb, stride, info, kperm, sv, view_of(s), (const u64*)t->ck, (u64)id_base, flags, n_tc, n_hi, n_lo, n_id, l_ck, \
      l_xr, l_dup, c_rows, c_new, c_leaves, c_xor, status, orig, list, l2, l1, ownbig, n_owner, preset, l512, wsrc,  \
      skip_stored, l_pfx, g_off, g_end
    // (the one-wave kernels: Zipf-tail owners of <= 128 / <= 256 messages, no cross-wave barriers;
    // source: true = the rows, false = packed records, SRC_WIRE = received records)
// (the 1,024 kernel with 512 threads, two messages each, measured slower:
// config 3 2.80 vs 2.59 ms, config-5 shape 4.87 vs 4.04)
#define K5_1024(SRCV)                                                                             \
  do {                                                                                              \
    if (leaf) KLAUNCH((k_svo_a<1024, SRCV, SVO_THREADS, true>), grid, dim3(SVO_THREADS), SVO_ARGS); \
    else KLAUNCH((k_svo_a<1024, SRCV>), grid, dim3(SVO_THREADS), SVO_ARGS);                          \
  } while (0)
#define SVO_PASS(SRCV)                                                                         \
  if (cap == 128) KLAUNCH((k_svo_a<128, SRCV, 64>), grid, dim3(64), SVO_ARGS);                  \
  else if (cap == 256) KLAUNCH((k_svo_a<256, SRCV, 64>), grid, dim3(64), SVO_ARGS);             \
  else if (cap == 512) KLAUNCH((k_svo_a<512, SRCV>), grid, dim3(SVO_THREADS), SVO_ARGS);        \
  else if (cap == 1024) K5_1024(SRCV);                                                          \
  else if (cap == 2048) KLAUNCH((k_svo_a<2048, SRCV>), grid, dim3(SVO_THREADS), SVO_ARGS);      \
  else KLAUNCH((k_svo_a<SVO_CAP, SRCV>), grid, dim3(SVO_THREADS), SVO_ARGS);
    if (fused && wire) {
      SVO_PASS(SRC_WIRE)
    } else if (fused) {
      SVO_PASS(true)
    } else {
      SVO_PASS(false)
    }
#undef SVO_PASS
#undef K5_1024
#undef SVO_ARGS
  };
  if (small) {
    // small segments on average (Zipf tails and ~560-message cuts): segments
    // listed by size class first, then one pass per class over exactly its
    // segments (the one-wave kernel for <= 128 messages)
    u32* lists = S.alloc<u32>(SEG_CLASSES * ((size_t)NS + 1));
    if (!lists) return EVM_ENOMEM;
    {
      static_assert(SEG_CLASSES <= ZERO_MAX, "one launch");
      ZeroList z;
      for (int c = 0; c < SEG_CLASSES; ++c) z.add(lists + (size_t)c * (NS + 1), sizeof(u32));
      if ((st = zero_small(ctx, z))) return st;
    }
    KLAUNCH(k_seg_classes, dim3(grid_for(NS, 256)), dim3(256), sv, NS, lists);
    u32 hc[SEG_CLASSES];
    {
      LandList l;
      for (int c = 0; c < SEG_CLASSES; ++c) l.add(lists + (size_t)c * (NS + 1), &hc[c], sizeof(u32));
      if ((st = land_words(ctx, l))) return st;
    }
    const u32 caps[SEG_CLASSES] = {128, 256, 512, 1024, 2048, SVO_CAP};
    for (int c = 0; c < SEG_CLASSES; ++c)
      if (hc[c])
        pass(caps[c], dim3(hc[c]), (const u32*)(lists + (size_t)c * (NS + 1) + 1), (u32*)nullptr, (u32*)nullptr,
             (u32*)nullptr);
  } else {
    pass(1024, dim3(NS), (const u32*)nullptr, (u32*)nullptr, mid, (u32*)nullptr);
    HIPR(hipMemcpyAsync(&hmid, mid, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    if (hmid) pass(SVO_CAP, dim3(hmid), (const u32*)(mid + 1), (u32*)nullptr, (u32*)nullptr, (u32*)nullptr);
  }
  KLAUNCH(k_seg_fix, dim3(grid_for(NS, 256)), dim3(256), sv, NS, ownbig, c_rows, c_new, c_leaves, c_xor);
  {
    const u32* ins[2] = {c_rows, c_leaves};
    u32* outs[2] = {pos, pos + NS};
    u32* tots[2] = {tot, tot + 1};
    if ((st = scan_exclusive_cols(ctx, S, 2, ins, NS, outs, tots))) return st;
  }
  // the empty store's commit copies (k_svo_copy) and writes the prefix XOR itself
  const bool by_copy = s->n == 0 && t->n_leaves == 0;
  int32_t* xpos = nullptr;
  if (by_copy) {
    xpos = S.alloc<int32_t>((size_t)NS + 1);
    if (!xpos) return EVM_ENOMEM;
    if ((st = scan_exclusive<int32_t, OpXor>(ctx, S, (const int32_t*)c_xor, NS, xpos, xpos + NS))) return st;
  }
  {
    // K5's status, the totals and (fused) the parse's verdict in one landing
    static_assert(sizeof(SvoStatus) % 4 == 0, "words");
    LandList l;
    l.add(status, &hs, sizeof(hs));
    l.add(tot, ht, sizeof(ht));
    if (fused) l.add(info, &hi, sizeof(Info));
    if ((st = land_words(ctx, l))) return st;
  }
  if (fused) {
    // the parse's verdict: a row outside the native domain -> pack to flag the culprits
    if (hi.bad_aux) return EVM_EINVAL;  // (the fused plan checks every owner in k_seg_key)
    if (hi.bad) {
      if ((st = unfuse())) return st;
      KLAUNCH(k_sv_bad, dim3(grid_for(n, 256)), dim3(256), rec, n, flags, orig);
      (void)evm_sync(ctx);
      return EVM_ENONCANON;
    }
  }
  if (hs.fallback) return unfuse();  // the sort path redoes every flag (from packed records)
  // a plan from sampled minutes may have cut owners although the batch's
  // minutes have two key lengths (then code order != minute order across an
  // owner's segments): the sort path
  if (seg_fused && !runs && nspl && __builtin_popcount(hs.lens) > 1) return unfuse();
  if (hs.big && bigmask && (st = unfuse())) return st;  // the big owners' sub-batch reads packed records
  if (hs.big) {
    if (!bigmask) return EVM_OK;
    // only some owners are too big for LDS: the rest commit here (the big
    // ones contribute no rows or leaves), the caller sends the big owners'
    // messages through the sort path
    KLAUNCH(k_big_mask, dim3(grid_for(n, 256)), dim3(256), owner, n, ownbig, bigmask);
    *big_only = true;
  }
  // new store and tree, exactly sized
  const int in_place = (n_owner && ht[0] == n) ? 1 : 0;
  if (in_place && gt && !hs.big) {
    // every message inserted, one segment per owner: K5 left the final rows
    // (at their batch positions: the owner offsets are the segment starts)
    // and the final gapped tree -- nothing is copied
    *ns = pre;
    ns->n = n;
    pre = evm_store{};
    HIPR(hipMemcpyAsync(ns->off, seg, sizeof(u64) * ((size_t)O + 1), hipMemcpyDeviceToDevice, ctx->stream));
    gt->n_leaves = ht[1];
    *new_tree = gt;
    gt = nullptr;
    *done = true;
    return hip_ok(hipGetLastError());
  }
  if (in_place) {
    *ns = pre;  // adopt the pre-allocated store (its rows are final)
    ns->n = n;
    pre = evm_store{};
  } else if ((st = store_alloc(ctx, ns, O, s->n + ht[0]))) {
    store_release_arrays(ctx, ns);
    return st;
  }
  evm_tree* nt = nullptr;
  if ((st = tree_alloc_cap(ctx, O, ht[1], &nt))) {
    store_release_arrays(ctx, ns);
    return st;
  }
  const StoreOut so{ns->owner, ns->tc, ns->hi, ns->lo, ns->id};
  u32* merr = nullptr;  // the merge's invariant checks (k_svo_b)
  if (!by_copy) {
    merr = S.alloc<u32>(1);
    if (!merr) {
      store_release_arrays(ctx, ns);
      tree_destroy(ctx, nt);
      return EVM_ENOMEM;
    }
    HIPR(hipMemsetAsync(merr, 0, sizeof(u32), ctx->stream));
  }
  if (s->n)
    // (fewer merge workgroups per CU -- an LDS pad of 40/80 KB -- made the
    // merge 19 %/100 % slower: its write traffic is not an L2 capacity effect)
    KLAUNCH(k_svo_b<true>, dim3(NS), dim3(SVO_THREADS), sv, NS, O, view_of(s),
                (const u64*)s->id, n_tc, n_hi, n_lo, n_id, c_rows, pos, (const u64*)t->ck, t->xr, l_ck, l_xr, l_dup,
                c_new, pos + NS, so, ns->off, nt->ck, nt->xr, nt->off, in_place, merr);
  else if (by_copy && NS == 0)
    HIPR(hipMemsetAsync(nt->pfx, 0, sizeof(int32_t), ctx->stream));
  else if (by_copy)
    KLAUNCH(k_svo_copy, dim3((NS + SVC_WAVES - 1) / SVC_WAVES), dim3(64 * SVC_WAVES), sv, NS, O, n_tc, n_hi, n_lo, n_id,
            c_rows, pos, l_ck, l_xr, c_new, pos + NS, so, ns->off, nt->ck, nt->xr, nt->off, in_place, xpos, nt->pfx);
  else
    KLAUNCH(k_svo_b<false>, dim3(NS), dim3(SVO_THREADS), sv, NS, O, view_of(s), (const u64*)s->id, n_tc, n_hi, n_lo, n_id,
          c_rows, pos, (const u64*)t->ck, t->xr, l_ck, l_xr, l_dup, c_new, pos + NS, so, ns->off, nt->ck, nt->xr,
          nt->off, in_place, merr);
  // (the prefix XOR inside the merge -- segments by decoupled look-back, each
  // re-reading its own leaves -- measured 1.88 vs 0.79 + 0.39 ms of scans on
  // config 3: the merge's workgroups then wait on each other)
  if (!by_copy && (st = scan_exclusive<int32_t, OpXor>(ctx, S, nt->xr, ht[1], nt->pfx, nt->pfx + ht[1]))) {
    store_release_arrays(ctx, ns);
    tree_destroy(ctx, nt);
    return st;
  }
  if (merr) {
    u32 herr = 0;
    st = hip_ok(hipMemcpyAsync(&herr, merr, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    if (!st) st = hip_ok(hipStreamSynchronize(ctx->stream));
    if (!st && herr) st = EVM_ESTATE;  // the store's invariants broke: nothing is committed
    if (st) {
      store_release_arrays(ctx, ns);
      tree_destroy(ctx, nt);
      return st;
    }
  }
  *new_tree = nt;
  *done = true;
  return EVM_OK;
}

}  // namespace

extern "C" {

int evm_store_new(evm_ctx* ctx, uint32_t n_owners, evm_store** out) {
  if (!ctx || !out) return EVM_EINVAL;
  evm_store* s = new evm_store();
  int st = store_alloc(ctx, s, n_owners, 0);
  if (!st) st = hip_ok(hipMemsetAsync(s->off, 0, sizeof(u64) * (n_owners + 1), ctx->stream));
  if (!st) st = evm_tree_new(ctx, n_owners, &s->tree);
  if (st) {
    store_release_arrays(ctx, s);
    delete s;
    return st;
  }
  *out = s;
  return evm_sync(ctx);
}

int evm_store_free(evm_ctx* ctx, evm_store* s) {
  if (!ctx) return EVM_EINVAL;
  if (!s) return EVM_OK;
  store_release_arrays(ctx, s);
  if (s->tree) tree_destroy(ctx, s->tree);
  delete s;
  return EVM_OK;
}

int evm_store_info(const evm_store* s, uint32_t* n_owners, uint64_t* n_messages) {
  if (!s) return EVM_EINVAL;
  if (n_owners) *n_owners = s->n_owners;
  if (n_messages) *n_messages = s->n;
  return EVM_OK;
}

const evm_tree* evm_store_tree(const evm_store* s) { return s ? s->tree : nullptr; }

int evm_store_messages(evm_ctx* ctx, const evm_store* s, uint64_t* owner_off, uint64_t* id) {
  if (!ctx || !s) return EVM_EINVAL;
  if (owner_off)
    HIPR(hipMemcpyAsync(owner_off, s->off, sizeof(u64) * (s->n_owners + 1), hipMemcpyDeviceToHost, ctx->stream));
  if (id && s->n) HIPR(hipMemcpyAsync(id, s->id, sizeof(u64) * s->n, hipMemcpyDeviceToHost, ctx->stream));
  return evm_sync(ctx);
}

}  // extern "C"

// Swap in the new store arrays and tree.
static int commit_store(evm_ctx* ctx, evm_store* s, evm_store& ns, evm_tree* new_tree) {
  store_release_arrays(ctx, s);
  tree_destroy(ctx, s->tree);
  s->n = ns.n;
  s->bytes = ns.bytes;
  s->off = ns.off;
  s->owner = ns.owner;
  s->tc = ns.tc;
  s->hi = ns.hi;
  s->lo = ns.lo;
  s->id = ns.id;
  s->tree = new_tree;
  return evm_sync(ctx);
}

// One ingest over the caller's batch, or over the sub-batch orig[0..n) of it
// (message k = the caller's message orig[k], its packed record prec[orig[k]];
// flags and ids refer to the caller's indices).
// mode 0: per-owner LDS path; when only some owners are too big for it, the
// rest commit and the big owners' messages then go through the sort path --
// owners are independent, so the result is the one of a single ingest;
// mode 2: the sort path.
static int ingest_impl(evm_ctx* ctx, evm_store* s, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                       const u32* orig, const evm_rec* prec, uint64_t id_base, uint8_t* flags, int mode,
                       const WireSrc* wire = nullptr) {
  if (orig && !prec) return EVM_EINVAL;
  int st;
  evm_store ns{};
  evm_tree* new_tree = nullptr;
  // an error return after the new arrays exist releases them (the store is untouched)
  struct Pending {
    evm_ctx* ctx;
    evm_store& ns;
    evm_tree*& t;
    bool armed = true;
    ~Pending() {
      if (!armed) return;
      store_release_arrays(ctx, &ns);
      if (t) tree_destroy(ctx, t);
    }
  } pending{ctx, ns, new_tree};
  {
    Scratch S(ctx);
    Info* info = nullptr;
    if ((st = new_info(ctx, S, &info))) return st;
    evm_rec* rec = S.alloc<evm_rec>(n);
    u32* perm = S.alloc<u32>(n);
    u64* fv = S.alloc<u64>(n);
    FieldRange* fr = S.alloc<FieldRange>(1);
    if (!rec || !perm || !fv || !fr) return EVM_ENOMEM;
    const u32* own = owner;
    // a sub-batch reads the caller's packed (and checked) records through
    // orig; its own copy is made only for the paths that index it directly
    bool have_rec = false;
    u32* own_sub = orig ? S.alloc<u32>(n) : nullptr;
    if (orig && !own_sub) return EVM_ENOMEM;
    auto materialize = [&]() {
      if (!have_rec && orig) {
        KLAUNCH(k_sv_rec_sel, dim3(grid_for(n, 256, 8192)), dim3(256), prec, orig, n, rec, own_sub);
        own = own_sub;
        have_rec = true;
      }
    };
    u32* minute = nullptr;  // compact minutes (segment keys); a sub-batch reads them from the records
    // the per-owner path parses 16-B aligned rows itself; the records are
    // packed only when a step needs them (cut owners, sort path, culprits)
    // (received route records: K5 reads them where they lie)
    const bool defer = !orig && mode == 0 && s->n_owners > 0 && ctx->server_path != 3 && ctx->server_path != 4 &&
                       (wire || (stride >= 48 && stride % 16 == 0 && ((uintptr_t)ts & 15) == 0));
    std::function<int()> pack_now;
    if (!orig) {
      minute = S.alloc<u32>(n);
      if (!minute) return EVM_ENOMEM;
      auto do_pack = [&, minute]() -> int {
        int e = wire ? launch_wire_pack(ctx, *wire, n, owner, s->n_owners, rec, info, minute)
                     : launch_pack(ctx, ts, stride, n, owner, s->n_owners, rec, info, minute);
        if (!e) have_rec = true;
        return e;
      };
      if (defer) {
        pack_now = do_pack;
      } else if ((st = do_pack())) {
        return st;
      }
    }
    if (mode != 2 && s->n_owners > 0) {
      materialize();
      bool done = false, big_only = false;
      uint8_t* bigmask = (mode == 0 && !orig) ? S.alloc<uint8_t>(n) : nullptr;
      if (mode == 0 && !orig && !bigmask) return EVM_ENOMEM;
      if ((st = ingest_by_owner(ctx, S, s, rec, minute, own, n, orig, id_base, flags, info, perm, &ns, &new_tree,
                                &done, bigmask, &big_only, ts, stride, pack_now, wire))) {
        if (st == EVM_ESTATE) {  // the merge refused: no message is reported inserted
          KLAUNCH(k_flags_clear, dim3(grid_for(n, 256)), dim3(256), n, flags, orig);
          (void)evm_sync(ctx);
        }
        return st;
      }
      if (done && big_only && !orig) {
        // the LDS path took every owner but the big ones: commit that, then
        // the big owners' messages (in batch order) through the sort path
        u32* bm = S.alloc<u32>(n);
        u32* bpos = S.alloc<u32>(n);
        u32* nbig = S.alloc<u32>(1);
        u32* sel_big = S.alloc<u32>(n);
        if (!bm || !bpos || !nbig || !sel_big) return EVM_ENOMEM;
        KLAUNCH(k_mask_u32, dim3(grid_for(n, 256)), dim3(256), bigmask, n, bm);
        if ((st = scan_exclusive<u32, OpAdd>(ctx, S, bm, n, bpos, nbig))) return st;
        KLAUNCH(k_pick, dim3(grid_for(n, 256)), dim3(256), bigmask, bpos, n, sel_big);
        u32 hbig = 0;
        HIPR(hipMemcpyAsync(&hbig, nbig, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
        HIPR(hipStreamSynchronize(ctx->stream));
        // phase 2 runs on the uncommitted phase-1 result: the caller's store
        // changes only when both phases succeed (index.ts:147-169 is one
        // transaction that rolls back on any error)
        evm_store mid = ns;
        mid.tree = new_tree;
        ns = evm_store{};
        new_tree = nullptr;
        st = ctx->test_fail == 1 ? EVM_ENOMEM
                                 : ingest_impl(ctx, &mid, ts, stride, hbig, owner, sel_big, rec, id_base, flags, 2);
        if (st) {
          store_release_arrays(ctx, &mid);
          tree_destroy(ctx, mid.tree);
          (void)hipMemsetAsync(flags, 0, n, ctx->stream);  // nothing inserted
          (void)evm_sync(ctx);
          return st;
        }
        return commit_store(ctx, s, mid, mid.tree);
      }
      if (done) goto commit;
    }
    if (!have_rec && pack_now && (st = pack_now())) return st;  // the sort path reads packed records
    FieldRange h0;
    for (int f = 0; f < N_FIELDS; ++f) {
      h0.mn[f] = ~0ull;
      h0.mx[f] = 0;
    }
    HIPR(hipMemcpyAsync(fr, &h0, sizeof(h0), hipMemcpyHostToDevice, ctx->stream));
    KLAUNCH(k_sv_ranges, dim3(grid_for(n, 256, 2048)), dim3(256), have_rec ? rec : prec, have_rec ? nullptr : orig, n,
            fr);
    Info hi;
    FieldRange hr;
    HIPR(hipMemcpyAsync(&hr, fr, sizeof(hr), hipMemcpyDeviceToHost, ctx->stream));
    if ((st = read_info(ctx, info, &hi))) return st;
    if (hi.bad_aux) return EVM_EINVAL;
    if (hi.bad) {
      // a timestamp the engine cannot canonicalise (toISOString would differ
      // or throw): flag the culprits, apply nothing -- the host falls back
      KLAUNCH(k_sv_bad, dim3(grid_for(n, 256)), dim3(256), rec, n, flags, orig);
      (void)evm_sync(ctx);
      return EVM_ENONCANON;
    }
    auto bits_of = [](u64 d) { return d ? 64 - __builtin_clzll(d) : 0; };
    const int ob = bits_of(hr.mx[F_OWNER] - hr.mn[F_OWNER]), mb = bits_of(hr.mx[F_MS] - hr.mn[F_MS]),
              cb = bits_of(hr.mx[F_CTR]);
    const u64* skeys = nullptr;
    evm_rec* srec = nullptr;  // records in sorted order
    u32* src = nullptr;       // sorted position -> srec index (tie runs permuted by node)
    bool sorted = false;
    if (ob + mb + cb <= 64) {
      // one radix sort on the compound (owner, millis, counter) key, then node-rank ties
      u64* kk = fv;
      u32* vv = perm;
      const CKey ck{hr.mn[F_OWNER], hr.mn[F_MS], mb, cb};
      // a sub-batch with the caller's packed records: the sort carries the
      // caller's indices, so nothing below maps through orig again
      const bool caller_idx = orig && prec;
      KLAUNCH(k_sv_ckey, dim3(grid_for(n, 256)), dim3(256), have_rec ? rec : prec, have_rec ? nullptr : orig, n, ck, kk,
              vv, caller_idx ? orig : (const u32*)nullptr);
      if ((st = radix_sort_pairs<u64>(ctx, S, kk, vv, n, 0, ob + mb + cb))) return st;
      u32* tl = S.alloc<u32>(1);
      srec = S.alloc<evm_rec>(n);
      src = S.alloc<u32>(n);
      if (!tl || !srec || !src) return EVM_ENOMEM;
      HIPR(hipMemsetAsync(tl, 0, sizeof(u32), ctx->stream));
      KLAUNCH(k_sv_gather, dim3(grid_for(n, 256)), dim3(256), caller_idx ? prec : rec, vv, n, srec);
      KLAUNCH(k_sv_ties, dim3(grid_for(n, 256)), dim3(256), kk, srec, n, src, tl);
      u32 too_long = 0;
      HIPR(hipMemcpyAsync(&too_long, tl, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
      HIPR(hipStreamSynchronize(ctx->stream));
      if (!too_long) {
        perm = vv;  // (scratch lives until the end of the call)
        if (caller_idx) orig = nullptr;
        skeys = kk;  // sorted compound keys (scratch lives until the end of the call)
        sorted = true;
      }
    }
    if (!sorted) {
      // stable LSD sort of the batch index by (owner, tc, rank_hi, rank_lo), field by field
      materialize();
      if ((st = launch_iota(ctx, perm, n))) return st;
      const int order[4] = {F_LO, F_HI, F_TC, F_OWNER};
      for (int f : order) {
        const u64 d = hr.mn[f] ^ hr.mx[f];
        if (!d) continue;
        const int hb = 64 - __builtin_clzll(d);
        KLAUNCH(k_sv_field, dim3(grid_for(n, 256)), dim3(256), rec, perm, n, f, fv);
        u64* kk = fv;
        u32* vv = perm;
        if ((st = radix_sort_pairs<u64>(ctx, S, kk, vv, n, 0, hb))) return st;
        if (vv != perm) HIPR(hipMemcpyAsync(perm, vv, sizeof(u32) * n, hipMemcpyDeviceToDevice, ctx->stream));
      }
      if (!srec && !(srec = S.alloc<evm_rec>(n))) return EVM_ENOMEM;
      src = nullptr;
      KLAUNCH(k_sv_gather, dim3(grid_for(n, 256)), dim3(256), rec, (const u32*)perm, n, srec);
    }
    // dedup within the batch and against the store
    u32* sel = S.alloc<u32>(n);
    u32* pos = S.alloc<u32>(n);
    u32* cnt = S.alloc<u32>(2);
    if (!sel || !pos || !cnt) return EVM_ENOMEM;
    const StoreView old = view_of(s);
    KLAUNCH(k_sv_mark, dim3(grid_for(n, 256)), dim3(256), (const evm_rec*)srec, (const u32*)src, (const u32*)perm, skeys,
            n, old, flags, sel, orig);
    if ((st = scan_exclusive<u32, OpAdd>(ctx, S, sel, n, pos, cnt))) return st;
    u32 m = 0;
    HIPR(hipMemcpyAsync(&m, cnt, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    // inserted rows (sorted), and their leaves
    u32* n_owner = S.alloc<u32>(m);
    u64* n_tc = S.alloc<u64>(m);
    u64* n_hi = S.alloc<u64>(m);
    u32* n_lo = S.alloc<u32>(m);
    u64* n_id = S.alloc<u64>(m);
    u64* l_ck = S.alloc<u64>(m);
    u32* l_h = S.alloc<u32>(m);
    if (!n_owner || !n_tc || !n_hi || !n_lo || !n_id || !l_ck || !l_h) return EVM_ENOMEM;
    HIPR(hipMemsetAsync(cnt + 1, 0, sizeof(u32), ctx->stream));
    KLAUNCH(k_sv_compact, dim3(grid_for(n, 256)), dim3(256), (const evm_rec*)srec, (const u32*)src, (const u32*)perm,
            sel, pos, n, (u64)id_base, n_owner, n_tc, n_hi, n_lo, n_id, l_ck, l_h, orig);
    if (m > 1) KLAUNCH(k_sv_sorted_check, dim3(grid_for(m, 256)), dim3(256), l_ck, (size_t)m, cnt + 1);
    // merged store
    if ((st = store_alloc(ctx, &ns, s->n_owners, s->n + m))) return st;
    u64* noff = S.alloc<u64>((size_t)s->n_owners + 1);  // the new rows' owner offsets
    if (!noff) return EVM_ENOMEM;
    KLAUNCH(k_sv_owner_off, dim3(grid_for(s->n_owners + 1, 256)), dim3(256), (const u32*)n_owner, (size_t)m,
            s->n_owners, noff);
    const StoreView nv{noff, n_owner, n_tc, n_hi, n_lo};
    const StoreOut so{ns.owner, ns.tc, ns.hi, ns.lo, ns.id};
    if (s->n)
      KLAUNCH(k_sv_merge_old, dim3(grid_for(s->n, 256)), dim3(256), old, (const u64*)s->id, (size_t)s->n, nv, (size_t)m,
              so);
    if (m)
      KLAUNCH(k_sv_merge_new, dim3(grid_for(m, 256)), dim3(256), nv, (const u64*)n_id, (size_t)m, old, (size_t)s->n,
              so);
    KLAUNCH(k_add_u64, dim3(grid_for(s->n_owners + 1, 256)), dim3(256), (const u64*)s->off, (const u64*)noff,
            (size_t)s->n_owners + 1, ns.off);
    // Merkle: XOR of the inserted rows into their owners' trees
    u32 unsorted = 0;
    HIPR(hipMemcpyAsync(&unsorted, cnt + 1, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    if (unsorted) {
      // mixed key lengths inside one owner's batch: sort the leaf keys
      Info fi = info_init();
      fi.ck_min = 0;
      fi.ck_max = ~0ull;
      fi.maxlen = CODE_DIGITS;
      st = fold_into_tree(ctx, S, s->tree, s->n_owners, l_ck, l_h, m, fi, &new_tree);
    } else {
      u64* rck = S.alloc<u64>(std::max<size_t>(m, 1));
      int32_t* rxr = S.alloc<int32_t>(std::max<size_t>(m, 1));
      if (!rck || !rxr) return EVM_ENOMEM;
      uint64_t L = 0;
      if ((st = reduce_runs(ctx, S, l_ck, (const int32_t*)l_h, m, rck, rxr, &L))) return st;
      st = merge_into_tree(ctx, S, s->tree, s->n_owners, rck, rxr, L, &new_tree);
    }
    if (st) return st;
  }
commit:
  pending.armed = false;
  return commit_store(ctx, s, ns, new_tree);
}

extern "C" {

int evm_server_ingest(evm_ctx* ctx, evm_store* s, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                      uint64_t id_base, uint8_t* flags) {
  if (!ctx || !s || stride < 46 || (n && (!ts || !owner || !flags))) return EVM_EINVAL;
  if (n == 0) return EVM_OK;  // index.ts:145 `if (req.messages.length === 0) return merkleTree`
  if (n >= 0xffffffffull) return EVM_EINVAL;
  return ingest_impl(ctx, s, ts, stride, n, owner, nullptr, nullptr, id_base, flags, ctx->server_path == 2 ? 2 : 0);
}

int evm_server_ingest_ex(evm_ctx* ctx, evm_store* s, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                         uint64_t id_base, uint8_t* flags, uint8_t* owner_status) {
  if (!ctx || !s || !owner_status || stride < 46 || (n && (!ts || !owner || !flags))) return EVM_EINVAL;
  if (n >= 0xffffffffull) return EVM_EINVAL;
  const u32 O = s->n_owners;
  if (O) HIPR(hipMemsetAsync(owner_status, 0, O, ctx->stream));
  if (n == 0) return evm_sync(ctx);
  const int mode = ctx->server_path == 2 ? 2 : 0;
  int st = ingest_impl(ctx, s, ts, stride, n, owner, nullptr, nullptr, id_base, flags, mode);
  if (st != EVM_ENONCANON) return st;
  // some owners' rows are outside the native domain: nothing was applied and
  // flags mark the culprits.  Those owners commit nothing (their requests
  // fail as one transaction, index.ts:147-169); every other owner commits.
  Scratch S(ctx);
  uint8_t* mask = S.alloc<uint8_t>(n);
  u32* keep = S.alloc<u32>(n);
  u32* pos = S.alloc<u32>(n);
  u32* nkeep = S.alloc<u32>(1);
  u32* sel = S.alloc<u32>(n);
  evm_rec* rec = S.alloc<evm_rec>(n);
  Info* info = nullptr;
  if (!mask || !keep || !pos || !nkeep || !sel || !rec) return EVM_ENOMEM;
  if ((st = new_info(ctx, S, &info))) return st;
  KLAUNCH(k_owner_bad, dim3(grid_for(n, 256)), dim3(256), flags, owner, n, O, owner_status);
  KLAUNCH(k_owner_keep, dim3(grid_for(n, 256)), dim3(256), owner, n, (const uint8_t*)owner_status, mask, keep);
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, keep, n, pos, nkeep))) return st;
  KLAUNCH(k_pick, dim3(grid_for(n, 256)), dim3(256), (const uint8_t*)mask, (const u32*)pos, n, sel);
  if ((st = launch_pack(ctx, ts, stride, n, owner, O, rec, info))) return st;
  u32 hkeep = 0;
  HIPR(hipMemcpyAsync(&hkeep, nkeep, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (hkeep) {
    // (the sub-batch writes the flags of its rows; the rejected owners' rows
    // keep the first pass's: EVM_MSG_BAD for the culprits, 0 otherwise)
    if ((st = ingest_impl(ctx, s, ts, stride, hkeep, owner, sel, rec, id_base, flags, mode))) return st;
  }
  return EVM_ENONCANON;
}

}  // extern "C"

int evm::server_ingest_wire(evm_ctx* ctx, evm_store* s, const WireSrc& w, size_t n, const u32* owner, uint64_t id_base,
                            uint8_t* flags) {
  if (!ctx || !s || (n && (!owner || !flags))) return EVM_EINVAL;
  if (n == 0) return EVM_OK;
  if (n >= 0xffffffffull) return EVM_EINVAL;
  return ingest_impl(ctx, s, nullptr, 48, n, owner, nullptr, nullptr, id_base, flags, ctx->server_path == 2 ? 2 : 0,
                     &w);
}

// Selection of each owner's rows after a per-owner bound (diff/since, < 0 =
// none), optionally excluding one node (server getMessages).
static int select_after(evm_ctx* ctx, Scratch& S, const evm_store* s, const int64_t* bound, const char* node,
                        const uint8_t* active, uint64_t* sel_off, uint64_t* sel_id, uint64_t* sel_key, uint64_t cap,
                        uint64_t* n_sel) {
  const u32 O = s->n_owners;
  int st;
  // candidate counts and their scans are u32: a store past 2^32 - 1 rows
  // would wrap them (and silently shorten the selection)
  if (s->n > 0xffffffffull) return EVM_ECAPACITY;
  u64* first = S.alloc<u64>(O);
  u32* cand = S.alloc<u32>(O);
  u32* cpos = S.alloc<u32>(O + 1);
  u64* req = S.alloc<u64>(O);
  u32* tot = S.alloc<u32>(2);
  if (!first || !cand || !cpos || !req || !tot) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(tot, 0, 2 * sizeof(u32), ctx->stream));
  const StoreView v = view_of(s);
  KLAUNCH(k_sv_sel_first, dim3(grid_for(O, 64, 65536)), dim3(64), v, O, bound, (const uint8_t*)node, active, first,
          cand, req, tot + 1);
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, cand, O, cpos, cpos + O))) return st;
  u32 h[2];
  {
    LandList l;
    l.add(cpos + O, &h[0], sizeof(u32));
    l.add(tot + 1, &h[1], sizeof(u32));
    if ((st = land_words(ctx, l))) return st;
  }
  if (h[1]) return EVM_EINVAL;  // a requester nodeId is not 16 hex chars
  const u32 C = h[0];
  const int grid = grid_for(C, SEL_THREADS, 16384);
  u32* keep = nullptr;
  u32* kpos = nullptr;
  u32 K = C;
  if (node && C && ctx->select_path == 0) {
    // keep + rank + emit in one pass (decoupled look-back over the candidate tiles)
    const u32 ntiles = (C + SEL_TILE - 1) / SEL_TILE;
    u32* kst = S.alloc<u32>(C);
    u64* status = S.alloc<u64>(ntiles);
    u32* ctr = S.alloc<u32>(2);  // tile counter, look-back error
    if (!kst || !status || !ctr) return EVM_ENOMEM;
    {
      ZeroList z;
      z.add(status, sizeof(u64) * ntiles);
      z.add(ctr, 2 * sizeof(u32));
      if ((st = zero_small(ctx, z))) return st;
    }
    KLAUNCH(k_sv_sel_scan, dim3(ntiles), dim3(SEL_THREADS), v, O, C, (const u32*)cpos, (const u64*)first,
            (const u64*)req, (const u64*)s->id, sel_id ? (u64)cap : 0ull, (u64*)sel_id, (u64*)sel_key, kst, status,
            ctr, tot, ctr + 1);
    KLAUNCH(k_sv_sel_off, dim3(grid_for(O + 1, 256)), dim3(256), O, C, (const u32*)cpos, (const u32*)kst,
            (const u32*)tot, (u64*)sel_off);
    u32 h2[2];
    {
      LandList l;
      l.add(tot, &K, sizeof(u32));
      l.add(ctr, h2, 2 * sizeof(u32));
      if ((st = land_words(ctx, l))) return st;
    }
    if (h2[1]) return EVM_EDEVICE;  // a look-back wait gave up
    *n_sel = K;
    if (K > cap || (K && !sel_id)) return EVM_ECAPACITY;
    return EVM_OK;
  }
  if (node && C) {
    keep = S.alloc<u32>(C);
    kpos = S.alloc<u32>(C);
    if (!keep || !kpos) return EVM_ENOMEM;
    KLAUNCH(k_sv_sel_keep, dim3(grid), dim3(SEL_THREADS), v, O, C, (const u32*)cpos, (const u64*)first,
            (const u64*)req, keep);
    if ((st = scan_exclusive<u32, OpAdd>(ctx, S, keep, C, kpos, tot))) return st;
    HIPR(hipMemcpyAsync(&K, tot, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
  }
  KLAUNCH(k_sv_sel_off, dim3(grid_for(O + 1, 256)), dim3(256), O, C, (const u32*)cpos, (const u32*)kpos,
          (const u32*)tot, (u64*)sel_off);
  *n_sel = K;
  if (K > cap || (K && !sel_id)) return EVM_ECAPACITY;
  if (K)
    KLAUNCH(k_sv_sel_emit, dim3(grid), dim3(SEL_THREADS), O, C, (const u32*)cpos, (const u64*)first,
            (const u32*)keep, (const u32*)kpos, (const u64*)s->id, (u64*)sel_id, v, (u64*)sel_key);
  return evm_sync(ctx);
}

extern "C" {

int evm_server_select(evm_ctx* ctx, const evm_store* s, const evm_tree* client, const char* node,
                      const uint8_t* active, int64_t* diff, uint64_t* sel_off, uint64_t* sel_id, uint64_t cap,
                      uint64_t* n_sel) {
  if (!ctx || !s || !client || !node || !diff || !sel_off || !n_sel) return EVM_EINVAL;
  if (client->n_owners != s->n_owners) return EVM_EINVAL;
  if (s->n_owners == 0) {
    *n_sel = 0;
    return EVM_OK;
  }
  int st;
  Scratch S(ctx);
  if ((st = launch_diff(ctx, s->tree, client, diff))) return st;
  return select_after(ctx, S, s, diff, node, active, sel_off, sel_id, nullptr, cap, n_sel);
}

int evm_store_since(evm_ctx* ctx, const evm_store* s, const int64_t* since, uint64_t* sel_off, uint64_t* sel_id,
                    uint64_t cap, uint64_t* n_sel) {
  if (!ctx || !s || !since || !sel_off || !n_sel) return EVM_EINVAL;
  if (s->n_owners == 0) {
    *n_sel = 0;
    return EVM_OK;
  }
  Scratch S(ctx);
  return select_after(ctx, S, s, since, nullptr, nullptr, sel_off, sel_id, nullptr, cap, n_sel);
}

int evm_store_select_after(evm_ctx* ctx, const evm_store* s, const int64_t* bound, const char* node,
                           const uint8_t* active, uint64_t* sel_off, uint64_t* sel_id, uint64_t* sel_key,
                           uint64_t cap, uint64_t* n_sel) {
  if (!ctx || !s || !bound || !sel_off || !n_sel) return EVM_EINVAL;
  if (s->n_owners == 0) {
    *n_sel = 0;
    return EVM_OK;
  }
  Scratch S(ctx);
  return select_after(ctx, S, s, bound, node, active, sel_off, sel_id, sel_key, cap, n_sel);
}

}  // extern "C"
