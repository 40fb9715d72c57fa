// applyMessages (packages/evolu/src/applyMessages.ts:26-131) on MI355X.
//
// Sequential reference semantics, per message i of the batch, in cell c:
//   t_i = max timestamp of c in __message before i  (prior rows + earlier batch rows)
//   ups_i = t_i == null || t_i < ts_i     (:93  upsert the user-table cell)
//   xor_i = t_i == null || t_i !== ts_i   (:105 INSERT ... ON CONFLICT DO NOTHING + Merkle XOR)
// With no timestamp repeated across cells (checked exactly, k_xcell), t_i is the
// exclusive running max of c in batch order seeded with the prior max, because a
// repeat of an older timestamp of c never moves the max.  Two device paths:
//   * fast path (one owner, <= CL_MAX_CELLS cells): wave-ranges stream the batch
//     twice, per-cell state in LDS, no global sort (evm_client.hip: k_cl_*);
//   * general path: stable radix sort by cell + segmented scan (k_lww_*).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_pack.hpp"
#include "evm_prims.hpp"

using namespace evm;
// ============================================================================
// applyMessages (applyMessages.ts:26-131)
// ============================================================================

// (1) Global __message PK: the same timestamp in two different cells of one
// batch makes the reference's INSERT fail silently for the later one and
// stops that cell's running max from advancing.  That interleaving is
// inherently sequential, so it is detected exactly and reported.
__global__ void k_xcell(const evm_rec* __restrict__ rec, size_t n, u64* __restrict__ table, u32 log2size,
                        Info* __restrict__ info) {
  const u64 mask = (1ull << log2size) - 1;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const evm_rec r = rec[i];
    if (!(r.meta & EVM_META_VALID)) continue;
    const u64 mine = ((u64)r.hash << 32) | (u64)(i + 1);
    u64 pos = ((u64)(r.hash * 2654435761u) ^ (r.node * 0x9E3779B97F4A7C15ull >> 20)) & mask;
    for (u64 probe = 0; probe <= mask; ++probe) {
      u64 s = __hip_atomic_load(&table[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (s == 0) {
        const u64 prev = atomicCAS(&table[pos], 0ull, mine);
        if (prev == 0) break;  // inserted
        s = prev;
      }
      if ((u32)(s >> 32) == r.hash) {
        const evm_rec o = rec[(size_t)(s & 0xffffffffu) - 1];
        if (o.tc == r.tc && o.node == r.node && (o.meta & EVM_META_CASEMASK) == (r.meta & EVM_META_CASEMASK)) {
          if (o.aux != r.aux) atomicOr(&info->collision, 1u);
          break;
        }
      }
      pos = (pos + 1) & mask;
    }
  }
}

// (2) Segmented (per cell) running max in batch order over the cell-sorted
// order.  Aggregate = (segment head seen, max since the last head).
struct SegAgg {
  u32 head;
  Key key;
};
__device__ __forceinline__ SegAgg seg_combine(const SegAgg& a, const SegAgg& b) {
  SegAgg r;
  r.head = a.head | b.head;
  r.key = b.head ? b.key : key_max(a.key, b.key);
  return r;
}

constexpr int LWW_THREADS = 256;
constexpr int LWW_ITEMS = 8;
constexpr int LWW_TILE = LWW_THREADS * LWW_ITEMS;

__device__ __forceinline__ SegAgg lww_elem(const evm_rec* rec, const u32* cell_s, const u32* idx_s, size_t p) {
  SegAgg e;
  e.head = (p == 0 || cell_s[p] != cell_s[p - 1]) ? 1u : 0u;
  e.key = key_of(rec[idx_s[p]]);
  return e;
}

struct SegLds {
  u32 head[LWW_THREADS];
  u64 tc[LWW_THREADS];
  u64 node[LWW_THREADS];
  u32 mask[LWW_THREADS];
};
__device__ __forceinline__ void seg_put(SegLds& L, int t, const SegAgg& a) {
  L.head[t] = a.head;
  L.tc[t] = a.key.tc;
  L.node[t] = a.key.node;
  L.mask[t] = a.key.mask;
}
__device__ __forceinline__ SegAgg seg_get(const SegLds& L, int t) {
  SegAgg a;
  a.head = L.head[t];
  a.key = Key{L.tc[t], L.node[t], L.mask[t]};
  return a;
}

// Block inclusive scan (Hillis-Steele over LDS) of one SegAgg per thread.
__device__ SegAgg seg_block_inclusive(SegLds& L, SegAgg v) {
  const int t = threadIdx.x;
  seg_put(L, t, v);
  __syncthreads();
  for (int d = 1; d < LWW_THREADS; d <<= 1) {
    SegAgg o;
    const bool has = t >= d;
    if (has) o = seg_get(L, t - d);
    __syncthreads();
    if (has) v = seg_combine(o, v);
    seg_put(L, t, v);
    __syncthreads();
  }
  return v;
}

__global__ __launch_bounds__(LWW_THREADS) void k_lww_reduce(const evm_rec* __restrict__ rec, const u32* __restrict__ cell_s,
                                                            const u32* __restrict__ idx_s, size_t n,
                                                            u32* __restrict__ t_head, Key* __restrict__ t_key) {
  __shared__ SegLds L;
  const size_t base = (size_t)blockIdx.x * LWW_TILE + (size_t)threadIdx.x * LWW_ITEMS;
  SegAgg acc{0u, key_none()};
  for (int k = 0; k < LWW_ITEMS; ++k) {
    const size_t p = base + k;
    if (p < n) acc = seg_combine(acc, lww_elem(rec, cell_s, idx_s, p));
  }
  const SegAgg inc = seg_block_inclusive(L, acc);
  if (threadIdx.x == LWW_THREADS - 1) {
    t_head[blockIdx.x] = inc.head;
    t_key[blockIdx.x] = inc.key;
  }
}

// Exclusive scan of the tile aggregates, in one block.
__global__ __launch_bounds__(LWW_THREADS) void k_lww_tiles(u32* __restrict__ t_head, Key* __restrict__ t_key, size_t nt) {
  __shared__ SegLds L;
  const size_t per = (nt + LWW_THREADS - 1) / LWW_THREADS;
  const size_t b = (size_t)threadIdx.x * per;
  SegAgg acc{0u, key_none()};
  for (size_t i = b; i < b + per && i < nt; ++i) acc = seg_combine(acc, SegAgg{t_head[i], t_key[i]});
  const SegAgg inc = seg_block_inclusive(L, acc);
  // exclusive for this thread = inclusive of thread-1
  __syncthreads();
  seg_put(L, threadIdx.x, inc);
  __syncthreads();
  SegAgg run = threadIdx.x ? seg_get(L, threadIdx.x - 1) : SegAgg{0u, key_none()};
  for (size_t i = b; i < b + per && i < nt; ++i) {
    const SegAgg here{t_head[i], t_key[i]};
    t_head[i] = run.head;
    t_key[i] = run.key;
    run = seg_combine(run, here);
  }
}

__global__ __launch_bounds__(LWW_THREADS) void k_lww_apply(const evm_rec* __restrict__ rec, const u32* __restrict__ cell_s,
                                                           const u32* __restrict__ idx_s, size_t n,
                                                           const u32* __restrict__ t_head, const Key* __restrict__ t_key,
                                                           const evm_rec* __restrict__ prior,
                                                           const uint8_t* __restrict__ prior_present,
                                                           uint8_t* __restrict__ flags, int32_t* __restrict__ winner) {
  __shared__ SegLds L;
  const size_t base = (size_t)blockIdx.x * LWW_TILE + (size_t)threadIdx.x * LWW_ITEMS;
  SegAgg e[LWW_ITEMS];
  SegAgg acc{0u, key_none()};
#pragma unroll
  for (int k = 0; k < LWW_ITEMS; ++k) {
    const size_t p = base + k;
    e[k] = p < n ? lww_elem(rec, cell_s, idx_s, p) : SegAgg{0u, key_none()};
    acc = seg_combine(acc, e[k]);
  }
  const SegAgg inc = seg_block_inclusive(L, acc);
  __syncthreads();
  seg_put(L, threadIdx.x, inc);
  __syncthreads();
  SegAgg run = SegAgg{t_head[blockIdx.x], t_key[blockIdx.x]};
  if (threadIdx.x) run = seg_combine(run, seg_get(L, threadIdx.x - 1));
#pragma unroll
  for (int k = 0; k < LWW_ITEMS; ++k) {
    const size_t p = base + k;
    if (p >= n) break;
    const Key excl = e[k].head ? key_none() : run.key;
    run = seg_combine(run, e[k]);
    const u32 c = cell_s[p];
    const u32 i = idx_s[p];
    Key t = excl;
    if (prior_present && prior_present[c]) t = key_max(t, key_of(prior[c]));
    const Key ts = e[k].key;
    // applyMessages.ts:93  t == null || t < message.timestamp
    const bool ups = key_cmp(t, ts) < 0;
    // applyMessages.ts:105 t == null || t !== message.timestamp
    const bool xr = !((t.mask & KEY_PRESENT) && key_eq(t, ts));
    flags[i] = (ups ? EVM_MSG_UPS : 0u) | (xr ? EVM_MSG_XOR : 0u);
    if (ups) atomicMax(&winner[c], (int32_t)i);
  }
}

__global__ void k_mark_bad(const evm_rec* __restrict__ rec, size_t n, uint8_t* __restrict__ flags) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    flags[i] = (rec[i].meta & EVM_META_VALID) ? 0u : EVM_MSG_BAD;
}

__global__ void k_fill_i32(int32_t* __restrict__ p, size_t n, int32_t v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}



// ============================================================================
// Fast path: one owner, n_cells <= CL_MAX_CELLS.
//
// The batch is cut into G contiguous wave-ranges (one 64-lane workgroup each).
// A range keeps per-cell state in LDS and walks its messages 64 at a time; the
// lanes of one round that hit the same cell are matched with ballots and
// combined in lane (= batch) order.
//   pass 1: per range and cell, the max timestamp and its first index
//   carry : per cell, exclusive scan over ranges (seeded with the prior max);
//           the final winner is the first index of the cell's overall max
//   pass 2: re-walk with the carried state: exclusive max t_i -> flags; write
//           (minute, hash) of every XOR message for the Merkle fold
// The timestamp bytes are streamed twice (re-parsing is cheaper than a round
// trip of a packed record), never sorted, never gathered.
// ============================================================================
constexpr u32 CL_MAX_CELLS = 2048;
constexpr int CL_RANGE_TARGET = 1280;  // ~5 ranges per CU
constexpr u32 FOLD_WIN = 32768;        // minutes per LDS histogram window (128 KiB)
constexpr u32 FOLD_MAXWIN = 4;
constexpr u32 FOLD_CHUNKS = 128;  // x windows: 256+ single-CU blocks for a 2-window batch
constexpr int FOLD_THREADS = 1024;


struct ClMsg {
  OKey key;
  u32 cell;
  bool ok;  // valid timestamp, cell in range, inside the range
};

struct ClRaw {
  uint4 key;  // tc, rh
  u32 rl;
  u32 cell;
};

__device__ __forceinline__ ClRaw cl_fetch(const uint4* __restrict__ key, const u32* __restrict__ rl,
                                          const u32* __restrict__ cell, size_t first, size_t end) {
  const size_t i = first + (threadIdx.x & 63);
  ClRaw r;
  if (i < end) {
    // non-temporal: shorter issue-to-land latency for the latency-bound walks
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u k = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(key) + i);
    r.key = make_uint4(k.x, k.y, k.z, k.w);
    r.rl = __builtin_nontemporal_load(rl + i);
    r.cell = __builtin_nontemporal_load(cell + i);
  } else {
    r.key = make_uint4(0, 0, 0, 0);
    r.rl = 0;
    r.cell = 0xffffffffu;
  }
  return r;
}

__device__ __forceinline__ ClMsg cl_decode(const ClRaw& r, u32 C) {
  ClMsg m;
  m.key = OKey{(u64)r.key.x | ((u64)r.key.y << 32), (u64)r.key.z | ((u64)r.key.w << 32), r.rl};
  m.cell = r.cell;
  m.ok = (r.rl & OKEY_PRESENT) && r.cell < C;
  return m;
}

__device__ __forceinline__ OKey shfl_okey(const OKey& k, int src) {
  OKey o;
  o.tc = ((u64)(u32)__shfl((int)(u32)(k.tc >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)k.tc, src, 64);
  o.rh = ((u64)(u32)__shfl((int)(u32)(k.rh >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)k.rh, src, 64);
  o.rl = (u32)__shfl((int)k.rl, src, 64);
  return o;
}

// Lanes whose `cell` equals this lane's (among `active`), by ballots on the bits.
__device__ __forceinline__ u64 match_cell(u32 c, bool active, int bits) {
  u64 peers = __ballot(active);
  for (int b = 0; b < bits; ++b) {
    const bool bit = (c >> b) & 1u;
    const u64 bal = __ballot(bit);
    peers &= bit ? bal : ~bal;
  }
  return active ? peers : 0ull;
}

struct ClState {
  u64* tc;
  u64* rh;
  u32* rl;
  u32* first;
};

__device__ __forceinline__ OKey cl_load(const ClState& S, u32 c) { return OKey{S.tc[c], S.rh[c], S.rl[c]}; }
__device__ __forceinline__ void cl_store(const ClState& S, u32 c, const OKey& k) {
  S.tc[c] = k.tc;
  S.rh[c] = k.rh;
  S.rl[c] = k.rl;
}

// Peer aggregate of one round of 64 messages (lane order == batch order):
// registers and cross-lane ops only, no per-cell state, so the rounds of a
// prefetch group are independent and only the short LDS read-compare-write
// (cl_commit*) is serial from round to round.
//   PASS 1: max key over this lane's same-cell peers up to and including
//           itself, with its batch index (ties: the earlier lane);
//   PASS 2: max key over the strictly earlier same-cell peers.
struct ClPeer {
  OKey acc;
  u32 acc_i;
  bool last;  // highest lane of its cell in the round: publishes the state
};

template <int PASS>
__device__ __forceinline__ ClPeer cl_peer(const ClMsg& m, size_t first, int cbits) {
  const int lane = threadIdx.x & 63;
  const u64 peers = match_cell(m.cell, m.ok, cbits);
  ClPeer r;
  r.last = m.ok && (peers >> lane) == 1ull;
  r.acc = okey_none();
  r.acc_i = 0xffffffffu;
  u64 rem = peers & lanemask_lt();
  while (__any(rem != 0)) {
    const int src = rem ? (int)__builtin_ctzll(rem) : lane;
    const OKey kp = shfl_okey(m.key, src);
    if (rem) {
      if (PASS == 1) {
        if (okey_gt(kp, r.acc)) {
          r.acc = kp;
          r.acc_i = (u32)(first + src);
        }
      } else {
        r.acc = okey_max(r.acc, kp);
      }
      rem &= rem - 1;
    }
  }
  if (PASS == 1 && m.ok && okey_gt(m.key, r.acc)) {
    r.acc = m.key;
    r.acc_i = (u32)(first + lane);
  }
  return r;
}

// pass 1: the round's last peer of a cell folds the round max into the range state
__device__ __forceinline__ void cl_commit1(const ClMsg& m, const ClPeer& p, const ClState& S) {
  if (p.last && okey_gt(p.acc, cl_load(S, m.cell))) {
    cl_store(S, m.cell, p.acc);
    S.first[m.cell] = p.acc_i;
  }
}

// pass 2: t_i = max(range state, earlier peers) -> flags; the last peer publishes
__device__ __forceinline__ void cl_commit2(const ClMsg& m, const ClPeer& p, const ClState& S,
                                           uint8_t* __restrict__ flags, size_t i, size_t end) {
  const OKey t = m.ok ? okey_max(cl_load(S, m.cell), p.acc) : okey_none();
  if (i < end) {
    // applyMessages.ts:93 / :105 with t (NULL is the all-zero key)
    const bool ups = m.ok && okey_gt(m.key, t);
    const bool xr = m.ok && !okey_eq(t, m.key);
    flags[i] = m.ok ? (uint8_t)((ups ? EVM_MSG_UPS : 0u) | (xr ? EVM_MSG_XOR : 0u)) : (uint8_t)EVM_MSG_BAD;
  }
  if (p.last) cl_store(S, m.cell, okey_max(t, m.key));
}

// The walk of one range by a 4-wave workgroup.  The range is cut into
// groups of 256 messages; wave w takes messages [64w, 64w + 64) of every
// group.  The peer phase (cl_peer: ballots and shuffles, the bulk of the
// work) runs in all four waves at once; the commits -- the short LDS
// read-compare-write on the range's per-cell state -- follow in batch order,
// wave 0 to 3, separated by barriers.  Other workgroups on the CU fill the
// SIMDs while one wave commits.
//   PASS 1: per-cell (max key, first index) of the range -> agg_*
//   PASS 2: state = the carried maxima (agg_*) -> flags
constexpr int WK_THREADS = 256;
constexpr int WK_PF = 4;  // groups in flight per wave

template <int PASS>
__device__ __forceinline__ void cl_walk(const uint4* __restrict__ key, const u32* __restrict__ rl,
                                        const u32* __restrict__ cell, size_t n, u32 C, int cbits, size_t range_len,
                                        u64* __restrict__ agg_tc, u64* __restrict__ agg_rh, u32* __restrict__ agg_rl,
                                        u32* __restrict__ agg_first, uint8_t* __restrict__ flags,
                                        Info* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  ClState S;
  S.tc = reinterpret_cast<u64*>(smem);
  S.rh = S.tc + C;
  S.rl = reinterpret_cast<u32*>(S.rh + C);
  S.first = PASS == 1 ? S.rl + C : nullptr;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t g = blockIdx.x;
  const size_t beg = g * range_len;
  const size_t end = min(n, beg + range_len);
  for (u32 c = threadIdx.x; c < C; c += WK_THREADS) {
    if (PASS == 1) {
      S.tc[c] = 0;
      S.rh[c] = 0;
      S.rl[c] = 0;
      S.first[c] = 0xffffffffu;
    } else {
      S.tc[c] = agg_tc[g * C + c];
      S.rh[c] = agg_rh[g * C + c];
      S.rl[c] = agg_rl[g * C + c];
    }
  }
  __syncthreads();
  ClRaw buf[WK_PF];
#pragma unroll
  for (int k = 0; k < WK_PF; ++k) buf[k] = cl_fetch(key, rl, cell, beg + 256 * k + 64 * w, end);
  bool aux_bad = false;
  for (size_t gfirst = beg; gfirst < end; gfirst += 256 * WK_PF) {  // uniform over the workgroup
#pragma unroll
    for (int k = 0; k < WK_PF; ++k) {
      const size_t f = gfirst + 256 * k + 64 * w;  // this wave's round
      if (PASS == 1) aux_bad |= f + lane < end && buf[k].cell >= C;
      const ClMsg m = cl_decode(buf[k], C);  // past the range: cell = ~0, not ok
      buf[k] = cl_fetch(key, rl, cell, f + 256 * WK_PF, end);
      const ClPeer p = cl_peer<PASS>(m, f, cbits);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (w == t) {
          if (PASS == 1) cl_commit1(m, p, S);
          else cl_commit2(m, p, S, flags, f + lane, end);
        }
        __syncthreads();
      }
    }
  }
  if (PASS == 1) {
    if (__ballot(aux_bad) && lane == 0) atomicOr(&info->bad_aux, 1u);
    for (u32 c = threadIdx.x; c < C; c += WK_THREADS) {
      agg_tc[g * C + c] = S.tc[c];
      agg_rh[g * C + c] = S.rh[c];
      agg_rl[g * C + c] = S.rl[c];
      agg_first[g * C + c] = S.first[c];
    }
  }
}

__global__ __launch_bounds__(WK_THREADS) void k_cl_scan1(const uint4* __restrict__ key, const u32* __restrict__ rl,
                                                         const u32* __restrict__ cell, size_t n, u32 C, int cbits,
                                                         size_t range_len, u64* __restrict__ agg_tc,
                                                         u64* __restrict__ agg_rh, u32* __restrict__ agg_rl,
                                                         u32* __restrict__ agg_first, Info* __restrict__ info) {
  cl_walk<1>(key, rl, cell, n, C, cbits, range_len, agg_tc, agg_rh, agg_rl, agg_first, nullptr, info);
}

__global__ __launch_bounds__(WK_THREADS) void k_cl_scan2(const uint4* __restrict__ key, const u32* __restrict__ rl,
                                                         const u32* __restrict__ cell, size_t n, u32 C, int cbits,
                                                         size_t range_len, u64* __restrict__ agg_tc,
                                                         u64* __restrict__ agg_rh, u32* __restrict__ agg_rl,
                                                         uint8_t* __restrict__ flags) {
  cl_walk<2>(key, rl, cell, n, C, cbits, range_len, agg_tc, agg_rh, agg_rl, nullptr, flags, nullptr);
}

// Carry: per cell, exclusive scan of the range aggregates in batch order,
// seeded with the prior max, as a 3-phase scan over SEG range segments.
// (max, first index) with ties kept left is associative.
constexpr u32 CARRY_SEGS = 64;

struct Agg {
  OKey key;
  u32 first;
};
__device__ __forceinline__ Agg agg_merge(const Agg& a, const Agg& b) { return okey_gt(b.key, a.key) ? b : a; }

__global__ void k_cl_carry_reduce(u32 C, size_t G, const u64* __restrict__ tc, const u64* __restrict__ rh,
                                  const u32* __restrict__ rl, const u32* __restrict__ firsti, u64* __restrict__ s_tc,
                                  u64* __restrict__ s_rh, u32* __restrict__ s_rl, u32* __restrict__ s_first) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x, p = blockIdx.y;
  if (c >= C) return;
  const size_t per = (G + CARRY_SEGS - 1) / CARRY_SEGS;
  const size_t a = p * per, e = min(G, a + per);
  Agg run{okey_none(), 0xffffffffu};
#pragma unroll 4
  for (size_t g = a; g < e; ++g) {
    const size_t k = g * C + c;
    run = agg_merge(run, Agg{OKey{tc[k], rh[k], rl[k]}, firsti[k]});
  }
  const size_t o = (size_t)p * C + c;
  s_tc[o] = run.key.tc;
  s_rh[o] = run.key.rh;
  s_rl[o] = run.key.rl;
  s_first[o] = run.first;
}

// One wave per cell, one lane per segment (CARRY_SEGS == 64): an exclusive
// wave scan of the segment aggregates seeded with the prior max.
static_assert(CARRY_SEGS == 64, "k_cl_carry_segs maps one segment per lane");
__global__ __launch_bounds__(256) void k_cl_carry_segs(u32 C, u64* __restrict__ s_tc, u64* __restrict__ s_rh,
                                                       u32* __restrict__ s_rl, u32* __restrict__ s_first,
                                                       const evm_rec* __restrict__ prior,
                                                       const uint8_t* __restrict__ prior_present,
                                                       int32_t* __restrict__ winner) {
  const u32 c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const size_t o = (size_t)lane * C + c;
  Agg v{OKey{s_tc[o], s_rh[o], s_rl[o]}, s_first[o]};
  // inclusive scan over lanes (segments in batch order); ties keep the left one
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    Agg u;
    u.key = shfl_okey(v.key, (int)lane - d < 0 ? (int)lane : (int)lane - d);
    u.first = (u32)__shfl((int)v.first, (int)lane - d < 0 ? (int)lane : (int)lane - d, 64);
    if ((int)lane >= d) v = agg_merge(u, v);
  }
  // exclusive: shift right by one, lane 0 gets the prior; the prior has no
  // batch index and wins ties (an equal batch copy is a no-op)
  const Agg seed{(prior_present && prior_present[c]) ? okey_of(prior[c]) : okey_none(), 0xffffffffu};
  Agg ex;
  ex.key = shfl_okey(v.key, lane == 0 ? 0 : (int)lane - 1);
  ex.first = (u32)__shfl((int)v.first, lane == 0 ? 0 : (int)lane - 1, 64);
  ex = lane == 0 ? seed : agg_merge(seed, ex);
  s_tc[o] = ex.key.tc;
  s_rh[o] = ex.key.rh;
  s_rl[o] = ex.key.rl;
  s_first[o] = ex.first;
  if (lane == 63) winner[c] = (int32_t)agg_merge(seed, v).first;  // 0xffffffff -> -1: no upsert survives
}

__global__ void k_cl_carry_down(u32 C, size_t G, u64* __restrict__ tc, u64* __restrict__ rh, u32* __restrict__ rl,
                                const u32* __restrict__ firsti, const u64* __restrict__ s_tc,
                                const u64* __restrict__ s_rh, const u32* __restrict__ s_rl) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x, p = blockIdx.y;
  if (c >= C) return;
  const size_t per = (G + CARRY_SEGS - 1) / CARRY_SEGS;
  const size_t a = p * per, e = min(G, a + per);
  const size_t o = (size_t)p * C + c;
  OKey run{s_tc[o], s_rh[o], s_rl[o]};
#pragma unroll 4
  for (size_t g = a; g < e; ++g) {
    const size_t k = g * C + c;
    const OKey here{tc[k], rh[k], rl[k]};
    tc[k] = run.tc;
    rh[k] = run.rh;
    rl[k] = run.rl;
    run = okey_max(run, here);
  }
}

// Exact cross-cell check over a persistent epoch-tagged hash set:
// slot = epoch:8 | hash low 24 bits:24 | (index + 1):32.  Equal fingerprints
// compare the raw 46 timestamp bytes.
__device__ __forceinline__ bool ts_bytes_equal(const uint8_t* ts, size_t stride, size_t a, size_t b) {
  u32 wa[12], wb[12];
  load_ts(ts, stride, a, wa);
  load_ts(ts, stride, b, wb);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 12; ++k) eq &= wa[k] == wb[k];
  return eq;
}

__global__ void k_cl_xcell(const uint8_t* __restrict__ ts, size_t stride, const u32* __restrict__ cell,
                           const u32* __restrict__ hash, size_t n, u64* __restrict__ table, u32 lg, u32 epoch,
                           Info* __restrict__ info) {
  const u64 mask = (1ull << lg) - 1;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32 h = hash[i];
    const u64 mine = ((u64)epoch << 56) | ((u64)(h & 0xffffffu) << 32) | (u64)(i + 1);
    u64 pos = ((u64)(h * 2654435761u) << 32 | (u64)(h * 0x85ebca6bu)) >> (64 - lg);
    for (u64 probe = 0; probe <= mask; ++probe) {
      u64 s = __hip_atomic_load(&table[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((u32)(s >> 56) != epoch) {
        const u64 prev = atomicCAS(&table[pos], s, mine);
        if (prev == s) break;  // inserted
        s = prev;
        if ((u32)(s >> 56) != epoch) continue;  // lost to a stale rewrite? retry this slot
      }
      if ((u32)(s >> 32 & 0xffffffu) == (h & 0xffffffu)) {
        const size_t j = (size_t)(s & 0xffffffffu) - 1;
        if (ts_bytes_equal(ts, stride, i, j)) {
          if (cell[i] != cell[j]) atomic_or_if(&info->collision, 1u);
          break;
        }
      }
      pos = (pos + 1) & mask;
    }
  }
}

// Rows already in __message (applyMessages.ts:42-45 PRIMARY KEY "timestamp"):
// the caller hands over the stored rows whose timestamp is in the batch
// (SELECT "timestamp", "table", "row", "column" FROM "__message" WHERE
// "timestamp" IN (...)).  A batch message whose timestamp is stored under
// another cell would have its INSERT ignored (:107-113) and its cell's running
// max frozen -- the sequential case the engine reports as a collision.  The
// stored rows go into an open-addressing set (slot = hash:32 | (row + 1):32);
// every batch message probes it with K1's hash, equal hashes compare the raw
// bytes.  Stored timestamps are unique (the PK), so one match ends a probe.
__global__ void k_st_insert(const evm_rec* __restrict__ srec, size_t m, u64* __restrict__ table, u32 lg) {
  const u64 mask = (1ull << lg) - 1;
  for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (size_t)gridDim.x * blockDim.x) {
    const evm_rec r = srec[j];
    if (!(r.meta & EVM_META_VALID)) continue;  // not canonical: no canonical batch timestamp equals it
    const u64 mine = ((u64)r.hash << 32) | (u64)(j + 1);
    u64 pos = (u64)(r.hash * 2654435761u) & mask;
    for (u64 probe = 0; probe <= mask; ++probe) {
      if (atomicCAS(&table[pos], 0ull, mine) == 0ull) break;
      pos = (pos + 1) & mask;
    }
  }
}

__global__ void k_st_probe(const u32* __restrict__ hash, size_t hstride, const uint8_t* __restrict__ ts, size_t stride,
                           const u32* __restrict__ cell, size_t n, const uint8_t* __restrict__ sts, size_t sstride,
                           const u32* __restrict__ scell, const u64* __restrict__ table, u32 lg,
                           Info* __restrict__ info) {
  const u64 mask = (1ull << lg) - 1;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32 h = hash[i * hstride];
    u64 pos = (u64)(h * 2654435761u) & mask;
    for (u64 probe = 0; probe <= mask; ++probe) {
      const u64 s = table[pos];
      if (s == 0) break;
      if ((u32)(s >> 32) == h) {
        const size_t j = (size_t)(s & 0xffffffffu) - 1;
        u32 wa[12], wb[12];
        load_ts(ts, stride, i, wa);
        load_ts(sts, sstride, j, wb);
        bool eq = true;
#pragma unroll
        for (int k = 0; k < 12; ++k) eq &= wa[k] == wb[k];
        if (eq) {
          if (cell[i] != scell[j]) atomic_or_if(&info->collision, 1u);
          break;
        }
      }
      pos = (pos + 1) & mask;
    }
  }
}

// Stored rows of the batch's timestamps (see k_st_insert), checked on the
// context stream.  hash: K1's hash of batch message i at hash[i * hstride].
struct Stored {
  const char* ts;
  size_t stride;
  size_t n;
  const u32* cell;
};

static int stored_check(evm_ctx* ctx, Scratch& S, const Stored& st, const u32* hash, size_t hstride, const char* ts,
                        size_t stride, const u32* cell, size_t n, Info* info) {
  if (!st.n || !n) return EVM_OK;
  const int lg = std::max(ceil_log2(2 * st.n), 6);
  evm_rec* srec = S.alloc<evm_rec>(st.n);
  u64* table = S.alloc<u64>((size_t)1 << lg);
  if (!srec || !table) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(table, 0, sizeof(u64) << lg, ctx->stream));
  int e;
  // the stored strings' murmur3 (their validity only gates the set)
  if ((e = launch_pack(ctx, st.ts, st.stride, st.n, nullptr, 0, srec, nullptr))) return e;
  KLAUNCH(k_st_insert, dim3(grid_for(st.n, 256, 2048)), dim3(256), (const evm_rec*)srec, st.n, table, (u32)lg);
  KLAUNCH(k_st_probe, dim3(grid_for(n, 256, 8192)), dim3(256), hash, hstride, (const uint8_t*)ts, stride, cell, n,
          (const uint8_t*)st.ts, st.stride, st.cell, (const u64*)table, (u32)lg, info);
  return EVM_OK;
}

// Partitioned cross-cell check (the default): messages are bucketed by the top
// bits of their hash (one counting-sort pass), then every bucket is checked in
// an LDS hash set.  Equal timestamps always share a bucket.  A bucket too big
// for LDS flags `xc_oversize` and the host reruns the global-table check.
constexpr int XP_THREADS = 1024;
constexpr int XP_ITEMS = 16;
constexpr int XP_TILE = XP_THREADS * XP_ITEMS;  // 16384 pairs staged in 128 KiB of LDS
constexpr u32 XP_SLOTS = 32768;                 // LDS set: u32 slots, 128 KiB
constexpr u32 XP_MAX_FILL = 24576;              // bucket capacity cap (75 % load)
constexpr u32 XP_AVG = 10000;                   // target mean bucket size (LDS set load <= ~0.4: short probe chains)
constexpr int XP_MAX_KB = 11;                   // 2048 buckets: n > 41M overfills them -> exact fallback
constexpr int XD_ITEMS = (XP_MAX_FILL + XP_THREADS - 1) / XP_THREADS;  // pairs per thread in k_xp_dedup

// Buckets have a fixed capacity `cap` in `out` (bucket b owns [b*cap, b*cap+cap));
// each tile reserves its run per bucket with one atomic on cursor[b], so no
// count matrix and no scan.  The tile is staged in LDS in bucket order and
// written back with consecutive lanes on consecutive addresses.  Order inside
// a bucket is irrelevant.  A full bucket flags xc_oversize (exact fallback).
__global__ __launch_bounds__(XP_THREADS) void k_xp_scatter(const u32* __restrict__ hash, size_t n, int kb, u32 cap,
                                                          u32* __restrict__ cursor, u64* __restrict__ out,
                                                          Info* __restrict__ info) {
  __shared__ u64 stage[XP_TILE];
  __shared__ u32 cnt[1u << XP_MAX_KB];  // per bucket: count, then local offset
  __shared__ u32 gb[1u << XP_MAX_KB];   // per bucket: this tile's base inside the bucket
  __shared__ u32 scan_tmp[XP_THREADS / 64 + 1];
  const u32 B = 1u << kb;
  const int sh = 32 - kb;
  for (u32 b = threadIdx.x; b < B; b += XP_THREADS) cnt[b] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * XP_TILE;
  u32 h[XP_ITEMS], r[XP_ITEMS];
#pragma unroll
  for (int k = 0; k < XP_ITEMS; ++k) {
    const size_t i = base + (size_t)k * XP_THREADS + threadIdx.x;
    h[k] = i < n ? __builtin_nontemporal_load(hash + i) : 0u;
    r[k] = i < n ? atomicAdd(&cnt[kb ? h[k] >> sh : 0u], 1u) : 0u;
  }
  __syncthreads();
  // exclusive scan of the bucket counts (B <= 16 * XP_THREADS), reserve global runs
  const u32 per = (B + XP_THREADS - 1) / XP_THREADS;
  u32 loc[(1u << XP_MAX_KB) / XP_THREADS];
  u32 sum = 0;
  for (u32 k = 0; k < per; ++k) {
    const u32 b = threadIdx.x * per + k;
    loc[k] = b < B ? cnt[b] : 0u;
    sum += loc[k];
  }
  u32 tot;
  const u32 incl = block_inclusive_scan<u32>(sum, scan_tmp, OpAdd<u32>(), &tot);
  u32 run = incl - sum;
  bool full = false;
  for (u32 k = 0; k < per; ++k) {
    const u32 b = threadIdx.x * per + k;
    if (b < B) {
      const u32 c = loc[k];
      cnt[b] = run;
      u32 g = 0;
      if (c) {
        g = atomicAdd(&cursor[b], c);
        full |= g + c > cap;
      }
      gb[b] = g;
      run += c;
    }
  }
  if (__ballot(full) && (threadIdx.x & 63) == 0) atomic_or_if(&info->xc_oversize, 1u);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < XP_ITEMS; ++k) {
    const size_t i = base + (size_t)k * XP_THREADS + threadIdx.x;
    if (i < n) stage[cnt[kb ? h[k] >> sh : 0u] + r[k]] = ((u64)h[k] << 32) | (u64)i;
  }
  __syncthreads();
  const u32 m = (u32)min((size_t)XP_TILE, n - base);
  for (u32 t = threadIdx.x; t < m; t += XP_THREADS) {
    const u64 v = stage[t];
    const u32 b = kb ? (u32)(v >> 32) >> sh : 0u;
    const u32 slot = gb[b] + (t - cnt[b]);
    if (slot < cap) out[(size_t)b * cap + slot] = v;
  }
}

// One bucket per workgroup: insert every (hash, index) into an LDS set of u32
// slots = tag:17 | (local index + 1):15; a tag match re-reads the other pair's
// full hash (L2-hot), and equal hashes compare the raw 46 timestamp bytes.
// (Probing past same-cell equal hashes to skip the byte reads of redeliveries
// measured slower: 82 vs 75 us per config-2 batch -- longer chains, and the
// two cell reads cost what the row reads did.)
// A pair gets XP_INLINE_PROBES probes in its wave's round; one still unplaced
// is queued (its next slot kept) and finished after the rounds, one per lane
// -- so a long probe chain no longer holds its whole wave at every round.
// Insertion order does not matter: slots never empty again, so two pairs of
// one hash (one start slot) always meet whichever goes first.
constexpr u32 XP_INLINE_PROBES = 2;
constexpr u32 XQ_CAP = 2048;
__device__ __forceinline__ bool xp_insert(u32* tab, const u64* bp, u64 p, u32 k, u32& pos, u32 budget,
                                          const uint8_t* ts, size_t stride, const u32* cell, Info* info) {
  const u32 h = (u32)(p >> 32), i = (u32)p;
  const u32 mine = ((h >> 15) << 15) | (k + 1);
  for (u32 probe = 0; probe < budget; ++probe) {
    const u32 prev = atomicCAS(&tab[pos], 0u, mine);
    if (prev == 0) return true;  // inserted
    if ((prev >> 15) == (h >> 15)) {
      const u64 q = bp[(prev & 0x7fffu) - 1];
      if ((u32)(q >> 32) == h) {
        const u32 j = (u32)q;
        if (ts_bytes_equal(ts, stride, i, j)) {  // equal strings <=> equal keys (both canonical)
          if (cell[i] != cell[j]) atomic_or_if(&info->collision, 1u);
          return true;
        }
      }
    }
    pos = (pos + 1) & (XP_SLOTS - 1);
  }
  return false;
}

__global__ __launch_bounds__(XP_THREADS) void k_xp_dedup(const u64* __restrict__ pairs, const u32* __restrict__ cursor,
                                                        u32 cap, size_t n, const uint8_t* __restrict__ ts,
                                                        size_t stride, const u32* __restrict__ cell,
                                                        Info* __restrict__ info) {
  __shared__ u32 tab[XP_SLOTS];  // 0 = empty
  __shared__ u32 q[XQ_CAP];      // queued pairs: next slot:15 | local index:15
  __shared__ u32 qn;
  const u32 b = blockIdx.x;
  const u32 cnt = min(cursor[b], cap);
  if (cnt < 2) return;
  const u64* bp = pairs + (size_t)b * cap;
  // every pair of this thread in flight at once (cap <= XP_MAX_FILL), then the set
  u64 it[XD_ITEMS];
#pragma unroll
  for (int r = 0; r < XD_ITEMS; ++r) {
    const u32 k = r * XP_THREADS + threadIdx.x;
    it[r] = k < cnt ? bp[k] : 0ull;
  }
  for (u32 s = threadIdx.x; s < XP_SLOTS; s += XP_THREADS) tab[s] = 0;
  if (threadIdx.x == 0) qn = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < XD_ITEMS; ++r) {
    const u32 k = r * XP_THREADS + threadIdx.x;
    if (k >= cnt) break;
    const u64 p = it[r];
    u32 pos = ((u32)(p >> 32) * 2654435761u) >> 17;  // 15 bits
    if (!xp_insert(tab, bp, p, k, pos, XP_INLINE_PROBES, ts, stride, cell, info)) {
      const u32 at = atomicAdd(&qn, 1u);
      if (at < XQ_CAP) q[at] = (pos << 15) | k;
      else xp_insert(tab, bp, p, k, pos, XP_SLOTS, ts, stride, cell, info);  // queue full: finish here
    }
  }
  __syncthreads();
  const u32 m = min(qn, XQ_CAP);
  for (u32 t = threadIdx.x; t < m; t += XP_THREADS) {
    const u32 e = q[t], k = e & 0x7fffu;
    u32 pos = e >> 15;
    xp_insert(tab, bp, bp[k], k, pos, XP_SLOTS, ts, stride, cell, info);
  }
}

// Dense Merkle fold over [minute_min, minute_min + FOLD_MAXWIN * FOLD_WIN):
// per (window, chunk) an LDS XOR histogram + presence bitmap.
// FLAGS: fold the EVM_MSG_XOR messages (both streaming paths); otherwise
// every message whose minute is in range (valid only for a batch in which
// every valid message is XORed).
template <bool FLAGS>
__global__ __launch_bounds__(FOLD_THREADS) void k_cl_fold_hist(const uint8_t* __restrict__ flags,
                                                              const u32* __restrict__ minute,
                                                              const u32* __restrict__ hash, size_t n,
                                                              u32* __restrict__ px, u32* __restrict__ pp,
                                                              Info* __restrict__ info) {
  __shared__ u32 hist[FOLD_WIN];
  __shared__ u32 pres[FOLD_WIN / 32];
  const u32 mlo = info->minute_min, mhi = info->minute_max;
  if (mlo > mhi) return;  // no valid message
  const u32 nwin = (mhi - mlo) / FOLD_WIN + 1;
  if (nwin > FOLD_MAXWIN || base3_len(mlo) != base3_len(mhi)) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicOr(&info->fold_overflow, 1u);
    return;
  }
  // (mapping the windows of one chunk to one XCD, for an L2 hit on the second
  // read, measured 1.6x slower: chunk-major dispatch order it is)
  const u32 w = blockIdx.y, chunk = blockIdx.x;
  if (w >= nwin) return;
  for (u32 b = threadIdx.x; b < FOLD_WIN; b += FOLD_THREADS) hist[b] = 0;
  for (u32 b = threadIdx.x; b < FOLD_WIN / 32; b += FOLD_THREADS) pres[b] = 0;
  __syncthreads();
  const u32 base = mlo + w * FOLD_WIN;
  const size_t per = ((n + FOLD_CHUNKS - 1) / FOLD_CHUNKS + 3) & ~(size_t)3;
  const size_t a = (size_t)chunk * per, e = min(n, a + per);
  // 4 messages per thread per step: one 32-bit load of flags
  for (size_t i = a + 4 * (size_t)threadIdx.x; i < e; i += 4 * FOLD_THREADS) {
    if (i + 4 <= e) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const u32 f4 = FLAGS ? __builtin_nontemporal_load(reinterpret_cast<const u32*>(flags + i)) : 0x02020202u;
      const v4u m4 = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(minute + i));
      const v4u h4 = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(hash + i));
      const u32 mm[4] = {m4.x, m4.y, m4.z, m4.w}, hh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32 off = mm[k] - base;
        if (((f4 >> (8 * k)) & EVM_MSG_XOR) && off < FOLD_WIN) {
          atomicXor(&hist[off], hh[k]);
          atomicOr(&pres[off >> 5], 1u << (off & 31));
        }
      }
    } else {
      for (size_t k = i; k < e; ++k) {
        const u32 off = minute[k] - base;
        if ((!FLAGS || (flags[k] & EVM_MSG_XOR)) && off < FOLD_WIN) {
          atomicXor(&hist[off], hash[k]);
          atomicOr(&pres[off >> 5], 1u << (off & 31));
        }
      }
    }
  }
  __syncthreads();
  const size_t slot = (size_t)w * FOLD_CHUNKS + chunk;
  for (u32 b = threadIdx.x; b < FOLD_WIN; b += FOLD_THREADS) px[slot * FOLD_WIN + b] = hist[b];
  for (u32 b = threadIdx.x; b < FOLD_WIN / 32; b += FOLD_THREADS) pp[slot * (FOLD_WIN / 32) + b] = pres[b];
}

// Per bin: XOR / OR of the chunk partials; per block of FR_THREADS bins: the
// number of present bins and the XOR of their hashes (the leaf kernel's
// output offsets and prefix-XOR carries).
constexpr int FR_THREADS = 256;
constexpr u32 FR_BLOCKS = FOLD_MAXWIN * FOLD_WIN / FR_THREADS;
__global__ __launch_bounds__(FR_THREADS) void k_cl_fold_reduce(const u32* __restrict__ px, const u32* __restrict__ pp,
                                                              const Info* __restrict__ info, u32* __restrict__ dx,
                                                              u32* __restrict__ dp, u32* __restrict__ bcnt,
                                                              u32* __restrict__ bxor) {
  __shared__ u32 tmp[FR_THREADS / 64 + 1];
  const u32 b = blockIdx.x * FR_THREADS + threadIdx.x;  // grid = FR_BLOCKS: every b < FOLD_MAXWIN * FOLD_WIN
  const u32 mlo = info->minute_min, mhi = info->minute_max;
  const bool usable = mlo <= mhi && !info->fold_overflow;
  const u32 w = b / FOLD_WIN, o = b % FOLD_WIN;
  u32 x = 0, p = 0;
  if (usable && w < (mhi - mlo) / FOLD_WIN + 1) {
    for (u32 k = 0; k < FOLD_CHUNKS; ++k) {
      const size_t slot = (size_t)w * FOLD_CHUNKS + k;
      x ^= px[slot * FOLD_WIN + o];
      p |= (pp[slot * (FOLD_WIN / 32) + (o >> 5)] >> (o & 31)) & 1u;
    }
  }
  x = p ? x : 0u;
  dx[b] = x;
  dp[b] = p;
  u32 tot, xtot;
  block_inclusive_scan<u32>(p, tmp, OpAdd<u32>(), &tot);
  block_inclusive_scan<u32>(x, tmp, OpXor<u32>(), &xtot);
  if (threadIdx.x == 0) {
    bcnt[blockIdx.x] = tot;
    bxor[blockIdx.x] = xtot;
  }
}

// Dense leaves, one bin per thread: block k's first output slot is the sum of
// the earlier blocks' counts and its prefix-XOR carry the XOR of their hashes
// (< FR_BLOCKS values, L2-resident); block scans place each leaf.  Minute
// order == code order here (one key length).  With `pfx` the leaves land
// directly in a one-owner tree: ck, xr, the exclusive prefix XOR and off.
__global__ __launch_bounds__(FR_THREADS) void k_cl_leaves(const u32* __restrict__ dx, const u32* __restrict__ dp,
                                                         const u32* __restrict__ bcnt, const u32* __restrict__ bxor,
                                                         Info* __restrict__ info, u64* __restrict__ ck,
                                                         int32_t* __restrict__ xr, int32_t* __restrict__ pfx,
                                                         u64* __restrict__ off) {
  __shared__ u32 tmp[FR_THREADS / 64 + 1];
  u32 s = 0, sx = 0;
  for (u32 k = threadIdx.x; k < blockIdx.x; k += FR_THREADS) {
    s += bcnt[k];
    sx ^= bxor[k];
  }
  u32 base, xbase;
  block_inclusive_scan<u32>(s, tmp, OpAdd<u32>(), &base);
  block_inclusive_scan<u32>(sx, tmp, OpXor<u32>(), &xbase);
  const u32 b = blockIdx.x * FR_THREADS + threadIdx.x;
  const u32 p = dp[b], x = dx[b];
  u32 tot, xtot;
  const u32 incl = block_inclusive_scan<u32>(p, tmp, OpAdd<u32>(), &tot);
  const u32 xincl = block_inclusive_scan<u32>(x, tmp, OpXor<u32>(), &xtot);
  if (p) {
    const u32 pos = base + incl - 1;
    ck[pos] = minute_code(info->minute_min + b);  // owner 0
    xr[pos] = (int32_t)x;
    if (pfx) pfx[pos] = (int32_t)(xbase ^ xincl ^ x);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const u32 L = base + tot;
    info->n_leaves = L;
    if (pfx) {
      pfx[L] = (int32_t)(xbase ^ xtot);
      off[0] = 0;
      off[1] = L;
    }
  }
}

// Fallback fold input (rare: wide minute range or mixed key lengths).
__global__ void k_cl_fold_ck(const uint8_t* __restrict__ flags, const u32* __restrict__ minute,
                             const u32* __restrict__ hash, const u32* __restrict__ pos, size_t n, u64* __restrict__ ck,
                             u32* __restrict__ h, Info* __restrict__ info) {
  u64 mn = ~0ull, mx = 0;
  u32 ml = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (!(flags[i] & EVM_MSG_XOR)) continue;
    const u64 c = minute_code(minute[i]);
    ck[pos[i]] = c;
    h[pos[i]] = hash[i];
    mn = min(mn, c);
    mx = max(mx, c);
    ml = max(ml, (u32)base3_len(minute[i]));
  }
  for (int d = 32; d >= 1; d >>= 1) {
    mn = min(mn, (u64)__shfl_xor(mn, d, 64));
    mx = max(mx, (u64)__shfl_xor(mx, d, 64));
    ml = max(ml, (u32)__shfl_xor(ml, d, 64));
  }
  if ((threadIdx.x & 63) == 0 && mx >= mn) {
    atomic_min_if(&info->ck_min, mn);
    atomic_max_if(&info->ck_max, mx);
    atomic_max_if(&info->maxlen, ml);
  }
}

__global__ void k_keep_bad(uint8_t* __restrict__ flags, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    flags[i] &= (uint8_t)EVM_MSG_BAD;
}

__global__ void k_prior_check(const evm_rec* __restrict__ prior, const uint8_t* __restrict__ present, u32 C,
                              Info* __restrict__ info) {
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C && present[c] && !(prior[c].meta & EVM_META_VALID)) atomicOr(&info->bad, 1u);
}

// ============================================================================
// tc path (the default streaming path).  Against its cell's running max t, a
// message's applyMessages decisions need only tc = millis << 16 | counter:
//     tc_i > tc(t): upsert + XOR        tc_i < tc(t): XOR only
// and only tc_i == tc(t) needs the node chars (a tie: equal millis and counter
// from two nodes, or a redelivery of the cell's current max).  Every running
// max is therefore carried as (tc, row) -- the row that holds it, or the
// prior max, or none -- and a tie compares the two timestamps' node ranks,
// read from the rows' bytes (applyMessages.ts:93 `t < timestamp`, :105
// `t !== timestamp`, string order).
//   TP1 k_tp_pack : K1 (parse, canonical check, murmur3, minute) + per (range,
//                   cell) the max tc in LDS and its row; cells where two rows
//                   share that max (or the row record raced) are resolved by
//                   node rank in a short rescan of the range
//   TP2 carry     : per cell, exclusive max over the ranges seeded with the
//                   prior max; the cell's final max -> its winner (the first
//                   occurrence of the final max key, applyMessages.ts:93)
//   TP3 k_tp_walk : a workgroup per range: rows below their cell's running max
//                   decided on the spot; the rest walked in batch order (LDS
//                   state) -> flags
// Bytes per message: TP1 46 + 4 in, 16 out; TP3 12 in, 1 out.
// ============================================================================
constexpr u64 TP_INVALID = ~0ull;  // tc of a message the walk skips (invalid timestamp or cell id)
constexpr u32 XF_SPAN_MAX = FOLD_MAXWIN * FOLD_WIN;  // minutes of the fused fold's dense arrays (k_cl_leaves)
// TP1's per-row word for the walk and the fused check: cell << 49 | millis << 8
// | counter while millis < 2^41 and counter < 256 (every row of a batch before
// 2039-09 with < 256 sends per node and millisecond), so neither reads the
// cell column again; any other valid row is TP_FAR with its tc in a side
// array (and its cell from the column).  The order of (millis, counter) is kept.
constexpr u64 TP_FAR = ~0ull - 1ull;
constexpr int TPC_CELL = 49;
__device__ __forceinline__ u64 tpc_pack(u64 tc, u32 c) {
  return ((u64)c << TPC_CELL) | ((tc >> 16) << 8) | (tc & 0xffull);
}
__device__ __forceinline__ void tpc_unpack(u64 v, const u64* __restrict__ far, const u32* __restrict__ cell, size_t i,
                                           u64* tc, u32* c) {
  if (v == TP_FAR) {
    *tc = far[i];
    *c = cell[i];
  } else {
    const u64 low = v & ((1ull << TPC_CELL) - 1ull);
    *tc = ((low >> 8) << 16) | (low & 0xffull);
    *c = (u32)(v >> TPC_CELL);
  }
}
__device__ __forceinline__ u32 minute_of_tc(u64 tc) { return (u32)((tc >> 16) / 60000ull); }
constexpr int TP_THREADS = 256;
constexpr int TP_RANGES = 2048;  // ~8 ranges per CU: TP1's occupancy
constexpr u32 ROW_NONE = 0xffffffffu;   // no max (SQL NULL: below every timestamp)
constexpr u32 ROW_PRIOR = 0xfffffffeu;  // the max is the caller's prior row of the cell
constexpr u32 TP_MATCH_MAX = 512;       // TP1 rescan: rows tied at a cell's range max

// Node ranks (OKey rh, rl) of a batch row: chars 30..45 of its timestamp.
struct NodeSrc {
  const uint8_t* ts;
  size_t stride;
  const evm_rec* prior;  // per cell (ROW_PRIOR)
};
__device__ __forceinline__ void node_ranks_of(const NodeSrc& N, u32 c, u32 row, u64* rh, u32* rl) {
  if (row == ROW_PRIOR) {
    const evm_rec& p = N.prior[c];
    node_rank(p.node, p.meta & EVM_META_CASEMASK, rh, rl);
    return;
  }
  const uint8_t* s = N.ts + (size_t)row * N.stride;
  u32 w[5];  // words 7..11 of the string (bytes 28..47; 46, 47 unused)
  if ((N.stride & 3) == 0 && N.stride >= 48) {
    const u32* p = reinterpret_cast<const u32*>(s + 28);
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = p[k];
  } else {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      u32 x = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (28 + 4 * k + j < 46) x |= (u32)s[28 + 4 * k + j] << (8 * j);
      w[k] = x;
    }
  }
  u64 h = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) h = (h << 20) | swar_rank20((w[k] >> 16) | (w[k + 1] << 16));
  *rh = h;
  *rl = swar_rank20((w[3] >> 16) | (w[4] << 16));
}

// A carried max: (tc, row).  Order = the timestamps' string order; ROW_NONE
// below everything; equal timestamps: the earlier one (prior, then the lower
// row) -- so the carried row of the final max is the first occurrence.
struct TK {
  u64 tc;
  u32 row;
};
__device__ __forceinline__ int tk_cmp(const NodeSrc& N, u32 c, const TK& a, const TK& b) {
  if (a.row == ROW_NONE) return b.row == ROW_NONE ? 0 : -1;
  if (b.row == ROW_NONE) return 1;
  if (a.tc != b.tc) return a.tc < b.tc ? -1 : 1;
  if (a.row == b.row) return 0;
  u64 ha, hb;
  u32 la, lb;
  node_ranks_of(N, c, a.row, &ha, &la);
  node_ranks_of(N, c, b.row, &hb, &lb);
  if (ha != hb) return ha < hb ? -1 : 1;
  if (la != lb) return la < lb ? -1 : 1;
  return 0;
}
__device__ __forceinline__ u32 tk_earlier(u32 a, u32 b) {
  if (a == ROW_PRIOR || b == ROW_PRIOR) return ROW_PRIOR;
  return a < b ? a : b;
}
__device__ __forceinline__ TK tk_max(const NodeSrc& N, u32 c, const TK& a, const TK& b) {
  const int k = tk_cmp(N, c, a, b);
  if (k > 0) return a;
  if (k < 0) return b;
  return TK{a.tc, tk_earlier(a.row, b.row)};
}
__device__ __forceinline__ TK shfl_tk(const TK& k, int src) {
  TK o;
  o.tc = ((u64)(u32)__shfl((int)(u32)(k.tc >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)k.tc, src, 64);
  o.row = (u32)__shfl((int)k.row, src, 64);
  return o;
}

// TP1: K1 + per (range, cell) the max tc and the row holding it.  One LDS
// 64-bit max per row on key = millis << 21 | counter << 13 | (8191 - row
// offset): exact for millis < 2^41 (until 2039-09), counter < 256 and ranges
// of <= 8,192 rows -- the largest key is the range's max tc at its first row.
// A row outside that (far) or a second row at a max tc (ds_max returns the key
// it replaced: equal tc bits) marks its cell; marked cells are resolved by a
// rescan of the range (true max tc, then the node ranks of the rows at it).
constexpr int TP_WPE = 8;  // waves per SIMD TP1 is compiled for (7: no spills, measured no faster)

constexpr u32 TP_ROWS_MAX = 8192;  // rows per range (the key's 13-bit row offset)

// Range g of the tc path.  The batch's first L rows are cut into five
// geometric sub-ranges (q, q, 2q, 4q, L - 8q; q = L/16 rounded down to 64):
// in the first rows every row is a candidate of the walk (no earlier maximum
// of its cell exists), so a full-length first range would hold the walk's
// longest serial chain; each sub-range starts from the maxima of all earlier
// ones.  Then ranges of L.  G' = ceil(n / L) + 4.
struct TpRanges {
  size_t L, q;
};
__host__ __device__ __forceinline__ void tp_range(const TpRanges& R, size_t g, size_t n, size_t* beg, size_t* end) {
  size_t b, e;
  if (g < 5) {
    b = g == 0 ? 0 : R.q << (g - 1);
    e = g == 4 ? R.L : R.q << g;
  } else {
    b = (g - 4) * R.L;
    e = b + R.L;
  }
  *beg = b < n ? b : n;
  *end = e < n ? e : n;
}
constexpr u64 TP_MS_FAST = 1ull << 41;

template <bool S48>
__global__ __launch_bounds__(TP_THREADS) __attribute__((amdgpu_waves_per_eu(TP_WPE, 8))) void k_tp_pack(const uint8_t* __restrict__ ts, size_t stride, size_t n,
                                                        const u32* __restrict__ cell, u32 C, TpRanges R,
                                                        u64* __restrict__ tcs, u64* __restrict__ tcs_far,
                                                        u32* __restrict__ hash, u64* __restrict__ agg,
                                                        u32* __restrict__ arow, Info* __restrict__ info,
                                                        u32* __restrict__ zero_buf, u32 zero_n,
                                                        u32* __restrict__ fold_zero, u32 fold_zero_n) {
  // LDS: [C] max key per cell of this range, [ceil(C/32)] the marked cells
  extern __shared__ __attribute__((aligned(16))) u64 cmax[];
  u32* cfix = reinterpret_cast<u32*>(cmax + C);
  // (the cross-cell check's bucket cursors, cleared here instead of by a
  // memset on the second stream, which forks after this kernel)
  if (blockIdx.x == 0)
    for (u32 k = threadIdx.x; k < zero_n; k += TP_THREADS) zero_buf[k] = 0u;
  // (and the fused fold's dense minute arrays, which the dedup kernel and the
  // walk add into afterwards -- a slice per workgroup)
  for (u32 k = blockIdx.x * TP_THREADS + threadIdx.x; k < fold_zero_n; k += gridDim.x * TP_THREADS) fold_zero[k] = 0u;
  __shared__ uint4 stage[TP_THREADS / 64][192];
  __shared__ u32 nmatch;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u32 bad = 0, aux_bad = 0, mn = 0xffffffffu, mx = 0;
  const size_t g = blockIdx.x;
  size_t beg, end;
  tp_range(R, g, n, &beg, &end);
  for (u32 c = threadIdx.x; c < C; c += TP_THREADS) cmax[c] = 0;
  for (u32 k = threadIdx.x; k < (C + 31) / 32; k += TP_THREADS) cfix[k] = 0;
  if (threadIdx.x == 0) nmatch = 0;
  __syncthreads();
  for (size_t first = beg + 64 * wv; first < end; first += TP_THREADS) {  // wave-uniform
    uint4 a, b, c;
    clp_fetch<S48>(ts, stride, end, first, a, b, c);
    const size_t i = first + lane;
    u32 w[12];
    if (S48) {
      stage[wv][lane] = a;
      stage[wv][lane + 64] = b;
      stage[wv][lane + 128] = c;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const uint4 x = stage[wv][3 * lane], y = stage[wv][3 * lane + 1], z = stage[wv][3 * lane + 2];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
      w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
      w[8] = z.x; w[9] = z.y; w[10] = z.z; w[11] = z.w & 0xffffu;
    } else {
      w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
      w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
      w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w & 0xffffu;
    }
    Parsed p = parse_ts46(w);  // (the node ranks it can compute are dead here)
    const bool valid = (p.meta & EVM_META_VALID) != 0;
    if (i < end) {
      const u32 ci = __builtin_nontemporal_load(cell + i);
      const bool ok = valid && ci < C;
      const bool fast = (p.tc >> 16) < TP_MS_FAST && ((u32)p.tc & 0xffffu) < 256u;
      __builtin_nontemporal_store(!ok ? TP_INVALID : fast ? tpc_pack(p.tc, ci) : TP_FAR, tcs + i);
      if (ok && !fast) tcs_far[i] = p.tc;
      if (!ok) p.minute = 0xffffffffu;  // outside every fold window (and the minute bounds)
      if (ok) {
        const u64 ms = p.tc >> 16;
        const u32 ctr = (u32)p.tc & 0xffffu;
        bool mark = true;  // far
        if (ms < TP_MS_FAST && ctr < 256u) {
          const u64 key = (ms << 21) | ((u64)ctr << 13) | (u64)(TP_ROWS_MAX - 1u - (u32)(i - beg));
          mark = (atomicMax(&cmax[ci], key) >> 13) == (key >> 13);  // a second row at this tc (or tc 0)
        }
        if (mark) atomicOr(&cfix[ci >> 5], 1u << (ci & 31));
      }
      bad |= valid ? 0u : 1u;
      aux_bad |= ci < C ? 0u : 1u;
    }
    // (the wave's 64 hashes are one contiguous 256-B store; the minute is not
    // stored: the fused check + fold re-derives it from tc)
    if (i < end) hash[i] = p.hash;
    // (lanes past the range end parsed zero bytes: their minute must not
    // widen the bounds, or the dense fold of a batch whose size is not a
    // multiple of 64 overflows into the sort-based fold)
    const bool in = i < end;
    mn = min(mn, in ? p.minute : 0xffffffffu);
    mx = max(mx, in && p.minute != 0xffffffffu ? p.minute : 0u);
  }
  __syncthreads();
  // the unmarked cells: tc and row straight from the key
  for (u32 c = threadIdx.x; c < C; c += TP_THREADS) {
    if ((cfix[c >> 5] >> (c & 31)) & 1u) continue;
    const u64 k = cmax[c];
    agg[g * C + c] = k ? (((k >> 21) << 16) | ((k >> 13) & 0xffu)) : 0ull;
    arow[g * C + c] = k ? (u32)(beg + (TP_ROWS_MAX - 1u - (u32)(k & (TP_ROWS_MAX - 1u)))) : ROW_NONE;
  }
  bool any_fix = false;
  for (u32 k = threadIdx.x; k < (C + 31) / 32; k += TP_THREADS) any_fix |= cfix[k] != 0;
  if (__syncthreads_or(any_fix)) {
    // rescan (rare): the marked cells' true max tc, then their rows at it with
    // their node ranks into LDS (the stage is free now), then per cell the
    // best: highest node ranks, the lowest row among equals
    struct Match {
      u64 rh;
      u32 rl, row, cell, pad;
    };
    Match* mt = reinterpret_cast<Match*>(&stage[0][0]);
    static_assert(sizeof(stage) >= TP_MATCH_MAX * sizeof(Match), "match list fits the stage");
    auto marked = [&](u32 c) { return ((cfix[c >> 5] >> (c & 31)) & 1u) != 0; };
    for (u32 c = threadIdx.x; c < C; c += TP_THREADS)
      if (marked(c)) cmax[c] = 0;
    __syncthreads();
    for (size_t i = beg + threadIdx.x; i < end; i += TP_THREADS) {
      const u64 v = __hip_atomic_load(tcs + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // written above
      if (v == TP_INVALID) continue;
      u64 t;
      u32 ci;
      tpc_unpack(v, tcs_far, cell, i, &t, &ci);
      if (marked(ci)) atomicMax(&cmax[ci], t);
    }
    __syncthreads();
    const NodeSrc N{ts, stride, nullptr};
    for (size_t i = beg + threadIdx.x; i < end; i += TP_THREADS) {
      const u64 v = __hip_atomic_load(tcs + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == TP_INVALID) continue;
      u64 t;
      u32 ci;
      tpc_unpack(v, tcs_far, cell, i, &t, &ci);
      if (!marked(ci) || t != cmax[ci]) continue;
      const u32 k = atomicAdd(&nmatch, 1u);
      if (k < TP_MATCH_MAX) {
        Match m;
        node_ranks_of(N, ci, (u32)i, &m.rh, &m.rl);
        m.row = (u32)i;
        m.cell = ci;
        m.pad = 0;
        mt[k] = m;
      }
    }
    __syncthreads();
    const u32 nm = nmatch;
    if (nm > TP_MATCH_MAX) {
      // too many: the exact walk path redoes the batch; until then the carry
      // and the walk must read in-bounds rows (no row: NONE)
      if (threadIdx.x == 0) atomicOr(&info->ties, 1u);
      for (u32 c = threadIdx.x; c < C; c += TP_THREADS)
        if (marked(c)) {
          agg[g * C + c] = 0;
          arow[g * C + c] = ROW_NONE;
        }
    } else {
      for (u32 k = threadIdx.x; k < nm; k += TP_THREADS) {
        const Match e = mt[k];
        bool best = true;
        for (u32 f = 0; f < nm && best; ++f) {
          const Match o = mt[f];
          if (f == k || o.cell != e.cell) continue;
          best = !(o.rh > e.rh || (o.rh == e.rh && (o.rl > e.rl || (o.rl == e.rl && o.row < e.row))));
        }
        if (best) {
          agg[g * C + e.cell] = cmax[e.cell];
          arow[g * C + e.cell] = e.row;
        }
      }
    }
  }
  if (__ballot(aux_bad) && lane == 0) atomicOr(&info->bad_aux, 1u);
  block_fold_bounds<u32, TP_THREADS>(mn, mx, bad, &info->minute_min, &info->minute_max, &info->bad);
}

// TP2: per cell, the exclusive max over the G range maxima seeded with the
// prior max, and the final max -> winner.  One workgroup per CT_CELLS cells:
// each of its CT_GROUPS lane groups reduces a contiguous segment of ranges
// (CT_CELLS consecutive cells = one 64-B read per range), one wave per cell
// scans the segment maxima in LDS (two per lane), and the groups write their
// segment's running maxima.  A segment of <= CT_CACHE ranges (G <= 2,048:
// the headline) is loaded once, every load in flight at once, and kept in
// registers for the write-back; equal tc in two ranges (rare: the node ranks
// decide) sends the lane to the exact loop, which re-reads memory.
constexpr u32 CT_CELLS = 8, CT_GROUPS = 128, CT_THREADS = CT_CELLS * CT_GROUPS;
constexpr int CT_BATCH = 8, CT_CACHE = 16;

__global__ __launch_bounds__(CT_THREADS) void k_tp_carry(u32 C, size_t G, u64* __restrict__ agg,
                                                         u32* __restrict__ arow, NodeSrc N,
                                                         const uint8_t* __restrict__ prior_present,
                                                         int32_t* __restrict__ winner) {
  __shared__ u64 s_tc[CT_GROUPS][CT_CELLS];
  __shared__ u32 s_row[CT_GROUPS][CT_CELLS];
  const u32 cl = threadIdx.x % CT_CELLS, grp = threadIdx.x / CT_CELLS;
  const u32 c = blockIdx.x * CT_CELLS + cl;
  const bool ok = c < C;
  const u32 cc = ok ? c : C - 1;  // (loads stay in bounds; the lane writes nothing)
  const size_t per = (G + CT_GROUPS - 1) / CT_GROUPS;
  const size_t a = min(G, grp * per), e = min(G, a + per);
  // (a range without rows holds (0, ROW_NONE); a row of tc 0 ties with it and
  // takes the exact loop, which ranks NONE below every row)
  const bool cached = per <= CT_CACHE;
  u64 tcache[CT_CACHE];
  u32 rcache[CT_CACHE];
  TK m{0, ROW_NONE};
  bool tie = false;
  if (cached) {
#pragma unroll
    for (int k = 0; k < CT_CACHE; ++k) {
      const size_t g = a + k;
      const size_t gi = min(g, G - 1) * C + cc;
      const u64 t = agg[gi];
      const u32 r = arow[gi];
      tcache[k] = g < e ? t : 0ull;
      rcache[k] = g < e ? r : ROW_NONE;
    }
#pragma unroll
    for (int k = 0; k < CT_CACHE; ++k) {
      if (tcache[k] > m.tc) m = TK{tcache[k], rcache[k]};
      else if (tcache[k] == m.tc && rcache[k] != m.row) tie = true;
    }
  }
  if (ok && (!cached || tie)) {
    m = TK{0, ROW_NONE};
    for (size_t g0 = a; g0 < e; g0 += CT_BATCH) {
      u64 t[CT_BATCH];
      u32 r[CT_BATCH];
#pragma unroll
      for (int k = 0; k < CT_BATCH; ++k) {
        const size_t g = g0 + k;
        t[k] = g < e ? agg[g * C + c] : 0ull;
        r[k] = g < e ? arow[g * C + c] : ROW_NONE;
      }
#pragma unroll
      for (int k = 0; k < CT_BATCH; ++k) {
        const TK x{t[k], r[k]};
        if (x.tc > m.tc) m = x;
        else if (x.tc == m.tc && x.row != m.row) m = tk_max(N, c, m, x);  // (rare: equal tc in two ranges)
      }
    }
  }
  s_tc[grp][cl] = m.tc;
  s_row[grp][cl] = m.row;
  __syncthreads();
  {
    // one wave per cell; lane l holds segments 2l and 2l + 1
    const u32 w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const u32 cw = blockIdx.x * CT_CELLS + w;
    static_assert(CT_GROUPS == 128 && CT_THREADS / 64 >= CT_CELLS, "one wave per cell, two groups per lane");
    if (w < CT_CELLS && cw < C) {
      const TK v0{s_tc[2 * lane][w], s_row[2 * lane][w]}, v1{s_tc[2 * lane + 1][w], s_row[2 * lane + 1][w]};
      TK v = tk_max(N, cw, v0, v1);
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const TK u = shfl_tk(v, (int)lane - d < 0 ? (int)lane : (int)lane - d);
        if ((int)lane >= d) v = tk_max(N, cw, u, v);
      }
      const TK seed = (prior_present && prior_present[cw]) ? TK{N.prior[cw].tc, ROW_PRIOR} : TK{0, ROW_NONE};
      const TK ex = shfl_tk(v, lane == 0 ? 0 : (int)lane - 1);
      const TK x0 = lane == 0 ? seed : tk_max(N, cw, seed, ex);  // before segment 2l
      const TK x1 = tk_max(N, cw, x0, v0);                       // before segment 2l + 1
      s_tc[2 * lane][w] = x0.tc;
      s_row[2 * lane][w] = x0.row;
      s_tc[2 * lane + 1][w] = x1.tc;
      s_row[2 * lane + 1][w] = x1.row;
      if (lane == 63) {
        // the last upsert is the first occurrence of the final max (none if
        // the prior max or nothing holds it)
        const TK f = tk_max(N, cw, seed, v);
        winner[cw] = (f.row == ROW_NONE || f.row == ROW_PRIOR) ? -1 : (int32_t)f.row;
      }
    }
  }
  __syncthreads();
  if (!ok) return;
  TK run{s_tc[grp][cl], s_row[grp][cl]};
  if (cached && !tie) {
    // the running max by tc alone unless it meets an equal tc (then the
    // exact loop, from memory: nothing is written before this check)
    u64 rt = run.tc;
    u32 rr = run.row;
#pragma unroll
    for (int k = 0; k < CT_CACHE; ++k) {
      if (tcache[k] > rt) {
        rt = tcache[k];
        rr = rcache[k];
      } else if (tcache[k] == rt && rcache[k] != rr) {
        tie = true;
      }
    }
    if (!tie) {
#pragma unroll
      for (int k = 0; k < CT_CACHE; ++k) {
        const size_t g = a + k;
        if (g < e) {
          agg[g * C + c] = run.tc;
          arow[g * C + c] = run.row;
        }
        if (tcache[k] > run.tc) run = TK{tcache[k], rcache[k]};
      }
      return;
    }
  }
  for (size_t g0 = a; g0 < e; g0 += CT_BATCH) {
    u64 t[CT_BATCH];
    u32 r[CT_BATCH];
#pragma unroll
    for (int k = 0; k < CT_BATCH; ++k) {
      const size_t g = g0 + k;
      t[k] = g < e ? agg[g * C + c] : 0ull;
      r[k] = g < e ? arow[g * C + c] : ROW_NONE;
    }
#pragma unroll
    for (int k = 0; k < CT_BATCH; ++k) {
      const size_t g = g0 + k;
      if (g < e) {
        agg[g * C + c] = run.tc;
        arow[g * C + c] = run.row;
      }
      const TK here{t[k], r[k]};
      if (here.tc > run.tc) run = here;
      else if (here.tc == run.tc && here.row != run.row) run = tk_max(N, c, run, here);
    }
  }
}

// TP3: one workgroup per range, the range in chunks of TPC_ROWS rows.  A row
// whose tc is below its cell's running max at the chunk start is decided on
// the spot (XOR only: applyMessages.ts:105 holds, :93 does not) -- in a
// shuffled stream that is nearly every row, so the pass streams at HBM speed.
// The rest (tc >= that max: possible new maxima, ties) are compacted in
// batch order into LDS and walked by one wave: 64 candidates per round, the
// round's lanes of each cell found through an LDS mask per cell (each lane
// ORs its bit in, reads the mask back, clears it), each lane takes the max of
// its lower peers (a wave prefix-max when the round is one cell), t =
// max(running max, that) decides its flags, and the round's last peer of the
// cell writes the new max.  Keys are (tc, row): equal tc compares node ranks
// (tk_cmp), so a tie costs two 16-byte reads.  An ascending stream makes
// every row a candidate and costs one walk.
constexpr int TP_WAVES = TP_THREADS / 64;
constexpr u32 TPC_ROWS = 64 * 4 * TP_WAVES;  // 4 rounds per wave per chunk

__global__ __launch_bounds__(TP_THREADS) void k_tp_walk(const u64* __restrict__ tcs, const u64* __restrict__ tcs_far,
                                                        const u32* __restrict__ cell,
                                                        size_t n, u32 C, TpRanges R,
                                                        const u64* __restrict__ carry, const u32* __restrict__ crow,
                                                        NodeSrc N, uint8_t* __restrict__ flags,
                                                        const u32* __restrict__ hash, u32* __restrict__ dx,
                                                        u32* __restrict__ dc, const Info* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) u64 tw_lds[];
  u64* T = tw_lds;                                       // [C] running max per cell: tc
  u64* M = T + C;                                        // [C] the walk round's lanes per cell (zero between rounds)
  u64* cx = M + C;                                       // [TPC_ROWS] candidates: tc
  u32* ci = reinterpret_cast<u32*>(cx + TPC_ROWS);       // [TPC_ROWS] row index
  uint16_t* cc = reinterpret_cast<uint16_t*>(ci + TPC_ROWS);  // [TPC_ROWS] cell
  u32* TR = reinterpret_cast<u32*>(cc + TPC_ROWS);       // [C] running max per cell: row
  __shared__ u32 seg[TP_WAVES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u64 lt = lanemask_lt();
  const size_t g = blockIdx.x;
  size_t beg, end;
  tp_range(R, g, n, &beg, &end);
  for (u32 c = threadIdx.x; c < C; c += TP_THREADS) {
    T[c] = carry[g * C + c];
    TR[c] = crow[g * C + c];
    M[c] = 0;
  }
  __syncthreads();
  for (size_t base = beg; base < end; base += TPC_ROWS) {
    // classify this wave's 256 rows; compact the candidates in batch order
    const size_t wb = base + 256 * wv;
    u64 x[4];
    u32 c[4];
    u64 v[4];  // (all four loads in flight before any decode)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t i = wb + 64 * r + lane;
      v[r] = i < end ? __builtin_nontemporal_load(tcs + i) : TP_INVALID;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const u64 low = v[r] & ((1ull << TPC_CELL) - 1ull);
      x[r] = v[r] == TP_INVALID ? TP_INVALID : ((low >> 8) << 16) | (low & 0xffull);
      c[r] = v[r] == TP_INVALID ? 0u : (u32)(v[r] >> TPC_CELL);
    }
    if (__any(v[0] == TP_FAR || v[1] == TP_FAR || v[2] == TP_FAR || v[3] == TP_FAR)) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (v[r] == TP_FAR) tpc_unpack(v[r], tcs_far, cell, wb + 64 * r + lane, &x[r], &c[r]);
    }
    u32 wcnt = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t i = wb + 64 * r + lane;
      const bool ok = x[r] != TP_INVALID;
      // (a cell without a max yet: TR == ROW_NONE and T == 0, every row a candidate)
      const bool cand = ok && x[r] >= T[c[r]];
      if (i < end && !cand) flags[i] = ok ? (uint8_t)EVM_MSG_XOR : (uint8_t)EVM_MSG_BAD;
      const u64 bal = __ballot(cand);
      if (cand) {
        const u32 k = 256 * wv + wcnt + (u32)__popcll(bal & lt);
        cx[k] = x[r];
        ci[k] = (u32)i;
        cc[k] = (uint16_t)c[r];
      }
      wcnt += (u32)__popcll(bal);
    }
    if (lane == 0) seg[wv] = wcnt;
    __syncthreads();
    if (wv == 0) {
      u32 s0 = seg[0], s1 = seg[1], s2 = seg[2], s3 = seg[3];
      const u32 total = s0 + s1 + s2 + s3;
      for (u32 k0 = 0; k0 < total; k0 += 64) {  // uniform
        const u32 k = k0 + lane;
        // candidate k of the concatenated wave segments
        u32 q = k;
        int sg = 0;
        if (q >= s0) {
          q -= s0;
          sg = 1;
          if (q >= s1) {
            q -= s1;
            sg = 2;
            if (q >= s2) {
              q -= s2;
              sg = 3;
            }
          }
        }
        const bool ok = k < total;
        const u32 slot = 256 * sg + q;
        const TK own{ok ? cx[slot] : 0ull, ok ? ci[slot] : ROW_NONE};
        const u32 cv = ok ? cc[slot] : 0u;
        if (ok) atomicOr(&M[cv], 1ull << lane);
        const u64 peers = ok ? __hip_atomic_load(&M[cv], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) : 0ull;
        if (ok) __hip_atomic_store(&M[cv], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const u64 act = __ballot(ok);
        TK pm{0, ROW_NONE};  // max key of the lower lanes of the same cell
        if (peers == act && act == ~0ull) {
          TK v = own;  // the round is one cell: exclusive wave prefix max
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const TK u = shfl_tk(v, lane >= d ? lane - d : lane);
            if (lane >= d) v = tk_max(N, cv, u, v);
          }
          pm = shfl_tk(v, lane >= 1 ? lane - 1 : lane);
          if (lane == 0) pm = TK{0, ROW_NONE};
        } else {
          u64 rem = peers & lt;
          while (__any(rem != 0)) {
            const int src = rem ? (int)__builtin_ctzll(rem) : lane;
            const TK v = shfl_tk(own, src);
            if (rem) {
              pm = tk_max(N, cv, pm, v);
              rem &= rem - 1;
            }
          }
        }
        int k3 = 1;
        if (ok) {
          const TK t = tk_max(N, cv, TK{T[cv], TR[cv]}, pm);
          k3 = tk_cmp(N, cv, own, t);
          // applyMessages.ts:93 `t < timestamp` -> upsert; :105 `t !== timestamp` -> INSERT + XOR
          flags[own.row] = k3 > 0 ? (uint8_t)(EVM_MSG_UPS | EVM_MSG_XOR) : k3 < 0 ? (uint8_t)EVM_MSG_XOR : (uint8_t)0;
          if ((peers >> lane) == 1ull) {  // the round's last peer of the cell
            const TK nt = k3 > 0 ? own : t;
            T[cv] = nt.tc;
            TR[cv] = nt.row;
          }
        }
        // an exact redelivery of the cell's max is the one row applyMessages.ts:105
        // does not XOR: out of the fused fold again (the dedup kernel XORs every
        // row; XOR and add commute, so the order against it does not matter)
        if (ok && k3 == 0) {
          const u32 mlo = info->minute_min, span = info->minute_max - mlo + 1u;
          const u32 d = minute_of_tc(own.tc) - mlo;
          if (span <= XF_SPAN_MAX && d < span) {
            atomicXor(&dx[d], hash[own.row]);
            atomicSub(&dc[d], 1u);
          }
        }
      }
    }
    __syncthreads();
  }
}

// ============================================================================
// XF: the tc path's cross-cell PK check fused with its Merkle fold.
//
// Messages are bucketed by MINUTE (contiguous minute ranges; a batch spanning
// fewer minutes than buckets splits each minute by hash bits), so one bucket
// holds every copy of a timestamp AND every message of its minutes: the
// bucket's workgroup checks the global `__message` PK in an LDS set and XORs
// the hashes into an LDS histogram of its minutes.  The fold XORs EVERY row;
// the rows the walk finds to be exact redeliveries of their cell's max (the
// only rows applyMessages.ts:105 does not XOR) are XORed out again afterwards
// (k_xf_fix) -- XOR is its own inverse, the presence count drops by one.
//
// The LDS set compares 64-bit fingerprints instead of the 46 raw bytes: a
// pair is hash32 | minute offset | tc bits | cell, so two copies of one
// timestamp carry equal fingerprints.  Equal fingerprints in two different
// cells are a *possible* collision: the batch is redone by the exact walk
// path, whose byte-exact check decides (two distinct timestamps need equal
// murmur3 AND equal minute AND equal mixed tc bits to get there).  A bucket
// that overflows, a span above XF_SPAN_MAX or two base-3 key lengths also
// redo the batch (`xf_redo`).  Bytes per message: scatter 16 in + 8 out,
// dedup + fold 8 in.
// ============================================================================
constexpr int XF_MIN_KB = 6;                         // >= 64 buckets
constexpr u32 XF_WMAX = XF_SPAN_MAX / (1u << XF_MIN_KB) + 2;  // minutes one bucket can touch (its LDS histogram)

// A message's place on the minute axis is K = d + hash / 2^32 (d = minute -
// mlo), and bucket b covers K in [b, b + 1) * span / B: equal lengths of the
// axis, so a batch spread over its minutes fills the buckets evenly whether
// it spans many minutes per bucket or many buckets per minute.  Every copy
// of a timestamp has one K.  floor(K * B) = d << kb | hash >> (32 - kb) is an
// exact integer below 2^28, divided by span with a multiply-high.
struct XfGeom {
  u32 mlo, span, magic;  // minutes [mlo, mlo + span); magic = ceil(2^32 / span) (span > 1)
  int kb, mb, xb, cb;    // bucket bits, minute-offset bits, tc bits, cell bits of a pair
  u32 W;                 // minutes a bucket can touch
  bool ok;
};
__device__ __forceinline__ XfGeom xf_geom(const Info* info, int kb, int cbits) {
  XfGeom g;
  g.mlo = info->minute_min;
  const u32 mhi = info->minute_max;
  g.ok = g.mlo <= mhi;
  g.span = g.ok ? mhi - g.mlo + 1u : 1u;
  g.ok = g.ok && g.span <= XF_SPAN_MAX && base3_len(g.mlo) == base3_len(mhi);
  if (!g.ok) g.span = 1;
  g.kb = kb;
  g.magic = g.span > 1 ? (u32)((0x100000000ull + g.span - 1) / g.span) : 0u;
  g.W = ((g.span + (1u << kb) - 1) >> kb) + 1u;
  g.mb = 32 - __builtin_clz(g.W - 1);  // W >= 2
  g.cb = cbits;
  g.xb = 32 - g.mb - cbits;
  return g;
}
__device__ __forceinline__ u32 xf_first_minute(const XfGeom& g, u32 b) { return (b * g.span) >> g.kb; }

// (d = minute - mlo, hash, tc, cell) -> bucket and pair (hash32 | minute
// offset in the bucket | mixed tc bits | cell)
__device__ __forceinline__ u64 xf_pair(const XfGeom& g, u32 d, u32 h, u64 tc, u32 c, u32* bucket) {
  const u32 N = (d << g.kb) | (g.kb ? h >> (32 - g.kb) : 0u);
  u32 b = N;
  if (g.span > 1) {
    b = __umulhi(N, g.magic);  // floor(N / span) or one above
    if (b * g.span > N) --b;
  }
  *bucket = b;
  const u32 moff = d - xf_first_minute(g, b);
  const u32 x = ((u32)tc ^ (u32)(tc >> 32)) * 0x9E3779B1u;  // every tc bit mixed into the top bits
  const u32 lo = (moff << (32 - g.mb)) | ((x >> (32 - g.xb)) << g.cb) | c;
  return ((u64)h << 32) | lo;
}


// d = minute(tc) - mlo without a 64-bit division: rel = millis - mlo * 60000
// fits 32 bits while the span is <= XF_SPAN32 minutes, and (rel >> 5) / 1875
// is exact as a multiply-high below 2^27 (M = ceil(2^42 / 1875)).
constexpr u32 XF_SPAN32 = 71582;  // floor(2^32 / 60000)
__device__ __forceinline__ u32 xf_minute_off(u64 tc, u64 base_ms, u32 mlo, bool narrow) {
  if (narrow) return __umulhi((u32)(((tc >> 16) - base_ms) >> 5), 2345624806u) >> 10;
  return minute_of_tc(tc) - mlo;
}

// A tile of THREADS x ITEMS pairs is staged in LDS with its bucket ids and
// written back bucket by bucket (EVM_XF_SCATTER picks the shape).
template <int THREADS, int ITEMS>
__global__ __launch_bounds__(THREADS) void k_xf_scatter(const u32* __restrict__ hash, const u64* __restrict__ tcs,
                                                          const u64* __restrict__ tcs_far,
                                                          const u32* __restrict__ cell, size_t n, int kb, int cbits,
                                                          u32 cap, u32* __restrict__ cursor, u64* __restrict__ out,
                                                          Info* __restrict__ info, u32 tl) {
  __shared__ u64 stage[(THREADS * ITEMS)];
  __shared__ uint16_t sbk[(THREADS * ITEMS)];      // the bucket of each staged pair
  __shared__ u32 cnt[1u << XP_MAX_KB];  // per bucket: count, then local offset
  __shared__ u32 gb[1u << XP_MAX_KB];   // per bucket: this tile's base inside the bucket
  __shared__ u32 scan_tmp[THREADS / 64 + 1];
  const XfGeom g = xf_geom(info, kb, cbits);
  if (!g.ok) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&info->xf_redo, 1u);
    return;
  }
  const u32 B = 1u << kb;
  const bool narrow = g.span <= XF_SPAN32;
  const u64 base_ms = (u64)g.mlo * 60000ull;
  for (u32 b = threadIdx.x; b < B; b += THREADS) cnt[b] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * tl;  // (tl <= THREADS * ITEMS rows per tile)
  u64 v[ITEMS];
  u32 bk[ITEMS], r[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const u32 t = (u32)k * THREADS + threadIdx.x;
    const size_t i = t < tl ? base + t : n;
    const u64 tv = i < n ? __builtin_nontemporal_load(tcs + i) : TP_INVALID;
    const u32 h = i < n ? __builtin_nontemporal_load(hash + i) : 0u;
    bk[k] = B;  // none (an invalid row: the batch is rejected anyway)
    v[k] = 0;
    if (tv != TP_INVALID) {
      const u64 low = tv & ((1ull << TPC_CELL) - 1ull);
      u64 tc = ((low >> 8) << 16) | (low & 0xffull);
      u32 c = (u32)(tv >> TPC_CELL);
      if (tv == TP_FAR) tpc_unpack(tv, tcs_far, cell, i, &tc, &c);
      v[k] = xf_pair(g, xf_minute_off(tc, base_ms, g.mlo, narrow), h, tc, c, &bk[k]);
    }
    r[k] = bk[k] < B ? atomicAdd(&cnt[bk[k]], 1u) : 0u;
  }
  __syncthreads();
  const u32 per = (B + THREADS - 1) / THREADS;
  u32 loc[(1u << XP_MAX_KB) / THREADS];
  u32 sum = 0;
  for (u32 k = 0; k < per; ++k) {
    const u32 b = threadIdx.x * per + k;
    loc[k] = b < B ? cnt[b] : 0u;
    sum += loc[k];
  }
  u32 tot;
  const u32 incl = block_inclusive_scan<u32>(sum, scan_tmp, OpAdd<u32>(), &tot);
  u32 run = incl - sum;
  bool full = false;
  for (u32 k = 0; k < per; ++k) {
    const u32 b = threadIdx.x * per + k;
    if (b < B) {
      const u32 c = loc[k];
      cnt[b] = run;
      u32 gg = 0;
      if (c) {
        gg = atomicAdd(&cursor[b], c);
        full |= gg + c > cap;
      }
      gb[b] = gg;
      run += c;
    }
  }
  if (__ballot(full) && (threadIdx.x & 63) == 0) atomic_or_if(&info->xf_redo, 1u);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ITEMS; ++k)
    if (bk[k] < B) {
      const u32 at = cnt[bk[k]] + r[k];
      stage[at] = v[k];
      sbk[at] = (uint16_t)bk[k];
    }
  __syncthreads();
  // write-back in bucket order: consecutive lanes on consecutive slots of a bucket
  for (u32 t = threadIdx.x; t < tot; t += THREADS) {
    const u32 b = sbk[t];
    const u32 slot = gb[b] + (t - cnt[b]);
    if (slot < cap) out[(size_t)b * cap + slot] = stage[t];
  }
}

// One bucket per workgroup: the PK check on fingerprints (LDS set of u32
// slots = hash tag:17 | (local index + 1):15; a tag match re-reads the other
// pair, L2-hot) and the fold of the bucket's minutes in LDS, flushed with one
// global XOR / add per minute of the bucket.
__device__ __forceinline__ bool xf_insert(u32* tab, const u64* bp, u64 p, u32 k, u32& pos, u32 budget, u32 cmask,
                                          Info* info) {
  const u32 h = (u32)(p >> 32);
  const u32 mine = ((h >> 15) << 15) | (k + 1);
  for (u32 probe = 0; probe < budget; ++probe) {
    const u32 prev = atomicCAS(&tab[pos], 0u, mine);
    if (prev == 0) return true;  // inserted
    if ((prev >> 15) == (h >> 15)) {
      const u64 q = bp[(prev & 0x7fffu) - 1];
      if ((q | cmask) == (p | cmask)) {  // equal fingerprints: a copy of one timestamp (or a near-impossible twin)
        if (((u32)q & cmask) != ((u32)p & cmask)) atomic_or_if(&info->xf_redo, 1u);
        return true;
      }
    }
    pos = (pos + 1) & (XP_SLOTS - 1);
  }
  return false;
}

// (a 16K-slot set with the minute histograms in dynamic LDS -- 74 KB, 20
// VGPRs, two workgroups per CU beside the next batch's TP1 -- made the
// headline step slower, 0.307/0.302 vs 0.2985/0.2977 ms in one run: the
// longer probe chains at 60 % load cost more than the occupancy gave)
__global__ __launch_bounds__(XP_THREADS) void k_xf_dedup(const u64* __restrict__ pairs, const u32* __restrict__ cursor,
                                                        u32 cap, int kb, int cbits, u32* __restrict__ dx,
                                                        u32* __restrict__ dc, Info* __restrict__ info) {
  __shared__ u32 tab[XP_SLOTS];  // 0 = empty
  __shared__ u32 q[XQ_CAP];      // queued pairs: next slot:15 | local index:15
  __shared__ u32 hx[XF_WMAX], hc[XF_WMAX];
  __shared__ u32 qn;
  const u32 b = blockIdx.x;
  const u32 cnt = min(cursor[b], cap);
  if (cnt == 0) return;
  const XfGeom g = xf_geom(info, kb, cbits);
  if (!g.ok) return;
  const u32 cmask = (1u << cbits) - 1u;
  const u64* bp = pairs + (size_t)b * cap;
  u64 it[XD_ITEMS];
#pragma unroll
  for (int r = 0; r < XD_ITEMS; ++r) {
    const u32 k = r * XP_THREADS + threadIdx.x;
    it[r] = k < cnt ? bp[k] : 0ull;
  }
  for (u32 s = threadIdx.x; s < XP_SLOTS; s += XP_THREADS) tab[s] = 0;
  for (u32 s = threadIdx.x; s < g.W; s += XP_THREADS) {
    hx[s] = 0;
    hc[s] = 0;
  }
  if (threadIdx.x == 0) qn = 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < XD_ITEMS; ++r) {
    const u32 k = r * XP_THREADS + threadIdx.x;
    if (k >= cnt) break;
    const u64 p = it[r];
    const u32 moff = (u32)p >> (32 - g.mb);
    atomicXor(&hx[moff], (u32)(p >> 32));
    atomicAdd(&hc[moff], 1u);
    if (cnt < 2) continue;
    u32 pos = ((u32)(p >> 32) * 2654435761u) >> 17;  // 15 bits
    if (!xf_insert(tab, bp, p, k, pos, XP_INLINE_PROBES, cmask, info)) {
      const u32 at = atomicAdd(&qn, 1u);
      if (at < XQ_CAP) q[at] = (pos << 15) | k;
      else xf_insert(tab, bp, p, k, pos, XP_SLOTS, cmask, info);  // queue full: finish here
    }
  }
  __syncthreads();
  const u32 m = min(qn, XQ_CAP);
  for (u32 t = threadIdx.x; t < m; t += XP_THREADS) {
    const u32 e = q[t], k = e & 0x7fffu;
    u32 pos = e >> 15;
    xf_insert(tab, bp, bp[k], k, pos, XP_SLOTS, cmask, info);
  }
  // the bucket's minutes (a minute split over buckets gets one XOR / add from each)
  const u32 m0 = xf_first_minute(g, b);
  for (u32 s = threadIdx.x; s < g.W; s += XP_THREADS) {
    const u32 c = hc[s];
    if (!c) continue;
    const u32 d = m0 + s;
    atomicXor(&dx[d], hx[s]);
    atomicAdd(&dc[d], c);
  }
}

// Per minute: presence (count > 0) and the XOR; per block of FR_THREADS
// minutes the present count and XOR (k_cl_leaves' offsets and carries).
__global__ __launch_bounds__(FR_THREADS) void k_xf_blocks(u32* __restrict__ dx, const u32* __restrict__ dc,
                                                         const Info* __restrict__ info, u32* __restrict__ dp,
                                                         u32* __restrict__ bcnt, u32* __restrict__ bxor) {
  __shared__ u32 tmp[FR_THREADS / 64 + 1];
  const u32 b = blockIdx.x * FR_THREADS + threadIdx.x;  // grid = FR_BLOCKS
  const u32 mlo = info->minute_min, mhi = info->minute_max;
  const bool usable = mlo <= mhi && !info->xf_redo && mhi - mlo < XF_SPAN_MAX;
  u32 x = 0, p = 0;
  if (usable && b <= mhi - mlo) {
    p = dc[b] != 0 ? 1u : 0u;
    x = p ? dx[b] : 0u;
  }
  dx[b] = x;
  dp[b] = p;
  u32 tot, xtot;
  block_inclusive_scan<u32>(p, tmp, OpAdd<u32>(), &tot);
  block_inclusive_scan<u32>(x, tmp, OpXor<u32>(), &xtot);
  if (threadIdx.x == 0) {
    bcnt[blockIdx.x] = tot;
    bxor[blockIdx.x] = xtot;
  }
}

// ============================================================================
// Host drivers
// ============================================================================
// An enqueued streaming batch (evm_apply_batch_async): the call's arguments
// (the caller keeps them valid until evm_apply_wait), the pinned landing slot
// of its status record, the event after its last kernel, and its outputs.
// (the status record lands by a kernel, k_info_land, not the runtime's copy:
// config 2 0.2938 / 0.2989 vs 0.2971 / 0.3027 ms per step, two pairs)
__global__ void k_info_land(const Info* __restrict__ info, Info* host) {
  static_assert(sizeof(Info) % 4 == 0, "word copy");
  const u32* src = reinterpret_cast<const u32*>(info);
  volatile u32* dst = reinterpret_cast<volatile u32*>(host);
  for (u32 k = threadIdx.x; k < sizeof(Info) / 4; k += blockDim.x) dst[k] = src[k];
  __threadfence_system();
}

struct evm_pending {
  const evm_tree* tree_in;
  const char* ts;
  size_t stride, n;
  const uint32_t* cell;
  uint32_t n_cells;
  const uint32_t* cell_owner;
  const char* prior_ts;
  size_t prior_stride;
  const uint8_t* prior_present;
  const char* stored_ts;
  size_t stored_stride, n_stored;
  const uint32_t* stored_cell;
  uint8_t* flags;
  int32_t* winner;
  bool enqueued = false;  // false: finished synchronously (status, done)
  int status = EVM_OK;
  evm_tree* done = nullptr;
  evm::Info* hinfo = nullptr;  // pinned
  hipEvent_t ev = nullptr;
  evm_tree* spec = nullptr;  // the output tree (an empty one-owner tree_in)
  void* leaves = nullptr;    // the batch's leaves (ck, xr) for a merge at the wait
  size_t leaves_bytes = 0;
  // the buffers the batch's cross-cell check (second stream) reads after the
  // call returns -- status record, K1's hashes, the check's buckets -- so the
  // next batch's kernels, which reuse the scratch arena, never touch them
  void* dev = nullptr;
  size_t dev_bytes = 0;
};

// Geometry of the partitioned cross-cell check for n messages.
struct XpGeom {
  int kb;
  u32 cap;
};
static XpGeom xp_geom(size_t n) {
  XpGeom x;
  x.kb = XF_MIN_KB;  // (the fused check + fold of the tc path needs >= 64 minute buckets)
  while (x.kb < XP_MAX_KB && (n >> x.kb) > XP_AVG) ++x.kb;
  const size_t avg = (n >> x.kb) + 1;
  x.cap = (u32)std::min<size_t>(XP_MAX_FILL, avg + avg / 8 + 1024);
  return x;
}
// The buffers a streaming batch's second-stream work (cross-cell check, and
// on the tc path the Merkle fold) reads: the status record, K1's hashes and
// minutes, the check's buckets, the fold's partials.  One block per pending
// batch (evm_apply_batch_async), so the next batch's kernels -- which reuse
// the scratch arena -- never touch them; a synchronous call takes the same
// layout from the scratch arena.
struct SideBufs {
  Info* info;
  u32* hash;
  u32* minute;
  u32* xcur;
  u64* xpairs;
  u32 *px, *pp, *dx, *dc, *dp, *bcnt, *bxor;  // (dc, the tc path's per-minute row counts, right after dx)
  u64 *tcs, *tcs_far;  // tc path: TP1's packed (cell, tc) per row (the second stream's scatter reads it) and far rows' tc
};
static size_t side_bufs(void* base, size_t n, SideBufs* v) {
  const XpGeom x = xp_geom(n);
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t B = (size_t)FOLD_MAXWIN * FOLD_WIN;
  const size_t sz[] = {up(sizeof(Info)), up(4 * n), up(4 * n), up(4ull << x.kb), up((8ull * x.cap) << x.kb),
                       up((size_t)4 * FOLD_MAXWIN * FOLD_CHUNKS * FOLD_WIN),
                       up((size_t)4 * FOLD_MAXWIN * FOLD_CHUNKS * (FOLD_WIN / 32)), up(4 * B), up(4 * B), up(4 * B),
                       up(4 * FR_BLOCKS), up(4 * FR_BLOCKS), up(8 * n), up(8 * n)};
  constexpr int NB = sizeof(sz) / sizeof(sz[0]);
  size_t off[NB], tot = 0;
  for (int k = 0; k < NB; ++k) {
    off[k] = tot;
    tot += sz[k];
  }
  if (v && base) {
    char* p = static_cast<char*>(base);
    v->info = reinterpret_cast<Info*>(p + off[0]);
    v->hash = reinterpret_cast<u32*>(p + off[1]);
    v->minute = reinterpret_cast<u32*>(p + off[2]);
    v->xcur = reinterpret_cast<u32*>(p + off[3]);
    v->xpairs = reinterpret_cast<u64*>(p + off[4]);
    v->px = reinterpret_cast<u32*>(p + off[5]);
    v->pp = reinterpret_cast<u32*>(p + off[6]);
    v->dx = reinterpret_cast<u32*>(p + off[7]);
    v->dc = reinterpret_cast<u32*>(p + off[8]);
    v->dp = reinterpret_cast<u32*>(p + off[9]);
    v->bcnt = reinterpret_cast<u32*>(p + off[10]);
    v->bxor = reinterpret_cast<u32*>(p + off[11]);
    v->tcs = reinterpret_cast<u64*>(p + off[12]);
    v->tcs_far = reinterpret_cast<u64*>(p + off[13]);
  }
  return tot;
}

// The streaming paths.  TC: the tc path (TP1-TP3); otherwise the exact walk
// path (K1 + pass 1 + carry + pass 2 over the full order key).  Both share
// the cross-cell check, the Merkle fold and the status handling.  The tc
// path returns TP_REDO when it met a tie (the caller reruns the exact path).
constexpr int TP_REDO = -100;
constexpr int ST_PENDING = -101;  // apply_stream enqueued the batch (evm_apply_batch_async)

template <bool TC>
static int apply_stream(evm_ctx* ctx, Scratch& S, Info* info, const evm_tree* tree_in, const char* ts, size_t stride,
                        size_t n, const u32* cell, u32 C, const evm_rec* prior, const uint8_t* prior_present,
                        const Stored& stored, uint8_t* flags, int32_t* winner, evm_tree** tree_out,
                        evm_pending* pend = nullptr) {
  int st;
  const int cbits = C > 1 ? 32 - __builtin_clz(C - 1) : 0;
  const bool s48 = stride == 48 && ((uintptr_t)ts & 15) == 0;
  SideBufs sb;
  void* sbase = pend ? pend->dev : static_cast<void*>(S.alloc<char>(side_bufs(nullptr, n, nullptr)));
  if (!sbase) return EVM_ENOMEM;
  side_bufs(sbase, n, &sb);
  u32* hash = sb.hash;
  u32* minute = sb.minute;
  u32* xcur = sb.xcur;
  u64* xpairs = sb.xpairs;
  // TC: ranges of TP1/TP3 (multiples of 256 rows); walk path: ranges of the walks
  size_t range, G;
  TpRanges TR{};
  if (TC) {
    range = std::max<size_t>(1024, ((n + TP_RANGES - 1) / TP_RANGES + 255) / 256 * 256);
    range = std::min<size_t>(range, TP_ROWS_MAX);  // (TP1's key holds a 13-bit row offset)
    TR = TpRanges{range, (range / 16) & ~(size_t)63};
    G = (n + range - 1) / range + 4;  // (the first range in five geometric pieces)
  } else {
    range = (n + CL_RANGE_TARGET - 1) / CL_RANGE_TARGET;
    range = std::max<size_t>(2048, (range + 255) / 256 * 256);
    G = (n + range - 1) / range;
  }
  uint4* key = nullptr;
  u32* rl = nullptr;
  u64* tcs = nullptr;
  u64* agg = nullptr;
  u32* arow = nullptr;
  u64* a_tc = nullptr;
  u64* a_rh = nullptr;
  u32* a_rl = nullptr;
  u32* a_first = nullptr;
  if (TC) {
    tcs = sb.tcs;  // (in the batch's own block: the second stream reads it after the call returns)
    agg = S.alloc<u64>(G * C);
    arow = S.alloc<u32>(G * C);
    if (!tcs || !agg || !arow) return EVM_ENOMEM;
    // TP1: parse + per (range, cell) max tc and its row, one workgroup per range
    evm::ProfScope ps_(ctx, "k_tp_pack");
    const size_t lds = (size_t)C * 8 + (size_t)((C + 31) / 32) * 4;
    const dim3 g1((u32)G);
    if (s48)
      hipLaunchKernelGGL(k_tp_pack<true>, g1, dim3(TP_THREADS), lds, ctx->stream, (const uint8_t*)ts, stride, n,
                         cell, C, TR, tcs, sb.tcs_far, hash, agg, arow, info, xcur, 1u << xp_geom(n).kb, sb.dx, 2u * XF_SPAN_MAX);
    else
      hipLaunchKernelGGL(k_tp_pack<false>, g1, dim3(TP_THREADS), lds, ctx->stream, (const uint8_t*)ts, stride, n,
                         cell, C, TR, tcs, sb.tcs_far, hash, agg, arow, info, xcur, 1u << xp_geom(n).kb, sb.dx, 2u * XF_SPAN_MAX);
  } else {
    key = S.alloc<uint4>(n);
    rl = S.alloc<u32>(n);
    a_tc = S.alloc<u64>(G * C);
    a_rh = S.alloc<u64>(G * C);
    a_rl = S.alloc<u32>(G * C);
    a_first = S.alloc<u32>(G * C);
    if (!key || !rl || !a_tc || !a_rh || !a_rl || !a_first) return EVM_ENOMEM;
    // K1: parse, canonical check, murmur3, minute -- at full occupancy
    evm::ProfScope ps_(ctx, "k_cl_pack");
    const dim3 g(std::min<size_t>((n + 255) / 256, 2048));  // (8192 measured 5 % slower inside the pipeline)
    if (s48)
      hipLaunchKernelGGL(k_cl_pack<true>, g, dim3(CLP_THREADS), 0, ctx->stream, (const uint8_t*)ts, stride, n, key,
                         rl, hash, minute, info);
    else
      hipLaunchKernelGGL(k_cl_pack<false>, g, dim3(CLP_THREADS), 0, ctx->stream, (const uint8_t*)ts, stride, n, key,
                         rl, hash, minute, info);
  }
  // batch timestamps already stored under another cell (global PK)
  if ((st = stored_check(ctx, S, stored, hash, 1, ts, stride, cell, n, info))) return st;
  // cross-cell PK check: partition by hash into fixed-capacity buckets, LDS set per bucket
  const XpGeom xg = xp_geom(n);
  const int kb = xg.kb;
  const u32 cap = xg.cap;
  const u32 xt = (u32)((n + XP_TILE - 1) / XP_TILE);
  // scatter tiles of 12,288 rows (rounding the tile count up to whole rounds
  // of the chip -- 1,024 tiles of 9,766 rows for 10M -- measured slower, 85
  // vs 78-81 us: shorter bucket runs cost more than the last round's sliver)
  const u32 xft = (u32)((n + 12287) / 12288);
  const u32 xf_tl = 12288;

  // it reads only the timestamps, cells and K1's hashes: a second stream runs
  // it beside the walks, forked right after K1 (joined before the status
  // read; forked after pass 1 instead: 0.502-0.506 vs 0.497 ms per config-2 step)
  // Merkle fold: LDS XOR histograms per (minute window, chunk), reduced into
  // leaves -- written straight into the output tree when it starts empty
  u32 *px = sb.px, *pp = sb.pp, *dx = sb.dx, *dp = sb.dp, *bcnt = sb.bcnt, *bxor = sb.bxor;
  const size_t B = (size_t)FOLD_MAXWIN * FOLD_WIN;
  const bool spec_out = tree_in->n_leaves == 0 && tree_in->n_owners == 1;
  u64* lck = nullptr;
  int32_t* lxr = nullptr;
  if (pend && !spec_out) {
    // the leaves outlive this call's scratch: the wait merges them
    pend->leaves_bytes = B * (sizeof(u64) + sizeof(int32_t));
    pend->leaves = block_alloc(ctx, &pend->leaves_bytes);
    if (!pend->leaves) return EVM_ENOMEM;
    lck = static_cast<u64*>(pend->leaves);
    lxr = reinterpret_cast<int32_t*>(lck + B);
  } else {
    lck = S.alloc<u64>(B);
    lxr = S.alloc<int32_t>(B);
  }
  if (!px || !pp || !dx || !dp || !bcnt || !bxor || !lck || !lxr) return EVM_ENOMEM;
  evm_tree* spec = nullptr;
  if (spec_out && (st = tree_alloc_cap(ctx, 1, B, &spec))) return st;
  struct SpecGuard {
    evm_ctx* ctx;
    evm_tree*& t;
    ~SpecGuard() {
      if (t) tree_destroy(ctx, t);
    }
  } guard{ctx, spec};
  auto leaves = [&](hipStream_t fs) {
    evm::ProfScope ps_(ctx, "k_cl_leaves", fs);
    if (spec)  // one owner, empty: the leaf kernel writes the tree itself
      hipLaunchKernelGGL(k_cl_leaves, dim3(FR_BLOCKS), dim3(FR_THREADS), 0, fs, dx, dp, bcnt, bxor, info, spec->ck,
                         spec->xr, spec->pfx, spec->off);
    else
      hipLaunchKernelGGL(k_cl_leaves, dim3(FR_BLOCKS), dim3(FR_THREADS), 0, fs, dx, dp, bcnt, bxor, info, lck, lxr,
                         (int32_t*)nullptr, (u64*)nullptr);
  };
  auto fold = [&](hipStream_t fs) {
    {
      evm::ProfScope ps_(ctx, "k_cl_fold_hist", fs);
      hipLaunchKernelGGL(k_cl_fold_hist<true>, dim3(FOLD_CHUNKS, FOLD_MAXWIN), dim3(FOLD_THREADS), 0, fs, flags, minute,
                         hash, n, px, pp, info);
    }
    {
      evm::ProfScope ps_(ctx, "k_cl_fold_reduce", fs);
      hipLaunchKernelGGL(k_cl_fold_reduce, dim3(FR_BLOCKS), dim3(FR_THREADS), 0, fs, px, pp, info, dx, dp, bcnt, bxor);
    }
    leaves(fs);
  };
  SideFork side(ctx);
  {
    const hipStream_t xs = side.stream();
    if (TC) {
      // the fused cross-cell check + Merkle fold (minute buckets; k_xf_fix
      // after the walk XORs its exact redeliveries out again)
      {
        evm::ProfScope ps_(ctx, "k_xf_scatter", xs);
        hipLaunchKernelGGL((k_xf_scatter<1024, 12>), dim3(xft), dim3(1024), 0, xs, hash, (const u64*)tcs,
                           (const u64*)sb.tcs_far, cell, n, kb, cbits, cap, xcur, xpairs, info, xf_tl);
      }
      evm::ProfScope ps_(ctx, "k_xf_dedup", xs);
      hipLaunchKernelGGL(k_xf_dedup, dim3(1u << kb), dim3(XP_THREADS), 0, xs, (const u64*)xpairs, (const u32*)xcur,
                         cap, kb, cbits, sb.dx, sb.dc, info);
    } else {
      HIPR(hipMemsetAsync(xcur, 0, sizeof(u32) << kb, xs));  // (the tc path's K1 clears them)
      {
        evm::ProfScope ps_(ctx, "k_xp_scatter", xs);
        hipLaunchKernelGGL(k_xp_scatter, dim3(xt), dim3(XP_THREADS), 0, xs, hash, n, kb, cap, xcur, xpairs, info);
      }
      evm::ProfScope ps_(ctx, "k_xp_dedup", xs);
      hipLaunchKernelGGL(k_xp_dedup, dim3(1u << kb), dim3(XP_THREADS), 0, xs, xpairs, xcur, cap, n,
                         (const uint8_t*)ts, stride, cell, info);
    }
  }
  if (TC) {
    // TP2: per cell, exclusive max over the ranges (in place in agg) + final max
    const NodeSrc N{(const uint8_t*)ts, stride, prior};
    KLAUNCH(k_tp_carry, dim3((C + CT_CELLS - 1) / CT_CELLS), dim3(CT_THREADS), C, G, agg, arow, N, prior_present,
            winner);
    // TP3: flags, a workgroup per range
    KLAUNCH_LDS(k_tp_walk, dim3(G), dim3(TP_THREADS), (size_t)2 * C * 8 + (size_t)TPC_ROWS * 14 + (size_t)C * 4,
                (const u64*)tcs, (const u64*)sb.tcs_far, cell, n, C, TR, (const u64*)agg, (const u32*)arow, N, flags,
                (const u32*)hash,
                sb.dx, sb.dc, (const Info*)info);
    // the Merkle fold reads the walk's flags (an exact redelivery of a cell's
    // max is not XORed): on the second stream after the walk, beside the
    // next batch's K1 when batches are pipelined
    const hipStream_t fs = side.stream();
    if (fs != ctx->stream) {
      HIPR(hipEventRecord(ctx->ev_fork, ctx->stream));
      HIPR(hipStreamWaitEvent(fs, ctx->ev_fork, 0));
    }
    {
      evm::ProfScope ps_(ctx, "k_xf_blocks", fs);
      hipLaunchKernelGGL(k_xf_blocks, dim3(FR_BLOCKS), dim3(FR_THREADS), 0, fs, sb.dx, (const u32*)sb.dc, info, sb.dp,
                         sb.bcnt, sb.bxor);
    }
    leaves(fs);
  } else {
    // pass 1: per range and cell, the max timestamp and its first index
    KLAUNCH_LDS(k_cl_scan1, dim3(G), dim3(WK_THREADS), (size_t)C * 24, key, rl, cell, n, C, cbits, range, a_tc, a_rh, a_rl,
                a_first, info);
    // carry: per cell, exclusive scan over ranges seeded with the prior max
    {
      u64* s_tc = S.alloc<u64>((size_t)CARRY_SEGS * C);
      u64* s_rh = S.alloc<u64>((size_t)CARRY_SEGS * C);
      u32* s_rl = S.alloc<u32>((size_t)CARRY_SEGS * C);
      u32* s_first = S.alloc<u32>((size_t)CARRY_SEGS * C);
      if (!s_tc || !s_rh || !s_rl || !s_first) return EVM_ENOMEM;
      const u32 cb = (C + 63) / 64;
      KLAUNCH(k_cl_carry_reduce, dim3(cb, CARRY_SEGS), dim3(64), C, G, a_tc, a_rh, a_rl, a_first, s_tc, s_rh, s_rl,
              s_first);
      KLAUNCH(k_cl_carry_segs, dim3((C + 3) / 4), dim3(256), C, s_tc, s_rh, s_rl, s_first, prior, prior_present, winner);
      KLAUNCH(k_cl_carry_down, dim3(cb, CARRY_SEGS), dim3(64), C, G, a_tc, a_rh, a_rl, a_first, s_tc, s_rh,
              s_rl);
    }
    KLAUNCH_LDS(k_cl_scan2, dim3(G), dim3(WK_THREADS), (size_t)C * 20, key, rl, cell, n, C, cbits, range, a_tc, a_rh, a_rl,
                flags);
  }
  if (!TC) fold(ctx->stream);
  if (!spec_out && !pend && tree_in->n_leaves == 0) {
    side.join();  // (the tc path's fold ran there)
    if ((st = tree_finalize_dev(ctx, S, tree_in->n_owners, lck, lxr, &info->n_leaves, B, &spec))) return st;
  }
  if (pend) {
    // asynchronous: the second stream finishes the cross-cell check beside the
    // NEXT batch's kernels; after the main stream's last kernel it lands the
    // status record in pinned memory.  No join: the main stream goes on.
    const hipStream_t xs = side.stream();
    if (xs != ctx->stream) {
      HIPR(hipEventRecord(ctx->ev_join, ctx->stream));
      HIPR(hipStreamWaitEvent(xs, ctx->ev_join, 0));
    }
    // (one workgroup writes the record into the pinned slot itself: the
    // runtime's copy of 64 bytes to the host was an 18-us blit per batch)
    hipLaunchKernelGGL(k_info_land, dim3(1), dim3(64), 0, xs, (const Info*)info, pend->hinfo);
    HIPR(hipGetLastError());
    HIPR(hipEventRecord(pend->ev, xs));
    side.detach();
    pend->spec = spec;
    spec = nullptr;
    return ST_PENDING;
  }
  side.join();
  Info hi;
  if ((st = read_info(ctx, info, &hi))) return st;
  if (hi.bad) {
    KLAUNCH(k_keep_bad, dim3(grid_for(n, 256)), dim3(256), flags, n);  // nothing applied: only the culprits
    return EVM_ENONCANON;
  }
  if (hi.bad_aux) return EVM_EINVAL;
  // an overflowed tie list, or the fused check + fold could not finish (a
  // possible collision, a full bucket, a wide minute range): the exact walk path redoes the batch
  if (TC && (hi.ties || hi.xf_redo)) return TP_REDO;
  if (!hi.collision && hi.xc_oversize) {
    // a hash bucket overflowed LDS (heavy skew): exact check on the global epoch-tagged set
    const int lg = std::max(ceil_log2(n + n / 2 + 1), 10);
    if (!ctx->xtab || ctx->xtab_lg < lg) {
      if (ctx->xtab) HIPR(hipFree(ctx->xtab));
      ctx->xtab = nullptr;
      HIPR(hipMalloc(&ctx->xtab, sizeof(u64) << lg));
      HIPR(hipMemsetAsync(ctx->xtab, 0, sizeof(u64) << lg, ctx->stream));
      ctx->xtab_lg = lg;
      ctx->xepoch = 0;
    }
    if (++ctx->xepoch == 256) {
      HIPR(hipMemsetAsync(ctx->xtab, 0, sizeof(u64) << ctx->xtab_lg, ctx->stream));
      ctx->xepoch = 1;
    }
    KLAUNCH(k_cl_xcell, dim3(grid_for(n, 256, 16384)), dim3(256), (const uint8_t*)ts, stride, cell, hash, n, ctx->xtab,
            (u32)ctx->xtab_lg, ctx->xepoch, info);
    if ((st = read_info(ctx, info, &hi))) return st;
  }
  if (hi.collision) return EVM_ECOLLISION;
  if (!hi.fold_overflow) {
    if (spec) {
      spec->n_leaves = hi.n_leaves;
      *tree_out = spec;
      spec = nullptr;
      return EVM_OK;
    }
    return merge_into_tree(ctx, S, tree_in, tree_in->n_owners, lck, lxr, hi.n_leaves, tree_out);
  }
  // wide minute range or mixed key lengths: sort-based fold
  u32* sel = S.alloc<u32>(n);
  u32* spos = S.alloc<u32>(n);
  u32* cnt = S.alloc<u32>(1);
  u64* ck = S.alloc<u64>(n);
  u32* h = S.alloc<u32>(n);
  if (!sel || !spos || !cnt || !ck || !h) return EVM_ENOMEM;
  if ((st = launch_sel(ctx, flags, (uint8_t)EVM_MSG_XOR, n, sel))) return st;
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, sel, n, spos, cnt))) return st;
  KLAUNCH(k_cl_fold_ck, dim3(grid_for(n, 256, 4096)), dim3(256), flags, minute, hash, spos, n, ck, h, info);
  u32 m = 0;
  HIPR(hipMemcpyAsync(&m, cnt, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  if ((st = read_info(ctx, info, &hi))) return st;
  return fold_into_tree(ctx, S, tree_in, tree_in->n_owners, ck, h, m, hi, tree_out);
}

// ============================================================================
// Small-batch path (send.ts:107-111: a client applies what one sync brings --
// hundreds to ~100k messages): the sort path's ~25 launches and 4 host
// synchronisations are latency at this size, so the same decisions run as
// five kernels and ONE status read:
//   K1 k_sm_pack    parse + canonical check + murmur3 (rec), rows per cell,
//                   the cross-cell PK set (raw-byte compare), minute bounds
//   K2 k_sm_scan_lb cell offsets (exclusive scan of the counts, look-back)
//   K3 k_sm_scatter rows -> their cell's slots (unordered within the cell)
//   K4 k_sm_lww     a thread per cell: its rows in batch order (repeated
//                   selection, <= SM_SEG of them; longer cells: a workgroup
//                   each, k_sm_long), the running max from the prior
//                   max -> flags and winner (applyMessages.ts:93,105); the
//                   XOR rows' hashes into dense minute bins
//   K5 k_sm_fold    one workgroup: bins -> leaves, merged with tree_in's
//                   leaves (equal keys XOR-combine), prefix XOR -> the tree
// A cell with more than SM_SEG rows, minutes wider than SM_BINS or of two
// base-3 lengths (leaf order != minute order) make the batch take the sort
// path instead (SM_FALLBACK).
// ============================================================================
constexpr size_t SM_MAX_N = 1u << 18;       // rows (the auto choice over > 2,048 cells; EVM_OPT_CLIENT_PATH 4 forces it)
constexpr size_t SM_AUTO_FEW = 1u << 14;    // rows: the auto choice over <= 2,048 cells too
constexpr u32 SM_MAX_CELLS = 1u << 22;
constexpr u32 SM_SEG = 8;                   // rows per cell a thread takes (longer cells: k_sm_long; its
                                            // O(k^2) selection made 20-32-row cells the kernel's tail at 32)
constexpr u32 SM_LONG_MAX = 4096;           // rows of one cell k_sm_long sorts in LDS
constexpr int SM_LONG_THREADS = 256;
constexpr u32 SM_BINS = 1u << 16;           // minutes (45 days) of the dense fold
constexpr int SM_FOLD_THREADS = 1024;
constexpr int SM_FALLBACK = -102;

__global__ __launch_bounds__(256) void k_sm_pack(const uint8_t* __restrict__ ts, size_t stride, size_t n,
                                                 const u32* __restrict__ cell, u32 C, evm_rec* __restrict__ rec,
                                                 u32* __restrict__ cnt, u64* __restrict__ table, u32 lg,
                                                 Info* __restrict__ info) {
  const u64 mask = (1ull << lg) - 1;
  u32 bad = 0, mn = 0xffffffffu, mx = 0;
  bool bad_aux = false, coll = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32 w[12];
    load_ts(ts, stride, i, w);
    const Parsed p = parse_ts46(w);
    const u32 c = cell[i];
    evm_rec r;
    r.tc = p.tc;
    r.node = p.node;
    r.meta = p.meta;
    r.hash = p.hash;
    r.minute = p.minute;
    r.aux = c;
    rec[i] = r;
    if (!(p.meta & EVM_META_VALID)) {
      bad = 1;
      continue;
    }
    mn = min(mn, p.minute);
    mx = max(mx, p.minute);
    if (c >= C) {
      bad_aux = true;
      continue;
    }
    atomicAdd(&cnt[c], 1u);
    // the global __message PK (applyMessages.ts:42-45): one timestamp in two cells
    const u64 mine = ((u64)p.hash << 32) | (u64)(i + 1);
    u64 pos = ((u64)(p.hash * 2654435761u) ^ (p.node * 0x9E3779B97F4A7C15ull >> 20)) & mask;
    for (u64 probe = 0; probe <= mask; ++probe) {
      u64 sl = __hip_atomic_load(&table[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (sl == 0) {
        const u64 prev = atomicCAS(&table[pos], 0ull, mine);
        if (prev == 0) break;  // inserted
        sl = prev;
      }
      if ((u32)(sl >> 32) == p.hash) {
        const size_t j = (size_t)(sl & 0xffffffffu) - 1;
        if (ts_bytes_equal(ts, stride, i, j)) {
          coll |= cell[j] != c;
          break;
        }
      }
      pos = (pos + 1) & mask;
    }
  }
  if (__ballot(bad_aux) && (threadIdx.x & 63) == 0) atomic_or_if(&info->bad_aux, 1u);
  if (__ballot(coll) && (threadIdx.x & 63) == 0) atomic_or_if(&info->collision, 1u);
  block_fold_bounds<u32, 256>(mn, mx, bad, &info->minute_min, &info->minute_max, &info->bad);
}

// cell offsets: off[c] = rows of cells < c (off[C] = all), and cnt[c] = off[c]
// (K3's cursors): 16 consecutive counts per thread (four 16-B loads).
constexpr u32 SM_SCAN_ITEMS = 16;
// (loads of 16 counts from a tile: 16-B loads where the tile is whole)
__device__ __forceinline__ void sm_scan_load(const u32* cnt, u32 C, u32 a, u32 (&v)[SM_SCAN_ITEMS]) {
  if (a + SM_SCAN_ITEMS <= C) {  // (cnt is 256-B aligned scratch: a is a multiple of 16)
    const uint4* p = reinterpret_cast<const uint4*>(cnt + a);
#pragma unroll
    for (u32 q = 0; q < SM_SCAN_ITEMS / 4; ++q) {
      const uint4 x = p[q];
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (u32 q = 0; q < SM_SCAN_ITEMS; ++q) v[q] = a + q < C ? cnt[a + q] : 0u;
  }
}
// Several workgroups (one tile of SM_FOLD_THREADS x 16 counts each, tiles in
// launch order from a counter): each tile's offsets after the counts of every
// tile before it, by decoupled look-back (status words and the counter zeroed
// with the batch's other scratch).  A 100k-message batch of ~55k cells: four
// tiles side by side (the one-workgroup scan it replaced: 23.4 vs 10.2 us).
constexpr u32 SM_SCAN_TILE = SM_FOLD_THREADS * SM_SCAN_ITEMS;
__global__ __launch_bounds__(SM_FOLD_THREADS) void k_sm_scan_lb(u32* __restrict__ cnt, u32 C, u32* __restrict__ off,
                                                                u64* __restrict__ status, u32* __restrict__ ctr,
                                                                u32* __restrict__ err) {
  __shared__ u32 lds[SM_FOLD_THREADS / 64 + 1];
  __shared__ u32 tile_s, excl_s;
  if (threadIdx.x == 0) tile_s = atomicAdd(ctr, 1u);
  __syncthreads();
  const u32 tile = tile_s;
  const u32 a = tile * SM_SCAN_TILE + threadIdx.x * SM_SCAN_ITEMS;
  u32 v[SM_SCAN_ITEMS];
  sm_scan_load(cnt, C, a, v);
  u32 sum = 0;
#pragma unroll
  for (u32 q = 0; q < SM_SCAN_ITEMS; ++q) sum += v[q];
  u32 tot;
  const u32 incl = block_inclusive_scan<u32, OpAdd<u32>>(sum, lds, OpAdd<u32>(), &tot);
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0)
      __hip_atomic_store(status + tile, (tile == 0 ? LB_PRE : LB_AGG) | (u64)tot, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    const u32 excl = tile ? (u32)lookback_wave(status, tile, LbAdd<u64>(), 1u << 24, err) : 0u;
    if (threadIdx.x == 0) {
      if (tile) __hip_atomic_store(status + tile, LB_PRE | (u64)(excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      excl_s = excl;
      if ((u64)(tile + 1) * SM_SCAN_TILE >= C) off[C] = excl + tot;
    }
  }
  __syncthreads();
  u32 run = excl_s + incl - sum;
  u32 x[SM_SCAN_ITEMS];
#pragma unroll
  for (u32 q = 0; q < SM_SCAN_ITEMS; ++q) {
    x[q] = run;
    run += v[q];
  }
  if (a + SM_SCAN_ITEMS <= C) {
    uint4* po = reinterpret_cast<uint4*>(off + a);
    uint4* pc = reinterpret_cast<uint4*>(cnt + a);
#pragma unroll
    for (u32 q = 0; q < SM_SCAN_ITEMS / 4; ++q) {
      const uint4 y = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
      po[q] = y;
      pc[q] = y;
    }
  } else {
#pragma unroll
    for (u32 q = 0; q < SM_SCAN_ITEMS; ++q)
      if (a + q < C) {
        off[a + q] = x[q];
        cnt[a + q] = x[q];
      }
  }
}

__global__ void k_sm_scatter(const evm_rec* __restrict__ rec, size_t n, u32 C, u32* __restrict__ cur,
                             u32* __restrict__ grp) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const evm_rec r = rec[i];
    if (!(r.meta & EVM_META_VALID) || r.aux >= C) continue;
    grp[atomicAdd(&cur[r.aux], 1u)] = (u32)i;
  }
}

// A thread per cell.  Its rows are taken in batch order by repeated
// selection (the smallest index above the last one: O(k^2) reads of the
// cell's L2-hot slots, no per-lane array, k <= SM_SEG).  The XOR rows' hashes
// go into a per-workgroup LDS copy of the minute bins when the batch's minutes
// fit it (a client batch spans minutes, not days: thousands of rows hit the
// same few bins, which global atomics would serialise), flushed once per
// workgroup; wider batches use the global bins directly.
constexpr u32 SM_LDS_BINS = 8192;
__global__ __launch_bounds__(256) void k_sm_lww(const evm_rec* __restrict__ rec, const u32* __restrict__ off,
                                                const u32* __restrict__ grp, u32 C,
                                                const evm_rec* __restrict__ prior,
                                                const uint8_t* __restrict__ prior_present, uint8_t* __restrict__ flags,
                                                int32_t* __restrict__ winner, u32* __restrict__ bins,
                                                u32* __restrict__ pres, u32* __restrict__ long_list,
                                                u32* __restrict__ long_n, Info* __restrict__ info) {
  __shared__ u32 lbins[SM_LDS_BINS];
  __shared__ u32 lpres[SM_LDS_BINS / 32];
  const u32 mlo = info->minute_min, mhi = info->minute_max;
  const u32 W = mhi >= mlo ? mhi - mlo + 1 : 0u;
  const bool lds = W <= SM_LDS_BINS;
  if (lds) {
    for (u32 k = threadIdx.x; k < W; k += blockDim.x) lbins[k] = 0;
    for (u32 k = threadIdx.x; k < (W + 31) / 32; k += blockDim.x) lpres[k] = 0;
  }
  __syncthreads();
  for (u32 c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    const u32 a = off[c], k = off[c + 1] - a;
    if (k == 0) continue;  // (winner -1 from the init)
    if (k > SM_SEG) {  // a long cell (a hot row of the app): a workgroup of k_sm_long takes it
      if (k > SM_LONG_MAX) atomic_or_if(&info->fold_overflow, 1u);  // (the sort path)
      else long_list[atomicAdd(long_n, 1u)] = c;
      continue;
    }
    Key run = (prior_present && prior_present[c]) ? key_of(prior[c]) : key_none();
    int32_t win = -1;
    u32 last = 0;
    for (u32 step = 0; step < k; ++step) {
      u32 i = 0xffffffffu;
      for (u32 q = 0; q < k; ++q) {
        const u32 v = grp[a + q];
        if ((step == 0 || v > last) && v < i) i = v;
      }
      last = i;
      const evm_rec r = rec[i];
      const Key ts = key_of(r);
      const bool ups = key_cmp(run, ts) < 0;                            // applyMessages.ts:93
      const bool xr = !((run.mask & KEY_PRESENT) && key_eq(run, ts));  // applyMessages.ts:105
      flags[i] = (ups ? EVM_MSG_UPS : 0u) | (xr ? EVM_MSG_XOR : 0u);
      if (ups) {
        win = (int32_t)i;
        run = ts;
      }
      if (xr) {
        const u32 d = r.minute - mlo;
        if (lds) {
          atomicXor(&lbins[d], r.hash);
          atomicOr(&lpres[d >> 5], 1u << (d & 31));
        } else if (d >= SM_BINS) {
          atomic_or_if(&info->fold_overflow, 1u);
        } else {
          atomicXor(&bins[d], r.hash);
          atomic_or_if(&pres[d >> 5], 1u << (d & 31));
        }
      }
    }
    winner[c] = win;
  }
  if (!lds) return;
  __syncthreads();
  for (u32 k = threadIdx.x; k < (W + 31) / 32; k += blockDim.x) {
    const u32 m = lpres[k];
    if (!m) continue;
    atomic_or_if(&pres[k], m);
    for (u32 b = 0; b < 32; ++b)
      if ((m >> b) & 1u) atomicXor(&bins[32 * k + b], lbins[32 * k + b]);
  }
}

// The long cells of up to 64 rows (every long cell of the config-1 todo app:
// hot rows of a few dozen updates), one WAVE each, no barriers: lane l takes
// the cell's row of batch rank l (ranks by 64 shuffled compares, placed
// through a per-wave LDS slot array), the exclusive running max is a wave
// prefix max of the keys seeded with the prior, and the XOR rows' hashes are
// reduced per minute inside the wave -- one global XOR / OR per distinct
// minute of the cell instead of one per row (a client batch spans a few
// minutes: per-row global atomics on the same bins serialise).
constexpr u32 SM_WAVE_MAX = 64;
__device__ __forceinline__ Key shfl_key(const Key& k, int src) {
  Key o;
  o.tc = ((u64)(u32)__shfl((int)(u32)(k.tc >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)k.tc, src, 64);
  o.node = ((u64)(u32)__shfl((int)(u32)(k.node >> 32), src, 64) << 32) | (u32)__shfl((int)(u32)k.node, src, 64);
  o.mask = (u32)__shfl((int)k.mask, src, 64);
  return o;
}
constexpr int SM_LW_WAVES = 16;  // waves per workgroup (one cell each at a time; the LDS bins shared)
__global__ __launch_bounds__(64 * SM_LW_WAVES) void k_sm_long_wave(const evm_rec* __restrict__ rec, const u32* __restrict__ off,
                                                      const u32* __restrict__ grp, const u32* __restrict__ long_list,
                                                      const u32* __restrict__ long_n, const evm_rec* __restrict__ prior,
                                                      const uint8_t* __restrict__ prior_present,
                                                      uint8_t* __restrict__ flags, int32_t* __restrict__ winner,
                                                      u32* __restrict__ bins, u32* __restrict__ pres,
                                                      Info* __restrict__ info) {
  __shared__ u32 slot[SM_LW_WAVES][SM_WAVE_MAX];
  __shared__ u32 lbins[SM_LDS_BINS];  // the workgroup's copy of the minute bins (as k_sm_lww)
  __shared__ u32 lpres[SM_LDS_BINS / 32];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u32 nl = *long_n;
  const u32 mlo = info->minute_min, mhi = info->minute_max;
  const u32 W = mhi >= mlo ? mhi - mlo + 1 : 0u;
  const bool lds = W <= SM_LDS_BINS;
  if (lds) {
    for (u32 q = threadIdx.x; q < W; q += blockDim.x) lbins[q] = 0;
    for (u32 q = threadIdx.x; q < (W + 31) / 32; q += blockDim.x) lpres[q] = 0;
  }
  __syncthreads();
  for (u32 li = blockIdx.x * SM_LW_WAVES + wv; li < nl; li += gridDim.x * SM_LW_WAVES) {  // wave-uniform
    const u32 c = long_list[li];
    const u32 a = off[c], k = off[c + 1] - a;
    if (k > SM_WAVE_MAX) continue;  // (k_sm_long)
    const bool in = (u32)lane < k;
    const u32 i = in ? grp[a + lane] : 0xffffffffu;
    u32 rank = 0;
    for (u32 j = 0; j < k; ++j) rank += (u32)__shfl((int)i, (int)j, 64) < i ? 1u : 0u;
    if (in) slot[wv][rank] = i;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const u32 row = in ? slot[wv][lane] : 0u;  // lane = batch rank
    __builtin_amdgcn_wave_barrier();
    evm_rec r{};
    if (in) r = rec[row];
    const Key ts = in ? key_of(r) : key_none();
    Key v = ts;  // inclusive prefix max over the lanes (batch order)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const Key o = shfl_key(v, lane >= d ? lane - d : lane);
      if (lane >= d) v = key_max(o, v);
    }
    Key run = (prior_present && prior_present[c]) ? key_of(prior[c]) : key_none();
    const Key ex = shfl_key(v, lane > 0 ? lane - 1 : 0);
    if (lane > 0) run = key_max(run, ex);
    const bool ups = in && key_cmp(run, ts) < 0;                             // applyMessages.ts:93
    const bool xr = in && !((run.mask & KEY_PRESENT) && key_eq(run, ts));  // applyMessages.ts:105
    if (in) flags[row] = (ups ? EVM_MSG_UPS : 0u) | (xr ? EVM_MSG_XOR : 0u);
    const u64 ub = __ballot(ups);  // the last upsert in batch order wins
    const u32 wrow = (u32)__shfl((int)row, ub ? 63 - __builtin_clzll(ub) : 0, 64);
    if (lane == 0) winner[c] = ub ? (int32_t)wrow : -1;
    const u32 d = xr ? r.minute - mlo : 0xffffffffu;
    if (lds) {
      if (xr) {
        atomicXor(&lbins[d], r.hash);
        atomicOr(&lpres[d >> 5], 1u << (d & 31));
      }
      continue;
    }
    // (wide batches) per distinct minute of the XOR rows: one reduction, one global update
    u64 left = __ballot(xr);
    while (left) {
      const int ld = __builtin_ctzll(left);
      const u32 dm = (u32)__shfl((int)d, ld, 64);
      const u64 mem = __ballot(xr && d == dm);
      u32 h = ((mem >> lane) & 1ull) ? r.hash : 0u;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) h ^= (u32)__shfl_xor((int)h, m, 64);
      if (lane == ld) {
        if (dm >= SM_BINS) {
          atomic_or_if(&info->fold_overflow, 1u);
        } else {
          atomicXor(&bins[dm], h);
          atomic_or_if(&pres[dm >> 5], 1u << (dm & 31));
        }
      }
      left &= ~mem;
    }
  }
  if (!lds) return;
  __syncthreads();
  for (u32 q = threadIdx.x; q < (W + 31) / 32; q += blockDim.x) {
    const u32 m = lpres[q];
    if (!m) continue;
    atomic_or_if(&pres[q], m);
    for (u32 b = 0; b < 32; ++b)
      if ((m >> b) & 1u) atomicXor(&bins[32 * q + b], lbins[32 * q + b]);
  }
}

// The long cells (SM_SEG < rows <= SM_LONG_MAX), a workgroup each: the rows'
// indices sorted in LDS (bitonic), the exclusive running max in batch order by
// a blocked scan with key_max (each thread a contiguous run of positions),
// then flags, the winner (the last upsert) and the XOR rows' bins.
__global__ __launch_bounds__(SM_LONG_THREADS) void k_sm_long(const evm_rec* __restrict__ rec,
                                                             const u32* __restrict__ off,
                                                             const u32* __restrict__ grp,
                                                             const u32* __restrict__ long_list,
                                                             const u32* __restrict__ long_n,
                                                             const evm_rec* __restrict__ prior,
                                                             const uint8_t* __restrict__ prior_present,
                                                             uint8_t* __restrict__ flags, int32_t* __restrict__ winner,
                                                             u32* __restrict__ bins, u32* __restrict__ pres,
                                                             Info* __restrict__ info) {
  __shared__ u32 idx[SM_LONG_MAX];
  __shared__ u64 s_tc[SM_LONG_THREADS], s_node[SM_LONG_THREADS];
  __shared__ u32 s_mask[SM_LONG_THREADS];
  __shared__ int32_t s_win;
  const u32 t = threadIdx.x;
  const u32 nl = *long_n;
  const u32 mlo = info->minute_min;
  for (u32 li = blockIdx.x; li < nl; li += gridDim.x) {
    const u32 c = long_list[li];
    const u32 a = off[c], k = off[c + 1] - a;
    if (k <= SM_WAVE_MAX) continue;  // (k_sm_long_wave; uniform over the workgroup)
    u32 P = 1;
    while (P < k) P <<= 1;
    for (u32 q = t; q < P; q += SM_LONG_THREADS) idx[q] = q < k ? grp[a + q] : 0xffffffffu;
    if (t == 0) s_win = -1;
    __syncthreads();
    for (u32 size = 2; size <= P; size <<= 1)  // bitonic sort of the row indices
      for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
        for (u32 q = t; q < P; q += SM_LONG_THREADS) {
          const u32 r = q ^ stride;
          if (r > q) {
            const u32 x = idx[q], y = idx[r];
            const bool up = (q & size) == 0;
            if ((x > y) == up) {
              idx[q] = y;
              idx[r] = x;
            }
          }
        }
        __syncthreads();
      }
    // this thread's positions [p0, p1): their max, then the block's exclusive scan
    const u32 per = (k + SM_LONG_THREADS - 1) / SM_LONG_THREADS;
    const u32 p0 = min(k, t * per), p1 = min(k, p0 + per);
    Key m = key_none();
    for (u32 q = p0; q < p1; ++q) m = key_max(m, key_of(rec[idx[q]]));
    s_tc[t] = m.tc;
    s_node[t] = m.node;
    s_mask[t] = m.mask;
    __syncthreads();
    for (u32 d = 1; d < SM_LONG_THREADS; d <<= 1) {  // inclusive max scan (Hillis-Steele)
      Key o = key_none();
      if (t >= d) o = Key{s_tc[t - d], s_node[t - d], s_mask[t - d]};
      __syncthreads();
      if (t >= d) {
        m = key_max(o, m);
        s_tc[t] = m.tc;
        s_node[t] = m.node;
        s_mask[t] = m.mask;
      }
      __syncthreads();
    }
    Key run = (prior_present && prior_present[c]) ? key_of(prior[c]) : key_none();
    if (t > 0) run = key_max(run, Key{s_tc[t - 1], s_node[t - 1], s_mask[t - 1]});
    int32_t win = -1;
    for (u32 q = p0; q < p1; ++q) {
      const u32 i = idx[q];
      const evm_rec r = rec[i];
      const Key ts = key_of(r);
      const bool ups = key_cmp(run, ts) < 0;                            // applyMessages.ts:93
      const bool xr = !((run.mask & KEY_PRESENT) && key_eq(run, ts));  // applyMessages.ts:105
      flags[i] = (ups ? EVM_MSG_UPS : 0u) | (xr ? EVM_MSG_XOR : 0u);
      if (ups) {
        win = (int32_t)i;
        run = ts;
      }
      if (xr) {
        const u32 d = r.minute - mlo;
        if (d >= SM_BINS) {
          atomic_or_if(&info->fold_overflow, 1u);
        } else {
          atomicXor(&bins[d], r.hash);
          atomic_or_if(&pres[d >> 5], 1u << (d & 31));
        }
      }
    }
    if (win >= 0) atomicMax(&s_win, win);
    __syncthreads();
    if (t == 0) winner[c] = s_win;
    __syncthreads();
  }
}

// One workgroup: the batch's leaves (present bins, minute order = code order
// for keys of one base-3 length) merged with tree_in's (ack/axr, L0 sorted
// unique, one owner) into the output tree's arrays; equal keys XOR-combine
// (a leaf whose XOR is 0 stays, as in evm_tree_merge).
__global__ __launch_bounds__(SM_FOLD_THREADS) void k_sm_fold(const u32* __restrict__ bins, const u32* __restrict__ pres,
                                                             const u64* __restrict__ ack, const int32_t* __restrict__ axr,
                                                             u32 L0, u64* __restrict__ nck, int32_t* __restrict__ nxr,
                                                             u64* __restrict__ mck, int32_t* __restrict__ mxr,
                                                             u64* __restrict__ off, u64* __restrict__ ock,
                                                             int32_t* __restrict__ oxr, int32_t* __restrict__ opfx,
                                                             Info* __restrict__ info) {
  __shared__ u32 lds[SM_FOLD_THREADS / 64 + 1];
  __shared__ int32_t xlds[SM_FOLD_THREADS / 64 + 1];
  const u32 t = threadIdx.x;
  if (info->bad || info->bad_aux || info->collision || info->fold_overflow) return;  // (the host reads why)
  const u32 mlo = info->minute_min, mhi = info->minute_max;
  const u32 W = mhi >= mlo ? min(SM_BINS, mhi - mlo + 1) : 0u;
  if (W && base3_len(mlo) != base3_len(mhi)) {
    if (t == 0) atomicOr(&info->fold_overflow, 1u);
    return;
  }
  // (1) the batch's leaves
  const u32 per = (W + SM_FOLD_THREADS - 1) / SM_FOLD_THREADS;
  const u32 a = min(W, t * per), e = min(W, a + per);
  u32 k = 0;
  for (u32 d = a; d < e; ++d) k += (pres[d >> 5] >> (d & 31)) & 1u;
  u32 L1;
  u32 pos = block_inclusive_scan<u32, OpAdd<u32>>(k, lds, OpAdd<u32>(), &L1) - k;
  for (u32 d = a; d < e; ++d)
    if ((pres[d >> 5] >> (d & 31)) & 1u) {
      nck[pos] = minute_code(mlo + d);
      nxr[pos] = (int32_t)bins[d];
      ++pos;
    }
  __syncthreads();
  // (2) merge positions: A[i] before the B keys >= it, B[j] after the A keys <= it
  for (u32 i = t; i < L0; i += SM_FOLD_THREADS) {
    const u64 x = ack[i];
    u32 lo = 0, hi = L1;
    while (lo < hi) {
      const u32 m = (lo + hi) >> 1;
      if (nck[m] < x) lo = m + 1;
      else hi = m;
    }
    mck[i + lo] = x;
    mxr[i + lo] = axr[i];
  }
  for (u32 j = t; j < L1; j += SM_FOLD_THREADS) {
    const u64 x = nck[j];
    u32 lo = 0, hi = L0;
    while (lo < hi) {
      const u32 m = (lo + hi) >> 1;
      if (ack[m] <= x) lo = m + 1;
      else hi = m;
    }
    mck[j + lo] = x;
    mxr[j + lo] = nxr[j];
  }
  __syncthreads();
  // (3) equal neighbours (one from each side) combine; compact
  const u32 M = L0 + L1;
  const u32 per2 = (M + SM_FOLD_THREADS - 1) / SM_FOLD_THREADS;
  const u32 b0 = min(M, t * per2), b1 = min(M, b0 + per2);
  u32 h = 0;
  for (u32 p = b0; p < b1; ++p) h += (p == 0 || mck[p] != mck[p - 1]) ? 1u : 0u;
  u32 L;
  const u32 o0 = block_inclusive_scan<u32, OpAdd<u32>>(h, lds, OpAdd<u32>(), &L) - h;
  u32 o = o0;
  int32_t xacc = 0;
  for (u32 p = b0; p < b1; ++p) {
    if (p != 0 && mck[p] == mck[p - 1]) continue;
    const int32_t x = mxr[p] ^ ((p + 1 < M && mck[p + 1] == mck[p]) ? mxr[p + 1] : 0);
    ock[o] = mck[p];
    oxr[o] = x;
    xacc ^= x;
    ++o;
  }
  // (4) exclusive prefix XOR of the leaves (node hash = range XOR): this
  // thread's leaves, after the XOR of every earlier thread's
  int32_t xtot;
  int32_t run = block_inclusive_scan<int32_t, OpXor<int32_t>>(xacc, xlds, OpXor<int32_t>(), &xtot) ^ xacc;
  for (u32 q = o0; q < o0 + h; ++q) {
    opfx[q] = run;
    run ^= oxr[q];
  }
  if (t == 0) {
    opfx[L] = xtot;
    off[0] = 0;
    off[1] = L;
    info->n_leaves = L;
  }
}

static int apply_small(evm_ctx* ctx, Scratch& S, Info* info, const evm_tree* tree_in, const char* ts, size_t stride,
                       size_t n, const u32* cell, u32 C, const evm_rec* prior, const uint8_t* prior_present,
                       uint8_t* flags, int32_t* winner, evm_tree** tree_out) {
  const int lg = ceil_log2(2 * n);
  const size_t a_cnt = ((size_t)(C + 1) * 4 + 255) & ~(size_t)255;
  const size_t a_bins = (size_t)SM_BINS * 4, a_pres = (size_t)SM_BINS / 8;
  const u32 n_scan_tiles = (u32)std::max<size_t>(1, (C + SM_SCAN_TILE - 1) / SM_SCAN_TILE);
  const size_t a_scan = ((size_t)n_scan_tiles * 8 + 16 + 255) & ~(size_t)255;  // look-back words, counter, error
  const size_t zero_bytes = a_cnt + a_bins + a_pres + (sizeof(u64) << lg) + a_scan;
  char* z = S.alloc<char>(zero_bytes);
  evm_rec* rec = S.alloc<evm_rec>(n);
  u32* off = S.alloc<u32>(C + 1);
  u32* grp = S.alloc<u32>(n);
  const u32 L0 = (u32)tree_in->n_leaves;
  const size_t nmax = std::min<size_t>(n, SM_BINS);
  u64* nck = S.alloc<u64>(nmax);
  int32_t* nxr = S.alloc<int32_t>(nmax);
  u64* mck = S.alloc<u64>(L0 + nmax);
  int32_t* mxr = S.alloc<int32_t>(L0 + nmax);
  if (!z || !rec || !off || !grp || !nck || !nxr || !mck || !mxr) return EVM_ENOMEM;
  u32* cnt = reinterpret_cast<u32*>(z);  // [C] counts, then the long-cell count at [C]
  u32* long_n = cnt + C;
  u32* long_list = S.alloc<u32>(std::max<size_t>(n / SM_SEG + 1, 1));
  if (!long_list) return EVM_ENOMEM;
  u32* bins = reinterpret_cast<u32*>(z + a_cnt);
  u32* pres = reinterpret_cast<u32*>(z + a_cnt + a_bins);
  u64* table = reinterpret_cast<u64*>(z + a_cnt + a_bins + a_pres);
  HIPR(hipMemsetAsync(z, 0, zero_bytes, ctx->stream));
  KLAUNCH(k_sm_pack, dim3(grid_for(n, 256, 1024)), dim3(256), (const uint8_t*)ts, stride, n, cell, C, rec, cnt, table,
          (u32)lg, info);
  {
    u64* lb_status = reinterpret_cast<u64*>(z + a_cnt + a_bins + a_pres + (sizeof(u64) << lg));
    u32* lb_ctr = reinterpret_cast<u32*>(lb_status + n_scan_tiles);
    // (a look-back that gives up sends the batch to the sort path; a partial
    // prefix keeps every slot in range meanwhile)
    KLAUNCH(k_sm_scan_lb, dim3(n_scan_tiles), dim3(SM_FOLD_THREADS), cnt, C, off, lb_status, lb_ctr,
            &info->fold_overflow);
  }
  KLAUNCH(k_sm_scatter, dim3(grid_for(n, 256, 1024)), dim3(256), (const evm_rec*)rec, n, C, cnt, grp);
  KLAUNCH(k_sm_lww, dim3(grid_for(C, 256, 4096)), dim3(256), (const evm_rec*)rec, (const u32*)off, (const u32*)grp, C,
          prior, prior_present, flags, winner, bins, pres, long_list, long_n, info);
  KLAUNCH(k_sm_long_wave, dim3(64), dim3(64 * SM_LW_WAVES), (const evm_rec*)rec, (const u32*)off,
          (const u32*)grp, (const u32*)long_list, (const u32*)long_n, prior, prior_present, flags, winner, bins, pres,
          info);
  KLAUNCH(k_sm_long, dim3(256), dim3(SM_LONG_THREADS), (const evm_rec*)rec, (const u32*)off, (const u32*)grp,
          (const u32*)long_list, (const u32*)long_n, prior, prior_present, flags, winner, bins, pres, info);
  evm_tree* t = nullptr;
  int st = tree_alloc_cap(ctx, 1, (uint64_t)L0 + nmax, &t);
  if (st) return st;
  KLAUNCH(k_sm_fold, dim3(1), dim3(SM_FOLD_THREADS), (const u32*)bins, (const u32*)pres, (const u64*)tree_in->ck,
          (const int32_t*)tree_in->xr, L0, nck, nxr, mck, mxr, t->off, t->ck, t->xr, t->pfx, info);
  Info hi;
  if ((st = read_info(ctx, info, &hi))) {
    tree_destroy(ctx, t);
    return st;
  }
  if (hi.bad) {
    tree_destroy(ctx, t);
    KLAUNCH(k_mark_bad, dim3(grid_for(n, 256)), dim3(256), rec, n, flags);
    return EVM_ENONCANON;
  }
  if (hi.bad_aux || hi.collision) {
    tree_destroy(ctx, t);
    return hi.bad_aux ? EVM_EINVAL : EVM_ECOLLISION;
  }
  if (hi.fold_overflow) {
    tree_destroy(ctx, t);
    return SM_FALLBACK;
  }
  t->n_leaves = hi.n_leaves;
  *tree_out = t;
  return EVM_OK;
}

static int apply_general(evm_ctx* ctx, Scratch& S, Info* info, const evm_tree* tree_in, const char* ts, size_t stride,
                         size_t n, const u32* cell, u32 n_cells, const u32* cell_owner, const evm_rec* prior,
                         const uint8_t* prior_present, const Stored& stored, uint8_t* flags, int32_t* winner,
                         evm_tree** tree_out) {
  int st;
  evm_rec* rec = S.alloc<evm_rec>(n);
  if (!rec) return EVM_ENOMEM;
  if ((st = launch_pack(ctx, ts, stride, n, cell, n_cells, rec, info))) return st;
  // (1) cross-cell PK collisions
  const int lg = ceil_log2(2 * n);
  u64* table = S.alloc<u64>((size_t)1 << lg);
  if (!table) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(table, 0, sizeof(u64) << lg, ctx->stream));
  KLAUNCH(k_xcell, dim3(grid_for(n, 256, 8192)), dim3(256), rec, n, table, (u32)lg, info);
  if ((st = stored_check(ctx, S, stored, &rec->hash, sizeof(evm_rec) / sizeof(u32), ts, stride, cell, n, info)))
    return st;
  // (2) stable sort (cell, index)
  u32* cell_s = S.alloc<u32>(n);
  u32* idx_s = S.alloc<u32>(n);
  if (!cell_s || !idx_s) return EVM_ENOMEM;
  HIPR(hipMemcpyAsync(cell_s, cell, sizeof(u32) * n, hipMemcpyDeviceToDevice, ctx->stream));
  if ((st = launch_iota(ctx, idx_s, n))) return st;
  const int cbits = n_cells > 1 ? 32 - __builtin_clz(n_cells - 1) : 0;
  if ((st = radix_sort_pairs<u32>(ctx, S, cell_s, idx_s, n, 0, cbits))) return st;
  // (3) segmented running max + decisions
  const size_t nt = (n + LWW_TILE - 1) / LWW_TILE;
  u32* t_head = S.alloc<u32>(nt);
  Key* t_key = S.alloc<Key>(nt);
  if (!t_head || !t_key) return EVM_ENOMEM;
  KLAUNCH(k_lww_reduce, dim3(nt), dim3(LWW_THREADS), rec, cell_s, idx_s, n, t_head, t_key);
  KLAUNCH(k_lww_tiles, dim3(1), dim3(LWW_THREADS), t_head, t_key, nt);
  KLAUNCH(k_lww_apply, dim3(nt), dim3(LWW_THREADS), rec, cell_s, idx_s, n, t_head, t_key, prior, prior_present, flags,
          winner);
  // (4) Merkle fold of the XOR messages
  u32* sel = S.alloc<u32>(n);
  u32* pos = S.alloc<u32>(n);
  u32* cnt = S.alloc<u32>(1);
  u64* ck = S.alloc<u64>(n);
  u32* h = S.alloc<u32>(n);
  if (!sel || !pos || !cnt || !ck || !h) return EVM_ENOMEM;
  if ((st = launch_sel(ctx, flags, (uint8_t)EVM_MSG_XOR, n, sel))) return st;
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, sel, n, pos, cnt))) return st;
  if ((st = launch_fold_prep(ctx, rec, flags, (uint8_t)EVM_MSG_XOR, pos, (int)(cell_owner ? OWNER_CELL : OWNER_ZERO),
                              cell_owner, n, ck, h, info)))
    return st;
  Info hi;
  if ((st = read_info(ctx, info, &hi))) return st;
  if (hi.bad) {
    KLAUNCH(k_mark_bad, dim3(grid_for(n, 256)), dim3(256), rec, n, flags);
    return EVM_ENONCANON;
  }
  if (hi.bad_aux) return EVM_EINVAL;
  if (hi.collision) return EVM_ECOLLISION;
  u32 m = 0;
  HIPR(hipMemcpyAsync(&m, cnt, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  return fold_into_tree(ctx, S, tree_in, tree_in->n_owners, ck, h, m, hi, tree_out);
}

__global__ void k_apply_init(Info* __restrict__ info, Info h, int32_t* __restrict__ winner, size_t n_cells) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *info = h;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_cells; i += (size_t)gridDim.x * blockDim.x)
    winner[i] = -1;
}

extern "C" {

int evm_apply_batch(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n, const uint32_t* cell,
                    uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts, size_t prior_stride,
                    const uint8_t* prior_present, uint8_t* flags, int32_t* winner, evm_tree** tree_out) {
  return evm_apply_batch_ex(ctx, tree_in, ts, stride, n, cell, n_cells, cell_owner, prior_ts, prior_stride,
                            prior_present, nullptr, 48, 0, nullptr, flags, winner, tree_out);
}

}  // extern "C"

// evm_apply_batch_ex, or (pend) its asynchronous form: a streaming batch is
// enqueued and ST_PENDING returned; anything else finishes here.
static int apply_entry(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n,
                       const uint32_t* cell, uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts,
                       size_t prior_stride, const uint8_t* prior_present, const char* stored_ts, size_t stored_stride,
                       size_t n_stored, const uint32_t* stored_cell, uint8_t* flags, int32_t* winner,
                       evm_tree** tree_out, int path, evm_pending* pend) {
  if (!ctx || !tree_in || !tree_out || stride < 46 || (n && (!ts || !cell || !flags))) return EVM_EINVAL;
  if (int e = tree_compact(ctx, tree_in)) return e;
  if (n_cells && !winner) return EVM_EINVAL;
  if (prior_present && (!prior_ts || prior_stride < 46)) return EVM_EINVAL;
  if (n_stored && (!stored_ts || !stored_cell || stored_stride < 46)) return EVM_EINVAL;
  const Stored stored{stored_ts, stored_stride, n_stored, stored_cell};
  if (n >= 0x7fffffffu) return EVM_EINVAL;
  *tree_out = nullptr;
  int st;
  {
    Scratch S(ctx);
    Info* info = nullptr;
    if (pend) {
      pend->dev_bytes = side_bufs(nullptr, n, nullptr);
      pend->dev = block_alloc(ctx, &pend->dev_bytes);
      if (!pend->dev) return EVM_ENOMEM;
      SideBufs v;
      side_bufs(pend->dev, n, &v);
      info = v.info;
    } else {
      info = S.alloc<Info>(1);
    }
    evm_rec* prior = S.alloc<evm_rec>(std::max<size_t>(n_cells, 1));
    if (!info || !prior) return EVM_ENOMEM;
    // one launch: the status record, and winner = -1 for every cell; the
    // cells' current maxima (SELECT ... ORDER BY timestamp DESC LIMIT 1)
    // the small-batch path: eligible batches up to SM_MAX_N over many cells,
    // and up to SM_AUTO_FEW over few (measured: 100 msgs 0.060 vs 0.106 ms on
    // the tc path, 1,000 msgs 0.097 vs 0.122 ms)
    const bool small_ok = n && !cell_owner && tree_in->n_owners == 1 && n_stored == 0 && n_cells <= SM_MAX_CELLS &&
                          ((uintptr_t)ts & 15) == 0 && n < 0x7fffffffu;
    const bool small_auto = small_ok && path == 0 && n <= SM_AUTO_FEW;
    // (the tc path's carry writes every cell's winner itself)
    const bool tc_path =
        n && path != 1 && (path == 3 || (path == 0 && !cell_owner && n_cells <= CL_MAX_CELLS && !small_auto));
    auto init = [&](bool winners) -> int {
      const size_t nw = winners ? n_cells : 0;
      KLAUNCH(k_apply_init, dim3(grid_for(std::max<size_t>(nw, 1), 256)), dim3(256), info, info_init(), winner, nw);
      if (prior_present && n_cells) {
        int e = launch_pack(ctx, prior_ts, prior_stride, n_cells, nullptr, 0, prior, nullptr);
        if (e) return e;
        KLAUNCH(k_prior_check, dim3((n_cells + 255) / 256), dim3(256), prior, prior_present, n_cells, info);
      }
      return EVM_OK;
    };
    if ((st = init(!tc_path))) return st;
    if (n == 0) {
      Info hi;
      if ((st = read_info(ctx, info, &hi))) return st;
      if (hi.bad) return EVM_ENONCANON;
      st = merge_into_tree(ctx, S, tree_in, tree_in->n_owners, nullptr, nullptr, 0, tree_out);
    } else if (path == 1 || path == 3 || (path == 0 && !cell_owner && n_cells <= CL_MAX_CELLS && !small_auto)) {
      if (cell_owner || n_cells > CL_MAX_CELLS) return EVM_EINVAL;
      st = TP_REDO;
      if (path != 1) {
        Scratch S2(ctx);  // released before a rerun
        st = apply_stream<true>(ctx, S2, info, tree_in, ts, stride, n, cell, n_cells, prior, prior_present, stored,
                                flags, winner, tree_out, pend);
        if (st == ST_PENDING) return st;
        if (st == TP_REDO) ++ctx->stats.tc_redos;
        else if (st == EVM_OK) ++ctx->stats.tc_batches;
      }
      if (st == TP_REDO) {
        // a tie (equal millis and counter in one cell): the exact walk path
        if (path != 1 && (st = init(true))) return st;
        st = apply_stream<false>(ctx, S, info, tree_in, ts, stride, n, cell, n_cells, prior, prior_present, stored,
                                 flags, winner, tree_out);
      }
    } else {
      // a small batch (one owner, no stored rows): five kernels and one status read
      st = SM_FALLBACK;
      if (small_ok && (path == 4 || small_auto || (path == 0 && n <= SM_MAX_N))) {
        {
          Scratch S2(ctx);  // released before a rerun
          st = apply_small(ctx, S2, info, tree_in, ts, stride, n, cell, n_cells, prior, prior_present, flags, winner,
                           tree_out);
        }
        if (st != SM_FALLBACK) {
          if (st) return st;
          ++ctx->stats.small_batches;
          return evm_sync(ctx);
        }
        ++ctx->stats.small_fallbacks;
        if ((st = init(true))) return st;  // the sort path, from a fresh status record
      }
      st = apply_general(ctx, S, info, tree_in, ts, stride, n, cell, n_cells, cell_owner, prior, prior_present, stored,
                         flags, winner, tree_out);
    }
  }
  if (st) return st;
  return evm_sync(ctx);
}

extern "C" {

int evm_apply_batch_ex(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n,
                       const uint32_t* cell, uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts,
                       size_t prior_stride, const uint8_t* prior_present, const char* stored_ts, size_t stored_stride,
                       size_t n_stored, const uint32_t* stored_cell, uint8_t* flags, int32_t* winner,
                       evm_tree** tree_out) {
  if (!ctx) return EVM_EINVAL;
  return apply_entry(ctx, tree_in, ts, stride, n, cell, n_cells, cell_owner, prior_ts, prior_stride, prior_present,
                     stored_ts, stored_stride, n_stored, stored_cell, flags, winner, tree_out, ctx->client_path,
                     nullptr);
}

int evm_apply_batch_async(evm_ctx* ctx, const evm_tree* tree_in, const char* ts, size_t stride, size_t n,
                          const uint32_t* cell, uint32_t n_cells, const uint32_t* cell_owner, const char* prior_ts,
                          size_t prior_stride, const uint8_t* prior_present, const char* stored_ts,
                          size_t stored_stride, size_t n_stored, const uint32_t* stored_cell, uint8_t* flags,
                          int32_t* winner, evm_pending** out) {
  if (!ctx || !out) return EVM_EINVAL;
  *out = nullptr;
  evm_pending* p;
  if (!ctx->pend_pool.empty()) {
    p = ctx->pend_pool.back();
    ctx->pend_pool.pop_back();
  } else {
    p = new evm_pending();
    if (hipHostMalloc((void**)&p->hinfo, sizeof(Info), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&p->ev, hipEventDisableTiming) != hipSuccess) {
      if (p->hinfo) (void)hipHostFree(p->hinfo);
      delete p;
      return EVM_EDEVICE;
    }
  }
  *p = evm_pending{tree_in, ts, stride, n, cell, n_cells, cell_owner, prior_ts, prior_stride, prior_present,
                   stored_ts, stored_stride, n_stored, stored_cell, flags, winner, false, EVM_OK, nullptr,
                   p->hinfo, p->ev, nullptr, nullptr, 0, nullptr, 0};
  const int st = apply_entry(ctx, tree_in, ts, stride, n, cell, n_cells, cell_owner, prior_ts, prior_stride,
                             prior_present, stored_ts, stored_stride, n_stored, stored_cell, flags, winner, &p->done,
                             ctx->client_path, p);
  if (st == ST_PENDING) {
    p->enqueued = true;
  } else {
    // finished (or failed) synchronously
    if (p->spec) tree_destroy(ctx, p->spec);
    if (p->leaves) block_free(ctx, p->leaves, p->leaves_bytes);
    if (p->dev) block_free(ctx, p->dev, p->dev_bytes);
    p->spec = nullptr;
    p->leaves = nullptr;
    p->dev = nullptr;
    p->status = st;
  }
  *out = p;
  return EVM_OK;
}

}  // extern "C"

void evm_pending_pool_clear(evm_ctx* ctx) {
  for (evm_pending* p : ctx->pend_pool) {
    if (p->hinfo) (void)hipHostFree(p->hinfo);
    if (p->ev) (void)hipEventDestroy(p->ev);
    delete p;
  }
  ctx->pend_pool.clear();
}

extern "C" {

int evm_apply_wait(evm_ctx* ctx, evm_pending* p, evm_tree** tree_out) {
  if (!ctx || !p || !tree_out) return EVM_EINVAL;
  *tree_out = nullptr;
  int st = EVM_OK;
  if (!p->enqueued) {
    st = p->status;
    *tree_out = p->done;
  } else {
    st = hip_ok(hipEventSynchronize(p->ev));
    Info hi = *p->hinfo;
    const bool exact = hi.ties || hi.xf_redo;  // (the tc path's redo: the exact walk path)
    const bool redo = !st && !hi.bad && !hi.bad_aux &&
                      (exact || (!hi.collision && (hi.xc_oversize || hi.fold_overflow)));
    if (st) {
    } else if (hi.bad) {
      KLAUNCH(k_keep_bad, dim3(grid_for(p->n, 256)), dim3(256), p->flags, p->n);  // nothing applied: the culprits
      st = EVM_ENONCANON;
    } else if (hi.bad_aux) {
      st = EVM_EINVAL;
    } else if (redo) {
      // a tie, an oversized hash bucket or a wide minute range: the synchronous paths redo the batch
      if (exact) ++ctx->stats.tc_redos;
      st = apply_entry(ctx, p->tree_in, p->ts, p->stride, p->n, p->cell, p->n_cells, p->cell_owner, p->prior_ts,
                       p->prior_stride, p->prior_present, p->stored_ts, p->stored_stride, p->n_stored, p->stored_cell,
                       p->flags, p->winner, tree_out, exact ? 1 : ctx->client_path, nullptr);
    } else if (hi.collision) {
      st = EVM_ECOLLISION;
    } else if (p->spec) {
      ++ctx->stats.tc_batches;
      p->spec->n_leaves = hi.n_leaves;
      *tree_out = p->spec;
      p->spec = nullptr;
    } else {
      ++ctx->stats.tc_batches;
      Scratch S(ctx);
      const size_t B = (size_t)FOLD_MAXWIN * FOLD_WIN;
      const u64* lck = static_cast<const u64*>(p->leaves);
      st = merge_into_tree(ctx, S, p->tree_in, p->tree_in->n_owners, lck, reinterpret_cast<const int32_t*>(lck + B),
                           hi.n_leaves, tree_out);
    }
    if (p->spec) tree_destroy(ctx, p->spec);
    if (p->leaves) block_free(ctx, p->leaves, p->leaves_bytes);
    if (p->dev) block_free(ctx, p->dev, p->dev_bytes);
    p->spec = nullptr;
    p->leaves = nullptr;
    p->dev = nullptr;
    if (!st) st = evm_sync(ctx);
  }
  p->enqueued = false;
  p->done = nullptr;
  ctx->pend_pool.push_back(p);
  return st;
}

int evm_cross_cell_check(evm_ctx* ctx, const char* ts, size_t stride, size_t n, const uint32_t* cell, uint32_t n_cells,
                         int32_t* found) {
  if (!ctx || !found || stride < 46 || (n && (!ts || !cell))) return EVM_EINVAL;
  if (n >= 0x7fffffffu) return EVM_EINVAL;
  *found = 0;
  if (n == 0) return EVM_OK;
  int st;
  Info hi;
  {
    Scratch S(ctx);
    Info* info = nullptr;
    if ((st = new_info(ctx, S, &info))) return st;
    evm_rec* rec = S.alloc<evm_rec>(n);
    const int lg = ceil_log2(2 * n);
    u64* table = S.alloc<u64>((size_t)1 << lg);
    if (!rec || !table) return EVM_ENOMEM;
    if ((st = launch_pack(ctx, ts, stride, n, cell, n_cells, rec, info))) return st;
    HIPR(hipMemsetAsync(table, 0, sizeof(u64) << lg, ctx->stream));
    KLAUNCH(k_xcell, dim3(grid_for(n, 256, 8192)), dim3(256), rec, n, table, (u32)lg, info);
    if ((st = read_info(ctx, info, &hi))) return st;
  }
  if (hi.bad) return EVM_ENONCANON;
  if (hi.bad_aux) return EVM_EINVAL;
  *found = hi.collision ? 1 : 0;
  return EVM_OK;
}

}  // extern "C"
