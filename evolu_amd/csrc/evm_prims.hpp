// Data-parallel primitives for the engine, written for CDNA4 (wave64, LDS).
//
//   * exclusive scan (add / xor) over u32 / u64 ............ reduce-then-scan, 3 launches
//   * stable LSD radix sort of (key, u32 value) pairs ........ per pass: tile histogram,
//     scan of the digit-major count matrix, stable scatter ranked with 64-lane ballots
//
// Nothing here is reference code: the reference is single-threaded JS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace evm {

constexpr int WAVE = 64;

__device__ __forceinline__ u64 lanemask_lt() {
  const u32 lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// ----------------------------------------------------------------------------
// Decoupled look-back by one whole wave (every lane of the calling wave must
// call it): tile `tile` has published its own aggregate; each step reads the
// status words of the 64 tiles before the window in parallel, and folds the
// aggregates of the tiles nearer than the nearest inclusive prefix -- so a
// tile walks back 64 predecessors per L2 round trip, not one.  Status word:
// LB_AGG | value, or LB_PRE | value (value: the low 62 bits); 0 = not ready.
// Returns the fold of every tile before `tile` (exclusive prefix); a wait
// past `spin_max` polls sets *err and returns what it has.
// ----------------------------------------------------------------------------
constexpr u64 LB_AGG = 1ull << 62, LB_PRE = 2ull << 62, LB_VAL = (1ull << 62) - 1;
template <typename Op>
__device__ __forceinline__ u64 lookback_wave(const u64* status, u32 tile, Op op, u32 spin_max, u32* err) {
  const int lane = __lane_id();
  u64 acc = Op::id();
  long t = (long)tile - 1;
  u32 spins = 0;
  while (t >= 0) {
    const long idx = t - lane;
    const u64 w = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : LB_PRE;
    const u64 pre = __ballot((w & LB_PRE) != 0);
    const u64 ready = __ballot((w & (LB_PRE | LB_AGG)) != 0);
    const int k = pre ? __builtin_ctzll(pre) : 63;  // the nearest inclusive prefix in the window
    const u64 need = k == 63 ? ~0ull : ((2ull << k) - 1ull);
    if ((ready & need) != need) {  // a tile in the way has not published yet
      if (++spins > spin_max) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    u64 v = lane <= k ? (w & LB_VAL) : Op::id();
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = op(v, __shfl_xor(v, d, 64));
    acc = op(acc, v);
    if (pre) break;
    t -= 64;
  }
  return acc;
}
template <typename T>
struct LbAdd {
  __device__ static T id() { return T(0); }
  __device__ T operator()(T a, T b) const { return a + b; }
};
template <typename T>
struct LbXor {
  __device__ static T id() { return T(0); }
  __device__ T operator()(T a, T b) const { return a ^ b; }
};

// ----------------------------------------------------------------------------
// Status bounds (Info.minute_min & co.).  Same-address atomics from every wave
// serialise at the memory side (a min+max per wave made the pack kernel 2-5x
// slower at 2-8k blocks): reduce over the block first, then touch the global
// word only when this block's value improves on what is already stored.
// ----------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const T o = __shfl_xor(v, d, 64);
    v = o < v ? o : v;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const T o = __shfl_xor(v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ void atomic_min_if(T* p, T v) {
  if (v < __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(p, v);
}
template <typename T>
__device__ __forceinline__ void atomic_max_if(T* p, T v) {
  if (v > __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(p, v);
}
template <typename T>
__device__ __forceinline__ void atomic_or_if(T* p, T v) {
  if ((v & ~__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0) atomicOr(p, v);
}

// Block-wide min / max / or of one (mn, mx, flags) triple per thread, folded
// into the global words by thread 0.  Every thread of the block must call it.
template <typename T, int THREADS>
__device__ __forceinline__ void block_fold_bounds(T mn, T mx, u32 flags, T* gmin, T* gmax, u32* gflags) {
  __shared__ T s_mn[THREADS / 64], s_mx[THREADS / 64];
  __shared__ u32 s_fl[THREADS / 64];
  mn = wave_min(mn);
  mx = wave_max(mx);
  const bool any = __ballot(flags != 0) != 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    s_mn[w] = mn;
    s_mx[w] = mx;
    s_fl[w] = any ? 1u : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 fl = 0;
    for (int k = 0; k < THREADS / 64; ++k) {
      mn = s_mn[k] < mn ? s_mn[k] : mn;
      mx = s_mx[k] > mx ? s_mx[k] : mx;
      fl |= s_fl[k];
    }
    if (fl && gflags) atomic_or_if(gflags, 1u);
    if (mx >= mn) {
      atomic_min_if(gmin, mn);
      atomic_max_if(gmax, mx);
    }
  }
}

// ----------------------------------------------------------------------------
// Exclusive scan.  Op is a functor with `static T id()` and `T operator()(T,T)`.
// ----------------------------------------------------------------------------
template <typename T>
struct OpAdd {
  __device__ static T id() { return T(0); }
  __device__ T operator()(T a, T b) const { return a + b; }
};
template <typename T>
struct OpXor {
  __device__ static T id() { return T(0); }
  __device__ T operator()(T a, T b) const { return a ^ b; }
};
template <typename T>
struct OpMax {  // unsigned types: identity 0
  __device__ static T id() { return T(0); }
  __device__ T operator()(T a, T b) const { return a > b ? a : b; }
};

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

// Block-wide inclusive scan of one value per thread (ordered, any associative op).
template <typename T, typename Op>
__device__ __forceinline__ T block_inclusive_scan(T v, T* lds /* >= blockDim.x/64 */, Op op, T* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(v, d, 64);
    if (lane >= d) v = op(o, v);
  }
  if (lane == 63) lds[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    T acc = Op::id();
    for (int w = 0; w < nw; ++w) {
      const T t = lds[w];
      lds[w] = acc;
      acc = op(acc, t);
    }
    lds[nw] = acc;
  }
  __syncthreads();
  v = op(lds[wid], v);
  if (total) *total = lds[nw];
  __syncthreads();
  return v;
}

template <typename T, typename Op>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_reduce(const T* __restrict__ in, size_t n, T* __restrict__ part) {
  __shared__ T lds[SCAN_THREADS / 64 + 1];
  Op op;
  const size_t base = (size_t)blockIdx.x * SCAN_TILE;
  T acc = Op::id();
  if (base + SCAN_TILE <= n) {  // full tile: every load in flight at once
    T v[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) v[k] = in[base + (size_t)k * SCAN_THREADS + threadIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) acc = op(acc, v[k]);
  } else {
    for (int k = 0; k < SCAN_ITEMS; ++k) {
      const size_t i = base + (size_t)k * SCAN_THREADS + threadIdx.x;
      if (i < n) acc = op(acc, in[i]);
    }
  }
  T tot;
  block_inclusive_scan<T, Op>(acc, lds, op, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// One block scans the partials in place (exclusive); *total_out = grand total.
template <typename T, typename Op>
__global__ __launch_bounds__(1024) void k_scan_partials(T* __restrict__ part, size_t np, T* __restrict__ total_out) {
  __shared__ T lds[1024 / 64 + 1];
  Op op;
  const size_t per = (np + blockDim.x - 1) / blockDim.x;
  const size_t b = threadIdx.x * per;
  T acc = Op::id();
  for (size_t i = b; i < b + per && i < np; ++i) acc = op(acc, part[i]);
  T tot;
  T incl = block_inclusive_scan<T, Op>(acc, lds, op, &tot);
  // exclusive prefix for this thread = incl minus own contribution: recompute serially
  T run = Op::id();
  {
    // exclusive of thread = inclusive of previous thread; get via shuffle over LDS
    __shared__ T ex[1024];
    ex[threadIdx.x] = incl;
    __syncthreads();
    run = threadIdx.x == 0 ? Op::id() : ex[threadIdx.x - 1];
  }
  for (size_t i = b; i < b + per && i < np; ++i) {
    const T t = part[i];
    part[i] = run;
    run = op(run, t);
  }
  if (threadIdx.x == 0 && total_out) *total_out = tot;
}

// Tile-local exclusive scan with the tile's carry from the scanned partials.
// The tile is loaded and stored coalesced (element k*THREADS + t) and
// transposed through LDS so that thread t scans elements t*ITEMS ..; the LDS
// index is padded by one word per 32 (conflict-free both ways for 4-B T).
__device__ __forceinline__ u32 scan_pad(u32 i) { return i + (i >> 5); }

template <typename T, typename Op>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_down(const T* __restrict__ in, size_t n, const T* __restrict__ part,
                                                            T* __restrict__ out) {
  __shared__ T tile[SCAN_TILE + SCAN_TILE / 32];
  __shared__ T lds[SCAN_THREADS / 64 + 1];
  __shared__ T ex[SCAN_THREADS];
  Op op;
  const size_t base = (size_t)blockIdx.x * SCAN_TILE;
  const bool full = base + SCAN_TILE <= n;
  if (full) {
    T w[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) w[k] = in[base + k * SCAN_THREADS + threadIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) tile[scan_pad(k * SCAN_THREADS + threadIdx.x)] = w[k];
  } else {
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
      const u32 i = k * SCAN_THREADS + threadIdx.x;
      tile[scan_pad(i)] = base + i < n ? in[base + i] : Op::id();
    }
  }
  __syncthreads();
  T v[SCAN_ITEMS];
  T acc = Op::id();
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = tile[scan_pad(threadIdx.x * SCAN_ITEMS + k)];
    acc = op(acc, v[k]);
  }
  const T incl = block_inclusive_scan<T, Op>(acc, lds, op, nullptr);
  ex[threadIdx.x] = incl;
  __syncthreads();
  T run = op(part[blockIdx.x], threadIdx.x == 0 ? Op::id() : ex[threadIdx.x - 1]);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    tile[scan_pad(threadIdx.x * SCAN_ITEMS + k)] = run;
    run = op(run, v[k]);
  }
  __syncthreads();
  if (full) {
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) out[base + k * SCAN_THREADS + threadIdx.x] = tile[scan_pad(k * SCAN_THREADS + threadIdx.x)];
  } else {
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
      const u32 i = k * SCAN_THREADS + threadIdx.x;
      if (base + i < n) out[base + i] = tile[scan_pad(i)];
    }
  }
}

// Small scans (at most SCAN_LB_TILES tiles) in one launch by decoupled
// look-back: per-owner / per-segment counts (~100k values) took three
// launches of ~20 us each, latency-bound.  Each workgroup takes the next
// tile from a counter (every earlier tile is then held by a running
// workgroup), publishes its aggregate and folds its predecessors' with one
// lookback_wave window.  status[0..nt) and *ticket are zero on entry.  (For
// large inputs the look-back walks long chains of aggregates: 0.44 vs 0.42 ms
// for the three launches at 94M values -- they keep those.)
constexpr u32 SCAN_LB_TILES = 64;
template <typename T, typename Op>
struct Lb32 {  // the look-back's fold of 32-bit values held in the status words' low bits
  __device__ static u64 id() { return (u64)(u32)Op::id(); }
  __device__ u64 operator()(u64 a, u64 b) const { return (u64)(u32)Op()((T)(u32)a, (T)(u32)b); }
};
// Up to SCAN_COLS scans of one length in one launch (blockIdx.y = the
// column; column c's look-back words and counter at status + c * (nt + 1)).
constexpr int SCAN_COLS = 3;
template <typename T>
struct ScanCols {
  const T* in[SCAN_COLS];
  T* out[SCAN_COLS];
  T* total[SCAN_COLS];
};
template <typename T, typename Op>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_small(ScanCols<T> cols, size_t n, u64* __restrict__ status_all) {
  static_assert(sizeof(T) == 4, "32-bit scan values");
  const u32 col = blockIdx.y;
  const T* __restrict__ in = cols.in[col];
  T* __restrict__ out = cols.out[col];
  T* __restrict__ total_out = cols.total[col];
  u64* __restrict__ status = status_all + (size_t)col * (gridDim.x + 1);
  u32* __restrict__ ticket = reinterpret_cast<u32*>(status + gridDim.x);
  __shared__ T tile_lds[SCAN_TILE + SCAN_TILE / 32];
  __shared__ T lds[SCAN_THREADS / 64 + 1];
  __shared__ T ex[SCAN_THREADS];
  __shared__ u32 tile_s, late_s;
  __shared__ T excl_s;
  Op op;
  if (threadIdx.x == 0) {
    tile_s = atomicAdd(ticket, 1u);
    late_s = 0;
  }
  __syncthreads();
  const u32 tile = tile_s;
  const size_t base = (size_t)tile * SCAN_TILE;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const u32 i = k * SCAN_THREADS + threadIdx.x;
    tile_lds[scan_pad(i)] = base + i < n ? in[base + i] : Op::id();
  }
  __syncthreads();
  T v[SCAN_ITEMS];
  T acc = Op::id();
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = tile_lds[scan_pad(threadIdx.x * SCAN_ITEMS + k)];
    acc = op(acc, v[k]);
  }
  T tot;
  const T incl = block_inclusive_scan<T, Op>(acc, lds, op, &tot);
  ex[threadIdx.x] = incl;
  if (threadIdx.x < 64) {  // wave 0: publish the aggregate, fold the predecessors, publish the prefix
    if (threadIdx.x == 0)
      __hip_atomic_store(status + tile, (tile == 0 ? LB_PRE : LB_AGG) | (u64)(u32)tot, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    const u64 e = tile ? lookback_wave(status, tile, Lb32<T, Op>(), 1u << 22, &late_s) : Lb32<T, Op>::id();
    if (threadIdx.x == 0) excl_s = (T)(u32)e;
  }
  __syncthreads();
  if (late_s) {  // (not expected: every predecessor is running) fold in[0, base) directly -- slow, still exact
    T a = Op::id();
    for (size_t i = threadIdx.x; i < base; i += SCAN_THREADS) a = op(a, in[i]);
    T all;
    block_inclusive_scan<T, Op>(a, lds, op, &all);
    if (threadIdx.x == 0) excl_s = all;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const T excl = excl_s;
    if (tile) __hip_atomic_store(status + tile, LB_PRE | (u64)(u32)op(excl, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (base + SCAN_TILE >= n && total_out) *total_out = op(excl, tot);
  }
  T run = op(excl_s, threadIdx.x == 0 ? Op::id() : ex[threadIdx.x - 1]);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    tile_lds[scan_pad(threadIdx.x * SCAN_ITEMS + k)] = run;
    run = op(run, v[k]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const u32 i = k * SCAN_THREADS + threadIdx.x;
    if (base + i < n) out[base + i] = tile_lds[scan_pad(i)];
  }
}

// ----------------------------------------------------------------------------
// Stable LSD radix sort of (key, value) pairs, RADIX_BITS per pass.
// Tile = 256 threads x 16 items.  Wave w owns items [w*64*16, (w+1)*64*16) of
// the tile, processed in 16 rounds of 64 consecutive items, so (round, lane)
// order == input order: ranks from per-wave running digit counters plus a
// 64-lane ballot match are stable.
// ----------------------------------------------------------------------------
constexpr int RADIX_BITS = 8;
constexpr int RADIX_BINS = 1 << RADIX_BITS;
constexpr int SORT_THREADS = 256;
// 24 keys per thread (6,144 per tile): measured over 8..32 on the config-5
// sort path (80M u64 keys, 6 passes): 8: 9.0 ms, 16: 7.6, 20: 6.9, 24: 6.6,
// 28: 8.6, 32: 8.4
constexpr int SORT_ITEMS = 24;
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;

template <typename K>
__device__ __forceinline__ u32 digit_of(K k, int shift, u32 mask) {
  return (u32)(k >> shift) & mask;
}

template <typename K>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_hist(const K* __restrict__ keys, size_t n, int shift, int bits,
                                                             u32* __restrict__ counts, u32 ntiles) {
  __shared__ u32 hist[RADIX_BINS];
  for (int d = threadIdx.x; d < RADIX_BINS; d += SORT_THREADS) hist[d] = 0;
  __syncthreads();
  const u32 mask = (1u << bits) - 1u;
  const size_t base = (size_t)blockIdx.x * SORT_TILE;
#pragma unroll 4
  for (int k = 0; k < SORT_ITEMS; ++k) {
    const size_t i = base + (size_t)k * SORT_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&hist[digit_of(keys[i], shift, mask)], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < (1 << bits); d += SORT_THREADS) counts[(size_t)d * ntiles + blockIdx.x] = hist[d];
}

template <typename K>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_scatter(const K* __restrict__ kin, const u32* __restrict__ vin,
                                                                K* __restrict__ kout, u32* __restrict__ vout, size_t n,
                                                                int shift, int bits, const u32* __restrict__ offsets,
                                                                u32 ntiles) {
  // ranks: per-wave running digit counters + 64-lane ballot match (stable);
  // the tile is then staged in LDS in digit order and written back with
  // consecutive lanes on consecutive addresses inside each digit run.
  __shared__ u32 wcnt[SORT_THREADS / WAVE][RADIX_BINS];
  __shared__ u32 toff[RADIX_BINS];
  __shared__ u32 lstart[RADIX_BINS];
  __shared__ u32 scan_tmp[SORT_THREADS / WAVE + 1];
  __shared__ K skey[SORT_TILE];
  __shared__ u32 sval[SORT_TILE];
  static_assert(RADIX_BINS <= SORT_THREADS, "one digit per thread in the tile scan");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const u32 nbins = 1u << bits, mask = nbins - 1u;
  for (u32 d = threadIdx.x; d < nbins; d += SORT_THREADS) {
    toff[d] = offsets[(size_t)d * ntiles + blockIdx.x];
#pragma unroll
    for (int ww = 0; ww < SORT_THREADS / WAVE; ++ww) wcnt[ww][d] = 0;
  }
  __syncthreads();
  const size_t tbase = (size_t)blockIdx.x * SORT_TILE;
  const size_t wbase = tbase + (size_t)w * WAVE * SORT_ITEMS;
  K key[SORT_ITEMS];
  u32 val[SORT_ITEMS], dig[SORT_ITEMS], rank[SORT_ITEMS];
  const u64 lt = lanemask_lt();
#pragma unroll
  for (int r = 0; r < SORT_ITEMS; ++r) {
    const size_t i = wbase + (size_t)r * WAVE + lane;
    const bool ok = i < n;
    key[r] = ok ? kin[i] : K(0);
    val[r] = ok ? (vin ? vin[i] : (u32)i) : 0u;  // no values: the identity
    const u32 d = digit_of(key[r], shift, mask);
    dig[r] = d;
    u64 peers = __ballot(ok);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (d >> b) & 1u;
      const u64 bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    if (ok) {
      const u32 pre = wcnt[w][d];
      rank[r] = pre + (u32)__popcll(peers & lt);
      // highest lane of the peer group publishes the new running count
      if ((peers >> lane) == 1ull) wcnt[w][d] = pre + (u32)__popcll(peers);
    }
  }
  __syncthreads();
  // per digit: exclusive prefix over waves, tile total, then the tile's digit starts
  u32 tot = 0;
  {
    const u32 d = threadIdx.x;
    if (d < nbins) {
#pragma unroll
      for (int ww = 0; ww < SORT_THREADS / WAVE; ++ww) {
        const u32 t = wcnt[ww][d];
        wcnt[ww][d] = tot;
        tot += t;
      }
    }
  }
  const u32 incl = block_inclusive_scan<u32>(tot, scan_tmp, OpAdd<u32>(), (u32*)nullptr);
  if (threadIdx.x < nbins) lstart[threadIdx.x] = incl - tot;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < SORT_ITEMS; ++r) {
    const size_t i = wbase + (size_t)r * WAVE + lane;
    if (i < n) {
      const u32 lp = lstart[dig[r]] + wcnt[w][dig[r]] + rank[r];
      skey[lp] = key[r];
      sval[lp] = val[r];
    }
  }
  __syncthreads();
  const u32 m = (u32)min((size_t)SORT_TILE, n - tbase);
  for (u32 t = threadIdx.x; t < m; t += SORT_THREADS) {
    const K k = skey[t];
    const u32 d = digit_of(k, shift, mask);
    const u32 dst = toff[d] + (t - lstart[d]);
    kout[dst] = k;
    vout[dst] = sval[t];
  }
}

// ----------------------------------------------------------------------------
// One-sweep variant: the digit histograms of every pass come from ONE read of
// the keys (k_radix_ghist), and each pass is ONE launch whose tiles find their
// per-digit offsets by decoupled look-back over the tiles before them (tile
// ids are taken in launch order from a counter, so every tile a tile waits
// for is already running).  Status word per (tile, digit): flag:2 | pass+1:4
// | count:58; AGG = this tile's count, PRE = inclusive prefix through this
// tile; a word tagged with another pass is not ready, so one clear serves
// every pass of a sort.  A wait that exceeds RADIX_SPIN_MAX polls sets *err
// and gives up (the host then fails the call) instead of hanging.
// ----------------------------------------------------------------------------
constexpr u64 RS_AGG = 1ull << 62, RS_PRE = 2ull << 62, RS_VAL = (1ull << 58) - 1;
constexpr int RS_TAG_SHIFT = 58;
constexpr u32 RADIX_SPIN_MAX = 1u << 24;
constexpr int RADIX_MAX_PASSES = 8;

// RB: bits per pass (8, or 10 when that saves a pass: 1,024 digits, each
// thread owning DPT = 4 consecutive digits in the per-digit phases).
template <typename K, int RB = RADIX_BITS>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_ghist(const K* __restrict__ keys, size_t n, int lo_bit,
                                                              int width, int hi_bit, int passes,
                                                              u32* __restrict__ ghist) {
  constexpr int BINS = 1 << RB;
  __shared__ u32 h[RADIX_MAX_PASSES][BINS];
  for (int i = threadIdx.x; i < RADIX_MAX_PASSES * BINS; i += SORT_THREADS) (&h[0][0])[i] = 0;
  __syncthreads();
  for (size_t i = (size_t)blockIdx.x * SORT_THREADS + threadIdx.x; i < n; i += (size_t)gridDim.x * SORT_THREADS) {
    const K k = keys[i];
    int shift = lo_bit;
    for (int p = 0; p < passes; ++p) {
      const int bits = min(width, hi_bit - shift);
      atomicAdd(&h[p][digit_of(k, shift, (1u << bits) - 1u)], 1u);
      shift += bits;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * BINS; i += SORT_THREADS) {
    const u32 v = (&h[0][0])[i];
    if (v) atomicAdd(&ghist[i], v);
  }
}

// exclusive scan of each pass's digit counts (one workgroup, DPT digits per thread)
template <int RB = RADIX_BITS>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_gscan(u32* __restrict__ ghist, int passes) {
  constexpr int BINS = 1 << RB, DPT = BINS / SORT_THREADS;
  static_assert(DPT >= 1, "at least one digit per thread");
  __shared__ u32 scan_tmp[SORT_THREADS / WAVE + 1];
  for (int p = 0; p < passes; ++p) {
    u32 v[DPT], sum = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      v[k] = ghist[p * BINS + threadIdx.x * DPT + k];
      sum += v[k];
    }
    u32 run = block_inclusive_scan<u32>(sum, scan_tmp, OpAdd<u32>(), (u32*)nullptr) - sum;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      ghist[p * BINS + threadIdx.x * DPT + k] = run;
      run += v[k];
    }
    __syncthreads();
  }
}

template <typename K, int RB = RADIX_BITS>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_onesweep(const K* __restrict__ kin, const u32* __restrict__ vin,
                                                                 K* __restrict__ kout, u32* __restrict__ vout, size_t n,
                                                                 int shift, int bits, const u32* __restrict__ goff,
                                                                 u64* __restrict__ status, u32* __restrict__ tile_ctr,
                                                                 int pass, u32* __restrict__ err) {
  constexpr int BINS = 1 << RB, DPT = BINS / SORT_THREADS;
  const u64 tag = (u64)(pass + 1) << RS_TAG_SHIFT, tag_mask = 15ull << RS_TAG_SHIFT;
  __shared__ u32 wcnt[SORT_THREADS / WAVE][BINS];
  __shared__ u32 toff[BINS];
  __shared__ u32 lstart[BINS];
  __shared__ u32 scan_tmp[SORT_THREADS / WAVE + 1];
  __shared__ u32 tile_s;
  __shared__ K skey[SORT_TILE];
  __shared__ u32 sval[SORT_TILE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const u32 nbins = 1u << bits, mask = nbins - 1u;
  if (threadIdx.x == 0) tile_s = atomicAdd(tile_ctr, 1u);
  for (u32 d = threadIdx.x; d < nbins; d += SORT_THREADS) {
#pragma unroll
    for (int ww = 0; ww < SORT_THREADS / WAVE; ++ww) wcnt[ww][d] = 0;
  }
  __syncthreads();
  const u32 tile = tile_s;
  const size_t tbase = (size_t)tile * SORT_TILE;
  const size_t wbase = tbase + (size_t)w * WAVE * SORT_ITEMS;
  K key[SORT_ITEMS];
  u32 val[SORT_ITEMS], dig[SORT_ITEMS], rank[SORT_ITEMS];
  const u64 lt = lanemask_lt();
#pragma unroll
  for (int r = 0; r < SORT_ITEMS; ++r) {
    const size_t i = wbase + (size_t)r * WAVE + lane;
    const bool ok = i < n;
    key[r] = ok ? kin[i] : K(0);
    val[r] = ok ? (vin ? vin[i] : (u32)i) : 0u;  // no values: the identity (the first pass of an index sort)
  }
#pragma unroll
  for (int r = 0; r < SORT_ITEMS; ++r) {
    const size_t i = wbase + (size_t)r * WAVE + lane;
    const bool ok = i < n;
    const u32 d = digit_of(key[r], shift, mask);
    dig[r] = d;
    u64 peers = __ballot(ok);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (d >> b) & 1u;
      const u64 bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    if (ok) {
      const u32 pre = wcnt[w][d];
      rank[r] = pre + (u32)__popcll(peers & lt);
      if ((peers >> lane) == 1ull) wcnt[w][d] = pre + (u32)__popcll(peers);
    }
  }
  __syncthreads();
  // per digit (DPT consecutive ones per thread): prefix over waves, then
  // publish this tile's count and look back for the tiles before it
  u32 tot[DPT], tsum = 0;
#pragma unroll
  for (int k = 0; k < DPT; ++k) {
    const u32 d = threadIdx.x * DPT + k;
    tot[k] = 0;
    if (d < nbins) {
#pragma unroll
      for (int ww = 0; ww < SORT_THREADS / WAVE; ++ww) {
        const u32 t = wcnt[ww][d];
        wcnt[ww][d] = tot[k];
        tot[k] += t;
      }
      u64* my = status + (size_t)tile * BINS + d;
      u64 excl = 0;
      if (tile == 0) {
        __hip_atomic_store(my, RS_PRE | tag | (u64)tot[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_store(my, RS_AGG | tag | (u64)tot[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        u32 spins = 0;
        for (int t = (int)tile - 1; t >= 0;) {
          const u64 s = __hip_atomic_load(status + (size_t)t * BINS + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const bool mine = (s & tag_mask) == tag;
          if (mine && (s & RS_PRE)) {
            excl += s & RS_VAL;
            break;
          }
          if (mine && (s & RS_AGG)) {
            excl += s & RS_VAL;
            --t;
            continue;
          }
          if (++spins > RADIX_SPIN_MAX) {
            atomicOr(err, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(my, RS_PRE | tag | (excl + tot[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      toff[d] = goff[d] + (u32)excl;
    }
    tsum += tot[k];
  }
  u32 run = block_inclusive_scan<u32>(tsum, scan_tmp, OpAdd<u32>(), (u32*)nullptr) - tsum;
#pragma unroll
  for (int k = 0; k < DPT; ++k) {
    const u32 d = threadIdx.x * DPT + k;
    if (d < nbins) lstart[d] = run;
    run += tot[k];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < SORT_ITEMS; ++r) {
    const size_t i = wbase + (size_t)r * WAVE + lane;
    if (i < n) {
      const u32 lp = lstart[dig[r]] + wcnt[w][dig[r]] + rank[r];
      skey[lp] = key[r];
      sval[lp] = val[r];
    }
  }
  __syncthreads();
  const u32 m = (u32)min((size_t)SORT_TILE, n - tbase);
  for (u32 t = threadIdx.x; t < m; t += SORT_THREADS) {
    const K k = skey[t];
    const u32 dd = digit_of(k, shift, mask);
    const u32 dst = toff[dd] + (t - lstart[dd]);
    kout[dst] = k;
    vout[dst] = sval[t];
  }
}

}  // namespace evm
