// MI355X (gfx950) batch-merge engine for Evolu's CRDT sync path: kernels +
// the C ABI declared in include/evm.h.
//
// Reference semantics restated here (harrywebdev/evolu @ 2025-01-31):
//   applyMessages.ts:26-131   LWW decisions per message, in batch order
//   merkleTree.ts:8-50        XOR of murmur3(ts) along the base-3 minute key
//   merkleTree.ts:52-91       greedy diff descent
//   apps/server/src/index.ts  per-owner INSERT OR IGNORE + XOR (see evm_server.hip)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <stdio.h>

#include <algorithm>
#include <string>
#include <vector>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_pack.hpp"
#include "evm_prims.hpp"

using namespace evm;

// ============================================================================
// K1: pack
// ============================================================================
constexpr int PACK_THREADS = 256;

__global__ __launch_bounds__(PACK_THREADS) void k_pack(const uint8_t* __restrict__ ts, size_t stride, size_t n,
                                                       const u32* __restrict__ aux, u32 aux_limit,
                                                       evm_rec* __restrict__ out, Info* __restrict__ info,
                                                       u32* __restrict__ minute_out) {
  u32 bad = 0, bad_aux = 0, mn = 0xffffffffu, mx = 0u;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32 w[12];
    load_ts(ts, stride, i, w);
    const Parsed p = parse_ts46(w);
    evm_rec r;
    r.tc = p.tc;
    r.node = p.node;
    r.meta = p.meta;
    r.hash = p.hash;
    r.minute = p.minute;
    r.aux = aux ? aux[i] : 0u;
    if (aux_limit && r.aux >= aux_limit) bad_aux = 1;
    out[i] = r;
    if (minute_out) minute_out[i] = p.minute;
    if (p.meta & EVM_META_VALID) {
      mn = min(mn, p.minute);
      mx = max(mx, p.minute);
    } else {
      bad = 1;
    }
  }
  // wave reduce then one atomic per wave
  for (int d = 32; d >= 1; d >>= 1) {
    bad |= __shfl_xor(bad, d, 64);
    bad_aux |= __shfl_xor(bad_aux, d, 64);
    mn = min(mn, (u32)__shfl_xor(mn, d, 64));
    mx = max(mx, (u32)__shfl_xor(mx, d, 64));
  }
  if ((threadIdx.x & 63) == 0 && info) {
    if (bad) atomic_or_if(&info->bad, 1u);
    if (bad_aux) atomic_or_if(&info->bad_aux, 1u);
    if (mn != 0xffffffffu) {
      atomic_min_if(&info->minute_min, mn);
      atomic_max_if(&info->minute_max, mx);
    }
  }
}

// The same for 16-B aligned 48-byte rows: a wave reads its 64 rows as three
// coalesced (non-temporal) 16-B loads per lane and redistributes them through
// LDS, as the client path's K1 does (evm_pack.hpp).
// REC = false: the minutes and the checks only (the server's segment keys
// when K5 parses the rows itself).
template <bool REC>
__device__ __forceinline__ void pack48_body(const uint8_t* __restrict__ ts, size_t n, const u32* __restrict__ aux,
                                            u32 aux_limit, evm_rec* __restrict__ out, Info* __restrict__ info,
                                            u32* __restrict__ minute_out) {
  __shared__ uint4 stage[PACK_THREADS / 64][192];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u32 bad = 0, bad_aux = 0, mn = 0xffffffffu, mx = 0u;
  const size_t step = (size_t)gridDim.x * PACK_THREADS;
  for (size_t first = ((size_t)blockIdx.x * (PACK_THREADS / 64) + wv) * 64; first < n; first += step) {
    uint4 a, b, c;
    clp_fetch<true>(ts, 48, n, first, a, b, c);
    stage[wv][lane] = a;
    stage[wv][lane + 64] = b;
    stage[wv][lane + 128] = c;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const uint4 x = stage[wv][3 * lane], y = stage[wv][3 * lane + 1], z = stage[wv][3 * lane + 2];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    u32 w[12] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, z.x, z.y, z.z, z.w & 0xffffu};
    const size_t i = first + lane;
    if (i >= n) continue;
    const Parsed p = parse_ts46(w);
    evm_rec r;
    r.tc = p.tc;
    r.node = p.node;
    r.meta = p.meta;
    r.hash = p.hash;
    r.minute = p.minute;
    r.aux = aux ? aux[i] : 0u;
    if (aux_limit && r.aux >= aux_limit) bad_aux = 1;
    if (REC) out[i] = r;  // (staging the records through LDS for 1-KiB stores measured slower: 1.92 vs 1.68 ms)
    if (minute_out) minute_out[i] = p.minute;  // compact copy for the server's segment keys
    if (p.meta & EVM_META_VALID) {
      mn = min(mn, p.minute);
      mx = max(mx, p.minute);
    } else {
      bad = 1;
    }
  }
  for (int d = 32; d >= 1; d >>= 1) {
    bad |= __shfl_xor(bad, d, 64);
    bad_aux |= __shfl_xor(bad_aux, d, 64);
    mn = min(mn, (u32)__shfl_xor(mn, d, 64));
    mx = max(mx, (u32)__shfl_xor(mx, d, 64));
  }
  if ((threadIdx.x & 63) == 0 && info) {
    if (bad) atomic_or_if(&info->bad, 1u);
    if (bad_aux) atomic_or_if(&info->bad_aux, 1u);
    if (mn != 0xffffffffu) {
      atomic_min_if(&info->minute_min, mn);
      atomic_max_if(&info->minute_max, mx);
    }
  }
}

__global__ __launch_bounds__(PACK_THREADS) void k_pack48(const uint8_t* __restrict__ ts, size_t n,
                                                         const u32* __restrict__ aux, u32 aux_limit,
                                                         evm_rec* __restrict__ out, Info* __restrict__ info,
                                                         u32* __restrict__ minute_out) {
  pack48_body<true>(ts, n, aux, aux_limit, out, info, minute_out);
}
__global__ __launch_bounds__(PACK_THREADS) void k_minute48(const uint8_t* __restrict__ ts, size_t n,
                                                           const u32* __restrict__ aux, u32 aux_limit,
                                                           Info* __restrict__ info, u32* __restrict__ minute_out) {
  pack48_body<false>(ts, n, aux, aux_limit, nullptr, info, minute_out);
}

int evm::launch_minutes(evm_ctx* ctx, const char* ts, size_t n, const u32* aux, u32 aux_limit, Info* info,
                        u32* minute_out) {
  if (n == 0) return EVM_OK;
  if (((uintptr_t)ts & 15) != 0) return EVM_EINVAL;
  KLAUNCH(k_minute48, dim3(grid_for(n, PACK_THREADS, 2048)), dim3(PACK_THREADS), (const uint8_t*)ts, n, aux, aux_limit,
          info, minute_out);
  return hip_ok(hipGetLastError());
}

int evm::launch_pack(evm_ctx* ctx, const char* ts, size_t stride, size_t n, const u32* aux, u32 aux_limit, evm_rec* out,
                     Info* info, u32* minute_out) {
  if (n == 0) return EVM_OK;
  if (stride == 48 && ((uintptr_t)ts & 15) == 0)
    KLAUNCH(k_pack48, dim3(grid_for(n, PACK_THREADS, 2048)), dim3(PACK_THREADS), (const uint8_t*)ts, n, aux,
            aux_limit, out, info, minute_out);
  else
    KLAUNCH(k_pack, dim3(grid_for(n, PACK_THREADS, 4096)), dim3(PACK_THREADS), (const uint8_t*)ts, stride, n, aux,
            aux_limit, out, info, minute_out);
  return hip_ok(hipGetLastError());
}

// ============================================================================
// Scans and sorts (host drivers for evm_prims.hpp)
// ============================================================================
// k columns (k <= SCAN_COLS) of n <= SCAN_LB_TILES tiles in one launch
template <typename T, template <typename> class Op>
static int scan_small_cols(evm_ctx* ctx, Scratch& S, int k, const T* const* ins, size_t n, T* const* outs,
                           T* const* tots) {
  const size_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  u64* status = S.alloc<u64>((size_t)k * (nt + 1));  // per column: look-back words, then the tile counter
  if (!status) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(status, 0, (size_t)k * (nt + 1) * sizeof(u64), ctx->stream));
  ScanCols<T> cols{};
  for (int c = 0; c < k; ++c) {
    cols.in[c] = ins[c];
    cols.out[c] = outs[c];
    cols.total[c] = tots[c];
  }
  KLAUNCH((k_scan_small<T, Op<T>>), dim3((unsigned)nt, (unsigned)k), dim3(SCAN_THREADS), cols, n, status);
  return hip_ok(hipGetLastError());
}

// Several exclusive add-scans of one length (per-owner / per-segment counts):
// one launch when they are small, else one scan after the other.
int evm::scan_exclusive_cols(evm_ctx* ctx, Scratch& S, int k, const u32* const* ins, size_t n, u32* const* outs,
                             u32* const* tots) {
  const size_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  bool ok = n > 0 && nt <= SCAN_LB_TILES && k <= SCAN_COLS;
  for (int c = 0; c < k && ok; ++c) ok = (const void*)ins[c] != (const void*)outs[c];
  if (ok) return scan_small_cols<u32, OpAdd>(ctx, S, k, ins, n, outs, tots);
  for (int c = 0; c < k; ++c) {
    const int st = scan_exclusive<u32, OpAdd>(ctx, S, ins[c], n, outs[c], tots[c]);
    if (st) return st;
  }
  return EVM_OK;
}

template <typename T, template <typename> class Op>
int evm::scan_exclusive(evm_ctx* ctx, Scratch& S, const T* in, size_t n, T* out, T* total_dev) {
  if (n == 0) {
    if (total_dev) HIPR(hipMemsetAsync(total_dev, 0, sizeof(T), ctx->stream));
    return EVM_OK;
  }
  const size_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  if constexpr (sizeof(T) == 4) {
    if (nt <= SCAN_LB_TILES && (const void*)in != (const void*)out) {
      const T* ins[1] = {in};
      T* outs[1] = {out};
      T* tots[1] = {total_dev};
      return scan_small_cols<T, Op>(ctx, S, 1, ins, n, outs, tots);
    }
  }
  T* part = S.alloc<T>(nt);
  if (!part) return EVM_ENOMEM;
  KLAUNCH((k_scan_reduce<T, Op<T>>), dim3(nt), dim3(SCAN_THREADS), in, n, part);
  KLAUNCH((k_scan_partials<T, Op<T>>), dim3(1), dim3(1024), part, nt, total_dev);
  KLAUNCH((k_scan_down<T, Op<T>>), dim3(nt), dim3(SCAN_THREADS), in, n, part, out);
  return hip_ok(hipGetLastError());
}
template int evm::scan_exclusive<u32, OpAdd>(evm_ctx*, Scratch&, const u32*, size_t, u32*, u32*);
template int evm::scan_exclusive<int32_t, OpXor>(evm_ctx*, Scratch&, const int32_t*, size_t, int32_t*, int32_t*);
template int evm::scan_exclusive<u64, OpMax>(evm_ctx*, Scratch&, const u64*, size_t, u64*, u64*);
template int evm::scan_exclusive<u64, OpAdd>(evm_ctx*, Scratch&, const u64*, size_t, u64*, u64*);

template <typename K>
int evm::radix_sort_pairs(evm_ctx* ctx, Scratch& S, K*& keys, u32*& vals, size_t n, int lo_bit, int hi_bit) {
  // vals == nullptr: the values are the identity 0..n-1 (made by the first pass)
  if (n <= 1 || hi_bit <= lo_bit) {
    if (!vals) {
      vals = S.alloc<u32>(std::max<size_t>(n, 1));
      if (!vals) return EVM_ENOMEM;
      return launch_iota(ctx, vals, n);
    }
    return EVM_OK;
  }
  const int B = hi_bit - lo_bit;
  // 10-bit digits when they save a pass (EVM_OPT_RADIX 2): 1,024 digits per
  // pass, 4 per thread in the look-back
  const bool wide = ctx->radix_onesweep == 2 && (B + 9) / 10 < (B + RADIX_BITS - 1) / RADIX_BITS;
  const int rb = wide ? 10 : RADIX_BITS;
  const int bins = 1 << rb;
  const int passes = (B + rb - 1) / rb;
  const int width = (B + passes - 1) / passes;
  const u32 ntiles = (u32)((n + SORT_TILE - 1) / SORT_TILE);
  K* k2 = S.alloc<K>(n);
  u32* v2 = S.alloc<u32>(n);
  u32* v3 = vals ? v2 : S.alloc<u32>(n);  // identity values: a second buffer for the ping-pong
  if (!k2 || !v2 || !v3) return EVM_ENOMEM;
  if (ctx->radix_onesweep && passes <= RADIX_MAX_PASSES) {
    // one read for every pass's digit histogram, then one launch per pass
    u64* status = S.alloc<u64>((size_t)bins * ntiles);
    u32* small = S.alloc<u32>((size_t)RADIX_MAX_PASSES * bins + RADIX_MAX_PASSES + 1);
    if (!status || !small) return EVM_ENOMEM;
    u32* gh = small;
    u32* ctr = small + RADIX_MAX_PASSES * bins;
    u32* err = ctr + RADIX_MAX_PASSES;
    HIPR(hipMemsetAsync(small, 0, sizeof(u32) * ((size_t)RADIX_MAX_PASSES * bins + RADIX_MAX_PASSES + 1),
                        ctx->stream));
    HIPR(hipMemsetAsync(status, 0, sizeof(u64) * bins * ntiles, ctx->stream));
    if (wide) {
      KLAUNCH((k_radix_ghist<K, 10>), dim3(std::min<u32>(ntiles, 2048)), dim3(SORT_THREADS), keys, n, lo_bit, width,
              hi_bit, passes, gh);
      KLAUNCH((k_radix_gscan<10>), dim3(1), dim3(SORT_THREADS), gh, passes);
    } else {
      KLAUNCH((k_radix_ghist<K>), dim3(std::min<u32>(ntiles, 2048)), dim3(SORT_THREADS), keys, n, lo_bit, width,
              hi_bit, passes, gh);
      KLAUNCH((k_radix_gscan<>), dim3(1), dim3(SORT_THREADS), gh, passes);
    }
    int shift = lo_bit;
    for (int p = 0; p < passes; ++p) {
      const int bits = std::min(width, hi_bit - shift);
      if (wide)
        KLAUNCH((k_radix_onesweep<K, 10>), dim3(ntiles), dim3(SORT_THREADS), keys, vals, k2, v2, n, shift, bits,
                gh + (size_t)p * bins, status, ctr + p, p, err);
      else
        KLAUNCH((k_radix_onesweep<K>), dim3(ntiles), dim3(SORT_THREADS), keys, vals, k2, v2, n, shift, bits,
                gh + (size_t)p * bins, status, ctr + p, p, err);
      std::swap(keys, k2);
      std::swap(vals, v2);
      if (!v2) v2 = v3;
      shift += bits;
    }
    u32 h_err = 0;
    HIPR(hipMemcpyAsync(&h_err, err, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
    return h_err ? EVM_EDEVICE : hip_ok(hipGetLastError());
  }
  u32* counts = S.alloc<u32>((size_t)RADIX_BINS * ntiles);
  u32* offs = S.alloc<u32>((size_t)RADIX_BINS * ntiles);
  if (!counts || !offs) return EVM_ENOMEM;
  int shift = lo_bit;
  // (8-bit passes: `wide` needs the one-sweep kernels)
  for (int p = 0; p < passes; ++p) {
    const int bits = std::min(width, hi_bit - shift);
    KLAUNCH((k_radix_hist<K>), dim3(ntiles), dim3(SORT_THREADS), keys, n, shift, bits, counts,
                       ntiles);
    int st = scan_exclusive<u32, OpAdd>(ctx, S, counts, (size_t)(1u << bits) * ntiles, offs, (u32*)nullptr);
    if (st) return st;
    KLAUNCH((k_radix_scatter<K>), dim3(ntiles), dim3(SORT_THREADS), keys, vals, k2, v2, n,
                       shift, bits, offs, ntiles);
    std::swap(keys, k2);
    std::swap(vals, v2);
    if (!v2) v2 = v3;
    shift += bits;
  }
  return hip_ok(hipGetLastError());
}
template int evm::radix_sort_pairs<u32>(evm_ctx*, Scratch&, u32*&, u32*&, size_t, int, int);
template int evm::radix_sort_pairs<u64>(evm_ctx*, Scratch&, u64*&, u32*&, size_t, int, int);

// ============================================================================
// Trees: leaf lists keyed by ck = owner << 40 | code, sorted, unique.
// ============================================================================
__global__ void k_iota(u32* __restrict__ v, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) v[i] = (u32)i;
}

// Fold input: for every selected message, (owner << 40 | code(minute), hash).
__global__ void k_fold_prep(const evm_rec* __restrict__ rec, const uint8_t* __restrict__ flags, uint8_t sel_mask,
                            const u32* __restrict__ pos, int owner_mode, const u32* __restrict__ cell_owner, size_t n,
                            u64* __restrict__ ck, u32* __restrict__ h, Info* __restrict__ info) {
  u64 mn = ~0ull, mx = 0ull;
  u32 maxlen = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (flags && !(flags[i] & sel_mask)) continue;
    const evm_rec r = rec[i];
    const u32 owner = owner_mode == OWNER_CELL ? cell_owner[r.aux] : (owner_mode == OWNER_AUX ? r.aux : 0u);
    const u64 c = ((u64)owner << 40) | minute_code(r.minute);
    const size_t o = pos ? pos[i] : i;
    ck[o] = c;
    h[o] = r.hash;
    mn = min(mn, c);
    mx = max(mx, c);
    maxlen = max(maxlen, (u32)base3_len(r.minute));
  }
  for (int d = 32; d >= 1; d >>= 1) {
    mn = min(mn, (u64)__shfl_xor(mn, d, 64));
    mx = max(mx, (u64)__shfl_xor(mx, d, 64));
    maxlen = max(maxlen, (u32)__shfl_xor(maxlen, d, 64));
  }
  if ((threadIdx.x & 63) == 0 && mx >= mn) {
    atomic_min_if(&info->ck_min, mn);
    atomic_max_if(&info->ck_max, mx);
    atomic_max_if(&info->maxlen, maxlen);
  }
}

__global__ void k_sel_u32(const uint8_t* __restrict__ flags, uint8_t mask, size_t n, u32* __restrict__ sel) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    sel[i] = (flags[i] & mask) ? 1u : 0u;
}

__global__ void k_info_set(Info* __restrict__ d, Info h) { *d = h; }

int evm::launch_info_set(evm_ctx* ctx, Info* d, const Info& h) {
  hipLaunchKernelGGL(k_info_set, dim3(1), dim3(1), 0, ctx->stream, d, h);
  return hip_ok(hipGetLastError());
}

int evm::launch_iota(evm_ctx* ctx, u32* v, size_t n) {
  KLAUNCH(k_iota, dim3(grid_for(n, 256)), dim3(256), v, n);
  return hip_ok(hipGetLastError());
}
int evm::launch_sel(evm_ctx* ctx, const uint8_t* flags, uint8_t mask, size_t n, u32* sel) {
  KLAUNCH(k_sel_u32, dim3(grid_for(n, 256)), dim3(256), flags, mask, n, sel);
  return hip_ok(hipGetLastError());
}
int evm::launch_fold_prep(evm_ctx* ctx, const evm_rec* rec, const uint8_t* flags, uint8_t sel_mask, const u32* pos,
                          int owner_mode, const u32* cell_owner, size_t n, u64* ck, u32* h, Info* info) {
  if (n == 0) return EVM_OK;
  KLAUNCH(k_fold_prep, dim3(grid_for(n, 256, 4096)), dim3(256), rec, flags, sel_mask, pos, owner_mode, cell_owner, n, ck,
          h, info);
  return hip_ok(hipGetLastError());
}

__global__ void k_heads(const u64* __restrict__ ck, size_t m, u32* __restrict__ head) {
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < m; p += (size_t)gridDim.x * blockDim.x)
    head[p] = (p == 0 || ck[p] != ck[p - 1]) ? 1u : 0u;
}

__global__ void k_run_starts(const u64* __restrict__ ck, const u32* __restrict__ head, const u32* __restrict__ lid,
                             size_t m, u32* __restrict__ start, u64* __restrict__ out_ck) {
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < m; p += (size_t)gridDim.x * blockDim.x)
    if (head[p]) {
      start[lid[p]] = (u32)p;
      out_ck[lid[p]] = ck[p];
    }
}

__global__ void k_run_xor(const u32* __restrict__ start, const int32_t* __restrict__ pfx, const u32* __restrict__ nrun,
                          size_t m, int32_t* __restrict__ out_xr) {
  const u32 L = *nrun;
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < L; r += (size_t)gridDim.x * blockDim.x) {
    const u32 a = start[r], b = (r + 1 < L) ? start[r + 1] : (u32)m;
    out_xr[r] = pfx[b] ^ pfx[a];
  }
}

// Reduces sorted (ck, h) runs of equal ck to unique leaves (ck, xor).
// Returns the leaf count (host sync).
int evm::reduce_runs(evm_ctx* ctx, Scratch& S, const u64* ck, const int32_t* h, size_t m, u64* out_ck, int32_t* out_xr,
                     uint64_t* out_count) {
  if (m == 0) {
    *out_count = 0;
    return EVM_OK;
  }
  u32* head = S.alloc<u32>(m);
  u32* lid = S.alloc<u32>(m);
  u32* start = S.alloc<u32>(m);
  int32_t* pfx = S.alloc<int32_t>(m + 1);
  u32* nrun = S.alloc<u32>(1);
  if (!head || !lid || !start || !pfx || !nrun) return EVM_ENOMEM;
  const int g = grid_for(m, 256);
  KLAUNCH(k_heads, dim3(g), dim3(256), ck, m, head);
  int st = scan_exclusive<u32, OpAdd>(ctx, S, head, m, lid, nrun);
  if (st) return st;
  st = scan_exclusive<int32_t, OpXor>(ctx, S, h, m, pfx, pfx + m);
  if (st) return st;
  KLAUNCH(k_run_starts, dim3(g), dim3(256), ck, head, lid, m, start, out_ck);
  KLAUNCH(k_run_xor, dim3(g), dim3(256), start, pfx, nrun, m, out_xr);
  u32 L = 0;
  HIPR(hipMemcpyAsync(&L, nrun, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  *out_count = L;
  return hip_ok(hipGetLastError());
}

__device__ __forceinline__ size_t lower_bound_u64(const u64* a, size_t lo, size_t hi, u64 x) {
  while (lo < hi) {
    const size_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ size_t upper_bound_u64(const u64* a, size_t lo, size_t hi, u64 x) {
  while (lo < hi) {
    const size_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Merge of two sorted unique leaf lists; equal keys land adjacent (A first).
__global__ void k_merge_a(const u64* __restrict__ ack, const int32_t* __restrict__ axr, size_t na, const u64* __restrict__ bck,
                          size_t nb, u64* __restrict__ ock, int32_t* __restrict__ oxr) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += (size_t)gridDim.x * blockDim.x) {
    const size_t j = lower_bound_u64(bck, 0, nb, ack[i]);
    ock[i + j] = ack[i];
    oxr[i + j] = axr[i];
  }
}
__global__ void k_merge_b(const u64* __restrict__ bck, const int32_t* __restrict__ bxr, size_t nb, const u64* __restrict__ ack,
                          size_t na, u64* __restrict__ ock, int32_t* __restrict__ oxr) {
  for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += (size_t)gridDim.x * blockDim.x) {
    const size_t i = upper_bound_u64(ack, 0, na, bck[j]);
    ock[i + j] = bck[j];
    oxr[i + j] = bxr[j];
  }
}

__global__ void k_owner_off(const u64* __restrict__ ck, size_t L, u32 n_owners, u64* __restrict__ off) {
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o <= n_owners; o += (size_t)gridDim.x * blockDim.x)
    off[o] = (o == n_owners) ? (u64)L : (u64)lower_bound_u64(ck, 0, L, (u64)o << 40);
}

// Device leaf lists (per-owner offsets + codes without the owner bits) <->
// tree leaves (ck = owner << 40 | code).  One wave per owner; codes must be
// valid, sorted and unique per owner.
__global__ void k_leaves_in(const u64* __restrict__ off, const u64* __restrict__ code, u32 n_owners,
                            u64* __restrict__ ck, u32* __restrict__ bad) {
  const u32 lane = threadIdx.x & 63;
  for (u32 o = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; o < n_owners; o += (gridDim.x * blockDim.x) >> 6) {
    const u64 a = off[o], b = off[o + 1];
    if (b < a) {
      if (lane == 0) atomicOr(bad, 1u);
      continue;
    }
    for (u64 k = a + lane; k < b; k += 64) {
      const u64 c = code[k];
      if ((c >> 40) || (k > a && code[k - 1] >= c)) atomicOr(bad, 1u);
      ck[k] = ((u64)o << 40) | (c & ((1ull << 40) - 1));
    }
  }
}

__global__ void k_leaves_out(const u64* __restrict__ off, const u64* __restrict__ ck, const int32_t* __restrict__ xr,
                             u32 owner_lo, u32 count, u64 base, u64 L, u64* __restrict__ o_off,
                             u64* __restrict__ o_code, int32_t* __restrict__ o_xr) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < L || i <= count; i += (u64)gridDim.x * blockDim.x) {
    if (i < L) {
      o_code[i] = ck[base + i] & ((1ull << 40) - 1);
      o_xr[i] = xr[base + i];
    }
    if (i <= count) o_off[i] = off[owner_lo + i] - base;
  }
}

static int tree_alloc(evm_ctx* ctx, evm_tree* t, u32 n_owners, uint64_t L) {
  t->n_owners = n_owners;
  t->n_leaves = L;
  t->off = nullptr;
  t->end = nullptr;
  t->ck = nullptr;
  t->xr = nullptr;
  t->pfx = nullptr;
  // one stream-ordered allocation per tree (the arrays 256-B aligned inside it)
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_off = up(sizeof(u64) * (n_owners + 1)), b_ck = up(sizeof(u64) * std::max<uint64_t>(L, 1)),
               b_xr = up(sizeof(int32_t) * std::max<uint64_t>(L, 1)), b_pfx = up(sizeof(int32_t) * (L + 1));
  size_t bytes = b_off + b_ck + b_xr + b_pfx;
  char* base = static_cast<char*>(block_alloc(ctx, &bytes));
  if (!base) return EVM_ENOMEM;
  t->bytes = bytes;
  t->off = reinterpret_cast<unsigned long long*>(base);
  t->end = t->off + 1;
  t->ck = reinterpret_cast<unsigned long long*>(base + b_off);
  t->xr = reinterpret_cast<int32_t*>(base + b_off + b_ck);
  t->pfx = reinterpret_cast<int32_t*>(base + b_off + b_ck + b_xr);
  t->cap = L;
  t->gapped = false;
  return EVM_OK;
}

static void tree_release(evm_ctx* ctx, evm_tree* t) {
  if (!t) return;
  if (t->off) block_free(ctx, t->off, t->bytes);  // the base of the tree's one block
  delete t;
}

constexpr size_t BLOCK_CACHE = 16;

void* evm::block_alloc(evm_ctx* ctx, size_t* bytes) {
  const size_t need = *bytes;
  size_t best = ctx->blocks.size();
  for (size_t k = 0; k < ctx->blocks.size(); ++k)
    if (ctx->blocks[k].second >= need && (best == ctx->blocks.size() || ctx->blocks[k].second < ctx->blocks[best].second))
      best = k;
  if (best < ctx->blocks.size()) {
    void* p = ctx->blocks[best].first;
    *bytes = ctx->blocks[best].second;
    ctx->blocks.erase(ctx->blocks.begin() + best);
    return p;
  }
  // new block, with headroom so a slowly growing workload keeps hitting the cache
  const size_t want = need + need / 8;
  void* p = nullptr;
  if (hipMallocAsync(&p, want, ctx->stream) != hipSuccess) return nullptr;
  ++ctx->stats.block_allocs;
  ctx->stats.block_bytes += want;
  *bytes = want;
  return p;
}

void evm::block_free(evm_ctx* ctx, void* p, size_t bytes) {
  if (!p) return;
  ctx->blocks.push_back({p, bytes});
  if (ctx->blocks.size() > BLOCK_CACHE) {  // drop the smallest
    size_t k = 0;
    for (size_t j = 1; j < ctx->blocks.size(); ++j)
      if (ctx->blocks[j].second < ctx->blocks[k].second) k = j;
    (void)hipFreeAsync(ctx->blocks[k].first, ctx->stream);
    ctx->blocks.erase(ctx->blocks.begin() + k);
  }
}

void evm::block_cache_clear(evm_ctx* ctx) {
  for (auto& b : ctx->blocks) (void)hipFreeAsync(b.first, ctx->stream);
  ctx->blocks.clear();
}

int evm::tree_alloc_cap(evm_ctx* ctx, u32 n_owners, uint64_t cap, evm_tree** out) {
  evm_tree* t = new evm_tree;
  const int st = tree_alloc(ctx, t, n_owners, cap);
  if (st) {
    tree_release(ctx, t);
    return st;
  }
  *out = t;
  return EVM_OK;
}

struct LandArgs {
  const u32* src[LAND_MAX];
  int n;
};
__global__ void k_land_words(LandArgs a, volatile u32* host) {
  const int k = threadIdx.x;
  if (k < a.n) host[k] = *a.src[k];
  __threadfence_system();
}
int evm::land_words(evm_ctx* ctx, const LandList& l) {
  if (l.n == 0) return EVM_OK;
  if (!ctx->hland) {  // (no pinned buffer: the runtime's copies)
    for (int k = 0; k < l.n; ++k) HIPR(hipMemcpyAsync(l.dst[k], l.src[k], 4, hipMemcpyDeviceToHost, ctx->stream));
    return hip_ok(hipStreamSynchronize(ctx->stream));
  }
  LandArgs a;
  for (int k = 0; k < l.n; ++k) a.src[k] = l.src[k];
  a.n = l.n;
  KLAUNCH(k_land_words, dim3(1), dim3(64), a, (volatile u32*)ctx->hland);
  HIPR(hipStreamSynchronize(ctx->stream));
  for (int k = 0; k < l.n; ++k) *static_cast<u32*>(l.dst[k]) = ctx->hland[k];
  return EVM_OK;
}

struct ZeroArgs {
  u32* p[ZERO_MAX];
  u32 words[ZERO_MAX];
  u32 fill[ZERO_MAX];
  int n;
};
__global__ void k_zero_small(ZeroArgs a) {
  const int b = blockIdx.x;
  if (b >= a.n) return;
  for (u32 k = threadIdx.x; k < a.words[b]; k += blockDim.x) a.p[b][k] = a.fill[b];
}
int evm::zero_small(evm_ctx* ctx, const ZeroList& z) {
  if (z.n == 0) return EVM_OK;
  ZeroArgs a;
  for (int k = 0; k < z.n; ++k) {
    a.p[k] = z.p[k];
    a.words[k] = z.words[k];
    a.fill[k] = z.fill[k];
  }
  a.n = z.n;
  KLAUNCH(k_zero_small, dim3(z.n), dim3(256), a);
  return hip_ok(hipGetLastError());
}

int evm::tree_alloc_gapped(evm_ctx* ctx, u32 n_owners, uint64_t cap, evm_tree** out) {
  evm_tree* t = new evm_tree;
  t->n_owners = n_owners;
  t->n_leaves = 0;
  t->off = t->end = t->ck = nullptr;
  t->xr = t->pfx = nullptr;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_off = up(sizeof(u64) * (n_owners + 1)), b_end = up(sizeof(u64) * std::max<u32>(n_owners, 1)),
               b_ck = up(sizeof(u64) * std::max<uint64_t>(cap, 1)), b_xr = up(sizeof(int32_t) * std::max<uint64_t>(cap, 1)),
               b_pfx = up(sizeof(int32_t) * (cap + 1));
  size_t bytes = b_off + b_end + b_ck + b_xr + b_pfx;
  char* base = static_cast<char*>(block_alloc(ctx, &bytes));
  if (!base) {
    delete t;
    return EVM_ENOMEM;
  }
  t->bytes = bytes;
  t->off = reinterpret_cast<unsigned long long*>(base);
  t->end = reinterpret_cast<unsigned long long*>(base + b_off);
  t->ck = reinterpret_cast<unsigned long long*>(base + b_off + b_end);
  t->xr = reinterpret_cast<int32_t*>(base + b_off + b_end + b_ck);
  t->pfx = reinterpret_cast<int32_t*>(base + b_off + b_end + b_ck + b_xr);
  t->cap = cap;
  t->gapped = true;
  *out = t;
  return EVM_OK;
}

// per owner: its leaf count and its root (the last entry of its own prefix)
__global__ void k_gap_counts(const u64* __restrict__ off, const u64* __restrict__ end, const int32_t* __restrict__ pfx,
                             u32 n_owners, u64* __restrict__ cnt, int32_t* __restrict__ root) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < n_owners; o += gridDim.x * blockDim.x) {
    const u64 a = off[o], b = end[o];
    cnt[o] = b - a;
    root[o] = b > a ? pfx[b] : 0;
  }
}

// one wave per owner: its leaves to their compact places; the global
// exclusive prefix = the XOR of the owners before (carry) ^ its own prefix
__global__ void k_gap_compact(const u64* __restrict__ off, const u64* __restrict__ end, const u64* __restrict__ ck,
                              const int32_t* __restrict__ xr, const int32_t* __restrict__ pfx, u32 n_owners,
                              const u64* __restrict__ pos, const int32_t* __restrict__ carry, u64* __restrict__ o_off,
                              u64* __restrict__ o_ck, int32_t* __restrict__ o_xr, int32_t* __restrict__ o_pfx) {
  const u32 lane = threadIdx.x & 63;
  for (u32 o = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; o < n_owners; o += (gridDim.x * blockDim.x) >> 6) {
    const u64 a = off[o], L = end[o] - a, w = pos[o];
    const int32_t c = carry[o];
    for (u64 k = lane; k < L; k += 64) {
      o_ck[w + k] = ck[a + k];
      o_xr[w + k] = xr[a + k];
      o_pfx[w + k] = c ^ pfx[a + k];
    }
    if (lane == 0) o_off[o] = w;
  }
}

int evm::tree_compact(evm_ctx* ctx, const evm_tree* tc) {
  if (!tc || !tc->gapped) return EVM_OK;
  evm_tree* t = const_cast<evm_tree*>(tc);  // (the same tree, another layout)
  const u32 O = t->n_owners;
  Scratch S(ctx);
  u64* cnt = S.alloc<u64>((size_t)O + 1);
  int32_t* root = S.alloc<int32_t>((size_t)O + 1);
  evm_tree nt{};
  if (!cnt || !root) return EVM_ENOMEM;
  int st = tree_alloc(ctx, &nt, O, t->n_leaves);
  if (st) return st;
  if (O) {
    KLAUNCH(k_gap_counts, dim3(grid_for(O, 256)), dim3(256), (const u64*)t->off, (const u64*)t->end,
            (const int32_t*)t->pfx, O, cnt, root);
    if (!st) st = scan_exclusive<u64, OpAdd>(ctx, S, cnt, O, nt.off, nt.off + O);
    int32_t* carry = S.alloc<int32_t>((size_t)O + 1);
    if (!st && !carry) st = EVM_ENOMEM;
    if (!st) st = scan_exclusive<int32_t, OpXor>(ctx, S, root, O, carry, nt.pfx + t->n_leaves);
    if (!st)
      KLAUNCH(k_gap_compact, dim3(grid_for((size_t)O * 64, 256, 1 << 14)), dim3(256), (const u64*)t->off,
              (const u64*)t->end, (const u64*)t->ck, (const int32_t*)t->xr, (const int32_t*)t->pfx, O,
              (const u64*)nt.off, (const int32_t*)carry, nt.off, nt.ck, nt.xr, nt.pfx);
  } else {
    st = hip_ok(hipMemsetAsync(nt.off, 0, sizeof(u64), ctx->stream));
    if (!st) st = hip_ok(hipMemsetAsync(nt.pfx, 0, sizeof(int32_t), ctx->stream));
  }
  if (st) {
    block_free(ctx, nt.off, nt.bytes);
    return st;
  }
  block_free(ctx, t->off, t->bytes);  // (stream-ordered: behind the copy)
  const uint64_t L = t->n_leaves;
  *t = nt;
  t->n_leaves = L;
  return hip_ok(hipGetLastError());
}

// Builds a tree object from device leaves (ck sorted unique, xr); copies them.
int evm::tree_finalize(evm_ctx* ctx, Scratch& S, u32 n_owners, const u64* ck, const int32_t* xr, uint64_t L,
                       evm_tree** out) {
  evm_tree* t = new evm_tree;
  int st = tree_alloc(ctx, t, n_owners, L);
  if (st) {
    tree_release(ctx, t);
    return st;
  }
  if (L) {
    HIPR(hipMemcpyAsync(t->ck, ck, sizeof(u64) * L, hipMemcpyDeviceToDevice, ctx->stream));
    HIPR(hipMemcpyAsync(t->xr, xr, sizeof(int32_t) * L, hipMemcpyDeviceToDevice, ctx->stream));
  }
  KLAUNCH(k_owner_off, dim3(grid_for(n_owners + 1, 256)), dim3(256), t->ck, (size_t)L,
                     n_owners, t->off);
  st = scan_exclusive<int32_t, OpXor>(ctx, S, t->xr, L, t->pfx, t->pfx + L);
  if (st) {
    tree_release(ctx, t);
    return st;
  }
  *out = t;
  return hip_ok(hipGetLastError());
}

__global__ void k_copy_leaves(const u64* __restrict__ ck, const int32_t* __restrict__ xr, const u32* __restrict__ d_count,
                              u64* __restrict__ ock, int32_t* __restrict__ oxr) {
  const size_t L = *d_count;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < L; i += (size_t)gridDim.x * blockDim.x) {
    ock[i] = ck[i];
    oxr[i] = xr[i];
  }
}

__global__ void k_owner_off_dev(const u64* __restrict__ ck, const u32* __restrict__ d_count, u32 n_owners,
                                u64* __restrict__ off) {
  const size_t L = *d_count;
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o <= n_owners; o += (size_t)gridDim.x * blockDim.x)
    off[o] = (o == n_owners) ? (u64)L : (u64)lower_bound_u64(ck, 0, L, (u64)o << 40);
}

int evm::tree_finalize_dev(evm_ctx* ctx, Scratch& S, u32 n_owners, const u64* ck, const int32_t* xr,
                           const u32* d_count, uint64_t cap, evm_tree** out) {
  evm_tree* t = new evm_tree;
  int st = tree_alloc(ctx, t, n_owners, cap);
  if (st) {
    tree_release(ctx, t);
    return st;
  }
  KLAUNCH(k_copy_leaves, dim3(grid_for(cap, 256, 1024)), dim3(256), ck, xr, d_count, t->ck, t->xr);
  KLAUNCH(k_owner_off_dev, dim3(grid_for(n_owners + 1, 256)), dim3(256), t->ck, d_count, n_owners, t->off);
  // prefix XOR over the whole capacity: entries past the count never feed pfx[0..count]
  st = scan_exclusive<int32_t, OpXor>(ctx, S, t->xr, cap, t->pfx, t->pfx + cap);
  if (st) {
    tree_release(ctx, t);
    return st;
  }
  *out = t;
  return hip_ok(hipGetLastError());
}

// Folds m selected (ck, hash) pairs into `in` (may be null = empty trees).
int evm::fold_into_tree(evm_ctx* ctx, Scratch& S, const evm_tree* in, u32 n_owners, u64* ck, u32* h, size_t m,
                        const Info& host_info, evm_tree** out) {
  // sort by the bits that vary
  int lo = 0, hi = 0;
  if (m > 1) {
    const u64 diff = host_info.ck_min ^ host_info.ck_max;
    hi = diff ? 64 - __builtin_clzll(diff) : 0;
    lo = 2 * (CODE_DIGITS - (int)host_info.maxlen);
    if (lo > hi) lo = hi;
  }
  int st = radix_sort_pairs<u64>(ctx, S, ck, h, m, lo, hi);
  if (st) return st;
  u64* nck = S.alloc<u64>(std::max<size_t>(m, 1));
  int32_t* nxr = S.alloc<int32_t>(std::max<size_t>(m, 1));
  if (!nck || !nxr) return EVM_ENOMEM;
  uint64_t L1 = 0;
  st = reduce_runs(ctx, S, ck, (const int32_t*)h, m, nck, nxr, &L1);
  if (st) return st;
  return merge_into_tree(ctx, S, in, n_owners, nck, nxr, L1, out);
}

// Merges sorted unique leaves (nck, nxr) into `in`; equal keys XOR-combine.
int evm::merge_into_tree(evm_ctx* ctx, Scratch& S, const evm_tree* in, u32 n_owners, const u64* nck,
                         const int32_t* nxr, uint64_t L1, evm_tree** out) {
  int st = in ? tree_compact(ctx, in) : EVM_OK;
  if (st) return st;
  const uint64_t L0 = in ? in->n_leaves : 0;
  if (L0 == 0) return tree_finalize(ctx, S, n_owners, nck, nxr, L1, out);
  if (L1 == 0) return tree_finalize(ctx, S, n_owners, in->ck, in->xr, L0, out);
  const size_t tot = L0 + L1;
  u64* mck = S.alloc<u64>(tot);
  int32_t* mxr = S.alloc<int32_t>(tot);
  u64* rck = S.alloc<u64>(tot);
  int32_t* rxr = S.alloc<int32_t>(tot);
  if (!mck || !mxr || !rck || !rxr) return EVM_ENOMEM;
  KLAUNCH(k_merge_a, dim3(grid_for(L0, 256)), dim3(256), in->ck, in->xr, (size_t)L0, nck,
                     (size_t)L1, mck, mxr);
  KLAUNCH(k_merge_b, dim3(grid_for(L1, 256)), dim3(256), nck, nxr, (size_t)L1, in->ck,
                     (size_t)L0, mck, mxr);
  uint64_t L = 0;
  st = reduce_runs(ctx, S, mck, mxr, tot, rck, rxr, &L);
  if (st) return st;
  return tree_finalize(ctx, S, n_owners, rck, rxr, L, out);
}

// ============================================================================
// Diff (merkleTree.ts:63-91), a 16-lane group per owner.
// ============================================================================
struct TreeView {
  const u64* off;
  const u64* end;  // owner o's leaves: [off[o], end[o])
  const u64* ck;
  const int32_t* pfx;
  const int32_t* xr;
};

__device__ __forceinline__ int32_t range_hash(const TreeView& t, size_t lo, size_t hi) { return t.pfx[hi] ^ t.pfx[lo]; }

constexpr int DIFF_LANES = 16;

// At each level the three children's leaf ranges in both trees are 6 lower
// bounds (child starts 1..3 in A and in B; the end of child 3 is the node's
// own end, known from the level above): lanes 0-2 / 4-6 of the group search
// them at once and fetch the prefix XOR at their bound, so a level costs one
// binary search + one load of latency instead of up to six searches in a row.
// The greedy choice (first child whose hash differs, a missing child counting
// as different) is then made by every lane of the group on the shuffled
// bounds.
//
// The top levels are not searched at all: every leaf of both trees lies in
// the code range of their longest common prefix (the first and the last
// leaf of each tree bound it), and above that depth every node has ONE
// child, present in both trees (or in the only non-empty one) and holding
// the whole range -- its hash is its parent's, which differs -- so the
// greedy path follows that prefix (for config-3 trees spanning 30 days: the
// first ~6 of 16 digits, each a full-range search before).  Searches of the
// same lines level after level were the kernel's HBM traffic: with thousands
// of owners in flight per XCD a line is evicted from L2 between one level
// and the next.
//
// Once both ranges hold at most 16 leaves (a few levels down: ranges shrink
// ~3x per level), the group loads them -- one leaf of A and one of B per
// lane -- and finishes every remaining level in registers: a child's
// presence is a ballot of the lanes whose digit at this depth selects it, its
// hash a 16-lane XOR reduction.
__device__ __forceinline__ int code_digits_equal(u64 a, u64 b) {
  const u64 x = (a ^ b) & ((1ull << (2 * CODE_DIGITS)) - 1);
  return x ? (__clzll(x) - (64 - 2 * CODE_DIGITS)) >> 1 : CODE_DIGITS;
}

__global__ __launch_bounds__(256) void k_diff(TreeView A, TreeView B, u32 n_owners, int64_t* __restrict__ millis) {
  const int sub = threadIdx.x & (DIFF_LANES - 1);
  const u32 groups = gridDim.x * (blockDim.x / DIFF_LANES);
  for (u32 o = (blockIdx.x * blockDim.x + threadIdx.x) / DIFF_LANES; o < n_owners; o += groups) {
    u64 alo = A.off[o], ahi = A.end[o], blo = B.off[o], bhi = B.end[o];
    // root: tree1.hash === tree2.hash (undefined for {})
    const bool ae = ahi > alo, be = bhi > blo;
    int32_t pa_lo = ae ? A.pfx[alo] : 0, pa_hi = ae ? A.pfx[ahi] : 0;
    int32_t pb_lo = be ? B.pfx[blo] : 0, pb_hi = be ? B.pfx[bhi] : 0;
    if (ae == be && (!ae || (pa_lo ^ pa_hi) == (pb_lo ^ pb_hi))) {
      if (sub == 0) millis[o] = EVM_DIFF_NONE;
      continue;
    }
    // the common prefix of every leaf of both trees (one 8-B load per lane of 4)
    u64 my = 0;
    if (sub < 4) {
      const bool inA = sub < 2;
      const bool live = inA ? ae : be;
      const u64* ck = inA ? A.ck : B.ck;
      const u64 at = inA ? ((sub & 1) ? ahi - 1 : alo) : ((sub & 1) ? bhi - 1 : blo);
      my = live ? ck[at] : ((sub & 1) ? 0ull : ~0ull);  // (an empty tree: neutral for min / max)
    }
    const int g0 = threadIdx.x & ~(DIFF_LANES - 1) & 63;
    const u64 first = min(__shfl(my, g0 + 0, 64), __shfl(my, g0 + 2, 64));
    const u64 last = max(__shfl(my, g0 + 1, 64), __shfl(my, g0 + 3, 64));
    int depth = code_digits_equal(first, last);
    u64 prefix = (u64)o << 40, kval = 0;
    for (int d = 0; d < depth; ++d) {
      const u32 dg = (u32)(first >> (2 * (CODE_DIGITS - 1 - d))) & 3u;
      if (dg == 0) {  // the key ends here (every leaf is this one code): no deeper node
        depth = d;
        break;
      }
      prefix |= (u64)dg << (2 * (CODE_DIGITS - 1 - d));
      kval = kval * 3 + (dg - 1);
    }
    bool in_regs = false;
    while (depth < CODE_DIGITS) {
      if (ahi - alo <= DIFF_LANES && bhi - blo <= DIFF_LANES) {
        in_regs = true;  // the rest in registers
        break;
      }
      const int sh = 2 * (CODE_DIGITS - 1 - depth);
      // lane s < 3: A bound of prefix + (s+1) << sh; 4 <= s < 7: B bound of prefix + (s-3) << sh
      u64 mb = 0;
      int32_t myx = 0;
      if ((sub & 3) != 3 && sub < 8) {
        const bool inA = sub < 4;
        const u64* ck = inA ? A.ck : B.ck;
        u64 lo = inA ? alo : blo, hi = inA ? ahi : bhi;
        const u64 x = prefix + ((u64)((sub & 3) + 1) << sh);
        while (lo < hi) {
          const u64 mid = (lo + hi) >> 1;
          if (ck[mid] < x) lo = mid + 1;
          else hi = mid;
        }
        mb = lo;
        myx = (inA ? A.pfx : B.pfx)[lo];
      }
      u64 a[4], b[4];
      int32_t xa[4], xb[4];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        a[k] = __shfl(mb, g0 + k, 64);
        b[k] = __shfl(mb, g0 + 4 + k, 64);
        xa[k] = __shfl(myx, g0 + k, 64);
        xb[k] = __shfl(myx, g0 + 4 + k, 64);
      }
      a[3] = ahi;  // the end of child 3 = the node's end
      b[3] = bhi;
      xa[3] = pa_hi;
      xb[3] = pb_hi;
      int pick = -1;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const bool ea = a[c + 1] > a[c], eb = b[c + 1] > b[c];
        if (pick < 0 && (ea || eb) && (ea != eb || (xa[c + 1] ^ xa[c]) != (xb[c + 1] ^ xb[c]))) pick = c;
      }
      if (pick < 0) break;
      prefix |= (u64)(pick + 1) << sh;
      kval = kval * 3 + (u64)pick;
      ++depth;
      alo = a[pick];
      ahi = a[pick + 1];
      blo = b[pick];
      bhi = b[pick + 1];
      pa_hi = xa[pick + 1];
      pb_hi = xb[pick + 1];
    }
    if (in_regs) {
      const u64 ia = alo + sub, ib = blo + sub;
      bool va = ia < ahi, vb = ib < bhi;
      const u64 ca = va ? A.ck[ia] : 0ull, cb = vb ? B.ck[ib] : 0ull;
      const int32_t xa = va ? A.xr[ia] : 0, xb = vb ? B.xr[ib] : 0;
      const u64 gmask = 0xFFFFull << (threadIdx.x & 63 & ~(DIFF_LANES - 1));
      while (depth < CODE_DIGITS) {
        const int sh = 2 * (CODE_DIGITS - 1 - depth);
        const u32 da = va ? (u32)(ca >> sh) & 3u : 0u, db = vb ? (u32)(cb >> sh) & 3u : 0u;
        int pick = -1;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const bool ina = da == (u32)c + 1u, inb = db == (u32)c + 1u;
          const bool ea = (__ballot(ina) & gmask) != 0, eb = (__ballot(inb) & gmask) != 0;
          int32_t ha = ina ? xa : 0, hb = inb ? xb : 0;
#pragma unroll
          for (int m = DIFF_LANES / 2; m >= 1; m >>= 1) {
            ha ^= __shfl_xor(ha, m, 64);
            hb ^= __shfl_xor(hb, m, 64);
          }
          if (pick < 0 && (ea || eb) && (ea != eb || ha != hb)) pick = c;
        }
        if (pick < 0) break;
        kval = kval * 3 + (u64)pick;
        ++depth;
        va = va && da == (u32)pick + 1u;
        vb = vb && db == (u32)pick + 1u;
      }
    }
    if (sub == 0) {
      if (depth > 16) {
        millis[o] = EVM_DIFF_RANGE_ERROR;  // "0".repeat(16 - k.length) throws (merkleTree.ts:58)
      } else {
        u64 v = kval;
        for (int i = depth; i < 16; ++i) v *= 3;  // padEnd(16, "0")
        millis[o] = (int64_t)(v * 60000ull);
      }
    }
  }
}

__global__ void k_roots(const u64* __restrict__ off, const u64* __restrict__ end, const int32_t* __restrict__ pfx,
                        u32 n_owners, int32_t* __restrict__ root, uint8_t* __restrict__ present) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < n_owners; o += gridDim.x * blockDim.x) {
    const u64 a = off[o], b = end[o];
    root[o] = pfx[b] ^ pfx[a];
    present[o] = b > a;
  }
}


// ============================================================================
// C ABI
// ============================================================================
static void prof_drain(evm_ctx* ctx);

extern "C" {

const char* evm_strerror(int s) {
  switch (s) {
    case EVM_OK: return "ok";
    case EVM_EINVAL: return "invalid argument";
    case EVM_ENONCANON: return "timestamp outside the native domain";
    case EVM_ECOLLISION: return "same timestamp in two cells of one batch";
    case EVM_ERANGE: return "diff reached a 17-digit key (RangeError)";
    case EVM_ETREE: return "tree is not a MerkleTree insertIntoMerkleTree can produce";
    case EVM_EDEVICE: return "HIP error";
    case EVM_ENOMEM: return "device out of memory";
    case EVM_ECAPACITY: return "output buffer too small";
    case EVM_EDIST: return "RCCL unavailable or a collective failed";
    case EVM_ESTATE: return "a store invariant broke in a merge; nothing committed";
    case EVM_EROUNDS: return "a userId in two requests of one call: split the call into rounds";
    case EVM_EHANDOVER: return "request not modelled here: the caller's reference path runs it";
  }
  return "unknown status";
}

int evm_create(int device, evm_ctx** out) {
  if (!out) return EVM_EINVAL;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return EVM_EDEVICE;
  if (hipSetDevice(device) != hipSuccess) return EVM_EDEVICE;
  evm_ctx* c = new evm_ctx;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return EVM_EDEVICE;
  }
  c->stream = c->own;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    c->n_cu = ncu;
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess)
    c->overlap = 0;
  // pinned landing buffer for the per-call status record (a pageable D2H
  // copy would stage through a bounce buffer on every call)
  if (hipHostMalloc((void**)&c->hinfo, sizeof(Info), hipHostMallocDefault) != hipSuccess) c->hinfo = nullptr;
  if (hipHostMalloc((void**)&c->hland, sizeof(uint32_t) * LAND_MAX, hipHostMallocDefault) != hipSuccess)
    c->hland = nullptr;
  // keep freed scratch in the stream-ordered pool between calls
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
    uint64_t thr = ~0ull;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  *out = c;
  return EVM_OK;
}

void evm_destroy(evm_ctx* ctx) {
  if (!ctx) return;
  prof_drain(ctx);
  for (hipEvent_t e : ctx->prof_pool) (void)hipEventDestroy(e);
  block_cache_clear(ctx);
  evm_pending_pool_clear(ctx);
  evm_host_stage_free(ctx);
  if (ctx->xtab) (void)hipFree(ctx->xtab);
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->side) (void)hipStreamSynchronize(ctx->side);
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  (void)hipStreamDestroy(ctx->own);
  if (ctx->hinfo) (void)hipHostFree(ctx->hinfo);
  if (ctx->hland) (void)hipHostFree(ctx->hland);
  delete ctx;
}

int evm_bind_thread(evm_ctx* ctx) {
  if (!ctx) return EVM_EINVAL;
  return hipSetDevice(ctx->device) == hipSuccess ? EVM_OK : EVM_EDEVICE;
}

int evm_get_stats(const evm_ctx* ctx, evm_stats* out) {
  if (!ctx || !out) return EVM_EINVAL;
  *out = ctx->stats;
  out->workspace_bytes = ctx->ws_bytes;
  return EVM_OK;
}

int evm_set_stream(evm_ctx* ctx, void* s) {
  if (!ctx) return EVM_EINVAL;
  (void)hipStreamSynchronize(ctx->stream);  // the workspace is ordered on one stream at a time
  ctx->stream = (hipStream_t)s;             // NULL: the HIP default (null) stream
  return EVM_OK;
}
void* evm_get_stream(evm_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int evm_sync(evm_ctx* ctx) {
  if (!ctx) return EVM_EINVAL;
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

int evm_set_option(evm_ctx* ctx, int option, int64_t value) {
  if (!ctx) return EVM_EINVAL;
  if (option == EVM_OPT_CLIENT_PATH && value >= 0 && value <= 4) {
    ctx->client_path = (int)value;
    return EVM_OK;
  }
  if (option == EVM_OPT_OVERLAP && (value == 0 || value == 1)) {
    ctx->overlap = (int)value;
    return EVM_OK;
  }
  if (option == EVM_OPT_RADIX && value >= 0 && value <= 2) {
    ctx->radix_onesweep = (int)value;
    return EVM_OK;
  }
  if (option == EVM_OPT_SELECT_PATH && (value == 0 || value == 1)) {
    ctx->select_path = (int)value;
    return EVM_OK;
  }
  if (option == EVM_OPT_DIFF_GRID && value >= 0 && value <= 64) {
    ctx->diff_grid = (int)value;
    return EVM_OK;
  }
  if (option == EVM_OPT_SERVER_PATH && value >= 0 && value <= 4) {
    ctx->server_path = (int)value;
    return EVM_OK;
  }
  return EVM_EINVAL;
}

// include/evm_test.h: fault injection for the atomicity tests, outside the
// product ABI (evm.h) and refused unless the process runs with
// EVM_TEST_HOOKS=1 -- no product caller can switch a check off by accident.
int evm_test_fault(evm_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 2) return EVM_EINVAL;
  const char* e = getenv("EVM_TEST_HOOKS");
  if (!e || strcmp(e, "1") != 0) return EVM_EINVAL;
  ctx->test_fail = mode;
  return EVM_OK;
}

int evm_prof_enable(evm_ctx* ctx, int on) {
  if (!ctx) return EVM_EINVAL;
  ctx->prof = on != 0;
  return EVM_OK;
}

int evm_prof_only(evm_ctx* ctx, const char* kernel) {
  if (!ctx) return EVM_EINVAL;
  ctx->prof_only = kernel ? kernel : "";
  return EVM_OK;
}

}  // extern "C"
static void prof_drain(evm_ctx* ctx) {
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->prof_events) {
    auto& tot = ctx->prof_total[kv.first];
    for (auto& ev : kv.second) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, ev.first, ev.second) == hipSuccess) tot.first += ms;
      tot.second += 1;
      ctx->prof_pool.push_back(ev.first);
      ctx->prof_pool.push_back(ev.second);
    }
  }
  ctx->prof_events.clear();
}
extern "C" {

int evm_prof_reset(evm_ctx* ctx) {
  if (!ctx) return EVM_EINVAL;
  prof_drain(ctx);
  ctx->prof_total.clear();
  return EVM_OK;
}

int evm_prof_report(evm_ctx* ctx, char* buf, size_t cap, size_t* len) {
  if (!ctx || !len) return EVM_EINVAL;
  prof_drain(ctx);
  std::string js = "{";
  bool first = true;
  char tmp[128];
  for (auto& kv : ctx->prof_total) {
    if (!first) js += ",";
    first = false;
    js += "\"" + kv.first + "\":";
    snprintf(tmp, sizeof tmp, "[%.6f,%llu]", kv.second.first, (unsigned long long)kv.second.second);
    js += tmp;
  }
  js += "}";
  *len = js.size();
  if (buf) {
    if (cap < js.size()) return EVM_ECAPACITY;
    memcpy(buf, js.data(), js.size());
  }
  return EVM_OK;
}

int evm_dev_alloc(evm_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return EVM_EINVAL;
  return hipMalloc(out, bytes ? bytes : 1) == hipSuccess ? EVM_OK : EVM_ENOMEM;
}
int evm_dev_free(evm_ctx* ctx, void* p) {
  if (!ctx) return EVM_EINVAL;
  return hip_ok(hipFree(p));
}
int evm_copy_h2d(evm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return EVM_EINVAL;
  if (!bytes) return EVM_OK;
  HIPR(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return hip_ok(hipStreamSynchronize(ctx->stream));
}
int evm_copy_d2h(evm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return EVM_EINVAL;
  if (!bytes) return EVM_OK;
  HIPR(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

int evm_pack(evm_ctx* ctx, const char* ts, size_t stride, size_t n, const uint32_t* aux, evm_rec* out) {
  if (!ctx || (n && (!ts || !out)) || stride < 46) return EVM_EINVAL;
  Scratch S(ctx);
  Info* info = nullptr;
  int st = new_info(ctx, S, &info);
  if (st) return st;
  st = launch_pack(ctx, ts, stride, n, aux, 0, out, info);
  if (st) return st;
  Info h;
  st = read_info(ctx, info, &h);
  if (st) return st;
  return h.bad ? EVM_ENONCANON : EVM_OK;
}

int evm_tree_new(evm_ctx* ctx, uint32_t n_owners, evm_tree** out) {
  if (!ctx || !out) return EVM_EINVAL;
  Scratch S(ctx);
  int st = tree_finalize(ctx, S, n_owners, nullptr, nullptr, 0, out);
  if (st) return st;
  return evm_sync(ctx);
}

int evm_tree_from_leaves(evm_ctx* ctx, uint32_t n_owners, const uint64_t* off_h, const uint64_t* code_h,
                         const int32_t* xr_h, evm_tree** out) {
  if (!ctx || !out || !off_h) return EVM_EINVAL;
  const uint64_t L = off_h[n_owners];
  std::vector<u64> ck(L);
  for (u32 o = 0; o < n_owners; ++o) {
    if (off_h[o + 1] < off_h[o]) return EVM_EINVAL;
    for (uint64_t k = off_h[o]; k < off_h[o + 1]; ++k) {
      if (code_h[k] >> 40) return EVM_EINVAL;
      ck[k] = ((u64)o << 40) | code_h[k];
      if (k > off_h[o] && code_h[k] <= code_h[k - 1]) return EVM_EINVAL;  // sorted, unique
    }
  }
  Scratch S(ctx);
  u64* dck = S.alloc<u64>(std::max<uint64_t>(L, 1));
  int32_t* dxr = S.alloc<int32_t>(std::max<uint64_t>(L, 1));
  if (!dck || !dxr) return EVM_ENOMEM;
  if (L) {
    HIPR(hipMemcpyAsync(dck, ck.data(), sizeof(u64) * L, hipMemcpyHostToDevice, ctx->stream));
    HIPR(hipMemcpyAsync(dxr, xr_h, sizeof(int32_t) * L, hipMemcpyHostToDevice, ctx->stream));
  }
  int st = tree_finalize(ctx, S, n_owners, dck, dxr, L, out);
  if (st) return st;
  return evm_sync(ctx);
}

int evm_tree_from_device_leaves(evm_ctx* ctx, uint32_t n_owners, const uint64_t* off, const uint64_t* code,
                                const int32_t* xr, evm_tree** out) {
  if (!ctx || !out || !off) return EVM_EINVAL;
  uint64_t L = 0;
  HIPR(hipMemcpyAsync(&L, off + n_owners, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (L && (!code || !xr)) return EVM_EINVAL;
  Scratch S(ctx);
  u64* ck = S.alloc<u64>(std::max<uint64_t>(L, 1));
  u32* bad = S.alloc<u32>(1);
  if (!ck || !bad) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  if (n_owners)
    KLAUNCH(k_leaves_in, dim3(grid_for(n_owners, 4, 1 << 16)), dim3(256), (const u64*)off, (const u64*)code, n_owners,
            ck, bad);
  u32 hb = 0;
  HIPR(hipMemcpyAsync(&hb, bad, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (hb) return EVM_EINVAL;
  const int st = tree_finalize(ctx, S, n_owners, ck, xr, L, out);
  return st ? st : evm_sync(ctx);
}

int evm_tree_slice(evm_ctx* ctx, const evm_tree* t, uint32_t owner_lo, uint32_t count, uint64_t* off, uint64_t* code,
                   int32_t* xr, uint64_t cap, uint64_t* n_leaves) {
  if (!ctx || !t || !n_leaves || owner_lo + (uint64_t)count > t->n_owners || (count && !off)) return EVM_EINVAL;
  if (int e = tree_compact(ctx, t)) return e;
  u64 ab[2] = {0, 0};
  HIPR(hipMemcpyAsync(&ab[0], t->off + owner_lo, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(&ab[1], t->off + owner_lo + count, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  *n_leaves = ab[1] - ab[0];
  if (*n_leaves > cap || (*n_leaves && (!code || !xr))) return EVM_ECAPACITY;
  if (count)
    KLAUNCH(k_leaves_out, dim3(grid_for(std::max<uint64_t>(*n_leaves, count + 1), 256, 8192)), dim3(256),
            (const u64*)t->off, (const u64*)t->ck, (const int32_t*)t->xr, owner_lo, count, ab[0], *n_leaves,
            (u64*)off, (u64*)code, xr);
  return evm_sync(ctx);
}

int evm_tree_free(evm_ctx* ctx, evm_tree* t) {
  if (!ctx) return EVM_EINVAL;
  if (t) tree_release(ctx, t);  // stream-ordered: safe behind queued readers
  return EVM_OK;
}

}  // extern "C"

void evm::tree_destroy(evm_ctx* ctx, evm_tree* t) { tree_release(ctx, t); }

extern "C" {

int evm_tree_info(const evm_tree* t, uint32_t* n_owners, uint64_t* n_leaves) {
  if (!t) return EVM_EINVAL;
  if (n_owners) *n_owners = t->n_owners;
  if (n_leaves) *n_leaves = t->n_leaves;
  return EVM_OK;
}

int evm_tree_device(const evm_tree* t, const uint64_t** off, const uint64_t** code, const int32_t** xr) {
  if (!t || t->gapped) return EVM_EINVAL;  // (a gapped tree: evm_tree_leaves / slice compact it)
  if (off) *off = (const uint64_t*)t->off;
  if (code) *code = (const uint64_t*)t->ck;
  if (xr) *xr = t->xr;
  return EVM_OK;
}

int evm_tree_leaves(evm_ctx* ctx, const evm_tree* t, uint64_t* off, uint64_t* code, int32_t* xr) {
  if (!ctx || !t) return EVM_EINVAL;
  if (int e = tree_compact(ctx, t)) return e;
  if (off) HIPR(hipMemcpyAsync(off, t->off, sizeof(u64) * (t->n_owners + 1), hipMemcpyDeviceToHost, ctx->stream));
  if (code && t->n_leaves)
    HIPR(hipMemcpyAsync(code, t->ck, sizeof(u64) * t->n_leaves, hipMemcpyDeviceToHost, ctx->stream));
  if (xr && t->n_leaves)
    HIPR(hipMemcpyAsync(xr, t->xr, sizeof(int32_t) * t->n_leaves, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (code)
    for (uint64_t k = 0; k < t->n_leaves; ++k) code[k] &= (1ull << 40) - 1;
  return EVM_OK;
}

int evm_tree_roots(evm_ctx* ctx, const evm_tree* t, int32_t* root, uint8_t* present) {
  if (!ctx || !t || !root || !present) return EVM_EINVAL;
  Scratch S(ctx);
  int32_t* dr = S.alloc<int32_t>(std::max<u32>(t->n_owners, 1));
  uint8_t* dp = S.alloc<uint8_t>(std::max<u32>(t->n_owners, 1));
  if (!dr || !dp) return EVM_ENOMEM;
  if (t->n_owners == 0) return EVM_OK;
  KLAUNCH(k_roots, dim3(grid_for(t->n_owners, 256)), dim3(256), t->off, t->end, t->pfx, t->n_owners, dr, dp);
  HIPR(hipMemcpyAsync(root, dr, sizeof(int32_t) * t->n_owners, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(present, dp, t->n_owners, hipMemcpyDeviceToHost, ctx->stream));
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

int evm_merkle_insert(evm_ctx* ctx, const evm_tree* in, const char* ts, size_t stride, size_t n, const uint32_t* owner,
                      evm_tree** out) {
  if (!ctx || !in || !out || stride < 46 || (n && !ts)) return EVM_EINVAL;
  if (int e = tree_compact(ctx, in)) return e;
  Scratch S(ctx);
  Info* info = nullptr;
  int st = new_info(ctx, S, &info);
  if (st) return st;
  evm_rec* rec = S.alloc<evm_rec>(std::max<size_t>(n, 1));
  u64* ck = S.alloc<u64>(std::max<size_t>(n, 1));
  u32* h = S.alloc<u32>(std::max<size_t>(n, 1));
  if (!rec || !ck || !h) return EVM_ENOMEM;
  st = launch_pack(ctx, ts, stride, n, owner, in->n_owners, rec, info);
  if (st) return st;
  if (n)
    KLAUNCH(k_fold_prep, dim3(grid_for(n, 256, 4096)), dim3(256), rec, (const uint8_t*)nullptr,
                       (uint8_t)0, (const u32*)nullptr, (int)(owner ? OWNER_AUX : OWNER_ZERO), (const u32*)nullptr, n, ck,
                       h, info);
  Info hi;
  st = read_info(ctx, info, &hi);
  if (st) return st;
  if (hi.bad_aux) return EVM_EINVAL;
  if (hi.bad) return EVM_ENONCANON;
  st = fold_into_tree(ctx, S, in, in->n_owners, ck, h, n, hi, out);
  if (st) return st;
  return evm_sync(ctx);
}

int evm_tree_merge(evm_ctx* ctx, const evm_tree* a, const evm_tree* b, evm_tree** out) {
  if (!ctx || !a || !b || !out || a->n_owners != b->n_owners) return EVM_EINVAL;
  if (int e = tree_compact(ctx, a)) return e;
  if (int e = tree_compact(ctx, b)) return e;
  Scratch S(ctx);
  // b's leaves are sorted and unique per owner; equal keys XOR-combine
  const int st = merge_into_tree(ctx, S, a, a->n_owners, (const u64*)b->ck, b->xr, b->n_leaves, out);
  if (st) return st;
  return evm_sync(ctx);
}

int evm_merkle_diff(evm_ctx* ctx, const evm_tree* a, const evm_tree* b, int64_t* millis) {
  if (!ctx || !a || !b || !millis || a->n_owners != b->n_owners) return EVM_EINVAL;
  int st = launch_diff(ctx, a, b, millis);
  return st ? st : evm_sync(ctx);
}

}  // extern "C"

int evm::launch_diff(evm_ctx* ctx, const evm_tree* a, const evm_tree* b, int64_t* millis) {
  if (a->n_owners == 0) return EVM_OK;
  TreeView A{a->off, a->end, a->ck, a->pfx, a->xr}, B{b->off, b->end, b->ck, b->pfx, b->xr};
  // EVM_OPT_DIFF_GRID: workgroups per CU (fewer owners in flight: each one's lines stay in L2)
  u32 grid = grid_for((size_t)a->n_owners * DIFF_LANES, 256, 1 << 16);
  if (ctx->diff_grid > 0) grid = std::min<u32>(grid, (u32)ctx->diff_grid * (u32)ctx->n_cu);
  KLAUNCH(k_diff, dim3(grid), dim3(256), A, B, a->n_owners, millis);
  return hip_ok(hipGetLastError());
}

extern "C" {

}  // extern "C"
