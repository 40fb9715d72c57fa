// K1 of the streaming client path (evm_client.hip): parse every timestamp of
// the batch once, at full occupancy, into SoA records.  A header so that
// tools/pack_probe.hip times exactly this kernel.
#pragma once
#include <hip/hip_runtime.h>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

namespace evm {

// K1 for the streaming path: parse every timestamp once, at full occupancy,
// into SoA records: order key (tc, rh) 16 B + rl 4 B (OKey; rl carries
// OKEY_PRESENT iff the timestamp is valid), hash 4 B, minute 4 B.
// For stride 48 each wave reads its 64 timestamps (3 KiB) with coalesced 16-B
// loads and redistributes them through LDS.
constexpr int CLP_THREADS = 256;

// One wave's 64 timestamps of round `first`.  S48: the 3 KiB block as three
// coalesced 16-B loads per lane (lane k holds bytes 16k..16k+15 of the block,
// redistributed through LDS by the caller); otherwise each lane loads its own.
template <bool S48>
__device__ __forceinline__ void clp_fetch(const uint8_t* __restrict__ ts, size_t stride, size_t n, size_t first,
                                          uint4& a, uint4& b, uint4& c) {
  const int lane = threadIdx.x & 63;
  const uint4 z = make_uint4(0, 0, 0, 0);
  if (S48) {
    const uint4* src = reinterpret_cast<const uint4*>(ts + first * 48);
    if (first + 64 <= n) {
      // read once: non-temporal
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const v4u* s4 = reinterpret_cast<const v4u*>(src);
      const v4u x = __builtin_nontemporal_load(s4 + lane), y = __builtin_nontemporal_load(s4 + lane + 64),
                z = __builtin_nontemporal_load(s4 + lane + 128);
      a = make_uint4(x.x, x.y, x.z, x.w);
      b = make_uint4(y.x, y.y, y.z, y.w);
      c = make_uint4(z.x, z.y, z.z, z.w);
    } else {
      const size_t nq = first < n ? (n - first) * 3 : 0;
      a = (size_t)lane < nq ? src[lane] : z;
      b = (size_t)lane + 64 < nq ? src[lane + 64] : z;
      c = (size_t)lane + 128 < nq ? src[lane + 128] : z;
    }
  } else {
    u32 w[12];
    const size_t i = first + lane;
    if (i < n) {
      load_ts(ts, stride, i, w);
    } else {
#pragma unroll
      for (int k = 0; k < 12; ++k) w[k] = 0;
    }
    a = make_uint4(w[0], w[1], w[2], w[3]);
    b = make_uint4(w[4], w[5], w[6], w[7]);
    c = make_uint4(w[8], w[9], w[10], w[11]);
  }
}

template <bool S48>
__global__ __launch_bounds__(CLP_THREADS) void k_cl_pack(const uint8_t* __restrict__ ts, size_t stride, size_t n,
                                                         uint4* __restrict__ key, u32* __restrict__ rl,
                                                         u32* __restrict__ hash, u32* __restrict__ minute,
                                                         Info* __restrict__ info) {
  __shared__ uint4 stage[CLP_THREADS / 64][192];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u32 bad = 0, mn = 0xffffffffu, mx = 0;
  const size_t step = (size_t)gridDim.x * CLP_THREADS;
  size_t first = ((size_t)blockIdx.x * (CLP_THREADS / 64) + wv) * 64;
  for (; first < n; first += step) {
    // no register prefetch: occupancy (~50 VGPRs) hides the load latency
    uint4 a, b, c;
    clp_fetch<S48>(ts, stride, n, first, a, b, c);
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
    const Parsed p = parse_ts46(w);  // lanes past n parse zeros; only their stores are masked
    const bool valid = (p.meta & EVM_META_VALID) != 0;
    if (i < n) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const v4u kv = {(u32)p.tc, (u32)(p.tc >> 32), (u32)p.rh, (u32)(p.rh >> 32)};
      __builtin_nontemporal_store(kv, reinterpret_cast<v4u*>(key) + i);
      bad |= valid ? 0u : 1u;
    }
    if (S48 && first + 64 <= n && (first & 3) == 0) {
      // rl / hash / minute of the wave's 64 rows: staged in LDS and written
      // as one 16-B-per-lane store (48 lanes) instead of three 4-B stores
      u32* st32 = reinterpret_cast<u32*>(&stage[wv][0]);
      st32[lane] = p.rl | (valid ? OKEY_PRESENT : 0u);
      st32[64 + lane] = p.hash;
      st32[128 + lane] = p.minute;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (lane < 48) {  // (a non-temporal store here measured slower: 150 vs 139 us)
        const uint4 v = stage[wv][lane];
        u32* dst = lane < 16 ? rl : lane < 32 ? hash : minute;
        reinterpret_cast<uint4*>(dst + first)[lane & 15] = v;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    } else if (i < n) {
      rl[i] = p.rl | (valid ? OKEY_PRESENT : 0u);
      hash[i] = p.hash;
      minute[i] = p.minute;
    }
    mn = min(mn, valid ? p.minute : 0xffffffffu);
    mx = max(mx, valid ? p.minute : 0u);
  }
  block_fold_bounds<u32, CLP_THREADS>(mn, mx, bad, &info->minute_min, &info->minute_max, &info->bad);
}

}  // namespace evm
