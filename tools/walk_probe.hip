// Microbenchmark: what bounds the tc path's walk (TP3, k_tp_walk)?  One wave
// per range of ~4.9k rows, 64 rows per round; variants add one piece each:
//   M0 loads (tc 8 B + cell 4 B) + flag byte store
//   M1 + the per-cell LDS state (read, compare, write)
//   M2 + the cell ballots (match_cell, 10 bits for 1,000 cells)
//   M3 + the lower-peer max loop (= the walk)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/walk_probe.hip -o tools/walk_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../evolu_amd/csrc/evm_device.hpp"
#include "../evolu_amd/csrc/evm_prims.hpp"

using namespace evm;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ u64 match_bits(u32 c, bool active, int bits) {
  u64 peers = __ballot(active);
  for (int b = 0; b < bits; ++b) {
    const bool bit = (c >> b) & 1u;
    const u64 bal = __ballot(bit);
    peers &= bit ? bal : ~bal;
  }
  return active ? peers : 0ull;
}

template <int MODE, int PF>
__global__ __launch_bounds__(256) void k_walk(const u64* __restrict__ tcs, const u32* __restrict__ cell, size_t n,
                                              u32 C, int cbits, size_t range_len, size_t G,
                                              uint8_t* __restrict__ flags, u32* __restrict__ sink) {
  extern __shared__ u64 lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t g = (size_t)blockIdx.x * 4 + wv;
  if (g >= G) return;
  u64* T = lds + (size_t)wv * C;
  for (u32 c = lane; c < C; c += 64) T[c] = 0;
  __builtin_amdgcn_wave_barrier();
  const u64 lt = lanemask_lt();
  const size_t beg = g * range_len, end = min(n, beg + range_len);
  u64 px[PF];
  u32 pc[PF];
#pragma unroll
  for (int r = 0; r < PF; ++r) {
    const size_t i = beg + 64 * r + lane;
    px[r] = i < end ? __builtin_nontemporal_load(tcs + i) : ~0ull;
    pc[r] = i < end ? __builtin_nontemporal_load(cell + i) : 0u;
  }
  u32 acc = 0;
  for (size_t first = beg; first < end; first += 64 * PF) {
#pragma unroll
    for (int r = 0; r < PF; ++r) {
      const size_t f = first + 64 * r;
      const u64 x = px[r];
      const u32 c = pc[r];
      {
        const size_t i = f + 64 * PF + lane;
        px[r] = i < end ? __builtin_nontemporal_load(tcs + i) : ~0ull;
        pc[r] = i < end ? __builtin_nontemporal_load(cell + i) : 0u;
      }
      if (f >= end) continue;
      const bool ok = x != ~0ull;
      uint8_t fl = 0;
      if (MODE == 0) {
        fl = (uint8_t)(x ^ c);
      } else {
        u64 pm = 0;
        u64 peers = 1ull << lane;
        if (MODE >= 2) peers = match_bits(c, ok, cbits);
        if (MODE >= 3) {
          u64 rem = peers & lt;
          while (__any(rem != 0)) {
            const int src = rem ? (int)__builtin_ctzll(rem) : lane;
            const u64 v = __shfl(x, src, 64);
            if (rem) {
              pm = max(pm, v);
              rem &= rem - 1;
            }
          }
        }
        if (ok) {
          const u64 t = max(T[c], pm);
          fl = x > t ? 3 : (x < t ? 2 : 0);
          if (MODE == 1) atomicMax(&T[c], x);
          else if ((peers >> lane) == 1ull) T[c] = max(t, x);
        }
      }
      if (f + lane < end) flags[f + lane] = fl;
      acc += fl;
    }
  }
  if (acc == 0xdeadbeef) sink[0] = acc;
}

template <int MODE, int PF>
static float run(const u64* tcs, const u32* cell, size_t n, u32 C, size_t G, uint8_t* flags, u32* sink) {
  const size_t range = ((n + G - 1) / G + 255) / 256 * 256;
  const int cbits = 32 - __builtin_clz(C - 1);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 grid((G + 3) / 4);
  hipLaunchKernelGGL((k_walk<MODE, PF>), grid, dim3(256), 4 * C * 8, 0, tcs, cell, n, C, cbits, range, G, flags, sink);
  CK(hipEventRecord(a, 0));
  for (int k = 0; k < 10; ++k)
    hipLaunchKernelGGL((k_walk<MODE, PF>), grid, dim3(256), 4 * C * 8, 0, tcs, cell, n, C, cbits, range, G, flags,
                       sink);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / 10 * 1e3f;
}

int main() {
  const size_t n = 10000000;
  const u32 C = 1000;
  std::vector<u64> h(n);
  std::vector<u32> hc(n);
  uint64_t s = 88172645463325252ull;
  for (size_t i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    h[i] = s >> 2;
    hc[i] = (u32)(s % C);
  }
  u64* tcs;
  u32* cell;
  uint8_t* flags;
  u32* sink;
  CK(hipMalloc(&tcs, n * 8));
  CK(hipMalloc(&cell, n * 4));
  CK(hipMalloc(&flags, n));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(tcs, h.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(cell, hc.data(), n * 4, hipMemcpyHostToDevice));
  for (size_t G : {2048, 4096, 8192}) {
    printf("G=%zu  M0 %.1f  M1 %.1f  M2 %.1f  M3 %.1f us  (PF 8)   M3 PF4 %.1f  M3 PF16 %.1f\n", G,
           run<0, 8>(tcs, cell, n, C, G, flags, sink), run<1, 8>(tcs, cell, n, C, G, flags, sink),
           run<2, 8>(tcs, cell, n, C, G, flags, sink), run<3, 8>(tcs, cell, n, C, G, flags, sink),
           run<3, 4>(tcs, cell, n, C, G, flags, sink), run<3, 16>(tcs, cell, n, C, G, flags, sink));
  }
  return 0;
}
