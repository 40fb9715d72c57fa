// Microbenchmark: the random-access costs of the server path on MI355X.
// n = 2^27 rows; perm = a multiplicative bijection of [0, n) (random-like).
//   gather32 -- out[p] = rec[perm[p]] (32-B records, what K5 phase A reads)
//   scatter1 -- flags[perm[p]] = v (1-B random stores, K5's per-message flags)
//   scatter4 -- 4-B random stores
//   seq1     -- flags[p] = v (coalesced reference)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gather_probe.hip -o tools/gather_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

struct Rec {
  uint4 a, b;
};

__global__ void k_perm(uint32_t* perm, size_t n) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    perm[p] = (uint32_t)((p * 2654435761ull) & (n - 1));
}
__global__ void k_gather(const Rec* __restrict__ rec, const uint32_t* __restrict__ perm, size_t n, Rec* __restrict__ out) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    out[p] = rec[perm[p]];
}
__global__ void k_scatter1(const uint32_t* __restrict__ perm, size_t n, uint8_t* __restrict__ f) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    f[perm[p]] = (uint8_t)p;
}
__global__ void k_scatter4(const uint32_t* __restrict__ perm, size_t n, uint32_t* __restrict__ f) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    f[perm[p]] = (uint32_t)p;
}
__global__ void k_seq1(const uint32_t* __restrict__ perm, size_t n, uint8_t* __restrict__ f) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    f[p] = (uint8_t)perm[p];
}

int main() {
  const size_t n = (size_t)1 << 27;
  Rec *rec, *out;
  uint32_t *perm, *f4;
  uint8_t* f1;
  CK(hipMalloc(&rec, n * sizeof(Rec)));
  CK(hipMalloc(&out, n * sizeof(Rec)));
  CK(hipMalloc(&perm, n * 4));
  CK(hipMalloc(&f4, n * 4));
  CK(hipMalloc(&f1, n));
  CK(hipMemset(rec, 1, n * sizeof(Rec)));
  hipLaunchKernelGGL(k_perm, dim3(8192), dim3(256), 0, 0, perm, n);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[] = {"gather32", "scatter1", "scatter4", "seq1"};
  const double bytes[] = {4.0 + 32 + 32, 4.0 + 1, 4.0 + 4, 4.0 + 1};
  for (int k = 0; k < 4; ++k) {
    float best = 1e9f;
    for (int it = 0; it < 5; ++it) {
      CK(hipEventRecord(a, 0));
      if (k == 0) hipLaunchKernelGGL(k_gather, dim3(8192), dim3(256), 0, 0, rec, perm, n, out);
      if (k == 1) hipLaunchKernelGGL(k_scatter1, dim3(8192), dim3(256), 0, 0, perm, n, f1);
      if (k == 2) hipLaunchKernelGGL(k_scatter4, dim3(8192), dim3(256), 0, 0, perm, n, f4);
      if (k == 3) hipLaunchKernelGGL(k_seq1, dim3(8192), dim3(256), 0, 0, perm, n, f1);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    printf("%-9s n=2^27: %.3f ms  %.1f ns/row  (%.0f GB/s of useful bytes)\n", names[k], best, best * 1e6 / n,
           bytes[k] * n / (best * 1e-3) / 1e9);
  }
  return 0;
}
