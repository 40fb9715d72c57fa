// Microbenchmark: what bounds the timestamp pack kernel (K1 of the streaming
// client path)?  Times variants that share its load/store pattern:
//   copy   -- loads 48 B/msg, stores 28 B/msg, no parsing
//   parse  -- full parse + canonical check, no murmur3
//   full   -- parse + murmur3 (what k_cl_pack does)
//   real   -- k_cl_pack<true> itself (evm_pack.hpp)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/pack_probe.hip -o tools/pack_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../evolu_amd/csrc/evm_device.hpp"
#include "../evolu_amd/csrc/evm_pack.hpp"

using namespace evm;

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

template <int MODE, int THREADS>
__global__ __launch_bounds__(THREADS) void k_probe(const uint8_t* __restrict__ ts, size_t n, uint4* __restrict__ key,
                                                    u32* __restrict__ meta, u32* __restrict__ hash,
                                                    u32* __restrict__ minute, u32* __restrict__ sink) {
  __shared__ uint4 stage[THREADS / 64][192];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t step = (size_t)gridDim.x * THREADS;
  u32 acc = 0;
  for (size_t first = ((size_t)blockIdx.x * (THREADS / 64) + wv) * 64; first < n; first += step) {
    const uint4* src = reinterpret_cast<const uint4*>(ts + first * 48);
    const uint4 a = src[lane], b = src[lane + 64], c = src[lane + 128];
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
    if (MODE == 0) {
      key[i] = make_uint4(w[0], w[1], w[2] ^ w[3], w[4] ^ w[5]);
      meta[i] = w[6] ^ w[7];
      hash[i] = w[8] ^ w[9];
      minute[i] = w[10] ^ w[11];
    } else {
      Parsed p = parse_ts46(w);
      if (MODE == 1) p.hash = 0;
      key[i] = make_uint4((u32)p.tc, (u32)(p.tc >> 32), (u32)p.node, (u32)(p.node >> 32));
      meta[i] = p.meta;
      hash[i] = p.hash;
      minute[i] = p.minute;
      acc |= p.meta;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

static void fmt_ts(char* s, unsigned long long millis, unsigned counter, unsigned long long node) {
  const long long days = (long long)(millis / 86400000ull);
  // civil from days (Howard Hinnant)
  long long z = days + 719468;
  const long long era = z / 146097;
  const unsigned doe = (unsigned)(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  long long y = (long long)yoe + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  const unsigned d = doy - (153 * mp + 2) / 5 + 1;
  const unsigned m = mp < 10 ? mp + 3 : mp - 9;
  y += m <= 2;
  const unsigned long long ms = millis % 86400000ull;
  char buf[64];
  snprintf(buf, sizeof(buf), "%04lld-%02u-%02uT%02llu:%02llu:%02llu.%03lluZ-%04X-%016llx", y, m, d, ms / 3600000,
           ms / 60000 % 60, ms / 1000 % 60, ms % 1000, counter, node);
  memcpy(s, buf, 46);
}

template <int MODE, int THREADS>
static float run(const uint8_t* ts, size_t n, uint4* key, u32* meta, u32* hash, u32* minute, u32* sink, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_probe<MODE, THREADS>), dim3(grid), dim3(THREADS), 0, 0, ts, n, key, meta, hash, minute, sink);
  CK(hipEventRecord(e0));
  const int R = 20;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL((k_probe<MODE, THREADS>), dim3(grid), dim3(THREADS), 0, 0, ts, n, key, meta, hash, minute, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / R;
}

int main() {
  const size_t n = 10000000;  // multiple of 64
  std::vector<char> h(n * 48, 0);
  unsigned long long t = 1700000000000ull;
  for (size_t i = 0; i < n; ++i) {
    t += (i * 2654435761ull) % 7;
    fmt_ts(&h[i * 48], t, (unsigned)(i % 5), 0x0123456789abcdefull ^ (i % 64));
  }
  uint8_t* ts;
  uint4* key;
  u32 *meta, *hash, *minute, *sink;
  CK(hipMalloc(&ts, n * 48));
  CK(hipMalloc(&key, n * 16));
  CK(hipMalloc(&meta, n * 4));
  CK(hipMalloc(&hash, n * 4));
  CK(hipMalloc(&minute, n * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(ts, h.data(), n * 48, hipMemcpyHostToDevice));
  const double bytes = n * 76.0;
  for (int grid : {1024, 2048, 4096, 8192}) {
    const float c = run<0, 256>(ts, n, key, meta, hash, minute, sink, grid);
    const float p = run<1, 256>(ts, n, key, meta, hash, minute, sink, grid);
    const float f = run<2, 256>(ts, n, key, meta, hash, minute, sink, grid);
    printf("grid %5d x256: copy %.4f ms (%.0f GB/s)  parse %.4f ms  full %.4f ms (%.0f GB/s)\n", grid, c, bytes / c / 1e6,
           p, f, bytes / f / 1e6);
  }
  Info* info;
  CK(hipMalloc(&info, sizeof(Info)));
  CK(hipMemset(info, 0, sizeof(Info)));
  for (int grid : {1024, 2048, 4096, 8192}) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w)
      hipLaunchKernelGGL(k_cl_pack<true>, dim3(grid), dim3(CLP_THREADS), 0, 0, ts, (size_t)48, n, key, meta, hash, minute, info);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 20; ++r)
      hipLaunchKernelGGL(k_cl_pack<true>, dim3(grid), dim3(CLP_THREADS), 0, 0, ts, (size_t)48, n, key, meta, hash, minute, info);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("grid %5d x256: real k_cl_pack %.4f ms (%.0f GB/s)\n", grid, ms / 20, bytes / (ms / 20) / 1e6);
  }
  for (int grid : {2048, 4096}) {
    const float f = run<2, 512>(ts, n, key, meta, hash, minute, sink, grid / 2);
    printf("grid %5d x512: full %.4f ms\n", grid / 2, f);
  }
  std::vector<u32> hm(16);
  CK(hipMemcpy(hm.data(), meta, 64, hipMemcpyDeviceToHost));
  printf("meta[0]=%x (valid bit %d)\n", hm[0], (hm[0] >> 16) & 1);
  return 0;
}
