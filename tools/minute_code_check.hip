// Host check of the fast minute_code (three divisions + base-3 digit tables)
// against the digit loop: all minutes < 3M, 5M random, powers of 3 +-2, the top
// 100k below 2^31.  Built and run by tests/test_minute_code.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../evolu_amd/csrc/evm_device.hpp"
using namespace evm;
int main() {
  for (uint32_t x = 0; x < 243; ++x) {
    uint32_t r = 0, y = x; for (int k = 0; k < 5; ++k) { r |= (y % 3) << (2 * k); y /= 3; }
    if (b3_raw5(x) != r) { printf("raw5 bad %u\n", x); return 1; }
  }
  uint64_t bad = 0, n = 0;
  for (uint64_t m = 0; m < 3000000ull; ++m, ++n) bad += minute_code((uint32_t)m) != minute_code_loop((uint32_t)m);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < 5000000; ++i, ++n) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; uint32_t m = (uint32_t)s & 0x7fffffffu; bad += minute_code(m) != minute_code_loop(m); }
  uint64_t p = 1; for (int k = 0; k < 20; ++k, p *= 3) for (int dlt = -2; dlt <= 2; ++dlt) { int64_t m = (int64_t)p + dlt; if (m >= 0 && m < 0x80000000ll) { ++n; bad += minute_code((uint32_t)m) != minute_code_loop((uint32_t)m); } }
  for (uint32_t m = 0x7fffffffu - 100000; m < 0x80000000u; ++m, ++n) bad += minute_code(m) != minute_code_loop(m);
  printf("checked %lu bad %lu\n", (unsigned long)n, (unsigned long)bad);
  return bad != 0;
}
