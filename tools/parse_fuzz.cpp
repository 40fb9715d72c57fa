// Host fuzz of the device timestamp parser (evm_device.hpp parse_ts46, SWAR)
// against the C restatement of the reference (oracle/c/evolu_oracle.c
// evo_parse / evo_murmur3).  Test infrastructure only.
//
//   gcc -O2 -c oracle/c/evolu_oracle.c -o /tmp/eo.o
//   hipcc -O2 -std=c++17 -I include tools/parse_fuzz.cpp -x none /tmp/eo.o -o /tmp/parse_fuzz && /tmp/parse_fuzz
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "../evolu_amd/csrc/evm_device.hpp"

extern "C" int evo_parse(const char* s, int64_t* millis, int* counter);
extern "C" uint32_t evo_murmur3(const uint8_t* d, size_t n);

using namespace evm;

static bool calendar_ok(int y, int mo, int d) {
  static const int t[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (mo < 1 || mo > 12 || d < 1) return false;
  int lim = t[mo - 1];
  if (mo == 2 && ((y % 4 == 0 && y % 100 != 0) || y % 400 == 0)) lim = 29;
  return d <= lim;
}

static int check(const char* s, long long* nvalid) {
  u32 w[12];
  memset(w, 0, sizeof(w));
  memcpy(w, s, 46);
  w[11] &= 0xffffu;
  const Parsed p = parse_ts46(w);
  int64_t millis = 0;
  int counter = 0;
  const bool ok = evo_parse(s, &millis, &counter) == 1;
  const bool valid = (p.meta & EVM_META_VALID) != 0;
  if (ok != valid) {
    printf("validity mismatch: %.46s oracle=%d meta=%x\n", s, ok, p.meta);
    return 1;
  }
  // node + mask
  u64 node = 0;
  u32 mask = 0;
  bool hex = true;
  for (int i = 0; i < 16; ++i) {
    const char c = s[30 + i];
    int v = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
    if (v < 0) hex = false;
    if (c >= 'A' && c <= 'F') mask |= 1u << i;
    node = (node << 4) | (u64)(v & 15);
  }
  if (ok) {
    ++*nvalid;
    u64 rh;
    u32 rl;
    node_rank(node, mask, &rh, &rl);
    if (p.rh != rh || p.rl != rl) {
      printf("rank mismatch: %.46s rh %llx/%llx rl %x/%x\n", s, (unsigned long long)p.rh, (unsigned long long)rh,
             p.rl, rl);
      return 1;
    }
    const u64 tc = ((u64)millis << 16) | (u32)counter;
    const u32 h = evo_murmur3((const uint8_t*)s, 46);
    if (p.tc != tc || p.node != node || (p.meta & EVM_META_CASEMASK) != mask || p.hash != h ||
        p.minute != (u32)(millis / 60000)) {
      printf("value mismatch: %.46s tc %llx/%llx node %llx/%llx hash %x/%x minute %u/%lld\n", s,
             (unsigned long long)p.tc, (unsigned long long)tc, (unsigned long long)p.node, (unsigned long long)node,
             p.hash, h, p.minute, (long long)(millis / 60000));
      return 1;
    }
  } else {
    // RANGE iff the string is canonical apart from the native domain
    int y = 0, mo = 0, d = 0;
    bool pat = sscanf(s, "%4d-%2d-%2d", &y, &mo, &d) == 3;
    for (int i : {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18, 20, 21, 22})
      pat &= s[i] >= '0' && s[i] <= '9';
    pat &= s[4] == '-' && s[7] == '-' && s[10] == 'T' && s[13] == ':' && s[16] == ':' && s[19] == '.' &&
           s[23] == 'Z' && s[24] == '-' && s[29] == '-' && hex;
    for (int i = 25; i < 29; ++i) pat &= (s[i] >= '0' && s[i] <= '9') || (s[i] >= 'A' && s[i] <= 'F');
    if (pat) {
      const int hh = (s[11] - '0') * 10 + s[12] - '0', mi = (s[14] - '0') * 10 + s[15] - '0',
                ss = (s[17] - '0') * 10 + s[18] - '0';
      pat &= calendar_ok(y, mo, d) && hh <= 23 && mi <= 59 && ss <= 59;
    }
    const u32 want = pat ? EVM_META_RANGE : EVM_META_NONCANON;
    if ((p.meta & (EVM_META_RANGE | EVM_META_NONCANON | EVM_META_VALID)) != want || p.hash != 0) {
      printf("class mismatch: %.46s meta %x want %x\n", s, p.meta, want);
      return 1;
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  const long long iters = argc > 1 ? atoll(argv[1]) : 20000000;
  std::mt19937_64 rng(12345);
  const char* hexs = "0123456789abcdefABCDEF";
  char s[64];
  long long nvalid = 0, fails = 0;
  for (long long it = 0; it < iters && fails < 10; ++it) {
    const int y = (int)(rng() % 10000), mo = (int)(rng() % 14), d = (int)(rng() % 33);
    const int hh = (int)(rng() % 26), mi = (int)(rng() % 62), ss = (int)(rng() % 62), ms = (int)(rng() % 1000);
    const unsigned c = (unsigned)(rng() % 65536);
    snprintf(s, sizeof(s), "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ-%04X-", y, mo, d, hh, mi, ss, ms, c);
    const int upper = (int)(rng() % 4);
    for (int i = 0; i < 16; ++i) s[30 + i] = hexs[rng() % (upper == 0 ? 22 : 16)];
    s[46] = 0;
    const u64 r = rng() % 8;
    if (r == 0) {  // one random byte anywhere
      s[rng() % 46] = (char)(rng() & 0xff);
    } else if (r == 1) {  // lower-case counter digit
      s[25 + rng() % 4] = "abcdef"[rng() % 6];
    } else if (r == 2) {  // near-class bytes
      static const char near[] = {'/', ':', '@', 'G', '`', 'g', 0x7f, (char)0x80, (char)0xb0, (char)0xff, ' ', '.'};
      s[rng() % 46] = near[rng() % sizeof(near)];
    }
    fails += check(s, &nvalid);
  }
  // calendar edges exhaustively: every year, Feb 28/29/30, Dec 31, Jan 1
  for (int y = 0; y < 10000 && fails < 10; ++y) {
    for (int k = 0; k < 6; ++k) {
      static const int md[6][2] = {{2, 28}, {2, 29}, {2, 30}, {12, 31}, {1, 1}, {3, 1}};
      snprintf(s, sizeof(s), "%04d-%02d-%02dT23:59:59.999Z-FFFF-0123456789abcdef", y, md[k][0], md[k][1]);
      fails += check(s, &nvalid);
    }
  }
  // order: (tc, rh, rl) lexicographic == byte order of the strings
  {
    char a[64], b[64];
    long long pairs = 0;
    for (long long it = 0; it < 2000000 && fails < 10; ++it) {
      for (char* s2 : {a, b}) {
        const unsigned long long t = 1700000000000ull + rng() % 5;
        const unsigned c = (unsigned)(rng() % 3);
        const int y = 2023 + (int)(t % 2);
        snprintf(s2, 64, "%04d-11-14T22:13:20.%03lluZ-%04X-", y, t % 1000, c);
        for (int i = 0; i < 16; ++i) s2[30 + i] = (rng() % 3) ? a[30 + i] : hexs[rng() % 22];
        if (s2 == a) for (int i = 0; i < 16; ++i) s2[30 + i] = hexs[rng() % 22];
        s2[46] = 0;
      }
      u32 wa[12] = {0}, wb[12] = {0};
      memcpy(wa, a, 46);
      memcpy(wb, b, 46);
      const Parsed pa = parse_ts46(wa), pb = parse_ts46(wb);
      const int want = memcmp(a, b, 46);
      const int got = pa.tc != pb.tc ? (pa.tc < pb.tc ? -1 : 1)
                                     : pa.rh != pb.rh ? (pa.rh < pb.rh ? -1 : 1) : pa.rl != pb.rl ? (pa.rl < pb.rl ? -1 : 1) : 0;
      if ((want > 0) - (want < 0) != got) {
        printf("order mismatch: %.46s vs %.46s got %d\n", a, b, got);
        ++fails;
      }
      ++pairs;
    }
    printf("order pairs: %lld\n", pairs);
  }
  printf("%s: %lld strings, %lld valid, %lld failures\n", fails ? "FAIL" : "OK", iters, nvalid, fails);
  return fails ? 1 : 0;
}
