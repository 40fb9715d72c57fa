// Device-side building blocks for the Evolu batch-merge engine (gfx950).
//
// Everything here restates reference arithmetic bit-exactly:
//   * timestamp parse / canonical check ... packages/evolu/src/timestamp.ts:43-55
//   * murmur3 of the canonical string ..... timestamp.ts:87-88 (murmurhash@2.0.1 = MurmurHash3_x86_32, seed 0)
//   * minute key ........................... merkleTree.ts:33  ((millis/1000/60)|0).toString(3)
//   * timestamp order ...................... applyMessages.ts:93 (JS string '<'), SQLite BINARY collation
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/evm.h"

namespace evm {

typedef unsigned long long u64;
typedef uint32_t u32;

// ----------------------------------------------------------------------------
// Timestamp key.  A canonical 46-byte string
//     YYYY-MM-DDTHH:mm:ss.sssZ-CCCC-NNNNNNNNNNNNNNNN
// packs losslessly into (tc, node, casemask):
//     tc   = millis << 16 | counter         (millis < 2^48)
//     node = 16 hex digits as a 64-bit value (case folded)
//     mask = bit i set <=> node char i is an upper-case letter A-F
// Byte-lexicographic order of the strings == (tc, node-with-case-rank) order,
// because every field is fixed width and zero padded.
// ----------------------------------------------------------------------------
struct Key {
  u64 tc;
  u64 node;
  u32 mask;  // casemask | KEY_PRESENT; 0 == "no timestamp" (SQL NULL), the minimum
};
constexpr u32 KEY_PRESENT = 0x80000000u;

__device__ __forceinline__ Key key_none() { return Key{0ull, 0ull, 0u}; }
__device__ __forceinline__ Key key_of(const evm_rec& r) {
  return Key{r.tc, r.node, (r.meta & EVM_META_CASEMASK) | KEY_PRESENT};
}

// Rank of one node char: '0'-'9' -> 0-9, 'A'-'F' -> 10-15, 'a'-'f' -> 16-21
// (ASCII order of the raw bytes).
__device__ __forceinline__ u32 node_char_rank(u32 v, u32 upper) {
  return v + ((v >= 10u && !upper) ? 6u : 0u);
}

// Three-way compare of two present keys, exactly as the raw strings compare.
__device__ __forceinline__ int key_cmp_present(const Key& a, const Key& b) {
  if (a.tc != b.tc) return a.tc < b.tc ? -1 : 1;
  if (a.mask == b.mask) {
    // Same case pattern: per char, rank is monotone in the hex value.
    if (a.node != b.node) return a.node < b.node ? -1 : 1;
    return 0;
  }
  // Different case patterns (rare): first differing char decides by rank.
  for (int i = 0; i < 16; ++i) {
    const u32 va = (u32)(a.node >> (60 - 4 * i)) & 15u;
    const u32 vb = (u32)(b.node >> (60 - 4 * i)) & 15u;
    const u32 ra = node_char_rank(va, (a.mask >> i) & 1u);
    const u32 rb = node_char_rank(vb, (b.mask >> i) & 1u);
    if (ra != rb) return ra < rb ? -1 : 1;
  }
  return 0;
}

// NULL (absent) is below every timestamp.
__device__ __forceinline__ int key_cmp(const Key& a, const Key& b) {
  const bool pa = a.mask & KEY_PRESENT, pb = b.mask & KEY_PRESENT;
  if (!pa || !pb) return (int)pa - (int)pb;
  return key_cmp_present(a, b);
}
__device__ __forceinline__ bool key_eq(const Key& a, const Key& b) {
  return a.tc == b.tc && a.node == b.node && a.mask == b.mask;
}
__device__ __forceinline__ Key key_max(const Key& a, const Key& b) { return key_cmp(a, b) >= 0 ? a : b; }

// ----------------------------------------------------------------------------
// MurmurHash3_x86_32, seed 0, specialised to 46 bytes = 11 blocks + 2-byte tail.
// w[0..11] are the string's little-endian 32-bit words (w[11] holds bytes 44,45).
// ----------------------------------------------------------------------------
__device__ __forceinline__ u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ __forceinline__ u32 murmur3_46(const u32 (&w)[12]) {
  const u32 c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  u32 h = 0u;
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    u32 k = w[i] * c1;
    k = rotl32(k, 15) * c2;
    h ^= k;
    h = rotl32(h, 13) * 5u + 0xe6546b64u;
  }
  u32 k = w[11] & 0xffffu;  // tail: bytes 44 (low) and 45
  k *= c1;
  k = rotl32(k, 15) * c2;
  h ^= k;
  h ^= 46u;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// ----------------------------------------------------------------------------
// Parse + canonical check of one 46-byte timestamp.
// ----------------------------------------------------------------------------
__device__ __forceinline__ u32 byte_at(const u32 (&w)[12], int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }

__device__ __forceinline__ bool is_digit(u32 c) { return c - 0x30u < 10u; }

// Days since 1970-01-01 of a proleptic Gregorian date (y >= 1970 here).
__device__ __forceinline__ int64_t days_from_civil(int y, int m, int d) {
  y -= m <= 2;
  const int era = y / 400;  // y >= 0 on the native path
  const int yoe = y - era * 400;
  const int doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return (int64_t)era * 146097 + doe - 719468;
}

// Millis below this bound give an int32 minute, so `(millis/1000/60)|0`
// (merkleTree.ts:33) equals floor(millis/60000) and no ToInt32 wrap occurs.
constexpr u64 NATIVE_MILLIS_END = 2147483648ull * 60000ull;

struct Parsed {
  u64 tc;
  u64 node;
  u32 meta;
  u32 hash;
  u32 minute;
};

__device__ __forceinline__ Parsed parse_ts46(const u32 (&w)[12]) {
  Parsed p;
  bool ok = true;
  // separators
  ok &= byte_at(w, 4) == '-' && byte_at(w, 7) == '-' && byte_at(w, 10) == 'T' && byte_at(w, 13) == ':' &&
        byte_at(w, 16) == ':' && byte_at(w, 19) == '.' && byte_at(w, 23) == 'Z' && byte_at(w, 24) == '-' &&
        byte_at(w, 29) == '-';
  // decimal fields
  u32 dig[17];
  const int dpos[17] = {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18, 20, 21, 22};
#pragma unroll
  for (int i = 0; i < 17; ++i) {
    const u32 c = byte_at(w, dpos[i]);
    ok &= is_digit(c);
    dig[i] = c - 0x30u;
  }
  const int year = dig[0] * 1000 + dig[1] * 100 + dig[2] * 10 + dig[3];
  const int mon = dig[4] * 10 + dig[5];
  const int day = dig[6] * 10 + dig[7];
  const int hh = dig[8] * 10 + dig[9];
  const int mi = dig[10] * 10 + dig[11];
  const int ss = dig[12] * 10 + dig[13];
  const int sss = dig[14] * 100 + dig[15] * 10 + dig[16];
  const bool leap = (year % 4 == 0 && year % 100 != 0) || year % 400 == 0;
  int dim = 31;
  if (mon == 4 || mon == 6 || mon == 9 || mon == 11) dim = 30;
  if (mon == 2) dim = leap ? 29 : 28;
  ok &= mon >= 1 && mon <= 12 && day >= 1 && day <= dim && hh <= 23 && mi <= 59 && ss <= 59;
  // counter: exactly 4 upper-case hex digits (canonical form of toString(16).toUpperCase())
  u32 counter = 0;
#pragma unroll
  for (int i = 25; i < 29; ++i) {
    const u32 c = byte_at(w, i);
    const bool d = is_digit(c), u = c - 0x41u < 6u;
    ok &= d || u;
    counter = counter * 16u + (d ? c - 0x30u : c - 0x37u);
  }
  // node: 16 hex digits, either case (types.ts:42 /^[0-9a-f]{16}$/i)
  u64 node = 0;
  u32 mask = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const u32 c = byte_at(w, 30 + i);
    const bool d = is_digit(c), u = c - 0x41u < 6u, l = c - 0x61u < 6u;
    ok &= d || u || l;
    const u32 v = d ? c - 0x30u : (u ? c - 0x37u : c - 0x57u);
    node = (node << 4) | v;
    mask |= (u ? 1u : 0u) << i;
  }
  u32 meta = mask;
  u64 millis = 0;
  u32 minute = 0;
  if (!ok) {
    meta |= EVM_META_NONCANON;
  } else if (year < 1970) {
    meta |= EVM_META_RANGE;
  } else {
    millis = (u64)(((days_from_civil(year, mon, day) * 24 + hh) * 60 + mi) * 60 + ss) * 1000ull + (u64)sss;
    if (millis >= NATIVE_MILLIS_END) {
      meta |= EVM_META_RANGE;
    } else {
      meta |= EVM_META_VALID;
      minute = (u32)(millis / 60000ull);
    }
  }
  p.tc = (millis << 16) | counter;
  p.node = node;
  p.meta = meta;
  p.hash = (meta & EVM_META_VALID) ? murmur3_46(w) : 0u;
  p.minute = minute;
  return p;
}

// Loads the 46 significant bytes of timestamp i into 12 words.
__device__ __forceinline__ void load_ts(const uint8_t* __restrict__ base, size_t stride, size_t i, u32 (&w)[12]) {
  const uint8_t* s = base + i * stride;
  if ((stride & 15) == 0) {
    const uint4* v = reinterpret_cast<const uint4*>(s);
    const uint4 a = v[0], b = v[1], c = v[2];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w & 0xffffu;
  } else if ((stride & 1) == 0) {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(s);
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const u32 lo = h[2 * k];
      const u32 hi = (k < 11) ? (u32)h[2 * k + 1] : 0u;
      w[k] = lo | (hi << 16);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      u32 x = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (4 * k + j < 46) x |= (u32)s[4 * k + j] << (8 * j);
      w[k] = x;
    }
  }
}

// ----------------------------------------------------------------------------
// Merkle key path.  key = minute.toString(3) (merkleTree.ts:33).  A path of
// L base-3 digits d_0..d_{L-1} is coded as sum (d_i + 1) * 4^(19 - i): the
// code order is the trie's depth-first order, and a node's subtree is the
// code range [code(prefix), code(prefix) + 4^(20 - depth)).
// ----------------------------------------------------------------------------
constexpr int CODE_DIGITS = 20;  // 3^20 > 2^31 > every native minute

__device__ __forceinline__ int base3_len(u32 m) {
  int L = 1;
  u64 p = 3;
  while (L < CODE_DIGITS && (u64)m >= p) {
    p *= 3;
    ++L;
  }
  return L;
}

__device__ __forceinline__ u64 minute_code(u32 m) {
  const int L = base3_len(m);
  u64 code = 0;
  // digits least significant first
  for (int i = L - 1; i >= 0; --i) {
    const u32 q = m / 3u;
    const u32 d = m - q * 3u;
    m = q;
    code |= (u64)(d + 1u) << (2 * (CODE_DIGITS - 1 - i));
  }
  return code;
}

}  // namespace evm
