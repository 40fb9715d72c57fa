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

// min / max of one unsigned long long and one unsigned long (uint64_t, size_t):
// HIP's overload set has no exact match for the mixed pair, and the call
// resolves to the double overload -- 53 bits: an HLC key (millis << 16 |
// counter, 57 bits) loses its counter.  These exact matches keep it integer.
__device__ __forceinline__ unsigned long long min(unsigned long long a, unsigned long b) {
  return a < (unsigned long long)b ? a : (unsigned long long)b;
}
__device__ __forceinline__ unsigned long long min(unsigned long a, unsigned long long b) {
  return (unsigned long long)a < b ? (unsigned long long)a : b;
}
__device__ __forceinline__ unsigned long long max(unsigned long long a, unsigned long b) {
  return a > (unsigned long long)b ? a : (unsigned long long)b;
}
__device__ __forceinline__ unsigned long long max(unsigned long a, unsigned long long b) {
  return (unsigned long long)a > b ? (unsigned long long)a : b;
}

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
#pragma unroll 1
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
// Order key: the raw-string order as three unsigned words, no case loop.
//   tc  = millis << 16 | counter
//   rh  = ranks of node chars 0..11, 5 bits each (rank: '0'-'9' 0-9,
//         'A'-'F' 10-15, 'a'-'f' 16-21 = ASCII order of the bytes)
//   rl  = ranks of node chars 12..15 (20 bits) | OKEY_PRESENT
// (tc, rh, rl) compare lexicographically exactly as the 46-byte strings, and
// are equal iff the strings are; the all-zero key is NULL, below every
// present key.  The streaming client path carries only this.
// ----------------------------------------------------------------------------
constexpr u32 OKEY_PRESENT = 0x80000000u;
struct OKey {
  u64 tc;
  u64 rh;
  u32 rl;
};
__device__ __forceinline__ OKey okey_none() { return OKey{0ull, 0ull, 0u}; }
__device__ __forceinline__ bool okey_gt(const OKey& a, const OKey& b) {
  return a.tc != b.tc ? a.tc > b.tc : (a.rh != b.rh ? a.rh > b.rh : a.rl > b.rl);
}
__device__ __forceinline__ bool okey_eq(const OKey& a, const OKey& b) {
  return a.tc == b.tc && a.rh == b.rh && a.rl == b.rl;
}
__device__ __forceinline__ OKey okey_max(const OKey& a, const OKey& b) { return okey_gt(b, a) ? b : a; }

// (node, case mask) -> (rh, rl without the present bit).
__host__ __device__ __forceinline__ void node_rank(u64 node, u32 mask, u64* rh, u32* rl) {
  u64 h = 0;
  u32 l = 0;
  for (int i = 0; i < 16; ++i) {
    const u32 v = (u32)(node >> (60 - 4 * i)) & 15u;
    const u32 r = v + ((v >= 10u && !((mask >> i) & 1u)) ? 6u : 0u);
    if (i < 12) h = (h << 5) | r;
    else l = (l << 5) | r;
  }
  *rh = h;
  *rl = l;
}
__device__ __forceinline__ OKey okey_of(const evm_rec& r) {
  OKey k;
  k.tc = r.tc;
  node_rank(r.node, r.meta & EVM_META_CASEMASK, &k.rh, &k.rl);
  k.rl |= OKEY_PRESENT;
  return k;
}

// ----------------------------------------------------------------------------
// MurmurHash3_x86_32, seed 0, specialised to 46 bytes = 11 blocks + 2-byte tail.
// w[0..11] are the string's little-endian 32-bit words (w[11] holds bytes 44,45).
// ----------------------------------------------------------------------------
__host__ __device__ __forceinline__ u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }

// h * 5 + c as a shift-add: left as a multiply, the compiler folds the
// rotate, the multiply and the 32-bit constant into a 64-bit multiply-add
// (v_mad_u64_u32, a quarter-rate instruction) once per block; the empty asm
// keeps the shifted copy opaque so the add stays two full-rate adds.
__host__ __device__ __forceinline__ u32 mul5_add(u32 h, u32 c) {
  u32 t = h << 2;
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(t));
#endif
  return h + t + c;
}

__host__ __device__ __forceinline__ u32 murmur3_46(const u32 (&w)[12]) {
  const u32 c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  u32 h = 0u;
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    u32 k = w[i] * c1;
    k = rotl32(k, 15) * c2;
    h ^= k;
    h = mul5_add(rotl32(h, 13), 0xe6546b64u);
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
// Parse + canonical check of one 46-byte timestamp, word-parallel (SWAR).
//
// The string is twelve little-endian words; every byte class test runs on a
// whole word at once, all date arithmetic is 32-bit with multiply-shift
// division (year <= 9999), and the minute comes straight from the fields, so
// no 64-bit division is left on the hot path.
//   w0 YYYY  w1 -MM-  w2 DDTH  w3 H:mm  w4 :ss.  w5 sssZ  w6 -CCC  w7 C-NN
//   w8..w10 NNNN  w11 NN (low half)
// ----------------------------------------------------------------------------
__host__ __device__ __forceinline__ u32 byte_at(const u32 (&w)[12], int k) {
  return (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
}

// Per byte: 0x80 where byte >= n, else 0 (every byte < 0x80, n <= 0x80).
__host__ __device__ __forceinline__ u32 swar_ge(u32 x, u32 n) {
  return ((x | 0x80808080u) - 0x01010101u * n) & 0x80808080u;
}
__host__ __device__ __forceinline__ u32 swar_digit(u32 x) { return swar_ge(x, 0x30) & ~swar_ge(x, 0x3a); }
__host__ __device__ __forceinline__ u32 swar_upper(u32 x) { return swar_ge(x, 0x41) & ~swar_ge(x, 0x47); }
__host__ __device__ __forceinline__ u32 swar_lower(u32 x) { return swar_ge(x, 0x61) & ~swar_ge(x, 0x67); }

// Four hex chars (first char in the low byte) -> their 16-bit value; any case.
__host__ __device__ __forceinline__ u32 swar_nibbles(u32 x) {  // per byte: hex value of the char
  return (x & 0x0f0f0f0fu) + ((x >> 6) & 0x01010101u) * 9u;
}
__host__ __device__ __forceinline__ u32 swar_hex16(u32 x) {
  const u32 v = swar_nibbles(x);
  const u32 t = (v << 4) | (v >> 8);  // byte0 = c0<<4|c1, byte2 = c2<<4|c3
  return ((t & 0xffu) << 8) | ((t >> 16) & 0xffu);
}
// Four node chars -> their four 5-bit ranks, first char most significant.
__host__ __device__ __forceinline__ u32 swar_rank20(u32 x) {
  const u32 r = swar_nibbles(x) + (swar_lower(x) >> 7) * 6u;  // lower-case letters rank above upper
  return ((r & 0xffu) << 15) | (((r >> 8) & 0xffu) << 10) | (((r >> 16) & 0xffu) << 5) | (r >> 24);
}
// 0x80-per-byte flags -> 4 bits (byte k -> bit k).
__host__ __device__ __forceinline__ u32 swar_bits4(u32 f) {
  const u32 m = f >> 7;
  return (m | (m >> 7) | (m >> 14) | (m >> 21)) & 0xfu;
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
  u64 rh;  // order key words (OKey); rl without OKEY_PRESENT
  u32 rl;
};

__host__ __device__ __forceinline__ u32 mul24(u32 a, u32 b) { return a * b; }  // a, b < 2^24: v_mul_u32_u24

__host__ __device__ __forceinline__ Parsed parse_ts46(const u32 (&w)[12]) {
  // byte classes: separators by template, digits / hex by SWAR ranges.  Every
  // failed check sets bits of `err` (no short-circuit `&&`: on the device a
  // chain of them compiles to one exec-mask branch per test)
  u32 err = (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7] | w[8] | w[9] | w[10] | (w[11] & 0xffffu)) &
            0x80808080u;
  err |= ((w[1] & 0xff0000ffu) ^ 0x2d00002du) | ((w[2] & 0x00ff0000u) ^ 0x00540000u) |
         ((w[3] & 0x0000ff00u) ^ 0x00003a00u) | ((w[4] & 0xff0000ffu) ^ 0x2e00003au) |
         ((w[5] & 0xff000000u) ^ 0x5a000000u) | ((w[6] & 0xffu) ^ 0x2du) | ((w[7] & 0xff00u) ^ 0x2d00u);
  // (swar_digit sets only 0x80 bits: a required digit missing leaves its bit in ~d & m)
  err |= (~swar_digit(w[0]) & 0x80808080u) | (~swar_digit(w[1]) & 0x00808000u) | (~swar_digit(w[2]) & 0x80008080u) |
         (~swar_digit(w[3]) & 0x80800080u) | (~swar_digit(w[4]) & 0x00808000u) | (~swar_digit(w[5]) & 0x00808080u);
  // counter: exactly 4 upper-case hex digits (canonical toString(16).toUpperCase())
  const u32 cw = (w[6] >> 8) | (w[7] << 24);
  err |= ~(swar_digit(cw) | swar_upper(cw)) & 0x80808080u;
  // node: 16 hex digits, either case (types.ts:42 /^[0-9a-f]{16}$/i)
  u32 nw[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) nw[k] = (w[7 + k] >> 16) | (w[8 + k] << 16);
  u32 mask = 0;
  u64 node = 0, rh = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32 up = swar_upper(nw[k]);
    err |= ~(swar_digit(nw[k]) | up | swar_lower(nw[k])) & 0x80808080u;
    mask |= swar_bits4(up) << (4 * k);
    node = (node << 16) | swar_hex16(nw[k]);
    if (k < 3) rh = (rh << 20) | swar_rank20(nw[k]);
  }
  bool ok = err == 0;
  const u32 counter = swar_hex16(cw);
  // decimal fields (digits already checked; garbage values only when !ok)
  const u32 d0 = w[0] - 0x30303030u;
  const u32 year = mul24(mul24(d0 & 0xffu, 10u) + ((d0 >> 8) & 0xffu), 100u) +
                   mul24((d0 >> 16) & 0xffu, 10u) + (d0 >> 24);
  auto two = [](u32 x, int sh) { return mul24((x >> sh) & 0xffu, 10u) + ((x >> (sh + 8)) & 0xffu) - 528u; };
  const u32 mon = two(w[1], 8), day = two(w[2], 0), mi = two(w[3], 16), ss = two(w[4], 8);
  const u32 hh = mul24((w[2] >> 24) - 0x30u, 10u) + (w[3] & 0xffu) - 0x30u;
  const u32 sss = mul24(mul24(w[5] & 0xffu, 10u) + ((w[5] >> 8) & 0xffu), 10u) + ((w[5] >> 16) & 0xffu) - 5328u;
  // calendar: leap year and month length without division
  const u32 cent = mul24(year, 5243u) >> 19;  // year / 100 for year < 43699
  const bool leap = ((year & 3u) == 0) & ((year != mul24(cent, 100u)) | ((cent & 3u) == 0));
  constexpr u32 MLEN = (3u << 2) | (0u << 4) | (3u << 6) | (2u << 8) | (3u << 10) | (2u << 12) | (3u << 14) |
                       (3u << 16) | (2u << 18) | (3u << 20) | (2u << 22) | (3u << 24);  // month length - 28, by 2*mon
  const bool mon_ok = mon - 1u < 12u;
  const u32 dim = 28u + ((MLEN >> (2u * (mon & 15u))) & 3u) + (((mon == 2u) & leap) ? 1u : 0u);
  ok = ok & mon_ok & (day - 1u < dim) & (hh <= 23u) & (mi <= 59u) & (ss <= 59u);
  // days since 1970-01-01 (March-based year): 365y + y/4 - y/100 + y/400 + doy - 719468;
  // computed for every row (garbage when !ok, then unused) -- a select, not a branch
  const u32 y = year - (mon <= 2u ? 1u : 0u);
  const u32 yc = mul24(y, 5243u) >> 19;
  const u32 mp = mon > 2u ? mon - 3u : mon + 9u;
  const u32 doy = (mul24(mul24(mp & 15u, 153u) + 2u, 52429u) >> 18) + day - 1u;  // (153 mp + 2) / 5
  const u32 days = mul24(y, 365u) + (y >> 2) - yc + (yc >> 2) + doy - 719468u;
  const u32 m32 = mul24(days & 0xffffffu, 1440u) + mul24(hh & 0xffu, 60u) + mi;  // < 2^32 for year <= 9999
  const bool valid = ok & (year >= 1970u) & (m32 < 0x80000000u);
  u32 meta = mask | (valid ? (u32)EVM_META_VALID : !ok ? (u32)EVM_META_NONCANON : (u32)EVM_META_RANGE);
  const u32 minute = valid ? m32 : 0u;
  const u64 millis = valid ? (u64)m32 * 60000ull + (mul24(ss & 0xffu, 1000u) + sss) : 0ull;
  Parsed p;
  p.tc = (millis << 16) | counter;
  p.node = node;
  p.meta = meta;
  p.hash = valid ? murmur3_46(w) : 0u;
  p.minute = minute;
  p.rh = rh;
  p.rl = swar_rank20(nw[3]);
  return p;
}

// The minute (floor(millis / 60000)) of a timestamp row from its first 16
// bytes, "YYYY-MM-DDTHH:MM" -- parse_ts46's minute on the native domain,
// without its checks (garbage for a row outside it, which the full parse
// flags later).
__host__ __device__ __forceinline__ u32 minute16(u32 w0, u32 w1, u32 w2, u32 w3) {
  const u32 d0 = w0 - 0x30303030u;
  const u32 year = mul24(mul24(d0 & 0xffu, 10u) + ((d0 >> 8) & 0xffu), 100u) + mul24((d0 >> 16) & 0xffu, 10u) +
                   (d0 >> 24);
  auto two = [](u32 x, int sh) { return mul24((x >> sh) & 0xffu, 10u) + ((x >> (sh + 8)) & 0xffu) - 528u; };
  const u32 mon = two(w1, 8), day = two(w2, 0), mi = two(w3, 16);
  const u32 hh = mul24((w2 >> 24) - 0x30u, 10u) + (w3 & 0xffu) - 0x30u;
  const u32 y = year - (mon <= 2u ? 1u : 0u);
  const u32 yc = mul24(y, 5243u) >> 19;
  const u32 mp = mon > 2u ? mon - 3u : mon + 9u;
  const u32 doy = (mul24(mul24(mp & 15u, 153u) + 2u, 52429u) >> 18) + day - 1u;
  const u32 days = mul24(y, 365u) + (y >> 2) - yc + (yc >> 2) + doy - 719468u;
  return mul24(days & 0xffffffu, 1440u) + mul24(hh & 0xffu, 60u) + mi;
}

// The inverse of parse_ts46 on the native domain: timestamp.ts:43-48
// timestampToString of (tc, node, case mask) as 12 little-endian words
// (bytes 46-47 zero).  Proleptic Gregorian civil date of the day count.
__host__ __device__ __forceinline__ void put_byte(u32 (&w)[12], int i, u32 c) {
  w[i >> 2] |= (c & 0xffu) << (8 * (i & 3));
}
__host__ __device__ __forceinline__ void put_dec(u32 (&w)[12], int at, u32 v, int digits) {
  for (int k = digits - 1; k >= 0; --k) {
    put_byte(w, at + k, 0x30u + v % 10u);
    v /= 10u;
  }
}
__host__ __device__ __forceinline__ void format_ts46(u64 tc, u64 node, u32 cmask, u32 (&w)[12]) {
  for (int k = 0; k < 12; ++k) w[k] = 0;
  const u64 ms = tc >> 16;
  const u32 ctr = (u32)(tc & 0xffffu);
  const u64 days = ms / 86400000ull;
  const u32 rem = (u32)(ms - days * 86400000ull);
  const u64 z = days + 719468ull;
  const u64 era = z / 146097ull;
  const u32 doe = (u32)(z - era * 146097ull);
  const u32 yoe = (doe - doe / 1460u + doe / 36524u - doe / 146096u) / 365u;
  const u32 doy = doe - (365u * yoe + yoe / 4u - yoe / 100u);
  const u32 mp = (5u * doy + 2u) / 153u;
  const u32 d = doy - (153u * mp + 2u) / 5u + 1u;
  const u32 m = mp < 10u ? mp + 3u : mp - 9u;
  const u32 y = (u32)(yoe + era * 400ull) + (m <= 2u ? 1u : 0u);
  put_dec(w, 0, y, 4);
  put_byte(w, 4, '-');
  put_dec(w, 5, m, 2);
  put_byte(w, 7, '-');
  put_dec(w, 8, d, 2);
  put_byte(w, 10, 'T');
  put_dec(w, 11, rem / 3600000u, 2);
  put_byte(w, 13, ':');
  put_dec(w, 14, rem / 60000u % 60u, 2);
  put_byte(w, 16, ':');
  put_dec(w, 17, rem / 1000u % 60u, 2);
  put_byte(w, 19, '.');
  put_dec(w, 20, rem % 1000u, 3);
  put_byte(w, 23, 'Z');
  put_byte(w, 24, '-');
  for (int k = 0; k < 4; ++k) {
    const u32 v = (ctr >> (12 - 4 * k)) & 15u;
    put_byte(w, 25 + k, v < 10u ? 0x30u + v : 0x37u + v);  // upper-case hex counter
  }
  put_byte(w, 29, '-');
  for (int k = 0; k < 16; ++k) {
    const u32 v = (u32)(node >> (60 - 4 * k)) & 15u;
    put_byte(w, 30 + k, v < 10u ? 0x30u + v : (((cmask >> k) & 1u) ? 0x37u : 0x57u) + v);
  }
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

__host__ __device__ __forceinline__ int base3_len(u32 m) {
  int L = 1;
  u64 p = 3;
  while (L < CODE_DIGITS && (u64)m >= p) {
    p *= 3;
    ++L;
  }
  return L;
}

// The five base-3 digits of x < 243 as 2-bit fields, most significant first:
// f = x / 243 in 16-bit fixed point, rounded up (270 > 2^16 / 243; the error
// after k steps, < 3^k * 0.0012, stays below the 3^(k-5) gap), then each
// digit is the integer part of f * 3.
__host__ __device__ __forceinline__ u32 b3_raw5(u32 x) {
  u32 f = x * 270u, r = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    f *= 3u;
    r = (r << 2) | (f >> 16);
    f &= 0xffffu;
  }
  return r;
}

// code of minute m from its 20 raw base-3 digits (R(x): the five digits of
// x < 243, from a table or b3_raw5): the L significant digits + 1 each, the
// most significant at the top digit (== the digit loop below, ~8x fewer
// instructions: three divisions instead of twenty, no 64-bit multiply).
template <typename R>
__host__ __device__ __forceinline__ u64 minute_code_from(u32 m, R raw5) {
  const u32 q1 = m / 59049u, r1 = m - q1 * 59049u;  // 3^10
  const u32 a = q1 / 243u, b = q1 - a * 243u, c = r1 / 243u, d = r1 - c * 243u;
  const u64 raw = ((u64)((raw5(a) << 10) | raw5(b)) << 20) | (u64)((raw5(c) << 10) | raw5(d));
  const int top = raw ? 63 - __builtin_clzll(raw) : 0;  // highest set bit
  const int L = top / 2 + 1;                            // significant digits (m == 0: one)
  const u64 ones = 0x5555555555ull >> (2 * (CODE_DIGITS - L));
  return (raw + ones) << (2 * (CODE_DIGITS - L));
}

__host__ __device__ __forceinline__ u64 minute_code(u32 m) {
  return minute_code_from(m, [](u32 x) { return b3_raw5(x); });
}

// The reference digit loop (tests check minute_code against it).
__host__ __device__ __forceinline__ u64 minute_code_loop(u32 m) {
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
