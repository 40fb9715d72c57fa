// Synthetic message streams on the device (bench and test input, not part of
// libevm).  Config 5 shape at the end of the file.  BASELINE config 4 -- O owners x P messages, 4 HLC nodes per owner,
// a 30-day span, every timestamp canonical.  Every byte is a
// pure function of (seed, owner, message index), so any rank can regenerate
// any owner's messages (the bench's self-check) and evolu_amd/synth.py has a
// numpy twin that tests compare byte for byte.
//
//   H(t, x, y)      = sm(sm(sm(seed ^ t) ^ x) ^ y), sm = splitmix64's finaliser
//   userId(o)       = 21 lower-case hex chars: H(1,o,0) (16) + H(1,o,1) >> 44 (5)
//   node(o, q)      = 16 lower-case hex chars of H(2, o, q), q < 4
//   message (o, j)  : q = j % 4, k = j / 4, slot = k / 2, counter = k % 2,
//                     millis = T0 + slot * GAP + H(3, o, q << 16 | slot) % GAP
//                     (two sends per node and slot: one millisecond, counters
//                     0 and 1 -- timestamp.ts:97-123 sendTimestamp)
//   client knows    : slot < keep_slots (the first ~90 % of each node's sends)
//   source rank s   : of G, the messages j = s, s + G, ... of every owner, one
//                     request per owner, requests in the order
//                     o = (p * A + seed) mod O (A = 1000003, coprime to O)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "evm_device.hpp"

using namespace evm;

namespace {

constexpr u64 T0 = 1704067200000ull;  // 2024-01-01T00:00:00.000Z
constexpr u64 SPAN = 30ull * 86400000ull;
constexpr u64 PERM_A = 1000003ull;

__host__ __device__ __forceinline__ u64 sm(u64 x) {
  u64 z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ u64 H(u64 seed, u64 t, u64 x, u64 y) { return sm(sm(sm(seed ^ t) ^ x) ^ y); }

struct Shape {
  u64 seed;
  u32 O, P;
  u32 slots;  // slots per node: ceil(ceil(P / 4) / 2)
  u64 gap;
  u32 keep_slots;
};

__device__ __forceinline__ void message(const Shape& S, u32 o, u32 j, u32 (&w)[12], bool* keep) {
  const u32 q = j & 3u, k = j >> 2, slot = k >> 1, ctr = k & 1u;
  const u64 ms = T0 + (u64)slot * S.gap + H(S.seed, 3, o, ((u64)q << 16) | slot) % S.gap;
  const u64 node = H(S.seed, 2, o, q);
  format_ts46((ms << 16) | ctr, node, 0u, w);
  *keep = slot < S.keep_slots;
}

__device__ __forceinline__ void store_row(char* out, size_t row, const u32 (&w)[12]) {
  uint4* d = reinterpret_cast<uint4*>(out + row * 48);
  d[0] = make_uint4(w[0], w[1], w[2], w[3]);
  d[1] = make_uint4(w[4], w[5], w[6], w[7]);
  d[2] = make_uint4(w[8], w[9], w[10], w[11]);
}

// source rank s of G: row p * m + t = message j = s + t * G of owner perm(p)
__global__ void k_source(Shape S, u32 G, u32 s, u32 m, u64 add, char* __restrict__ ts, u32* __restrict__ owner,
                         uint8_t* __restrict__ keep) {
  const size_t n = (size_t)S.O * m;
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    const u64 p = r / m;
    const u32 t = (u32)(r - p * m);
    const u32 o = (u32)((p * PERM_A + add) % S.O);
    u32 w[12];
    bool kp;
    message(S, o, s + t * G, w, &kp);
    store_row(ts, r, w);
    if (owner) owner[r] = o;
    if (keep) keep[r] = kp ? 1 : 0;
  }
}

// all P messages of each listed owner, in the order a rank receives them
// from G sources (source-major: j = s + t * G for s = 0.., t = 0..); owner
// out = the list index
__global__ void k_list(Shape S, u32 G, const u32* __restrict__ list, u32 n_list, char* __restrict__ ts,
                       u32* __restrict__ owner, uint8_t* __restrict__ keep) {
  const size_t n = (size_t)n_list * S.P;
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    const u32 li = (u32)(r / S.P);
    u32 pos = (u32)(r - (size_t)li * S.P);
    // position -> (s, t): source s holds m_s = ceil((P - s) / G) messages
    u32 s = 0;
    for (; s < G; ++s) {
      const u32 ms = (S.P > s) ? (S.P - s + G - 1) / G : 0u;
      if (pos < ms) break;
      pos -= ms;
    }
    u32 w[12];
    bool kp;
    message(S, list[li], s + pos * G, w, &kp);
    store_row(ts, r, w);
    if (owner) owner[r] = li;
    if (keep) keep[r] = kp ? 1 : 0;
  }
}

__global__ void k_owner_ids(u64 seed, u32 n, size_t stride, uint8_t* __restrict__ out) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x) {
    const u64 a = H(seed, 1, o, 0), b = H(seed, 1, o, 1) >> 44;
    uint8_t* d = out + (size_t)o * stride;
    for (int k = 0; k < 16; ++k) {
      const u32 v = (u32)(a >> (60 - 4 * k)) & 15u;
      d[k] = (uint8_t)(v < 10u ? 0x30u + v : 0x57u + v);
    }
    for (int k = 0; k < 5; ++k) {
      const u32 v = (u32)(b >> (16 - 4 * k)) & 15u;
      d[16 + k] = (uint8_t)(v < 10u ? 0x30u + v : 0x57u + v);
    }
    for (size_t k = 21; k < stride; ++k) d[k] = 0;
  }
}

Shape shape(uint64_t seed, uint32_t O, uint32_t P) {
  Shape S;
  S.seed = seed;
  S.O = O;
  S.P = P;
  S.slots = ((P + 3) / 4 + 1) / 2;
  if (S.slots == 0) S.slots = 1;
  S.gap = SPAN / S.slots;
  S.keep_slots = S.slots * 9 / 10;
  return S;
}

int grid(size_t n) {
  size_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 65536) g = 65536;
  return (int)g;
}

u64 gcd(u64 a, u64 b) {
  while (b) {
    const u64 t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// ---------------------------------------------------------------------------
// BASELINE config 5 shape (the server side): n messages, owners Zipf(s) by
// the inverse of `cdf` (host-built, cumulative, O doubles), shuffled, the
// last n / 10 rows exact redeliveries of earlier ones.  Message r (source
// index src = r, or a redelivery's H(9, r, 0) % base):
//   owner o = upper_bound(cdf, u) with u = (H(4, src, 0) >> 11) * 2^-53
//   node    = H(2, o, q), q = H(5, src, 0) & 3 (4 nodes per owner); a node
//             with H(6, o, q) % 100 == 0 spells its hex letters upper-case
//   millis  = T0 + (H(7, src, 0) % slots(o)) * 1000: a 1-second grid of
//             slots(o) = max(1, floor(base * p_o) / 4) -- ~4 messages per slot
//             per owner, so equal millis across nodes are frequent
//   counter = H(8, src, 0) % 1024
//   keep    = H(10, src, 0) % 10 != 0 (the client already holds it)
// ---------------------------------------------------------------------------
struct C5 {
  u64 seed;
  u32 O;
  u64 n, base;
  const double* cdf;
};

__device__ __forceinline__ void c5_message(const C5& S, u64 src, u32 (&w)[12], u32* owner, bool* keep) {
  const double u = (double)(H(S.seed, 4, src, 0) >> 11) * (1.0 / 9007199254740992.0);
  u32 lo = 0, hi = S.O;  // upper_bound
  while (lo < hi) {
    const u32 m = (lo + hi) >> 1;
    if (S.cdf[m] <= u) lo = m + 1;
    else hi = m;
  }
  const u32 o = lo < S.O ? lo : S.O - 1;
  const u32 q = (u32)(H(S.seed, 5, src, 0) & 3u);
  const u64 node = H(S.seed, 2, o, q);
  u32 mask = 0;
  if (H(S.seed, 6, o, q) % 100u == 0u)
    for (int k = 0; k < 16; ++k)
      if (((node >> (60 - 4 * k)) & 15u) >= 10u) mask |= 1u << k;
  const double p = S.cdf[o] - (o ? S.cdf[o - 1] : 0.0);
  u64 slots = (u64)((double)S.base * p) / 4u;
  if (slots < 1) slots = 1;
  const u64 ms = T0 + (H(S.seed, 7, src, 0) % slots) * 1000ull;
  const u32 ctr = (u32)(H(S.seed, 8, src, 0) % 1024u);
  format_ts46((ms << 16) | ctr, node, mask, w);
  *owner = o;
  *keep = H(S.seed, 10, src, 0) % 10u != 0u;
}

__global__ void k_c5(C5 S, char* __restrict__ ts, u32* __restrict__ owner, uint8_t* __restrict__ keep) {
  for (u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x; r < S.n; r += (u64)gridDim.x * blockDim.x) {
    const u64 src = r < S.base ? r : H(S.seed, 9, r, 0) % S.base;
    u32 w[12], o;
    bool kp;
    c5_message(S, src, w, &o, &kp);
    store_row(ts, r, w);
    if (owner) owner[r] = o;
    if (keep) keep[r] = kp ? 1 : 0;
  }
}

}  // namespace

extern "C" {

// BASELINE config 5 shape: n rows of 48 bytes, owner ids, keep flags (see
// above); cdf: device, O cumulative owner probabilities.  0, or -1.
int evs_config5_shape(void* stream, uint64_t seed, uint32_t O, uint64_t n, const double* cdf, char* ts,
                      uint32_t* owner, uint8_t* keep) {
  if (!O || !cdf || (n && !ts)) return -1;
  if (!n) return 0;
  C5 S{seed, O, n, n - n / 10, cdf};
  if (S.base == 0) S.base = n;
  hipLaunchKernelGGL(k_c5, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, S, ts, owner, keep);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"

namespace {
}  // namespace

extern "C" {

// rows of source rank s (of G): O * ceil((P - s) / G) rows of 48 bytes; owner
// = global owner id; keep = the client knows the message.  Returns 0, or -1
// on bad arguments.
int evs_config4_source(void* stream, uint64_t seed, uint32_t O, uint32_t P, uint32_t G, uint32_t s, char* ts,
                       uint32_t* owner, uint8_t* keep) {
  if (!O || !P || !G || s >= G || s >= P || !ts || gcd(PERM_A, O) != 1) return -1;
  const u32 m = (P - s + G - 1) / G;
  const Shape S = shape(seed, O, P);
  hipLaunchKernelGGL(k_source, dim3(grid((size_t)O * m)), dim3(256), 0, (hipStream_t)stream, S, G, s, m, seed % O, ts,
                     owner, keep);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// all P messages of each of n_list owners (global ids, device), source-major
// for G sources; owner = list index
int evs_config4_owners(void* stream, uint64_t seed, uint32_t O, uint32_t P, uint32_t G, const uint32_t* list,
                       uint32_t n_list, char* ts, uint32_t* owner, uint8_t* keep) {
  if (!O || !P || !G || (n_list && (!list || !ts))) return -1;
  if (!n_list) return 0;
  const Shape S = shape(seed, O, P);
  hipLaunchKernelGGL(k_list, dim3(grid((size_t)n_list * P)), dim3(256), 0, (hipStream_t)stream, S, G, list, n_list, ts,
                     owner, keep);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// userId strings of owners 0..n-1 (21 bytes, zero padded to stride >= 21)
int evs_owner_ids(void* stream, uint64_t seed, uint32_t n, size_t stride, uint8_t* out) {
  if (stride < 21 || (n && !out)) return -1;
  if (!n) return 0;
  hipLaunchKernelGGL(k_owner_ids, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, seed, n, stride, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
