// The server's per-request tree JSON (apps/server/src/index.ts:160-163, :240;
// types.ts:80-84 merkleTreeToString = JSON.stringify) for many owners in one
// launch: every owner's text straight from its leaf list, on the device.
//
// JSON.stringify of a trie node is {"0":..,"1":..,"2":..,"hash":h}: integer-
// like keys ascending, then "hash" (evm_json.cpp's host emitter, pinned by
// node).  Over an owner's leaves in code order (= depth-first order) the
// text is a concatenation of one piece per leaf i:
//   opens   the nodes on leaf i's path below its common prefix cp_i with leaf
//           i-1: `"d":{` each, a comma before the first one when leaf i-1
//           went deeper than cp_i (the new node has an elder sibling);
//   closes  the nodes on leaf i's path below its common prefix cn_i with leaf
//           i+1 (all of them after the last leaf), deepest first:
//           `"hash":H}`, with a comma in front unless the node is leaf i's
//           own node (a node closed later than its own leaf has children);
// wrapped in the root's `{` ... `,"hash":R}` (an empty tree: `{}`).  A node's
// hash H is the XOR of its leaves: the owner's prefix XOR after leaf i (the
// node's last leaf) ^ before the node's first leaf, which is the last leaf j
// <= i that opened a node at that depth (cp_j < d).
//
// Work unit: a wave per requested owner, its leaves 64 at a time (a chunk,
// one leaf per lane).  The node starts come from 20 ballots (lane j: cp_j <
// d) -- the last opener at or below a lane -- and, for nodes opened before
// the chunk, from the owner's previous chunks: their last opener per depth,
// carried in LDS.  k_jp_len sums each owner's text; after the caller's scan
// of the lengths k_jp_emit writes each chunk's pieces into LDS and copies
// them out (a chunk too long for the stage writes its bytes directly).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

namespace {

constexpr int JW = 64;                 // leaves per chunk: one wave
constexpr int JW_WAVES = 4;            // waves (chunks) per workgroup
constexpr u32 JW_STAGE = 8 * 1024;     // bytes of a chunk's text staged in LDS (after the destination's offset mod 16)
constexpr u64 CODE_MASK = (1ull << 40) - 1;

struct TreeJ {  // the tree as the kernels read it (gapped or compact: owner o's leaves [off[o], end[o]))
  const u64* off;
  const u64* end;
  const u64* ck;
  const int32_t* pfx;
  u32 n_owners;
};

__device__ __forceinline__ int code_depth(u64 c) {  // digits of a (non-zero) code
  return CODE_DIGITS - (__builtin_ctzll(c) >> 1);
}
__device__ __forceinline__ int code_lcp(u64 a, u64 b) {  // common leading digits
  const u64 x = a ^ b;
  return x ? (__clzll(x) - (64 - 2 * CODE_DIGITS)) >> 1 : CODE_DIGITS;
}
__device__ __forceinline__ u64 code_prefix(u64 c, int d) {  // the first d digits of c
  return d >= CODE_DIGITS ? c : c & ~((1ull << (2 * (CODE_DIGITS - d))) - 1ull);
}
__device__ __forceinline__ u32 dec_len(int32_t v) {  // (compares, not a division loop)
  const u32 x = v < 0 ? 0u - (u32)v : (u32)v;
  return 1u + (x >= 10u) + (x >= 100u) + (x >= 1000u) + (x >= 10000u) + (x >= 100000u) + (x >= 1000000u) +
         (x >= 10000000u) + (x >= 100000000u) + (x >= 1000000000u) + (v < 0 ? 1u : 0u);
}
// the root's tail after the last leaf: `,"hash":R}`
__device__ __forceinline__ u32 root_tail_len(int32_t r) { return 9u + dec_len(r); }

// A wave's chunk: its owner and its leaves' places
struct Chunk {
  u32 j;      // the request (owners[j])
  u32 L;      // the owner's leaves
  u64 a;      // its first leaf's slot
  u32 k;      // chunk number inside the owner
  int32_t p0; // pfx at the owner's first leaf (a compact tree's prefix is global)
  bool in;    // owner in range
};
__device__ __forceinline__ Chunk chunk_of(const TreeJ& t, const u32* owners, const u64* cbase, const u32* cj, u64 c) {
  const u32 lo = cj[c];  // (the request whose chunks hold c: k_jp_chunk_req)
  Chunk ch;
  ch.j = lo;
  const u32 o = owners ? owners[lo] : lo;
  ch.in = o < t.n_owners;
  const u64 a = ch.in ? t.off[o] : 0, b = ch.in ? t.end[o] : 0;
  ch.L = (u32)(b - a);
  ch.a = a;
  ch.k = (u32)(c - cbase[lo]);
  ch.p0 = ch.L ? t.pfx[a] : 0;
  return ch;
}

// Per wave, in LDS: the ballot of openers per depth, the prefix at the start
// of every node open before the chunk, and each lane's prefix before its leaf.
struct WaveLds {
  u64 opener[CODE_DIGITS + 1];
  int32_t carry[CODE_DIGITS + 1];
  int32_t p[JW];
};

// One lane's leaf: its code and neighbours, and (after chunk_setup) what
// its piece needs.
struct Lane {
  bool valid;
  u32 l, i;
  u64 c;
  int D, cp, cn, prevD;
  int32_t pn;  // prefix XOR after the leaf
};

__device__ __forceinline__ Lane chunk_setup(const TreeJ& t, const Chunk& ch, WaveLds* w) {
  Lane ln;
  ln.l = threadIdx.x & (JW - 1);
  ln.i = ch.k * JW + ln.l;
  ln.valid = ln.i < ch.L;
  const u64 base = ch.a;
  ln.c = ln.valid ? (t.ck[base + ln.i] & CODE_MASK) : 0ull;
  const int32_t p = ln.valid ? (t.pfx[base + ln.i] ^ ch.p0) : 0;
  ln.pn = ln.valid ? (t.pfx[base + ln.i + 1] ^ ch.p0) : 0;
  u64 prevc = __shfl_up(ln.c, 1, 64);
  u64 nextc = __shfl_down(ln.c, 1, 64);
  if (ln.l == 0 && ln.i > 0 && ln.valid) prevc = t.ck[base + ln.i - 1] & CODE_MASK;
  if (ln.l == JW - 1 && ln.i + 1 < ch.L) nextc = t.ck[base + ln.i + 1] & CODE_MASK;
  ln.cp = ln.valid && ln.i > 0 ? code_lcp(prevc, ln.c) : 0;
  ln.cn = ln.valid && ln.i + 1 < ch.L ? code_lcp(ln.c, nextc) : 0;
  ln.D = ln.valid ? code_depth(ln.c) : 0;
  ln.prevD = ln.valid && ln.i > 0 ? code_depth(prevc) : 0;
  w->p[ln.l] = p;
#pragma unroll
  for (int d = 1; d <= CODE_DIGITS; ++d) {
    const u64 m = __ballot(ln.valid && ln.cp < d);
    if (ln.l == 0) w->opener[d] = m;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ln;
}

// After a chunk: the start of each depth's node open at its end (its last
// opener at that depth, else the node open before it) for the owner's next chunk.
__device__ __forceinline__ void chunk_carry(WaveLds* w, u32 lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();  // (the chunk's reads of carry first)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < CODE_DIGITS) {
    const u64 m = w->opener[lane + 1];
    if (m) w->carry[lane + 1] = w->p[63 - __clzll(m)];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the prefix before the first leaf of leaf ln's node at depth d
__device__ __forceinline__ int32_t node_start(const WaveLds* w, const Lane& ln, int d) {
  const u64 m = w->opener[d] & (ln.l == 63 ? ~0ull : ((2ull << ln.l) - 1ull));
  return m ? w->p[63 - __clzll(m)] : w->carry[d];
}

// Leaf ln's piece: its length, and (put) its bytes.
template <typename Put>
__device__ __forceinline__ u32 leaf_piece(const WaveLds* w, const Lane& ln, Put put) {
  if (!ln.valid) return 0;
  const u64 c = ln.c;
  const int D = ln.D, cp = ln.cp, cn = ln.cn;
  u32 n = 0;
  if (ln.i && ln.prevD > cp) put(n++, ',');
  for (int k = cp + 1; k <= D; ++k) {
    const u32 dg = (u32)(c >> (2 * (CODE_DIGITS - k))) & 3u;  // digit + 1
    put(n++, '"');
    put(n++, (char)('0' + dg - 1));
    put(n++, '"');
    put(n++, ':');
    put(n++, '{');
  }
  for (int d = D; d > cn; --d) {
    const int32_t h = ln.pn ^ node_start(w, ln, d);
    if (d < D) put(n++, ',');
    put(n++, '"');
    put(n++, 'h');
    put(n++, 'a');
    put(n++, 's');
    put(n++, 'h');
    put(n++, '"');
    put(n++, ':');
    const u32 len = dec_len(h);
    u32 x = h < 0 ? 0u - (u32)h : (u32)h;
    for (u32 k = len; k-- > (h < 0 ? 1u : 0u);) {
      put(n + k, (char)('0' + x % 10u));
      x /= 10u;
    }
    if (h < 0) put(n, '-');
    n += len;
    put(n++, '}');
  }
  return n;
}

// n (<= 8) bytes of v (the first in the low byte) at p in LDS, written in
// at most three stores of exactly those bytes (LDS takes unaligned 2-, 4- and
// 8-byte accesses; a neighbour lane's bytes next to them are not touched)
typedef uint64_t __attribute__((aligned(1))) lu64;
typedef uint32_t __attribute__((aligned(1))) lu32;
typedef uint16_t __attribute__((aligned(1))) lu16;
__device__ __forceinline__ void lds_put(unsigned char* p, u64 v, u32 n) {
  if (n == 8) {
    *reinterpret_cast<lu64*>(p) = v;
    return;
  }
  if (n & 4) {
    *reinterpret_cast<lu32*>(p) = (u32)v;
    p += 4;
    v >>= 32;
  }
  if (n & 2) {
    *reinterpret_cast<lu16*>(p) = (uint16_t)v;
    p += 2;
    v >>= 16;
  }
  if (n & 1) *p = (unsigned char)v;
}
// the last n (1..8) decimal digits of v < 10^8, the first in the low byte:
// four 2-digit pairs from two divisions by 10^4 and 10^2 (no digit loop)
__device__ __forceinline__ u64 dec_chars(u32 v, u32 n) {
  const u32 hi = v / 10000u, lo = v - hi * 10000u;
  const u32 h1 = hi / 100u, h2 = hi - h1 * 100u, l1 = lo / 100u, l2 = lo - l1 * 100u;
  auto two = [](u32 d) -> u64 {
    const u32 t = d / 10u;
    return (u64)((t | ((d - t * 10u) << 8)) + 0x3030u);
  };
  const u64 s = two(h1) | two(h2) << 16 | two(l1) << 32 | two(l2) << 48;
  return s >> (8 * (8 - n));
}

// leaf_piece's bytes into the LDS stage at p, a few bytes per store
__device__ __forceinline__ void leaf_piece_wide(const WaveLds* w, const Lane& ln, unsigned char* p) {
  if (!ln.valid) return;
  const u64 c = ln.c;
  const int D = ln.D, cp = ln.cp, cn = ln.cn;
  if (ln.i && ln.prevD > cp) *p++ = ',';
  for (int k = cp + 1; k <= D; ++k) {
    const u32 dg = (u32)(c >> (2 * (CODE_DIGITS - k))) & 3u;  // digit + 1
    lds_put(p, 0x7B3A220022ull | (u64)('0' + dg - 1) << 8, 5);  // `"d":{`
    p += 5;
  }
  for (int d = D; d > cn; --d) {
    const int32_t h = ln.pn ^ node_start(w, ln, d);
    if (d < D) {
      lds_put(p, 0x3A2268736168222Cull, 8);  // `,"hash":`
      p += 8;
    } else {
      lds_put(p, 0x3A22687361682200ull >> 8, 7);  // `"hash":`
      p += 7;
    }
    const u32 x = h < 0 ? 0u - (u32)h : (u32)h;
    if (h < 0) *p++ = '-';
    if (x >= 100000000u) {
      const u32 hi = x / 100000000u, lo = x - hi * 100000000u, nh = hi >= 10u ? 2u : 1u;
      lds_put(p, dec_chars(hi, nh), nh);
      p += nh;
      lds_put(p, dec_chars(lo, 8u), 8);
      p += 8;
      *p++ = '}';
    } else {
      const u32 nd = dec_len((int32_t)x);
      const u64 ds = dec_chars(x, nd);
      if (nd < 8) {
        lds_put(p, ds | (u64)'}' << (8 * nd), nd + 1);
      } else {
        lds_put(p, ds, 8);
        p[8] = '}';
      }
      p += nd + 1;
    }
  }
}

__device__ __forceinline__ u32 wave_excl_sum(u32 v, u32* total) {
  u32 x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = __shfl_up(x, d, 64);
    if ((int)(threadIdx.x & 63) >= d) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

// A wave per requested owner, its chunks in order (the node starts carried
// from chunk to chunk in LDS).  k_jp_len: each owner's text length (an empty
// or out-of-range owner: `{}`, the latter flagged in *bad).
__global__ __launch_bounds__(JW * JW_WAVES) void k_jp_len(TreeJ t, const u32* __restrict__ owners, u32 n,
                                                          u64* __restrict__ len, u32* __restrict__ bad,
                                                          uint16_t* __restrict__ plen) {
  __shared__ WaveLds lds[JW_WAVES];
  WaveLds* w = &lds[threadIdx.x / JW];
  const u32 lane = threadIdx.x & 63;
  for (u32 j = blockIdx.x * JW_WAVES + threadIdx.x / JW; j < n; j += gridDim.x * JW_WAVES) {
    const u32 o = owners ? owners[j] : j;
    if (o >= t.n_owners && lane == 0) atomicOr(bad, 1u);
    const u64 a = o < t.n_owners ? t.off[o] : 0;
    const u32 L = o < t.n_owners ? (u32)(t.end[o] - a) : 0u;
    if (L == 0) {
      if (lane == 0) len[j] = 2;
      continue;
    }
    const int32_t p0 = t.pfx[a];
    u64 total = 1;
    for (u32 k = 0; (u64)k * JW < L; ++k) {
      const Chunk ch{j, L, a, k, p0, true};
      const Lane ln = chunk_setup(t, ch, w);
      u32 tot;
      const u32 my = leaf_piece(w, ln, [](u32, char) {});
      if (plen && ln.valid) plen[ch.a + ln.i] = (uint16_t)my;  // (k_jp_emit reads it: no second length pass)
      wave_excl_sum(my, &tot);
      total += tot;
      chunk_carry(w, lane);
    }
    if (lane == 0) len[j] = total + root_tail_len(t.pfx[a + L] ^ p0);
  }
}

// k_jp_emit: owner j's text at out + off[j], a chunk at a time (staged in LDS)
__global__ __launch_bounds__(JW * JW_WAVES) void k_jp_emit(TreeJ t, const u32* __restrict__ owners, u32 n,
                                                           const u64* __restrict__ off, char* __restrict__ out,
                                                           const uint16_t* __restrict__ plen) {
  __shared__ WaveLds lds[JW_WAVES];
  __shared__ __attribute__((aligned(16))) unsigned char stage[JW_WAVES][JW_STAGE + 16];
  const u32 wv = threadIdx.x / JW, lane = threadIdx.x & 63;
  WaveLds* w = &lds[wv];
  unsigned char* sg = stage[wv];
  for (u32 j = blockIdx.x * JW_WAVES + wv; j < n; j += gridDim.x * JW_WAVES) {
    const u32 o = owners ? owners[j] : j;
    const u64 a = o < t.n_owners ? t.off[o] : 0;
    const u32 L = o < t.n_owners ? (u32)(t.end[o] - a) : 0u;
    char* dst0 = out + off[j];
    if (L == 0) {
      if (lane == 0) {
        dst0[0] = '{';
        dst0[1] = '}';
      }
      continue;
    }
    const int32_t p0 = t.pfx[a];
    u64 run = 0;  // the owner's bytes written
    for (u32 k = 0; (u64)k * JW < L; ++k) {
      const Chunk ch{j, L, a, k, p0, true};
      char* dst = dst0 + run;
      const Lane ln = chunk_setup(t, ch, w);
      const u32 my = plen ? (ln.valid ? (u32)plen[ch.a + ln.i] : 0u) : leaf_piece(w, ln, [](u32, char) {});
      u32 tot;
      const u32 head = ch.k == 0 ? 1u : 0u;
      const u32 pos = head + wave_excl_sum(my, &tot);
      const bool last = (u64)(ch.k + 1) * JW >= ch.L;
      const int32_t R = last ? (t.pfx[ch.a + ch.L] ^ ch.p0) : 0;
      const u32 total = head + tot + (last ? root_tail_len(R) : 0u);
      auto tail = [&](auto put) {  // `,"hash":R}` at head + tot
        const char* h = ",\"hash\":";
        u32 q = head + tot;
        for (int k = 0; k < 8; ++k) put(q + k, h[k]);
        const u32 len = dec_len(R);
        u32 x = R < 0 ? 0u - (u32)R : (u32)R;
        for (u32 k = len; k-- > (R < 0 ? 1u : 0u);) {
          put(q + 8 + k, (char)('0' + x % 10u));
          x /= 10u;
        }
        if (R < 0) put(q + 8, '-');
        put(q + 8 + len, '}');
      };
      if (total <= JW_STAGE) {
        // staged at the destination's offset mod 16: the copy out is whole 16-B
        // LDS reads and stores between the ends
        const u32 s0 = (u32)((uintptr_t)dst & 15u);
        unsigned char* sgo = sg + s0;
        leaf_piece_wide(w, ln, sgo + pos);  // (a byte per store: encode 9.3 -> 8.8 ms on config 3's round)
        if (lane == 0) {
          if (head) sgo[0] = '{';
          if (last) tail([&](u32 k, char b) { sgo[k] = (unsigned char)b; });
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        char* d16 = dst - s0;  // 16-B aligned
        const u32 end = s0 + total;
        const u32 first = std::min<u32>(end, 16u);  // bytes [s0, first) of the first 16
        if (lane >= s0 && lane < first) d16[lane] = (char)sg[lane];
        const u32 full = end >> 4;  // 16-B blocks [1, full) whole; the last block's bytes below `end`
        for (u32 q = 1 + lane; q < full; q += JW)
          reinterpret_cast<uint4*>(d16)[q] = reinterpret_cast<const uint4*>(sg)[q];
        const u32 t0 = std::max<u32>(16u, full << 4);
        if (t0 + lane < end) d16[t0 + lane] = (char)sg[t0 + lane];
      } else {  // (a chunk of very deep, sparse leaves: its bytes straight out)
        leaf_piece(w, ln, [&](u32 k, char b) { dst[pos + k] = b; });
        if (lane == 0) {
          if (head) dst[0] = '{';
          if (last) tail([&](u32 k, char b) { dst[k] = b; });
        }
      }
      run += total;
      chunk_carry(w, lane);  // (also: the stage is rewritten by the next chunk)
    }
  }
}

}  // namespace

// The plan (chunks, their places, each owner's text length) and the emit, for
// a caller that places the texts itself (the device SyncResponse encoder:
// each text straight into its response).  The plan's arrays live in S.
int evm::json_plan(evm_ctx* ctx, Scratch& S, const evm_tree* t, const uint32_t* owners, uint32_t n, uint64_t* len,
                   uint32_t* bad, JsonPlan* plan) {
  const TreeJ tv{t->off, t->end, t->ck, t->pfx, t->n_owners};
  const u32 grid = (u32)std::min<u64>((n + JW_WAVES - 1) / JW_WAVES, (u64)ctx->n_cu * 32);
  // each leaf's piece length, by leaf slot, for the emit
  plan->plen = S.alloc<uint16_t>((size_t)(t->gapped ? t->cap : t->n_leaves) + 1);
  if (!plan->plen) return EVM_ENOMEM;
  if (n)
    KLAUNCH(k_jp_len, dim3(std::max<u32>(grid, 1)), dim3(JW * JW_WAVES), tv, owners, n, (u64*)len, bad, plan->plen);
  plan->n = n;
  return hip_ok(hipGetLastError());
}
int evm::json_emit(evm_ctx* ctx, const evm_tree* t, const uint32_t* owners, uint32_t n, const JsonPlan& plan,
                   const uint64_t* off, char* out) {
  const TreeJ tv{t->off, t->end, t->ck, t->pfx, t->n_owners};
  const u32 grid = (u32)std::min<u64>((n + JW_WAVES - 1) / JW_WAVES, (u64)ctx->n_cu * 32);
  if (n)
    KLAUNCH(k_jp_emit, dim3(std::max<u32>(grid, 1)), dim3(JW * JW_WAVES), tv, owners, n, (const u64*)off, out,
            (const uint16_t*)plan.plen);
  return hip_ok(hipGetLastError());
}

extern "C" int evm_tree_to_json_batch(evm_ctx* ctx, const evm_tree* t, const uint32_t* owners, uint32_t n, char* out,
                                      size_t cap, uint64_t* off, uint64_t* total) {
  if (!ctx || !t || !off || !total || (n && !owners && n > t->n_owners)) return EVM_EINVAL;
  *total = 0;
  Scratch S(ctx);
  u64* len = S.alloc<u64>((size_t)n + 1);
  u32* bad = S.alloc<u32>(1);
  if (!len || !bad) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  JsonPlan plan;
  int st = json_plan(ctx, S, t, owners, n, reinterpret_cast<uint64_t*>(len), bad, &plan);
  if (st) return st;
  u64* doff = reinterpret_cast<u64*>(off);
  if ((st = scan_exclusive<u64, OpAdd>(ctx, S, len, n, doff, doff + n))) return st;
  u64 h = 0;
  u32 hb = 0;
  {
    LandList l;
    l.add(doff + n, &h, sizeof(u64));
    l.add(bad, &hb, sizeof(u32));
    if ((st = land_words(ctx, l))) return st;
  }
  if (hb) return EVM_EINVAL;
  *total = h;
  if (!out) return EVM_OK;
  if (h > cap) return EVM_ECAPACITY;
  return json_emit(ctx, t, owners, n, plan, off, out);
}
