// The server's per-request tree JSON (apps/server/src/index.ts:160-163, :240;
// types.ts:80-84 merkleTreeToString = JSON.stringify) for many owners in one
// launch: every owner's text straight from its leaf list, on the device.
//
// JSON.stringify of a trie node is {"0":..,"1":..,"2":..,"hash":h}: integer-
// like keys ascending, then "hash" (evm_json.cpp's host emitter, pinned by
// node).  Over an owner's leaves in code order (= depth-first order) the
// text is a concatenation of one piece per leaf i:
//   opens   the nodes on leaf i's path below its common prefix c_i with leaf
//           i-1: `"d":{` each, a comma before the first one when leaf i-1
//           went deeper than c_i (the new node has an elder sibling);
//   closes  the nodes on leaf i's path below its common prefix with leaf i+1
//           (all of them after the last leaf), deepest first: `"hash":H}`,
//           with a comma in front unless the node is leaf i's own node (a
//           node closed later than its own leaf has children);
// wrapped in the root's `{` ... `,"hash":R}` (an empty tree: `{}`).  A node's
// hash H is the XOR of its leaves: the owner's prefix XOR at leaf i + 1 (the
// node's last leaf is i) ^ at its first leaf (a lower bound of its code
// prefix among leaves 0..i).
//
// Two passes, each a workgroup per owner over chunks of 256 leaves (one per
// thread): k_json_len sums the pieces' lengths; after a scan of the owners'
// lengths k_json_emit writes each chunk's pieces into LDS and copies them
// out coalesced (a chunk too long for the stage writes its bytes directly).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

namespace {

constexpr int JT = 256;            // threads per owner (one leaf each per chunk)
constexpr u32 JCAP = 2048;         // an owner's leaves staged in LDS (more: read from global memory)
constexpr u32 JSTAGE = 24 * 1024;  // bytes of a chunk's text staged in LDS
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
__device__ __forceinline__ u32 dec_len(int32_t v) {
  u32 x = v < 0 ? 0u - (u32)v : (u32)v;
  u32 n = 1;
  while (x >= 10u) {
    x /= 10u;
    ++n;
  }
  return n + (v < 0 ? 1u : 0u);
}

// An owner's leaves: codes (without the owner bits) and the owner-local
// exclusive prefix XOR, from LDS when staged there, else from the tree.
struct Leaves {
  const u64* g_ck;
  const int32_t* g_pfx;
  u64 base;
  int32_t p0;  // pfx at the owner's first leaf (a compact tree's prefix is global)
  const u64* s_ck;
  const int32_t* s_pfx;
  __device__ __forceinline__ u64 code(u32 i) const { return s_ck ? s_ck[i] : (g_ck[base + i] & CODE_MASK); }
  __device__ __forceinline__ int32_t pfx(u32 i) const { return s_pfx ? s_pfx[i] : (g_pfx[base + i] ^ p0); }
  __device__ __forceinline__ u32 lower(u32 hi, u64 x) const {  // first k < hi with code(k) >= x
    u32 lo = 0;
    while (lo < hi) {
      const u32 mid = (lo + hi) >> 1;
      if (code(mid) < x) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
};

// Leaf i's piece: its length, and (out != null) its bytes.
template <typename Put>
__device__ __forceinline__ u32 leaf_piece(const Leaves& lv, u32 i, u32 L, Put put) {
  const u64 c = lv.code(i);
  const int D = code_depth(c);
  const int cp = i ? code_lcp(lv.code(i - 1), c) : 0;
  const int cn = i + 1 < L ? code_lcp(c, lv.code(i + 1)) : 0;
  u32 n = 0;
  if (i && code_depth(lv.code(i - 1)) > cp) put(n++, ',');
  for (int k = cp + 1; k <= D; ++k) {
    const u32 dg = (u32)(c >> (2 * (CODE_DIGITS - k))) & 3u;  // digit + 1
    put(n++, '"');
    put(n++, (char)('0' + dg - 1));
    put(n++, '"');
    put(n++, ':');
    put(n++, '{');
  }
  const int32_t after = lv.pfx(i + 1);
  u32 lo = i + 1;
  for (int d = D; d > cn; --d) {
    lo = lv.lower(lo, code_prefix(c, d));  // (shallower nodes start no later)
    const int32_t h = after ^ lv.pfx(lo);
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

// the root's tail after the last leaf: `,"hash":R}`
__device__ __forceinline__ u32 root_tail_len(int32_t r) { return 9u + dec_len(r); }

__device__ __forceinline__ Leaves stage_leaves(const TreeJ& t, u32 o, u32* L_out, u64* s_ck, int32_t* s_pfx) {
  const bool in = o < t.n_owners;  // (an owner out of range: reported by k_json_len, emitted as {})
  const u64 a = in ? t.off[o] : 0, b = in ? t.end[o] : 0;
  const u32 L = (u32)(b - a);
  *L_out = L;
  Leaves lv{t.ck, t.pfx, a, L ? t.pfx[a] : 0, nullptr, nullptr};
  if (L <= JCAP) {
    for (u32 i = threadIdx.x; i <= L; i += JT) {
      if (i < L) s_ck[i] = t.ck[a + i] & CODE_MASK;
      s_pfx[i] = t.pfx[a + i] ^ lv.p0;
    }
    __syncthreads();
    lv.s_ck = s_ck;
    lv.s_pfx = s_pfx;
  }
  return lv;
}

__global__ __launch_bounds__(JT) void k_json_len(TreeJ t, const u32* __restrict__ owners, u32 n,
                                                 u64* __restrict__ len, u32* __restrict__ bad) {
  __shared__ u64 s_ck[JCAP];
  __shared__ int32_t s_pfx[JCAP + 1];
  __shared__ u32 tmp[JT / 64 + 1];
  for (u32 j = blockIdx.x; j < n; j += gridDim.x) {
    const u32 o = owners ? owners[j] : j;
    if (o >= t.n_owners && threadIdx.x == 0) atomicOr(bad, 1u);
    u32 L;
    const Leaves lv = stage_leaves(t, o, &L, s_ck, s_pfx);
    u32 sum = 0;
    for (u32 i = threadIdx.x; i < L; i += JT) sum += leaf_piece(lv, i, L, [](u32, char) {});
    u32 tot;
    block_inclusive_scan<u32>(sum, tmp, OpAdd<u32>(), &tot);
    if (threadIdx.x == 0) len[j] = L ? 1u + tot + root_tail_len(lv.pfx(L)) : 2u;
    __syncthreads();  // (the staged leaves of the next owner)
  }
}

__global__ __launch_bounds__(JT) void k_json_emit(TreeJ t, const u32* __restrict__ owners, u32 n,
                                                  const u64* __restrict__ off, char* __restrict__ out) {
  __shared__ u64 s_ck[JCAP];
  __shared__ int32_t s_pfx[JCAP + 1];
  __shared__ u32 tmp[JT / 64 + 1];
  __shared__ unsigned char stage[JSTAGE];
  for (u32 j = blockIdx.x; j < n; j += gridDim.x) {
    const u32 o = owners ? owners[j] : j;
    u32 L;
    const Leaves lv = stage_leaves(t, o, &L, s_ck, s_pfx);
    char* dst = out + off[j];
    if (L == 0) {
      if (threadIdx.x == 0) {
        dst[0] = '{';
        dst[1] = '}';
      }
      __syncthreads();
      continue;
    }
    if (threadIdx.x == 0) dst[0] = '{';
    u64 at = 1;  // bytes of the owner's text written so far
    for (u32 i0 = 0; i0 < L; i0 += JT) {
      const u32 i = i0 + threadIdx.x;
      const u32 my = i < L ? leaf_piece(lv, i, L, [](u32, char) {}) : 0u;
      u32 tot;
      const u32 pos = block_inclusive_scan<u32>(my, tmp, OpAdd<u32>(), &tot) - my;
      if (tot <= JSTAGE) {
        if (i < L) leaf_piece(lv, i, L, [&](u32 k, char ch) { stage[pos + k] = (unsigned char)ch; });
        __syncthreads();
        // copy out: 4-B stores from the first 4-B aligned byte, single bytes at the ends
        char* d = dst + at;
        const u32 head = std::min<u32>(tot, (u32)((4u - ((uintptr_t)d & 3u)) & 3u));
        if (threadIdx.x < head) d[threadIdx.x] = (char)stage[threadIdx.x];
        const u32 words = (tot - head) >> 2;
        u32* dw = reinterpret_cast<u32*>(d + head);
        for (u32 w = threadIdx.x; w < words; w += JT) {
          const u32 b = head + 4u * w;
          dw[w] = (u32)stage[b] | ((u32)stage[b + 1] << 8) | ((u32)stage[b + 2] << 16) | ((u32)stage[b + 3] << 24);
        }
        const u32 tail = head + 4u * words;
        if (threadIdx.x < tot - tail) d[tail + threadIdx.x] = (char)stage[tail + threadIdx.x];
        __syncthreads();  // (the stage is reused by the next chunk)
      } else if (i < L) {  // (a chunk of very deep, sparse leaves: its bytes straight out)
        char* d = dst + at + pos;
        leaf_piece(lv, i, L, [&](u32 k, char ch) { d[k] = ch; });
      }
      at += tot;
    }
    if (threadIdx.x == 0) {  // the root: `,"hash":R}`
      const int32_t r = lv.pfx(L);
      char* d = dst + at;
      const char* h = ",\"hash\":";
      for (int k = 0; k < 8; ++k) d[k] = h[k];
      const u32 len = dec_len(r);
      u32 x = r < 0 ? 0u - (u32)r : (u32)r;
      for (u32 k = len; k-- > (r < 0 ? 1u : 0u);) {
        d[8 + k] = (char)('0' + x % 10u);
        x /= 10u;
      }
      if (r < 0) d[8] = '-';
      d[8 + len] = '}';
    }
    __syncthreads();  // (the staged leaves of the next owner)
  }
}

}  // namespace

// the two passes for a caller that places the texts itself (the device
// SyncResponse encoder: each text straight into its response)
int evm::json_lengths(evm_ctx* ctx, const evm_tree* t, const uint32_t* owners, uint32_t n, uint64_t* len, uint32_t* bad) {
  const TreeJ tv{t->off, t->end, t->ck, t->pfx, t->n_owners};
  const u32 grid = (u32)std::min<size_t>(std::max<u32>(n, 1), (size_t)ctx->n_cu * 8);
  if (n) KLAUNCH(k_json_len, dim3(grid), dim3(JT), tv, owners, n, (u64*)len, bad);
  return hip_ok(hipGetLastError());
}
int evm::json_emit(evm_ctx* ctx, const evm_tree* t, const uint32_t* owners, uint32_t n, const uint64_t* off, char* out) {
  const TreeJ tv{t->off, t->end, t->ck, t->pfx, t->n_owners};
  const u32 grid = (u32)std::min<size_t>(std::max<u32>(n, 1), (size_t)ctx->n_cu * 8);
  if (n) KLAUNCH(k_json_emit, dim3(grid), dim3(JT), tv, owners, n, (const u64*)off, out);
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
  const TreeJ tv{t->off, t->end, t->ck, t->pfx, t->n_owners};
  const u32 grid = (u32)std::min<size_t>(std::max<u32>(n, 1), (size_t)ctx->n_cu * 8);
  if (n) KLAUNCH(k_json_len, dim3(grid), dim3(JT), tv, owners, n, len, bad);
  u64* doff = reinterpret_cast<u64*>(off);
  int st = scan_exclusive<u64, OpAdd>(ctx, S, len, n, doff, doff + n);
  if (st) return st;
  u64 h = 0;
  u32 hb = 0;
  HIPR(hipMemcpyAsync(&h, doff + n, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(&hb, bad, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (hb) return EVM_EINVAL;
  *total = h;
  if (!out) return EVM_OK;
  if (h > cap) return EVM_ECAPACITY;
  if (n) KLAUNCH(k_json_emit, dim3(grid), dim3(JT), tv, owners, n, (const u64*)doff, out);
  return hip_ok(hipGetLastError());
}
