// The sync server's wire work on the device: a round's SyncRequest bodies
// decoded where they lie in HBM, their client trees parsed, and the
// SyncResponse bodies built in HBM (apps/server/src/index.ts:112-116
// parseBody = SyncRequest.fromBinary, :121-136 merkleTreeFromString of the
// request's tree, :233-241 SyncResponse.toBinary with merkleTreeToString).
//
// Same grammar, same results as the host codecs (evm_proto.cpp's Reader /
// walk / read_msg, evm_json.cpp's Parser, evm_pb_encode_responses): one
// thread per body or tree runs the same sequential walk, so the accept /
// reject decisions are the host's by construction -- the tests compare the
// two byte for byte.  A tree the device reads in an order the leaf list
// cannot hold without a sort (children keys not ascending: JSON.stringify
// never writes that, a hand-made client might) is reported per owner
// (EVM_TREE_UNSORTED) and left to the host parser.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <functional>
#include <type_traits>
#include <vector>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

namespace {

// ------------------------------------------------------------------ protobuf
// Sequential reads of device bytes through a 64-B register window: one
// refill (four independent 16-B loads) per 64 bytes walked instead of one
// dependent load per byte.  A refill loads only the 16-B chunks below
// `lim` (the chunk boundary after the last byte of the buffer): the callers'
// buffers are readable in whole 16-B chunks (evm.h).
struct Win {
  const uint8_t* w;    // window start (16-B aligned)
  const uint8_t* lim;  // loads stay below this (16-B aligned)
  uint4 v0, v1, v2, v3;
  __device__ __forceinline__ void init(const uint8_t* end) {
    lim = reinterpret_cast<const uint8_t*>(((uintptr_t)end + 15) & ~(uintptr_t)15);
    w = nullptr;
  }
  __device__ __forceinline__ uint4 chunk(const uint8_t* c) const {
    return c < lim ? *reinterpret_cast<const uint4*>(c) : make_uint4(0, 0, 0, 0);
  }
  __device__ __forceinline__ void refill(const uint8_t* p) {
    w = reinterpret_cast<const uint8_t*>((uintptr_t)p & ~(uintptr_t)15);
    v0 = chunk(w);
    v1 = chunk(w + 16);
    v2 = chunk(w + 32);
    v3 = chunk(w + 48);
  }
  // (selects of values: a select of the members' addresses would keep the
  // window in scratch memory)
  static __device__ __forceinline__ u32 pick(u32 j, u32 a, u32 b, u32 c, u32 d) {
    const u32 lo = (j & 1u) ? b : a, hi = (j & 1u) ? d : c;
    return (j & 2u) ? hi : lo;
  }
  __device__ __forceinline__ u32 word(u32 i) const {  // i < 16
    return pick(i >> 2, pick(i & 3u, v0.x, v0.y, v0.z, v0.w), pick(i & 3u, v1.x, v1.y, v1.z, v1.w),
                pick(i & 3u, v2.x, v2.y, v2.z, v2.w), pick(i & 3u, v3.x, v3.y, v3.z, v3.w));
  }
  // bytes p .. p + 7, little-endian (past the buffer: whatever the chunk holds, or 0)
  __device__ __forceinline__ u64 get8(const uint8_t* p) {
    if (p < w || p + 8 > w + 64) refill(p);
    const u32 k = (u32)(p - w), j = k >> 2, sh = (k & 3u) * 8u;
    const u32 a = word(j), b = word(j + 1), c = word(min(j + 2, 15u));
    const u32 lo = sh ? (a >> sh) | (b << (32u - sh)) : a;
    const u32 hi = sh ? (b >> sh) | (c << (32u - sh)) : b;
    return ((u64)hi << 32) | lo;
  }
  __device__ __forceinline__ uint8_t get(const uint8_t* p) {
    if (p < w || p >= w + 64) refill(p);
    const u32 k = (u32)(p - w);
    const u32 j = (k >> 2) & 3u, c = k >> 4;
    const u32 word = pick(c, pick(j, v0.x, v0.y, v0.z, v0.w), pick(j, v1.x, v1.y, v1.z, v1.w),
                          pick(j, v2.x, v2.y, v2.z, v2.w), pick(j, v3.x, v3.y, v3.z, v3.w));
    return (uint8_t)(word >> ((k & 3u) * 8u));
  }
};

// The same reads through a window in LDS: NC 16-B chunks per lane (a refill
// issues NC independent loads -- a long walk takes a few messages per
// refill; the per-lane windows 4*65*.. bytes apart so a wave's reads spread
// over the banks).  The window lives at lds[lane * LW_STRIDE ..].
// (12 chunks, a 192-B window: config 3's scan 3.3 ms; 8: 3.7, 10: 3.6, 14: 3.4,
// 16: 4.1-4.3, 24: 8.0, 32: 31.6 -- same box, alternating builds)
#ifndef EVM_LW_NC
#define EVM_LW_NC 12
#endif
constexpr int LW_NC = EVM_LW_NC;
constexpr u32 LW_STRIDE = LW_NC * 4 + 1;  // dwords per lane
struct LWin {
  u32* lds;
  const uint8_t* w;
  const uint8_t* lim;
  __device__ __forceinline__ void init(const uint8_t* end, u32* mine) {
    lim = reinterpret_cast<const uint8_t*>(((uintptr_t)end + 15) & ~(uintptr_t)15);
    w = nullptr;
    lds = mine;
  }
  __device__ __forceinline__ void refill(const uint8_t* p) {
    w = reinterpret_cast<const uint8_t*>((uintptr_t)p & ~(uintptr_t)15);
    uint4 v[LW_NC];
#pragma unroll
    for (int c = 0; c < LW_NC; ++c)
      v[c] = w + 16 * c < lim ? *reinterpret_cast<const uint4*>(w + 16 * c) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int c = 0; c < LW_NC; ++c) {
      lds[4 * c] = v[c].x;
      lds[4 * c + 1] = v[c].y;
      lds[4 * c + 2] = v[c].z;
      lds[4 * c + 3] = v[c].w;
    }
  }
  __device__ __forceinline__ uint8_t get(const uint8_t* p) {
    if (p < w || p >= w + 16 * LW_NC) refill(p);
    const u32 k = (u32)(p - w);
    return (uint8_t)(lds[k >> 2] >> ((k & 3u) * 8u));
  }
};

// evm_proto.cpp's Reader on device bytes (the same checks, in the same order)
template <class W>
struct DReaderT {
  const uint8_t* p;
  const uint8_t* e;
  bool ok;
  W* win;
  __device__ __forceinline__ bool more() const { return ok && p < e; }
  __device__ __forceinline__ u64 varint() {
    u64 v = 0;
    for (int sh = 0; sh < 70; sh += 7) {
      if (p >= e) {
        ok = false;
        return 0;
      }
      const uint8_t b = win->get(p++);
      if (sh == 63 && b > 1) {
        ok = false;
        return 0;
      }
      v |= (u64)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  __device__ __forceinline__ bool bytes(const uint8_t** q, u64* n) {
    const u64 len = varint();
    if (!ok || len > (u64)(e - p)) return ok = false;
    *q = p;
    *n = len;
    p += len;
    return true;
  }
  __device__ __forceinline__ bool skip(u32 wt) {
    switch (wt) {
      case 0:
        varint();
        return ok;
      case 1:
        if (e - p < 8) return ok = false;
        p += 8;
        return true;
      case 2: {
        const uint8_t* q;
        u64 n;
        return bytes(&q, &n);
      }
      case 5:
        if (e - p < 4) return ok = false;
        p += 4;
        return true;
      default:
        return ok = false;
    }
  }
};

using DReader = DReaderT<Win>;

struct DMsg {
  const uint8_t* ts;
  u64 ts_len;
  const uint8_t* content;
  u64 content_len;
};

template <class W>
__device__ __forceinline__ bool d_read_msg(const uint8_t* q, u64 n, DMsg* m, W* win) {
  DReaderT<W> r{q, q + n, true, win};
  *m = DMsg{nullptr, 0, nullptr, 0};
  while (r.more()) {
    const u64 tag = r.varint();
    if (!r.ok) return false;
    const u32 field = (u32)(tag >> 3), wt = (u32)(tag & 7);
    if (field == 1 || field == 2) {
      if (wt != 2) return false;
      if (field == 1) r.bytes(&m->ts, &m->ts_len);
      else r.bytes(&m->content, &m->content_len);
    } else if (field == 0 || !r.skip(wt)) {
      return false;
    }
  }
  return r.ok;
}

// One top-level field of a body at r.p (the loop body of evm_proto.cpp's
// walk()): EVM_OK or EVM_EINVAL; on_msg(index, msg, its field's tag) per message
template <class W, typename F>
__device__ __forceinline__ int d_field(int kind, DReaderT<W>& r, const uint8_t* buf, evm_pb_sync& s, F on_msg) {
  const u32 tree_field = kind == EVM_PB_SYNC_REQUEST ? 4u : 2u;
  const uint8_t* at = r.p;
  const u64 tag = r.varint();
  if (!r.ok) return EVM_EINVAL;
  const u32 field = (u32)(tag >> 3), wt = (u32)(tag & 7);
  if (field == 0) return EVM_EINVAL;
  const bool is_str = field == 1 || field == tree_field || (kind == EVM_PB_SYNC_REQUEST && (field == 2 || field == 3));
  if (!is_str) return r.skip(wt) ? EVM_OK : EVM_EINVAL;
  if (wt != 2) return EVM_EINVAL;
  const uint8_t* q;
  u64 n;
  if (!r.bytes(&q, &n)) return EVM_EINVAL;
  const u64 off = (u64)(q - buf);
  if (field == 1) {
    DMsg m;
    if (!d_read_msg(q, n, &m, r.win)) return EVM_EINVAL;
    if (m.ts_len != 46) ++s.nonstd_ts;
    s.content_bytes += m.content_len;
    on_msg(s.n_messages, m, at);
    ++s.n_messages;
  } else if (field == tree_field) {
    s.tree_off = off;
    s.tree_len = n;
  } else if (field == 2) {
    s.user_off = off;
    s.user_len = n;
  } else {
    s.node_off = off;
    s.node_len = n;
  }
  return EVM_OK;
}

// evm_proto.cpp's walk() over a whole body
template <class W, typename F>
__device__ __forceinline__ int d_walk(int kind, const uint8_t* buf, u64 len, evm_pb_sync* info, W* win, F on_msg) {
  DReaderT<W> r{buf, buf + len, true, win};
  evm_pb_sync s{0, 0, 0, 0, 0, 0, 0, 0, 0};
  while (r.more())
    if (d_field(kind, r, buf, s, on_msg)) return EVM_EINVAL;
  if (!r.ok) return EVM_EINVAL;
  if (info) *info = s;
  return EVM_OK;
}

// (slots: where each message's field starts, body k's i-th at slots[a / 50 + i]
// -- a message with a 46-byte timestamp takes >= 50 bytes, so the bodies'
// ranges [a / 50, b / 50) do not overlap; a body with a shorter message may
// not have room for every one: its nonstd_ts count is nonzero)
constexpr u64 PB_MIN_MSG = 50;
__global__ void k_pb_scan(int kind, const uint8_t* __restrict__ arena, const u64* __restrict__ off, u32 n,
                          evm_pb_sync* __restrict__ info, int32_t* __restrict__ status, u64* __restrict__ slots) {
  __shared__ u32 lw[64 * LW_STRIDE];  // (a 64-thread block)
  for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const u64 a = off[k], b = off[k + 1];
    evm_pb_sync s{0, 0, 0, 0, 0, 0, 0, 0, 0};
    LWin win;
    win.init(arena + b, lw + threadIdx.x * LW_STRIDE);
    const u64 s0 = a / PB_MIN_MSG, room = b / PB_MIN_MSG - s0;
    int st = b < a ? EVM_EINVAL : d_walk(kind, arena + a, b - a, &s, &win, [&](u64 i, const DMsg&, const uint8_t* at) {
      if (slots && i < room) slots[s0 + i] = (u64)(at - arena);
    });
    if (st) s = evm_pb_sync{0, 0, 0, 0, 0, 0, 0, 0, 0};
    info[k] = s;
    status[k] = st;
  }
}

// The split in three parallel steps: the bodies' top-level walk only finds
// their messages (a thread per body, the walk's loads one window refill per
// message or so), then a thread per message parses it into its row, and
// after a scan of the content lengths copies its content.
__global__ void k_pb_offsets(int kind, const uint8_t* __restrict__ arena, const u64* __restrict__ off, u32 n,
                             const int32_t* __restrict__ status, const u64* __restrict__ msg_base,
                             const u32* __restrict__ owner_of, u64* __restrict__ mat, u32* __restrict__ mlen,
                             u32* __restrict__ owner, u32* __restrict__ bad) {
  for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    if (status[k]) continue;
    const u64 a = off[k], m0 = msg_base[k], mn = msg_base[k + 1] - m0;
    const u32 ow = owner_of ? owner_of[k] : 0u;
    Win win;
    win.init(arena + off[k + 1]);
    DReader r{arena + a, arena + off[k + 1], true, &win};
    const u32 tree_field = kind == EVM_PB_SYNC_REQUEST ? 4u : 2u;
    u64 i = 0;
    // (the body scanned fine: the same grammar as d_walk, inner messages not re-read)
    while (r.more()) {
      const u64 tag = r.varint();
      const u32 field = (u32)(tag >> 3), wt = (u32)(tag & 7);
      const bool is_str = field == 1 || field == tree_field || (kind == EVM_PB_SYNC_REQUEST && (field == 2 || field == 3));
      if (!is_str) {
        r.skip(wt);
        continue;
      }
      const uint8_t* q;
      u64 len;
      if (!r.bytes(&q, &len)) break;
      if (field == 1) {
        if (i < mn) {
          mat[m0 + i] = (u64)(q - arena);
          mlen[m0 + i] = (u32)len;
          if (owner) owner[m0 + i] = ow;
        }
        ++i;
      }
    }
    if (!r.ok || i != mn) atomicOr(bad, 1u);  // (cannot happen for a body that scanned fine)
  }
}

__global__ void k_pb_rows(const uint8_t* __restrict__ arena, const u64* __restrict__ mat, const u32* __restrict__ mlen,
                          u64 N, char* __restrict__ ts, u64 stride, u64* __restrict__ cat, u64* __restrict__ clen) {
  for (u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x; m < N; m += (u64)gridDim.x * blockDim.x) {
    const uint8_t* q = arena + mat[m];
    Win win;
    win.init(q + mlen[m]);
    DMsg msg;
    d_read_msg(q, mlen[m], &msg, &win);
    u64* row = reinterpret_cast<u64*>(ts + m * stride);
    const bool std46 = msg.ts_len == 46;
    for (int j = 0; j < 5; ++j) row[j] = std46 ? win.get8(msg.ts + 8 * j) : ~0ull;
    row[5] = (std46 ? win.get8(msg.ts + 40) : ~0ull) & 0x0000FFFFFFFFFFFFull;
    for (u64 j = 48; j < stride; j += 8) row[j >> 3] = 0ull;
    cat[m] = msg.content ? (u64)(msg.content - arena) : 0ull;
    clen[m] = msg.content_len;
  }
}

// bytes in global memory: a pointer read from LDS would be flat, and a flat
// load makes every later store wait for it and for every store before it
typedef __attribute__((address_space(1))) uint8_t gu8;

// s_waitcnt vmcnt(0) on the common path: the loads above it are complete.
// (Each store below sits in its own exec-masked block; without a wait every
// block could have been skipped, so each one waited again -- for the stores
// before it as well.)
__device__ __forceinline__ void vm_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

constexpr u32 PB_ROW_WORDS = 6;  // a row's 46 timestamp bytes as 8-B words (the rest of the stride is 0)
// Reads of a span of device bytes staged in LDS ([A, Z), A 16-B aligned),
// anything outside it from global memory
typedef uint64_t __attribute__((aligned(1))) ulu64;
typedef uint4 __attribute__((aligned(1))) u4u;
typedef __attribute__((address_space(3))) const unsigned char lds_u8;
typedef __attribute__((address_space(3))) const ulu64 lds_u64;
struct SWin {
  lds_u8* st;
  const uint8_t* A;
  const uint8_t* Z;
  __device__ __forceinline__ uint8_t get(const uint8_t* p) const { return p >= A && p < Z ? st[p - A] : *p; }
  __device__ __forceinline__ u64 get8(const uint8_t* p) const {
    if (p >= A && p + 8 <= Z) return *reinterpret_cast<lds_u64*>(st + (p - A));
    u64 v = 0;
    for (int k = 0; k < 8; ++k) v |= (u64)get(p + k) << (8 * k);
    return v;
  }
};
__device__ __forceinline__ u64 readlane64(u64 x, int l) {
  return ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(x >> 32), l) << 32) |
         (u32)__builtin_amdgcn_readlane((int)(u32)x, l);
}
constexpr u32 PB_STAGE = 8192;  // bytes of a chunk's 64 messages staged in LDS per wave (more: read in place)

// k_pb_rows from the scan's slots: a wave per body, a lane per message.  Each
// 64 messages' bytes are loaded into LDS by the wave (coalesced 16-B loads;
// each lane reading its own message through a register window fetched ~1.7x
// the bytes) and parsed there; the 64 rows are staged in LDS and stored as one
// contiguous run (a lane writing its own row made every store a
// 48-B-strided partial-line write); each content is copied by its lane in
// unaligned 16-B pieces (a byte loop: 6.9 ms for config 3's round, 16-B
// pieces 4.9 ms; the wave copying the 64 contents one after another, a byte
// per lane, 7.5-8 ms)

__global__ __launch_bounds__(256) void k_pb_rows_idx(const uint8_t* __restrict__ arena, const u64* __restrict__ off, u32 n,
                                                     const int32_t* __restrict__ status, const u64* __restrict__ msg_base,
                                                     const u64* __restrict__ content_base, const u64* __restrict__ slots,
                                                     const u32* __restrict__ owner_of, char* __restrict__ ts, u64 stride,
                                                     u64* __restrict__ content_off, uint8_t* __restrict__ content,
                                                     u32* __restrict__ owner, u32* __restrict__ bad) {
  __shared__ u64 srow[4][64 * PB_ROW_WORDS];
  __shared__ uint4 sstage[4][PB_STAGE / 16];
  const u32 lane = threadIdx.x & 63;
  u64* sr = srow[threadIdx.x >> 6];
  uint4* stg = sstage[threadIdx.x >> 6];
  const u32 SW = (u32)(stride / 8);  // (stride: a multiple of 16, >= 48)
  for (u32 k = blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += gridDim.x * 4) {
    if (status[k]) continue;
    const u64 a = off[k], b = off[k + 1], m0 = msg_base[k], mn = msg_base[k + 1] - m0;
    const u64 s0 = a / PB_MIN_MSG;
    const u32 ow = owner_of ? owner_of[k] : 0u;
    u64 cpos = content_base[k];  // the body's contents go here, message after message
    if (mn > b / PB_MIN_MSG - s0) {  // (a message shorter than 50 bytes: its timestamp is not 46)
      if (lane == 0) atomicOr(bad, 1u);
      for (u64 i = lane; i < mn; i += 64) {  // (its rows empty, no content: the call fails)
        u64* row = reinterpret_cast<u64*>(ts + (m0 + i) * stride);
        for (u64 j = 0; j < stride; j += 8) row[j >> 3] = ~0ull;
        content_off[m0 + i] = cpos;
        if (owner) owner[m0 + i] = ow;
      }
      continue;
    }
    // 64 messages at a time, a lane each (mn is wave-uniform: every lane runs
    // every chunk, so the contents' prefix sum is a wave scan)
    for (u64 i0 = 0; i0 < mn; i0 += 64) {
      const u64 i = i0 + lane;
      const u32 cnt = (u32)min<u64>(64, mn - i0);
      const u64 fpos = i < mn ? slots[s0 + i] : 0;
      // the chunk's bytes: its first message field up to the next chunk's
      // first (the body's last chunk: to its last message's end), loaded
      // into LDS by the wave with coalesced 16-B loads -- each lane reading
      // its own message through a window fetched ~1.7x the bytes
      u64 E;
      if (i0 + 64 < mn) {
        E = slots[s0 + i0 + 64];
      } else {
        u64 e = 0;
        if (lane == cnt - 1) {
          Win w2;
          w2.init(arena + b);
          DReader r{arena + fpos, arena + b, true, &w2};
          r.varint();
          const u64 len = r.varint();
          e = (u64)(r.p - arena) + len;
        }
        E = readlane64(e, (int)cnt - 1);
      }
      const u64 A0 = readlane64(fpos, 0) & ~15ull;
      const bool staged = E >= A0 && E - A0 <= PB_STAGE;  // (wave-uniform)
      if (staged) {
        const u32 nq = (u32)((E - A0 + 15) >> 4);
        for (u32 q = lane; q < nq; q += 64) stg[q] = *reinterpret_cast<const uint4*>(arena + A0 + 16ull * q);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      // (an unstaged chunk -- a content of kilobytes -- reads its bytes one by one)
      SWin sw{(lds_u8*)stg, arena + A0, arena + (staged ? E : A0)};
      u64 cl = 0;
      const uint8_t* csrc = nullptr;
      if (i < mn) {
        DReaderT<SWin> r{arena + fpos, arena + b, true, &sw};
        r.varint();  // (the field's tag: 1, length-delimited -- the scan read it)
        const uint8_t* q;
        u64 len;
        r.bytes(&q, &len);
        DMsg msg;
        d_read_msg(q, len, &msg, &sw);
        const bool std46 = msg.ts_len == 46;
#pragma unroll
        for (int j = 0; j < 5; ++j) sr[lane * PB_ROW_WORDS + j] = std46 ? sw.get8(msg.ts + 8 * j) : ~0ull;
        sr[lane * PB_ROW_WORDS + 5] = (std46 ? sw.get8(msg.ts + 40) : ~0ull) & 0x0000FFFFFFFFFFFFull;
        csrc = msg.content;
        cl = msg.content ? msg.content_len : 0;
        if (owner) owner[m0 + i] = ow;
      }
      // this message's content offset: the body's base + the contents before it
      u64 x = cl;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const u64 y = __shfl_up(x, d, 64);
        if ((int)lane >= d) x += y;
      }
      const u64 dst = cpos + x - cl;
      cpos += __shfl(x, 63, 64);
      if (i < mn) content_off[m0 + i] = dst;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // the chunk's rows are one contiguous run of cnt * SW words
      u64* rows = reinterpret_cast<u64*>(ts + (m0 + i0) * stride);
      for (u32 w = lane; w < cnt * SW; w += 64) {
        const u32 r = SW == PB_ROW_WORDS ? w / PB_ROW_WORDS : w / SW, f = w - r * SW;
        rows[w] = f < PB_ROW_WORDS ? sr[r * PB_ROW_WORDS + f] : 0ull;
      }
      if (i < mn) {
        // whole 16-B pieces by unaligned 16-B loads (from the staged copy when
        // the content lies in it) and stores (inside this message's bytes: no
        // other lane's), four in flight; the tail by bytes
        const u64 n16 = cl >> 4;
        const u64 t0 = n16 * 16;
        if (csrc >= sw.A && csrc + cl <= sw.Z) {  // (from the staged copy)
          typedef unsigned int v4u __attribute__((ext_vector_type(4), aligned(1)));
          typedef __attribute__((address_space(3))) const v4u lds_v4;
          lds_u8* src = sw.st + (csrc - sw.A);
          for (u64 j = 0; j < n16; ++j)
            *reinterpret_cast<v4u*>(content + dst + 16 * j) = *reinterpret_cast<lds_v4*>(src + 16 * j);
          for (u64 t = t0; t < cl; ++t) content[dst + t] = src[t];
        } else {  // (a chunk too long for the stage: in place)
          for (u64 j = 0; j < n16; ++j)
            *reinterpret_cast<u4u*>(content + dst + 16 * j) = *reinterpret_cast<const u4u*>(csrc + 16 * j);
          for (u64 t = t0; t < cl; ++t) content[dst + t] = csrc[t];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // (sr and the stage are rewritten by the next chunk)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

__global__ void k_pb_content(const uint8_t* __restrict__ arena, const u64* __restrict__ cat,
                             const u64* __restrict__ content_off, u64 N, uint8_t* __restrict__ content) {
  for (u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x; m < N; m += (u64)gridDim.x * blockDim.x) {
    const u64 d = content_off[m], len = content_off[m + 1] - d;
    const uint8_t* src = arena + cat[m];
    // 16 bytes at a time, every load issued before the stores (a byte loop
    // waited out one load latency per byte: 2.2 ms for config 3's round)
    for (u64 j0 = 0; j0 < len; j0 += 16) {
      uint8_t b[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) b[k] = j0 + k < len ? src[j0 + k] : 0;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (j0 + k < len) content[d + j0 + k] = b[k];
    }
  }
}

// packed copies of n byte spans: dst[dst_off[k] ..] = src[src_off[k] .. + len[k])
__global__ void k_gather_spans(const uint8_t* __restrict__ src, const u64* __restrict__ src_off,
                               const u64* __restrict__ len, const u64* __restrict__ dst_off, u32 n,
                               uint8_t* __restrict__ dst) {
  for (u32 k = blockIdx.x; k < n; k += gridDim.x)
    for (u64 j = threadIdx.x; j < len[k]; j += blockDim.x) dst[dst_off[k] + j] = src[src_off[k] + j];
}

// ---------------------------------------------------------------- tree JSON
// evm_json.cpp's Parser as an explicit stack (depth <= CODE_DIGITS), one
// thread per owner; the frames of a block's threads live in LDS.
constexpr int JP_THREADS = 64;
constexpr int JP_LEVELS = CODE_DIGITS + 1;
constexpr u64 CODE_MASK40 = (1ull << 40) - 1;

__device__ __forceinline__ bool jws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

struct JText {
  const uint8_t* p;
  const uint8_t* e;
  Win win;
  __device__ __forceinline__ uint8_t at(const uint8_t* q) { return win.get(q); }
  __device__ __forceinline__ void ws() {
    while (p < e && jws(at(p))) ++p;
  }
  __device__ __forceinline__ bool lit(uint8_t c) {
    ws();
    if (p < e && at(p) == c) {
      ++p;
      return true;
    }
    return false;
  }
  __device__ __forceinline__ int key() {  // 0, 1, 2 for the digits, 3 for "hash", -1 otherwise
    ws();
    if (p >= e || at(p) != '"') return -1;
    const uint8_t* q = ++p;
    uint8_t c;
    while (p < e && (c = at(p)) != '"') {
      if (c == '\\') return -1;
      ++p;
    }
    if (p >= e) return -1;
    const u64 len = (u64)(p - q);
    ++p;
    if (len == 1) {
      c = at(q);
      return c >= '0' && c <= '2' ? c - '0' : -1;
    }
    if (len == 4 && at(q) == 'h' && at(q + 1) == 'a' && at(q + 2) == 's' && at(q + 3) == 'h') return 3;
    return -1;
  }
  __device__ __forceinline__ bool integer(int32_t* v) {
    ws();
    bool neg = false;
    if (p < e && at(p) == '-') {
      neg = true;
      ++p;
    }
    if (p >= e || at(p) < '0' || at(p) > '9') return false;
    if (at(p) == '0' && p + 1 < e && at(p + 1) >= '0' && at(p + 1) <= '9') return false;
    int64_t x = 0;
    uint8_t c;
    while (p < e && (c = at(p)) >= '0' && c <= '9') {
      x = x * 10 + (c - '0');
      if (x > 2147483648LL) return false;
      ++p;
    }
    if (p < e && ((c = at(p)) == '.' || c == 'e' || c == 'E')) return false;
    if (neg) x = -x;
    if (x < (int64_t)INT32_MIN || x > (int64_t)INT32_MAX || (neg && x == 0)) return false;
    *v = (int32_t)x;
    return true;
  }
};

// The common text first: JSON.stringify's own form, `{` then tokens --
// OPEN `"d":{` (a child, digits ascending), HASH `"hash":N}` (closes the
// node; a `,` follows unless it is the root's) -- read a wave per tree, 3 KB
// per step.  A token starts at every `"` after `{` or `,` and nowhere else in
// that form, so the lanes find them in their 16 bytes independently; each
// token checks that its successor starts right after it (through a `,` after
// a HASH), hence the chain from the first token covers the text exactly.  The
// structure then comes from wave scans over the tokens: the depth (+1 / -1),
// the code (each token an operation "keep the digits above depth a, then set
// B": composable), and the XOR of the leaves (childless nodes) before each
// token; an internal node's hash must equal its leaves' XOR (the leaves XOR
// at its close ^ at its open: the open is the last OPEN one depth up, found
// by a ballot per depth or, from an earlier step, kept per depth in LDS).
// Such a tree's leaves are its childless nodes in text order, exactly what
// k_json_parse emits for it.  Anything else -- whitespace, another key
// order, an internal node whose hash is not its leaves' XOR (a shorter key
// of its own), a malformed text -- leaves the owner JP_SLOW for
// k_json_parse, which decides exactly as the host parser.
constexpr int32_t JP_SLOW = -1;
constexpr u64 JP_KEY_MASK = 0xFFFFFF00FFull, JP_KEY = 0x7B3A220022ull;          // `"?":{`
constexpr u64 JP_HASH_MASK = 0x00FFFFFFFFFFFFFFull, JP_HASH = 0x003A226873616822ull;  // `"hash":`
constexpr int JV_WAVES = 4;
constexpr u32 JV_STEP = 3072;                // text bytes per step: 48 per lane (~4 chunks of 64 tokens in config 3's trees)
constexpr u32 JV_BUF = 16 + JV_STEP + 48;    // the chunk before (a token's `{` / `,`), the step, lookahead
constexpr u32 JV_TOK = JV_STEP / 2;          // token starts in a step (>= 2 bytes apart: `,"` in a malformed text)
constexpr u32 JV_HASH = 3, JV_END = 4, JV_BAD = 5, JV_ROOT = 6, JV_NONE = 7;  // token kinds (0-2: OPEN digit)
constexpr u64 CODE_ALL = (1ull << (2 * CODE_DIGITS)) - 1ull;

struct alignas(16) JvLds {
  u32 buf[JV_BUF / 4];
  unsigned long long bal[CODE_DIGITS];  // a chunk's OPEN lanes by depth
  uint16_t pos[JV_TOK];      // the step's token starts (buffer bytes), in text order
  int32_t stk[CODE_DIGITS];  // the leaves' XOR before the last OPEN at each depth (earlier chunks)
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 0x80 in each zero byte of x; the four bytes' top bits as bits 0-3
__device__ __forceinline__ u32 zero_bytes(u32 x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu); }
__device__ __forceinline__ u32 gather4(u32 t) { return ((((t >> 7) & 0x01010101u) * 0x00204081u) >> 21) & 0xFu; }

// bit k: byte k of w equals c (c4 = c in every byte)
__device__ __forceinline__ u32 bytes_eq(u32 w, u32 c4) {
  const u32 x = w ^ c4;
  const u32 t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // 0x80 in the zero bytes
  return ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
}

// the code's bits of the digits above depth a (digit d at bits 2 * (CODE_DIGITS - 1 - d))
__device__ __forceinline__ u64 digits_above(int a) {
  const int sh = min(max(2 * (CODE_DIGITS - a), 0), 2 * CODE_DIGITS);
  return CODE_ALL & ~((1ull << sh) - 1ull);
}

__device__ __forceinline__ u64 shfl_up_u64(u64 v, int d) {
  return ((u64)(u32)__shfl_up((int)(u32)(v >> 32), d, 64) << 32) | (u32)__shfl_up((int)(u32)v, d, 64);
}

// Wave scans on the DPP network (row shifts 1, 2, 4, 8, then the row
// broadcasts of lanes 15 and 31): combine(earlier, later) at each step.
template <int CTRL>
__device__ __forceinline__ u32 dpp(u32 x) {
  return (u32)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ u32 rl(u32 x, int l) { return (u32)__builtin_amdgcn_readlane((int)x, l); }
template <int CTRL>
__device__ __forceinline__ u64 dpp64(u64 x) {
  return ((u64)dpp<CTRL>((u32)(x >> 32)) << 32) | dpp<CTRL>((u32)x);
}
template <class T, class Comb>
__device__ __forceinline__ T wave_scan(T x, int lane, Comb comb) {
  const int r = lane & 15;
  T y = x.template shift<0x111>();
  x = r >= 1 ? comb(y, x) : x;
  y = x.template shift<0x112>();
  x = r >= 2 ? comb(y, x) : x;
  y = x.template shift<0x114>();
  x = r >= 4 ? comb(y, x) : x;
  y = x.template shift<0x118>();
  x = r >= 8 ? comb(y, x) : x;
  // across the rows: lane 15 of each row into the next, then lane 31 into rows 2 and 3
  y = x.template shift<0x142>();
  x = (lane & 31) >= 16 ? comb(y, x) : x;
  y = x.template shift<0x143>();
  x = lane >= 32 ? comb(y, x) : x;
  return x;
}
// (the scanned values: a count; depth change and leaf XOR; the code operation
// "keep the digits above depth a, then set B")
struct JvCount {
  u32 n;
  template <int CTRL>
  __device__ __forceinline__ JvCount shift() const { return JvCount{dpp<CTRL>(n)}; }
  __device__ __forceinline__ JvCount at(int l) const { return JvCount{rl(n, l)}; }
};
struct JvDepth {
  int dx;
  u32 px;
  template <int CTRL>
  __device__ __forceinline__ JvDepth shift() const { return JvDepth{(int)dpp<CTRL>((u32)dx), dpp<CTRL>(px)}; }
  __device__ __forceinline__ JvDepth at(int l) const { return JvDepth{(int)rl((u32)dx, l), rl(px, l)}; }
};
struct JvOp {
  int a;
  u64 B;
  template <int CTRL>
  __device__ __forceinline__ JvOp shift() const { return JvOp{(int)dpp<CTRL>((u32)a), dpp64<CTRL>(B)}; }
  __device__ __forceinline__ JvOp at(int l) const { return JvOp{(int)rl((u32)a, l), ((u64)rl((u32)(B >> 32), l) << 32) | rl((u32)B, l)}; }
};

// The token at buffer byte pb (text position p, the text ends at E): its kind
// (0-2, JV_HASH, JV_END, or JV_BAD) and hash.
__device__ __forceinline__ u32 jv_token(const JvLds* w, u32 pb, u64 p, u64 E, int32_t* hv) {
  const u32 a = pb >> 2, s = pb & 3u;
  const u32 w0 = w->buf[a], w1 = w->buf[a + 1], w2 = w->buf[a + 2], w3 = w->buf[a + 3], w4 = w->buf[a + 4],
            w5 = w->buf[a + 5], w6 = w->buf[a + 6];
  const u64 X = ((u64)__builtin_amdgcn_alignbyte(w2, w1, s) << 32) | __builtin_amdgcn_alignbyte(w1, w0, s);
  const u64 X1 = ((u64)__builtin_amdgcn_alignbyte(w4, w3, s) << 32) | __builtin_amdgcn_alignbyte(w3, w2, s);
  const u64 X2 = ((u64)__builtin_amdgcn_alignbyte(w6, w5, s) << 32) | __builtin_amdgcn_alignbyte(w5, w4, s);
  auto byte = [&](int k) -> u32 {
    return (u32)((k < 8 ? X >> (8 * k) : k < 16 ? X1 >> (8 * (k - 8)) : X2 >> (8 * (k - 16))) & 0xffu);
  };
  *hv = 0;
  if ((X & JP_KEY_MASK) == JP_KEY) {
    const u32 d = byte(1) - '0';
    return d < 3u && byte(5) == '"' && p + 5 < E ? d : JV_BAD;
  }
  if ((X & JP_HASH_MASK) != JP_HASH) return JV_BAD;
  // -?(0|[1-9][0-9]*) within int32, `}`, then `,"` or the end of the text: the
  // 16 bytes after the sign as two words, the digits found and read 8 at a time
  const bool neg = byte(7) == '-';
  const u64 lo = neg ? X1 : (X >> 56) | (X1 << 8), hi = neg ? X2 : (X1 >> 56) | (X2 << 8);
  auto nondigit = [](u64 x) -> u64 {  // 0x80 in the bytes that are not '0'-'9'
    const u64 y = ((x & 0xF0F0F0F0F0F0F0F0ull) ^ 0x3030303030303030ull) |
                  (((x & 0x0F0F0F0F0F0F0F0Full) + 0x0606060606060606ull) & 0x1010101010101010ull);
    return (((y & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | y) & 0x8080808080808080ull;
  };
  auto eight = [](u64 x) -> u64 {  // 8 digits, the first in the low byte
    x = (x & 0x0F0F0F0F0F0F0F0Full) * 2561 >> 8;
    x = (x & 0x00FF00FF00FF00FFull) * 6553601 >> 16;
    return (x & 0x0000FFFF0000FFFFull) * 42949672960001ull >> 32;
  };
  const u64 ml = nondigit(lo), mh = nondigit(hi);
  const u32 nd = ml ? (u32)__builtin_ctzll(ml) >> 3 : 8u + (mh ? (u32)__builtin_ctzll(mh) >> 3 : 8u);
  if (nd == 0 || nd > 10) return JV_BAD;
  const u32 sh = 8 * nd;
  const u64 tail = sh < 64 ? (lo >> sh) | (hi << (64 - sh)) : hi >> (sh - 64);
  const u32 t0 = (u32)tail & 0xffu, t1 = (u32)(tail >> 8) & 0xffu, t2 = (u32)(tail >> 16) & 0xffu;
  const u32 d0 = (u32)lo & 0xffu;
  const u64 e8 = eight(nd >= 8 ? lo : lo << (64 - sh));
  const u64 d8 = (hi & 0xffu) - '0', d9 = ((hi >> 8) & 0xffu) - '0';
  const u64 v = nd <= 8 ? e8 : nd == 9 ? e8 * 10u + d8 : e8 * 100u + d8 * 10u + d9;
  if (nd == 0 || nd > 10 || (nd > 1 && d0 == '0') || (neg && v == 0) || t0 != '}' ||
      v > (neg ? 2147483648ull : 2147483647ull))
    return JV_BAD;
  *hv = (int32_t)(neg ? 0ull - v : v);
  const u64 end = p + 8 + (neg ? 1 : 0) + nd;
  if (end == E) return JV_END;
  return t1 == ',' && t2 == '"' && end + 1 < E ? JV_HASH : JV_BAD;
}

__global__ __launch_bounds__(64 * JV_WAVES) void k_json_wave(const uint8_t* __restrict__ json, const u64* __restrict__ jat,
                                                              const u64* __restrict__ jlen, u32 n_owners,
                                                              const u64* __restrict__ base, u64* __restrict__ t_off,
                                                              u64* __restrict__ t_end, u64* __restrict__ ck,
                                                              int32_t* __restrict__ xr, int32_t* __restrict__ pfx,
                                                              int32_t* __restrict__ status, u64* __restrict__ n_leaves) {
  __shared__ JvLds lds[JV_WAVES];
  JvLds* w = &lds[threadIdx.x >> 6];
  const int lane = (int)(threadIdx.x & 63);
  const u32 o = blockIdx.x * JV_WAVES + (threadIdx.x >> 6);
  if (o >= n_owners) return;  // (the whole wave)
  const u64 lt = (1ull << lane) - 1ull;
  const u64 b0 = base[o];
  const u64 bound = base[o + 1] - b0 - 1;
  const u64 L = jlen[o];
  int st = JP_SLOW;
  u64 cnt = 0;
  int32_t P = 0;  // the leaves' XOR so far
  if (L == 0) {
    st = 0;
  } else if (L >= 2) {
    const uint8_t* tx = json + jat[o];
    const uint8_t c0 = tx[0], c1 = tx[1];
    if (L == 2 && c0 == '{' && c1 == '}') {
      st = 0;
    } else if (c0 == '{' && c1 == '"') {
      const uint8_t* A = reinterpret_cast<const uint8_t*>((uintptr_t)tx & ~(uintptr_t)15);
      const uint8_t* lim = reinterpret_cast<const uint8_t*>(((uintptr_t)(tx + L) + 15) & ~(uintptr_t)15);
      const u64 s0 = (u64)(tx - A), E = s0 + L;  // text positions from A
      auto chunk = [lim](const uint8_t* c) -> uint4 {
        if (c < lim) return *reinterpret_cast<const uint4*>(c);
        return make_uint4(0, 0, 0, 0);
      };
      int depth = 0;
      u64 code = 0, lastcode = 0;
      u32 lastk = JV_ROOT;
      bool bad = false;
      // the step's 32 bytes per lane and the 48 after the step (lanes 0-2), loaded
      // one step ahead
      uint4 v0 = chunk(A + 48 * lane), v1 = chunk(A + 48 * lane + 16), v2 = chunk(A + 48 * lane + 32),
            la = make_uint4(0, 0, 0, 0);
      if (lane < 3) la = chunk(A + JV_STEP + 16 * lane);
      uint4 last2 = make_uint4(0, 0, 0, 0);  // (lane 63: the step before's last 16 bytes)
      for (u64 P0 = 0; P0 < E && !bad; P0 += JV_STEP) {
        const uint8_t* S1 = A + P0 + JV_STEP;
        const uint4 n0 = chunk(S1 + 48 * lane), n1 = chunk(S1 + 48 * lane + 16), n2 = chunk(S1 + 48 * lane + 32);
        uint4 nla = make_uint4(0, 0, 0, 0);
        if (lane < 3) nla = chunk(S1 + JV_STEP + 16 * lane);
        // stage the step's bytes, the chunk before them and the lookahead in LDS
        uint4* b4 = reinterpret_cast<uint4*>(w->buf);
        b4[1 + 3 * lane] = v0;
        b4[2 + 3 * lane] = v1;
        b4[3 + 3 * lane] = v2;
        if (lane < 3) b4[1 + 3 * 64 + lane] = la;
        if (lane == 63) b4[0] = last2;
        wave_sync();
        // token starts in this lane's 48 bytes: `"` after `{` or `,`, within [s0 + 1, E)
        const u32 prev = w->buf[3 + 12 * lane] >> 24;
        auto oc4 = [](u32 x) { return gather4(zero_bytes(x ^ 0x7B7B7B7Bu) | zero_bytes(x ^ 0x2C2C2C2Cu)); };
        auto q4 = [](u32 x) { return gather4(zero_bytes(x ^ 0x22222222u)); };
        auto q16 = [&](uint4 v) { return q4(v.x) | q4(v.y) << 4 | q4(v.z) << 8 | q4(v.w) << 12; };
        auto oc16 = [&](uint4 v) { return oc4(v.x) | oc4(v.y) << 4 | oc4(v.z) << 8 | oc4(v.w) << 12; };
        const u64 q = (u64)q16(v0) | (u64)q16(v1) << 16 | (u64)q16(v2) << 32;
        const u64 oc = (u64)oc16(v0) | (u64)oc16(v1) << 16 | (u64)oc16(v2) << 32;
        u64 starts = q & ((oc << 1) | (prev == '{' || prev == ',' ? 1ull : 0ull)) & 0xFFFFFFFFFFFFull;
        const u64 pos0 = P0 + 48 * (u64)lane;
        const int64_t lo = (int64_t)(s0 + 1) - (int64_t)pos0, hi = (int64_t)E - (int64_t)pos0;
        if (lo > 0) starts &= lo >= 48 ? 0ull : ~((1ull << lo) - 1ull);
        if (hi < 48) starts &= hi <= 0 ? 0ull : (1ull << hi) - 1ull;
        last2 = v2;
        v0 = n0;
        v1 = n1;
        v2 = n2;
        la = nla;
        const u32 nt = __popcll(starts);
        u32 tb = wave_scan(JvCount{nt}, lane, [](JvCount y, JvCount x) { return JvCount{x.n + y.n}; }).n;
        const u32 T = __builtin_amdgcn_readlane(tb, 63);
        tb -= nt;
        while (starts) {
          const u32 j = __ffsll((unsigned long long)starts) - 1;
          starts &= starts - 1;
          w->pos[tb++] = (uint16_t)(16 + 48 * lane + j);
        }
        wave_sync();
        // the tokens, 64 at a time, one per lane
        for (u32 c = 0; c < T; c += 64) {
          const u32 i = c + lane;
          int32_t h = 0;
          u32 k = JV_NONE;
          if (i < T) {
            const u32 pb = w->pos[i];
            k = jv_token(w, pb, P0 + pb - 16, E, &h);
          }
          const bool open = k < 3, hash = k == JV_HASH || k == JV_END;
          const int dlt = open ? 1 : hash ? -1 : 0;
          // the token before: its kind, and (below) the code before it
          u32 pk = (u32)__shfl_up((int)k, 1, 64);
          if (lane == 0) pk = lastk;
          const bool leaf = hash && pk < 3;
          const int32_t lv = leaf ? h : 0;
          // depth and leaf XOR: inclusive scans
          const JvDepth sc = wave_scan(JvDepth{dlt, (u32)lv}, lane,
                                       [](JvDepth y, JvDepth x) { return JvDepth{x.dx + y.dx, x.px ^ y.px}; });
          const int db = depth + sc.dx - dlt;  // the depth before each token
          const int32_t pb = P ^ (int32_t)sc.px ^ lv;
          bool bl = k == JV_BAD || (open && db >= CODE_DIGITS) || (k == JV_HASH && db <= 0) || (k == JV_END && db != 0);
          // the code before each token: the composition of the operations before it
          JvOp op{63, 0};
          if (open && db < CODE_DIGITS) {
            op.a = db;
            op.B = (u64)(k + 1) << (2 * (CODE_DIGITS - 1 - db));
          } else if (hash) {
            op.a = db > 0 ? db - 1 : 0;
          }
          const JvOp oc2 = wave_scan(op, lane, [](JvOp y, JvOp x) {  // (y before x)
            return JvOp{min(x.a, y.a), (y.B & digits_above(x.a)) | x.B};
          });
          int ea = __shfl_up(oc2.a, 1, 64);
          u64 eB = shfl_up_u64(oc2.B, 1);
          if (lane == 0) {
            ea = 63;
            eB = 0;
          }
          const u64 cb = (code & digits_above(ea)) | eB;
          u64 pc = shfl_up_u64(cb, 1);
          if (lane == 0) pc = lastcode;
          // an internal node's open: the last OPEN one depth up (in this chunk: a
          // ballot per depth present; before it: the depth's entry in stk)
          const int need = hash && !leaf && db >= 1 ? db - 1 : -1;
          // (the chunk's OPEN lanes per depth: one LDS OR per lane, not a ballot per depth)
          const bool o2 = open && db < CODE_DIGITS;
          if (lane < CODE_DIGITS) w->bal[lane] = 0;
          wave_sync();
          if (o2) atomicOr(&w->bal[db], 1ull << lane);
          wave_sync();
          const u64 mneed = need >= 0 ? w->bal[need] : 0ull;
          const u64 mown = o2 ? w->bal[db] : 0ull;
          const u64 mm = mneed & lt;
          const int32_t po_lane = __shfl(pb, mm ? 63 - __clzll(mm) : lane, 64);
          if (hash && !leaf) {
            if (db == 0) bl |= pk != JV_HASH || h != pb;  // the root: children, their leaves' XOR
            else if (db > 0) bl |= h != (pb ^ (mm ? po_lane : w->stk[need]));
          }
          if (open && pk == JV_HASH && db < CODE_DIGITS)  // the previous sibling's digit below this one
            bl |= ((pc >> (2 * (CODE_DIGITS - 1 - db))) & 3u) > k;
          // the leaves out, in text order
          const u64 lb = __ballot(leaf);
          const u64 at = cnt + __popcll(lb & lt);
          if (leaf) {
            if (at >= bound) {
              bl = true;
            } else {
              ck[b0 + at] = ((u64)o << 40) | cb;
              xr[b0 + at] = h;
              pfx[b0 + at] = pb;
            }
          }
          wave_sync();
          if (open && db < CODE_DIGITS && (mown >> lane) == 1ull) w->stk[db] = pb;
          wave_sync();
          cnt += __popcll(lb);
          depth = __builtin_amdgcn_readlane(depth + sc.dx, 63);
          P = __builtin_amdgcn_readlane(pb ^ lv, 63);
          const u64 ca = (cb & digits_above(op.a)) | op.B;
          code = ((u64)rl((u32)(ca >> 32), 63) << 32) | rl((u32)ca, 63);
          const int last = (int)min<u32>(T - c, 64u) - 1;
          lastk = __builtin_amdgcn_readlane(k, last);
          lastcode = ((u64)rl((u32)(cb >> 32), last) << 32) | rl((u32)cb, last);
          if (__ballot(bl)) {
            bad = true;
            break;
          }
        }
      }
      if (!bad && lastk == JV_END) st = 0;
    }
  }
  if (st) cnt = 0;
  if (lane == 0) {
    t_off[o] = b0;
    pfx[b0 + cnt] = st ? 0 : P;
    t_end[o] = b0 + cnt;
    status[o] = st;
    if (cnt) atomicAdd(n_leaves, cnt);
  }
}

// owner o's text at json + jat[o], jlen[o] bytes (jlen 0: no request, the
// empty tree); its leaves from slot base[o] (room for the bound), the
// owner-local exclusive prefix XOR beside them; status[o]: 0, EVM_ETREE, or
// EVM_TREE_UNSORTED
__global__ __launch_bounds__(JP_THREADS) void k_json_parse(const uint8_t* __restrict__ json, const u64* __restrict__ jat,
                                                           const u64* __restrict__ jlen, u32 n_owners,
                                                           const u64* __restrict__ base, u64* __restrict__ t_off,
                                                           u64* __restrict__ t_end, u64* __restrict__ ck,
                                                           int32_t* __restrict__ xr, int32_t* __restrict__ pfx,
                                                           int32_t* __restrict__ status, u64* __restrict__ n_leaves) {
  __shared__ int32_t s_h[JP_LEVELS][JP_THREADS];
  __shared__ int32_t s_cx[JP_LEVELS][JP_THREADS];
  __shared__ uint8_t s_fl[JP_LEVELS][JP_THREADS];  // seen keys (bits 0-3) | any child (bit 4)
  __shared__ u32 s_first[JP_LEVELS][JP_THREADS];    // leaves emitted when the node opened
  const u32 o = blockIdx.x * JP_THREADS + threadIdx.x;
  if (o >= n_owners || status[o] != JP_SLOW) return;  // (k_json_wave read it)
  const u32 me = threadIdx.x;
  const u64 b0 = base[o];
  const u64 bound = base[o + 1] - b0 - 1;  // leaf slots (one more holds the root's prefix)
  t_off[o] = b0;
  u64 cnt = 0;
  int32_t run = 0;
  int st = 0;
  const u64 L = jlen[o];
  if (L) {
    JText tx;
    tx.p = json + jat[o];
    tx.e = tx.p + L;
    tx.win.init(tx.e);
    // the frame of the node being read at depth d: prefix = the code so far
    u64 prefix = 0;
    int d = 0;
    if (!tx.lit('{')) st = EVM_ETREE;
    s_fl[0][me] = 0;
    s_h[0][me] = 0;
    s_cx[0][me] = 0;
    s_first[0][me] = 0;
    bool fresh = true;  // just after a node's '{'
    while (!st) {
      // next member of the node at depth d, or its end
      bool close = false;
      if (fresh) {
        close = tx.lit('}');
      } else if (tx.lit(',')) {
        close = false;
      } else if (tx.lit('}')) {
        close = true;
      } else {
        st = EVM_ETREE;
        break;
      }
      fresh = false;
      if (!close) {
        const int k = tx.key();
        const uint8_t fl = s_fl[d][me];
        if (k < 0 || (fl >> k) & 1u || !tx.lit(':')) {
          st = EVM_ETREE;
          break;
        }
        s_fl[d][me] = fl | (uint8_t)(1u << k);
        if (k == 3) {
          int32_t h;
          if (!tx.integer(&h)) {
            st = EVM_ETREE;
            break;
          }
          s_h[d][me] = h;
          continue;
        }
        if (d >= CODE_DIGITS) {
          st = EVM_ETREE;
          break;
        }
        const int sh = 2 * (CODE_DIGITS - 1 - d);
        prefix |= (u64)(k + 1) << sh;
        ++d;
        s_fl[d][me] = 0;
        s_h[d][me] = 0;
        s_cx[d][me] = 0;
        s_first[d][me] = (u32)cnt;
        if (!tx.lit('{')) {
          st = EVM_ETREE;
          break;
        }
        fresh = true;
        continue;
      }
      // the node at depth d ends
      const uint8_t fl = s_fl[d][me];
      const bool seen_h = (fl >> 3) & 1u, any = (fl >> 4) & 1u;
      const int32_t h = s_h[d][me], cx = s_cx[d][me];
      if (d == 0) {  // the root: {} only, or children + a hash equal to their XOR
        if (seen_h ? !(any && (h ^ cx) == 0) : any) st = EVM_ETREE;
        break;
      }
      if (!seen_h) {
        st = EVM_ETREE;
        break;
      }
      const int32_t t = h ^ cx;
      if (!any || t != 0) {
        // a node closes after its subtree's leaves, whose codes extend its
        // own: it goes in front of them (a node with children and its own
        // leaf -- a shorter key -- is rare), after every leaf read before
        const u64 at = s_first[d][me];
        if (at && (ck[b0 + at - 1] & CODE_MASK40) >= prefix) {
          st = EVM_TREE_UNSORTED;  // (children keys not ascending: the host parser sorts)
          break;
        }
        if (cnt >= bound) {
          st = EVM_ETREE;
          break;
        }
        for (u64 i = cnt; i > at; --i) {
          ck[b0 + i] = ck[b0 + i - 1];
          xr[b0 + i] = xr[b0 + i - 1];
          pfx[b0 + i] = pfx[b0 + i - 1] ^ t;
        }
        ck[b0 + at] = ((u64)o << 40) | prefix;
        xr[b0 + at] = t;
        if (at == cnt) pfx[b0 + at] = run;
        run ^= t;
        ++cnt;
      }
      // back to the parent: its children's XOR and presence
      --d;
      s_cx[d][me] ^= h;
      s_fl[d][me] |= 0x10;
      prefix &= ~((4ull << (2 * (CODE_DIGITS - 1 - d))) - 1ull);  // (the digit at depth d and below)
    }
    if (!st) {
      tx.ws();
      if (tx.p != tx.e) st = EVM_ETREE;
    }
  }
  if (st) cnt = 0;
  pfx[b0 + cnt] = st ? 0 : run;
  t_end[o] = b0 + cnt;
  status[o] = st;
  if (cnt) atomicAdd(n_leaves, cnt);
}

// leaf slots per owner: the bound on its nodes + 1 (the root's prefix slot)
__global__ void k_json_bound(const u64* __restrict__ jlen, u32 n, u64* __restrict__ slots) {
  for (u32 o = blockIdx.x * blockDim.x + threadIdx.x; o < n; o += gridDim.x * blockDim.x)
    slots[o] = json_slot_bound(jlen[o]);
}

// -------------------------------------------------------------- responses
// A message log segment as the device reads it (evm_pb_encode_responses'
// seg_* arrays): ids [base, next base), row = id - base or row[id - base],
// 46-B timestamp at ts + row * stride, content [coff[row], coff[row + 1]).
struct DSeg {
  u64 base;
  const u64* row;
  const char* ts;
  const u64* coff;
  const uint8_t* content;
};

__device__ __forceinline__ u32 vlen(u64 v) {
  u32 k = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++k;
  }
  return k;
}
__device__ __forceinline__ u32 put_varint(uint8_t* d, u64 v) {
  u32 k = 0;
  while (v >= 0x80) {
    d[k++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  d[k++] = (uint8_t)v;
  return k;
}

__device__ __forceinline__ bool locate(const DSeg* segs, u32 n_seg, u64 id, u64 stride, const char** t,
                                       const uint8_t** c, u64* cl) {
  u32 lo = 0, hi = n_seg;  // first segment with base > id
  while (lo < hi) {
    const u32 m = (lo + hi) >> 1;
    if (segs[m].base <= id) lo = m + 1;
    else hi = m;
  }
  if (lo == 0) return false;
  const DSeg& s = segs[lo - 1];
  const u64 k = id - s.base;
  const u64 row = s.row ? s.row[k] : k;
  *t = s.ts + row * stride;
  const u64 a = s.coff[row], b = s.coff[row + 1];
  *c = s.content + a;
  *cl = b - a;
  return true;
}

// response r's selection: owner owners[r]'s ids (a getMessages selection by
// owner), none when skip[r] -- counts, then the ids back to back
__global__ void k_resp_count(u32 n, const u32* __restrict__ owners, const u64* __restrict__ osel_off,
                             const uint8_t* __restrict__ skip, u32 n_owners, u64* __restrict__ cnt,
                             u32* __restrict__ bad) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const u32 o = owners[r];
    if (o >= n_owners) {
      atomicOr(bad, 1u);
      cnt[r] = 0;
      continue;
    }
    cnt[r] = skip && skip[r] ? 0ull : osel_off[o + 1] - osel_off[o];
  }
}
__global__ void k_resp_expand(u32 n, const u32* __restrict__ owners, const u64* __restrict__ osel_off,
                              const u64* __restrict__ osel_id, const u64* __restrict__ roff, u64* __restrict__ sel) {
  const u32 lane = threadIdx.x & 63;
  for (u32 r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += (gridDim.x * blockDim.x) >> 6) {
    const u64 a = roff[r], m = roff[r + 1] - a;
    if (!m) continue;
    const u64 b = osel_off[owners[r]];
    for (u64 j = lane; j < m; j += 64) sel[a + j] = osel_id[b + j];
  }
}

// bytes of selected message m: `messages` field (1) around {timestamp (1), content (2)}
__global__ void k_resp_msg_size(const u64* __restrict__ sel_id, u64 S, const DSeg* __restrict__ segs, u32 n_seg,
                                u64 stride, u64* __restrict__ msz, u32* __restrict__ bad) {
  for (u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x; m < S; m += (u64)gridDim.x * blockDim.x) {
    const char* t;
    const uint8_t* c;
    u64 cl = 0;
    u64 body = 48;
    if (!locate(segs, n_seg, sel_id[m], stride, &t, &c, &cl)) atomicOr(bad, 1u);
    else if (cl) body += 1 + vlen(cl) + cl;
    msz[m] = 1 + vlen(body) + body;
  }
}

// per response: its messages' bytes + the merkleTree field (2)
__global__ void k_resp_len(u32 n, const u64* __restrict__ sel_off, const u64* __restrict__ mpos,
                           const u64* __restrict__ jlen, u64* __restrict__ rlen) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const u64 jl = jlen[r];
    rlen[r] = (mpos[sel_off[r + 1]] - mpos[sel_off[r]]) + (jl ? 1 + vlen(jl) + jl : 0);
  }
}

// the merkleTree field's header; jdst[r] = where its text goes
__global__ void k_resp_tree_hdr(u32 n, const u64* __restrict__ sel_off, const u64* __restrict__ mpos,
                                const u64* __restrict__ jlen, const u64* __restrict__ out_off, uint8_t* __restrict__ out,
                                u64* __restrict__ jdst) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const u64 jl = jlen[r];
    u64 at = out_off[r] + (mpos[sel_off[r + 1]] - mpos[sel_off[r]]);
    if (jl) {
      out[at++] = (uint8_t)(2u << 3 | 2u);
      at += put_varint(out + at, jl);
    }
    jdst[r] = at;
  }
}

// every selected message's bytes: a wave per 64 messages -- each lane works
// out one message's place, header and sources, then the wave writes the
// messages one after another, a byte per lane (64-B coalesced stores instead
// of ~70 scattered byte stores per lane)
struct RespMsg {
  uint8_t* d;
  const char* t;
  const uint8_t* c;
  u32 cl, hdr, len;
  uint8_t h[12];  // `messages` tag + body length, timestamp tag + 46
};
__global__ __launch_bounds__(256) void k_resp_msgs(u32 n, const u64* __restrict__ sel_off,
                                                   const u64* __restrict__ sel_id, u64 S, const DSeg* __restrict__ segs,
                                                   u32 n_seg, u64 stride, const u64* __restrict__ mpos,
                                                   const u64* __restrict__ out_off, uint8_t* __restrict__ out) {
  __shared__ RespMsg meta[4][64];
  const u32 wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (u64 m0 = ((u64)blockIdx.x * 4 + wv) * 64; m0 < S; m0 += (u64)gridDim.x * 4 * 64) {
    const u64 m = m0 + lane;
    RespMsg& r = meta[wv][lane];  // (built in LDS: a local copy with its byte array would live in scratch)
    r.len = 0;
    if (m < S) {
      u32 lo = 0, hi = n;  // the response: last q with sel_off[q] <= m
      while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (sel_off[mid + 1] <= m) lo = mid + 1;
        else hi = mid;
      }
      const char* t;
      const uint8_t* c;
      u64 cl = 0;
      if (locate(segs, n_seg, sel_id[m], stride, &t, &c, &cl)) {  // (a miss: reported by k_resp_msg_size)
        r.d = out + out_off[lo] + (mpos[m] - mpos[sel_off[lo]]);
        r.t = t;
        r.c = c;
        r.cl = (u32)cl;
        const u64 body = 48 + (cl ? 1 + vlen(cl) + cl : 0);
        u32 k = 0;
        r.h[k++] = (uint8_t)(1u << 3 | 2u);
        k += put_varint(r.h + k, body);
        r.h[k++] = (uint8_t)(1u << 3 | 2u);
        r.h[k++] = 46;
        r.hdr = k;
        r.len = k + 46 + (cl ? 1 + vlen(cl) + (u32)cl : 0);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // RG messages x RU passes of 64 bytes loaded before any is stored (a
    // message at a time waited out a load latency per 64 bytes)
    constexpr int RG = 4, RU = 3;
    for (int j0 = 0; j0 < 64; j0 += RG) {
      u32 lmax = 0;
#pragma unroll
      for (int g = 0; g < RG; ++g) lmax = max(lmax, meta[wv][j0 + g].len);
      for (u32 b0 = 0; b0 < lmax; b0 += 64 * RU) {
        // first the loaded bytes (timestamp, content: one load each, no other
        // write to its register while it is in flight), then the headers'
        // bytes and the stores
        uint8_t v[RG][RU];
#pragma unroll
        for (int g = 0; g < RG; ++g)
#pragma unroll
          for (int u = 0; u < RU; ++u) {
            const RespMsg& q = meta[wv][j0 + g];
            const u32 k = b0 + 64 * u + lane, ts_end = q.hdr + 46, vl = vlen(q.cl);
            const gu8* p = nullptr;
            if (k < q.len && k >= q.hdr) p = k < ts_end ? (const gu8*)(uintptr_t)q.t + (k - q.hdr)
                                           : k > ts_end + vl ? (const gu8*)(uintptr_t)q.c + (k - ts_end - 1 - vl) : nullptr;
            v[g][u] = p ? *p : (uint8_t)0;
          }
        vm_wait_all();
#pragma unroll
        for (int g = 0; g < RG; ++g)
#pragma unroll
          for (int u = 0; u < RU; ++u) {
            const RespMsg& q = meta[wv][j0 + g];
            const u32 k = b0 + 64 * u + lane, ts_end = q.hdr + 46;
            if (k >= q.len) continue;
            uint8_t b = v[g][u];
            if (k < q.hdr) b = q.h[k];
            else if (k >= ts_end) {  // the content field's tag and varint length
              const u32 e = k - ts_end, vl = vlen(q.cl);
              if (e == 0) b = (uint8_t)(2u << 3 | 2u);
              else if (e <= vl) {
                u64 x = q.cl;
                for (u32 z = 1; z < e; ++z) x >>= 7;
                b = (uint8_t)((x & 0x7f) | (e < vl ? 0x80 : 0));
              }
            }
            ((gu8*)(uintptr_t)q.d)[k] = b;
          }
      }
    }
    __builtin_amdgcn_wave_barrier();  // (meta is rewritten by the next round)
  }
}

}  // namespace

// Each owner's leaf slots (the bound on its nodes + 1: json_slot_bound) and
// their exclusive scan, *slots[O] = the total -- launches only (S owns slots).
int evm::json_tree_slots(evm_ctx* ctx, Scratch& S, u32 n_owners, const u64* len, u64** slots) {
  u64* bnd = S.alloc<u64>((size_t)n_owners + 1);
  u64* sl = S.alloc<u64>((size_t)n_owners + 1);
  if (!bnd || !sl) return EVM_ENOMEM;
  if (n_owners) KLAUNCH(k_json_bound, dim3(grid_for(n_owners, 256)), dim3(256), len, n_owners, bnd);
  *slots = sl;
  return scan_exclusive<u64, OpAdd>(ctx, S, bnd, n_owners, sl, sl + n_owners);
}

// The owners' texts into t (gapped, cap >= the slots' total): the wave parser,
// then the exact one for the texts it left; *nl = the leaves (launches only:
// the caller reads *nl into t->n_leaves once the stream has run).
int evm::json_tree_parse(evm_ctx* ctx, u32 n_owners, const uint8_t* json, const u64* at, const u64* len,
                         const u64* slots, int32_t* status, evm_tree* t, u64* nl) {
  HIPR(hipMemsetAsync(nl, 0, sizeof(u64), ctx->stream));
  HIPR(hipMemsetAsync(t->off + n_owners, 0, sizeof(u64), ctx->stream));
  if (n_owners)
    KLAUNCH(k_json_wave, dim3((n_owners + JV_WAVES - 1) / JV_WAVES), dim3(64 * JV_WAVES), json, at, len, n_owners,
            slots, (u64*)t->off, (u64*)t->end, (u64*)t->ck, t->xr, t->pfx, status, nl);
  if (n_owners)
    KLAUNCH(k_json_parse, dim3((n_owners + JP_THREADS - 1) / JP_THREADS), dim3(JP_THREADS), json, at, len, n_owners,
            slots, (u64*)t->off, (u64*)t->end, (u64*)t->ck, t->xr, t->pfx, status, nl);
  return hip_ok(hipGetLastError());
}

extern "C" {

int evm_pb_scan_index_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n,
                          evm_pb_sync* info, int32_t* status, uint64_t* slots) {
  if (!ctx || (n && (!arena || !off || !info || !status)) ||
      (kind != EVM_PB_SYNC_REQUEST && kind != EVM_PB_SYNC_RESPONSE))
    return EVM_EINVAL;
  if (n)
    KLAUNCH(k_pb_scan, dim3(grid_for(n, 64, 1 << 16)), dim3(64), kind, arena, (const u64*)off, n, info, status,
            (u64*)slots);
  return hip_ok(hipGetLastError());
}

int evm_pb_scan_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n, evm_pb_sync* info,
                    int32_t* status) {
  return evm_pb_scan_index_dev(ctx, kind, arena, off, n, info, status, nullptr);
}

int evm_pb_split_index_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n,
                           const int32_t* status, const uint64_t* msg_base, const uint64_t* content_base,
                           const uint32_t* owner_of, char* ts, size_t stride, uint64_t* content_off, uint8_t* content,
                           uint32_t* owner, const uint64_t* slots) {
  if (!ctx || (n && (!arena || !off || !status || !msg_base || !content_base || !ts || !content_off || !content)) ||
      stride < 48 || stride % 16 || (kind != EVM_PB_SYNC_REQUEST && kind != EVM_PB_SYNC_RESPONSE))
    return EVM_EINVAL;
  if (!n) return EVM_OK;
  Scratch S(ctx);
  int st;
  u64 N = 0;
  {
    LandList l;
    l.add(msg_base + n, &N, sizeof(u64));
    if ((st = land_words(ctx, l))) return st;
  }
  u32* bad = S.alloc<u32>(1);
  if (!bad) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  u64* co = reinterpret_cast<u64*>(content_off);
  if (slots) {
    // rows, contents and their offsets in one pass (the bodies' content bases
    // from the caller): no offsets array for a second kernel, no scan
    KLAUNCH(k_pb_rows_idx, dim3(grid_for(n, 4, 1 << 16)), dim3(256), arena, (const u64*)off, n, status,
            (const u64*)msg_base, (const u64*)content_base, (const u64*)slots, owner_of, ts, (u64)stride, co, content,
            owner, bad);
    HIPR(hipMemcpyAsync(co + N, content_base + n, sizeof(u64), hipMemcpyDeviceToDevice, ctx->stream));
  } else {
    u64* cat = S.alloc<u64>(N + 1);
    u64* clen = S.alloc<u64>(N + 1);
    if (!cat || !clen) return EVM_ENOMEM;
    u64* mat = S.alloc<u64>(N + 1);
    u32* mlen = S.alloc<u32>(N + 1);
    if (!mat || !mlen) return EVM_ENOMEM;
    KLAUNCH(k_pb_offsets, dim3(grid_for(n, 64, 1 << 16)), dim3(64), kind, arena, (const u64*)off, n, status,
            (const u64*)msg_base, owner_of, mat, mlen, owner, bad);
    if (N)
      KLAUNCH(k_pb_rows, dim3(grid_for(N, 256, 1 << 16)), dim3(256), arena, (const u64*)mat, (const u32*)mlen, N, ts,
              (u64)stride, cat, clen);
    if ((st = scan_exclusive<u64, OpAdd>(ctx, S, clen, N, co, co + N))) return st;
    if (N) KLAUNCH(k_pb_content, dim3(grid_for(N, 256, 1 << 16)), dim3(256), arena, (const u64*)cat, (const u64*)co, N,
                   content);
  }
  u32 hb = 0;
  {
    LandList l;
    l.add(bad, &hb, sizeof(u32));
    if ((st = land_words(ctx, l))) return st;
  }
  return hb ? EVM_EINVAL : EVM_OK;
}

int evm_pb_split_dev(evm_ctx* ctx, int kind, const uint8_t* arena, const uint64_t* off, uint32_t n,
                     const int32_t* status, const uint64_t* msg_base, const uint64_t* content_base,
                     const uint32_t* owner_of, char* ts, size_t stride, uint64_t* content_off, uint8_t* content,
                     uint32_t* owner) {
  return evm_pb_split_index_dev(ctx, kind, arena, off, n, status, msg_base, content_base, owner_of, ts, stride,
                                content_off, content, owner, nullptr);
}

int evm_gather_spans_dev(evm_ctx* ctx, const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                         const uint64_t* dst_off, uint32_t n, uint8_t* dst) {
  if (!ctx || (n && (!src || !src_off || !len || !dst_off || !dst))) return EVM_EINVAL;
  if (n) KLAUNCH(k_gather_spans, dim3(grid_for(n, 1, 1 << 16)), dim3(64), src, (const u64*)src_off, (const u64*)len,
                 (const u64*)dst_off, n, dst);
  return hip_ok(hipGetLastError());
}

int evm_tree_from_json_dev(evm_ctx* ctx, uint32_t n_owners, const uint8_t* json, const uint64_t* at,
                           const uint64_t* len, int32_t* status, evm_tree** out) {
  if (!ctx || !out || !status || (n_owners && (!json || !at || !len))) return EVM_EINVAL;
  *out = nullptr;
  Scratch S(ctx);
  u64* slots = nullptr;
  u64* nl = S.alloc<u64>(1);
  if (!nl) return EVM_ENOMEM;
  int st = json_tree_slots(ctx, S, n_owners, reinterpret_cast<const u64*>(len), &slots);
  if (st) return st;
  u64 cap = 0;
  HIPR(hipMemcpyAsync(&cap, slots + n_owners, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  evm_tree* t = nullptr;
  if ((st = tree_alloc_gapped(ctx, n_owners, std::max<u64>(cap, 1), &t))) return st;
  st = json_tree_parse(ctx, n_owners, json, reinterpret_cast<const u64*>(at), reinterpret_cast<const u64*>(len), slots,
                       status, t, nl);
  u64 hl = 0;
  if (!st) st = hip_ok(hipMemcpyAsync(&hl, nl, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  if (!st) st = hip_ok(hipStreamSynchronize(ctx->stream));
  if (st) {
    tree_destroy(ctx, t);
    return st;
  }
  t->n_leaves = hl;
  *out = t;
  return EVM_OK;
}

}  // extern "C"

// SyncResponse bodies in one pass over the plan: the sizes, then `out(total)`
// (the caller's buffer of >= total bytes, or null: sizes only), then the bytes.
int evm::encode_responses_dev(evm_ctx* ctx, uint32_t n, const evm_tree* tree, const uint32_t* owners,
                              const uint64_t* osel_off, const uint64_t* osel_id, const uint8_t* skip, uint32_t n_seg,
                              const uint64_t* seg_base, const uint64_t* const* seg_row, const char* const* seg_ts,
                              size_t stride, const uint64_t* const* seg_coff, const uint8_t* const* seg_content,
                              const std::function<uint8_t*(uint64_t)>& out_for, uint64_t* out_off, uint64_t* total,
                              const JsonPlan* pre, const uint64_t* pre_jlen, const uint32_t* pre_bad) {
  if (!ctx || !tree || !total || (n && (!owners || !osel_off || !out_off)) || stride < 46 ||
      (n_seg && (!seg_base || !seg_ts || !seg_coff || !seg_content)))
    return EVM_EINVAL;
  *total = 0;
  Scratch S(ctx);
  int st;
  // the responses' selections back to back: sel_off (n + 1), sel_id
  u64* rcnt = S.alloc<u64>((size_t)n + 1);
  u64* sel_off = S.alloc<u64>((size_t)n + 1);
  u32* bad0 = S.alloc<u32>(1);
  if (!rcnt || !sel_off || !bad0) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(bad0, 0, sizeof(u32), ctx->stream));
  if (n)
    KLAUNCH(k_resp_count, dim3(grid_for(n, 256)), dim3(256), n, owners, (const u64*)osel_off, skip, tree->n_owners,
            rcnt, bad0);
  if ((st = scan_exclusive<u64, OpAdd>(ctx, S, rcnt, n, sel_off, sel_off + n))) return st;
  u64 hs[2] = {0, 0};
  u32 hb0 = 0;
  {
    LandList l;
    l.add(sel_off + n, &hs[0], sizeof(u64));
    l.add(bad0, &hb0, sizeof(u32));
    if ((st = land_words(ctx, l))) return st;
  }
  if (hb0) return EVM_EINVAL;
  const u64 NS = hs[0];
  if (NS && !osel_id) return EVM_EINVAL;
  u64* sel_id = S.alloc<u64>(NS + 1);
  if (!sel_id) return EVM_ENOMEM;
  if (NS)
    KLAUNCH(k_resp_expand, dim3(grid_for((size_t)n * 64, 256)), dim3(256), n, owners, (const u64*)osel_off,
            (const u64*)osel_id, (const u64*)sel_off, sel_id);
  std::vector<DSeg> hseg(n_seg);
  for (u32 s = 0; s < n_seg; ++s) {
    hseg[s] = DSeg{seg_base[s], seg_row ? (const u64*)seg_row[s] : nullptr, seg_ts[s], (const u64*)seg_coff[s],
                   seg_content[s]};
    if (s && seg_base[s] < seg_base[s - 1]) return EVM_EINVAL;
  }
  DSeg* dseg = S.alloc<DSeg>(std::max<u32>(n_seg, 1));
  u64* jlen = S.alloc<u64>((size_t)n + 1);
  u64* msz = S.alloc<u64>(NS + 1);
  u64* mpos = S.alloc<u64>(NS + 1);
  u64* rlen = S.alloc<u64>((size_t)n + 1);
  u64* jdst = S.alloc<u64>((size_t)n + 1);
  u32* bad = S.alloc<u32>(1);
  if (!dseg || !jlen || !msz || !mpos || !rlen || !jdst || !bad) return EVM_ENOMEM;
  if (n_seg) HIPR(hipMemcpyAsync(dseg, hseg.data(), sizeof(DSeg) * n_seg, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  // (the emitter reads a gapped tree as it lies -- an empty store's ingest
  // leaves one: no compaction pass, 1.2 ms of config 3's round)
  JsonPlan jplan;
  if (pre) {
    jplan = *pre;
    jlen = reinterpret_cast<u64*>(const_cast<uint64_t*>(pre_jlen));
  } else if ((st = json_plan(ctx, S, tree, owners, n, reinterpret_cast<uint64_t*>(jlen), bad, &jplan))) {
    return st;
  }
  if (NS)
    KLAUNCH(k_resp_msg_size, dim3(grid_for(NS, 256)), dim3(256), (const u64*)sel_id, NS, (const DSeg*)dseg, n_seg,
            (u64)stride, msz, bad);
  if ((st = scan_exclusive<u64, OpAdd>(ctx, S, msz, NS, mpos, mpos + NS))) return st;
  if (n)
    KLAUNCH(k_resp_len, dim3(grid_for(n, 256)), dim3(256), n, (const u64*)sel_off, (const u64*)mpos, (const u64*)jlen,
            rlen);
  u64* doff = reinterpret_cast<u64*>(out_off);
  if ((st = scan_exclusive<u64, OpAdd>(ctx, S, rlen, n, doff, doff + n))) return st;
  u32 hb = 0, hpb = 0;
  {
    LandList l;
    l.add(doff + n, &hs[1], sizeof(u64));
    l.add(bad, &hb, sizeof(u32));
    if (pre_bad) l.add(pre_bad, &hpb, sizeof(u32));
    if ((st = land_words(ctx, l))) return st;
  }
  if (hb || hpb) return EVM_EINVAL;  // (an owner out of range, or an id in no segment)
  *total = hs[1];
  uint8_t* out = out_for(hs[1]);
  if (!out) return EVM_OK;
  if (n)
    KLAUNCH(k_resp_tree_hdr, dim3(grid_for(n, 256)), dim3(256), n, (const u64*)sel_off, (const u64*)mpos,
            (const u64*)jlen, (const u64*)doff, out, jdst);
  // the messages' bytes (memory-bound) on the second stream beside the tree
  // texts (VALU-bound): disjoint bytes of the responses, joined on the way out
  SideFork side(ctx);
  if (NS) {
    const hipStream_t ms = side.stream();
    evm::ProfScope ps_(ctx, "k_resp_msgs", ms);
    hipLaunchKernelGGL(k_resp_msgs, dim3(grid_for((NS + 63) / 64, 4)), dim3(256), 0, ms, n, (const u64*)sel_off,
                       (const u64*)sel_id, NS, (const DSeg*)dseg, n_seg, (u64)stride, (const u64*)mpos,
                       (const u64*)doff, out);
  }
  if ((st = json_emit(ctx, tree, owners, n, jplan, reinterpret_cast<const uint64_t*>(jdst), reinterpret_cast<char*>(out))))
    return st;
  side.join();
  return hip_ok(hipGetLastError());
}

extern "C" int evm_pb_encode_responses_dev(evm_ctx* ctx, uint32_t n, const evm_tree* tree, const uint32_t* owners,
                                           const uint64_t* osel_off, const uint64_t* osel_id, const uint8_t* skip,
                                           uint32_t n_seg, const uint64_t* seg_base, const uint64_t* const* seg_row,
                                           const char* const* seg_ts, size_t stride,
                                           const uint64_t* const* seg_coff, const uint8_t* const* seg_content,
                                           uint8_t* out, size_t cap, uint64_t* out_off, uint64_t* total) {
  bool small = false;
  const int st = evm::encode_responses_dev(
      ctx, n, tree, owners, osel_off, osel_id, skip, n_seg, seg_base, seg_row, seg_ts, stride, seg_coff, seg_content,
      [&](uint64_t need) -> uint8_t* {
        if (out && need > cap) {
          small = true;
          return nullptr;
        }
        return out;
      },
      out_off, total);
  return st ? st : small ? EVM_ECAPACITY : EVM_OK;
}
