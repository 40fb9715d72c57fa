// The sync server's request handler as one native call
// (apps/server/src/index.ts:204-251): SyncRequest bodies in, SyncResponse
// bodies out, for every request of a round at once.
//
//   parseBody (:108-116)         evm_pb_scan_index_dev + evm_pb_split_index_dev
//   userId -> the owner's rows   k_dir_find / k_dir_commit: a device hash table
//     (the "message" table's      of userIds -> owner slots (new users take
//     userId column, :64-75)      slots in request order)
//   addMessages (:136-171)       evm_server_ingest_ex (per-request transactions)
//   getMerkleTree + merkleTreeFromString (:118-134, :187)
//                                evm_tree_from_json_dev (+ the host parser for
//                                the rare text whose keys are out of order)
//   getMessages (:173-202)       evm_server_select
//   SyncResponse.toBinary (:233-241)
//                                evm_pb_encode_responses_dev
//
// Host bodies (where = EVM_SYNC_HOST) reach the device through pinned
// chunks: host threads copy chunk k + 1 into one pinned buffer while the
// copy engine moves chunk k out of the other; responses come back the same
// way (evm_sync_fetch).  Nothing in the round is a torch call.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

// (the ABI's uint64_t is unsigned long; the kernels' u64 is unsigned long long)
#define U64P(x) reinterpret_cast<uint64_t*>(x)
#define U64C(x) reinterpret_cast<const uint64_t*>(x)

namespace evm {

// Pinned staging chunks on a copy stream of their own (one set per context).
struct HostStage {
  static constexpr int NB = 3;
  static constexpr size_t CHUNK = (size_t)128 << 20;
  uint8_t* pin[NB] = {};
  hipEvent_t ev[NB] = {};
  hipStream_t cs = nullptr;
  bool ok = false;
};

}  // namespace evm

namespace {

constexpr u32 DIR_EMPTY = 0xffffffffu;
constexpr u32 DIR_PEND = 0x80000000u;  // a provisional entry of this call: DIR_PEND | request

enum : uint8_t { RQ_NEW = 1, RQ_DUP = 2, RQ_NODEBAD = 4, RQ_HANDED = 8, RQ_FULL = 16, RQ_USE = 32, RQ_NONASCII = 64 };

__device__ __forceinline__ u64 key_hash(const uint8_t* p, u32 len) {
  u64 h = 1469598103934665603ull ^ (u64)len;
  for (u32 i = 0; i < len; ++i) {
    h ^= p[i];
    h *= 1099511628211ull;
  }
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  return h ^ (h >> 32);
}

__device__ __forceinline__ bool key_eq(const uint8_t* a, u32 la, const uint8_t* b, u32 lb) {
  if (la != lb) return false;
  for (u32 i = 0; i < la; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__device__ __forceinline__ bool is_hex(uint8_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}

struct Dir {
  u32* table;  // [mask + 1]: a slot, DIR_EMPTY, or DIR_PEND | request (inside one call)
  u32 mask;
  const u64* koff;  // [cap] slot s's key: kbytes[koff[s] .. koff[s] + klen[s])
  const u32* klen;
  const uint8_t* kbytes;
  u32* claim;  // [cap] the epoch of the last call that named the slot (a user twice in one call)
  u32 epoch;
  const uint8_t* flag;  // [cap] 1: handed to the caller
};

// Per request of a round: its userId span in the arena (the directory's key),
// whether it takes part (the body parsed), and whether its nodeId is the
// 16 hex chars NOT LIKE '%' || nodeId is modelled for.
__global__ void k_sync_req(const uint8_t* __restrict__ arena, const u64* __restrict__ off,
                           const evm_pb_sync* __restrict__ info, const int32_t* __restrict__ st, u32 n,
                           u64* __restrict__ koff, u32* __restrict__ klen, uint8_t* __restrict__ rf) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    uint8_t f = 0;
    u64 ko = 0;
    u32 kl = 0;
    if (st[r] == 0) {
      const evm_pb_sync& s = info[r];
      f = RQ_USE;
      ko = off[r] + s.user_off;
      kl = (u32)s.user_len;
      bool ok = s.node_len == 16;
      for (u32 i = 0; ok && i < 16; ++i) ok = is_hex(arena[off[r] + s.node_off + i]);
      if (!ok) f |= RQ_NODEBAD;
      // a userId with a byte >= 0x80: protobuf-ts decodes it as UTF-8 (an
      // invalid sequence becomes U+FFFD, so two byte strings can be one user);
      // the directory keys bytes, so such a request goes to the caller
      bool ascii = true;
      for (u32 i = 0; ascii && i < kl; ++i) ascii = arena[ko + i] < 0x80;
      if (!ascii) f = RQ_NONASCII;
    }
    koff[r] = ko;
    klen[r] = kl;
    rf[r] = f;
  }
}

// Look each request's key up; a key not in the table is entered
// provisionally (DIR_PEND | r) so two requests of one new user meet.  Every
// probe sequence ends: after mask + 1 probes the table counts as full.
__global__ void k_dir_find(Dir d, const uint8_t* __restrict__ src, const u64* __restrict__ soff,
                           const u32* __restrict__ slen, u32 n, uint8_t* __restrict__ rf, u32* __restrict__ slot,
                           u32* __restrict__ tpos, u32* __restrict__ isnew, u64* __restrict__ newlen,
                           u32* __restrict__ cnt) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    uint8_t f = rf[r];
    u32 sl = DIR_EMPTY, tp = DIR_EMPTY;
    if (f & RQ_USE) {
      const uint8_t* k = src + soff[r];
      const u32 L = slen[r];
      u32 p = (u32)key_hash(k, L) & d.mask;
      for (u32 step = 0;; ++step) {
        if (step > d.mask) {
          f |= RQ_FULL;
          atomicOr(&cnt[2], 1u);
          break;
        }
        u32 e = __hip_atomic_load(&d.table[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e == DIR_EMPTY) {
          const u32 old = atomicCAS(&d.table[p], DIR_EMPTY, DIR_PEND | r);
          if (old == DIR_EMPTY) {
            f |= RQ_NEW;
            tp = p;
            break;
          }
          e = old;
        }
        if (e & DIR_PEND) {
          const u32 q = e & ~DIR_PEND;
          if (key_eq(k, L, src + soff[q], slen[q])) {
            f |= RQ_DUP;
            atomicOr(&cnt[1], 1u);
            break;
          }
        } else if (key_eq(k, L, d.kbytes + d.koff[e], d.klen[e])) {
          sl = e;
          if (atomicExch(&d.claim[e], d.epoch) == d.epoch) {
            f |= RQ_DUP;
            atomicOr(&cnt[1], 1u);
          }
          if (d.flag[e]) f |= RQ_HANDED;
          break;
        }
        p = (p + 1) & d.mask;
      }
    }
    rf[r] = f;
    slot[r] = sl;
    tpos[r] = tp;
    isnew[r] = (f & RQ_NEW) ? 1u : 0u;
    newlen[r] = (f & RQ_NEW) ? (u64)slen[r] : 0ull;
  }
}

// Commit the new users (slots in request order: users0 + rank, key bytes
// appended) or take the provisional entries back out (rollback: the table is
// exactly as before the call -- the entries only ever filled empty places).
// A user whose nodeId is not modelled is handed over for good.
__global__ void k_dir_commit(u32* __restrict__ table, u32 n, const uint8_t* __restrict__ rf,
                             const u32* __restrict__ tpos, const u32* __restrict__ rank, const u64* __restrict__ kpos,
                             u32 users0, u64 kused0, const uint8_t* __restrict__ src, const u64* __restrict__ soff,
                             const u32* __restrict__ slen, u64* __restrict__ koff, u32* __restrict__ klen,
                             uint8_t* __restrict__ kbytes, u32* __restrict__ slot, uint8_t* __restrict__ flag,
                             u32* __restrict__ claim, u32 epoch, int rollback) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const uint8_t f = rf[r];
    if (f & RQ_NEW) {
      if (rollback) {
        table[tpos[r]] = DIR_EMPTY;
        continue;
      }
      const u32 s = users0 + rank[r];
      const u64 ko = kused0 + kpos[r];
      const u32 L = slen[r];
      const uint8_t* k = src + soff[r];
      for (u32 i = 0; i < L; ++i) kbytes[ko + i] = k[i];
      koff[s] = ko;
      klen[s] = L;
      claim[s] = epoch;
      flag[s] = 0;
      slot[r] = s;
      __threadfence();
      table[tpos[r]] = s;
    }
    if (!rollback && (f & RQ_NODEBAD) && slot[r] != DIR_EMPTY) flag[slot[r]] = 1;
  }
}

__global__ void k_set_u8(uint8_t* p, u32 i, uint8_t v) { p[i] = v; }
__global__ void k_fill_u32(u32* p, size_t n, u32 v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// Rounds' per-request bookkeeping on the device (request r of the call):
// which owner slot it answers and where its client tree lies.
enum : uint8_t { RC_ACTIVE = 0, RC_OUT = 1, RC_REJECTED = 2, RC_ETREE = 3, RC_UNSORTED = 4 };

// at/len of each included request's client tree (by slot; the kernel that
// parses reads the texts where they lie).  It runs beside the ingest, so the
// owners the ingest rejects are parsed too and turned away by k_sync_reject.
__global__ void k_sync_trees(const u64* __restrict__ off, const evm_pb_sync* __restrict__ info, u32 n,
                             const uint8_t* __restrict__ incl, const u32* __restrict__ slot, u64* __restrict__ at,
                             u64* __restrict__ len, uint8_t* __restrict__ rc) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    uint8_t c = RC_OUT;
    if (incl[r]) {
      const u32 s = slot[r];
      if (info[r].tree_len == 0) {
        c = RC_ETREE;  // JSON.parse("") throws (an absent merkleTree decodes as "")
      } else {
        at[s] = off[r] + info[r].tree_off;
        len[s] = info[r].tree_len;
        c = RC_ACTIVE;
      }
    }
    rc[r] = c;
  }
}

// the owners the ingest rejected (a row outside the domain: the request's
// transaction rolled back) answer nothing, whatever their trees
__global__ void k_sync_reject(u32 n, const uint8_t* __restrict__ incl, const u32* __restrict__ slot,
                              const uint8_t* __restrict__ ostat, uint8_t* __restrict__ rc) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x)
    if (incl[r] && ostat[slot[r]]) rc[r] = RC_REJECTED;
}

// the parse's verdict per request; the requester's nodeId and the active
// mask by slot for getMessages
__global__ void k_sync_active(const uint8_t* __restrict__ arena, const u64* __restrict__ off,
                              const evm_pb_sync* __restrict__ info, u32 n, const u32* __restrict__ slot,
                              const int32_t* __restrict__ tst, uint8_t* __restrict__ rc, uint8_t* __restrict__ node,
                              uint8_t* __restrict__ active) {
  for (u32 r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    if (rc[r] != RC_ACTIVE) continue;
    const u32 s = slot[r];
    const int32_t t = tst[s];
    if (t == EVM_TREE_UNSORTED) {
      rc[r] = RC_UNSORTED;
      continue;
    }
    if (t != 0) {
      rc[r] = RC_ETREE;
      continue;
    }
    const uint8_t* nd = arena + off[r] + info[r].node_off;
    for (int i = 0; i < 16; ++i) node[(size_t)s * 16 + i] = nd[i];
    active[s] = 1;
  }
}

// answered requests (request order): their owner slots; their RangeError skips
__global__ void k_sync_owners(const u32* __restrict__ ans, u32 na, const u32* __restrict__ slot,
                              u32* __restrict__ owners) {
  for (u32 j = blockIdx.x * blockDim.x + threadIdx.x; j < na; j += gridDim.x * blockDim.x) owners[j] = slot[ans[j]];
}
__global__ void k_sync_answer(const u32* __restrict__ ans, u32 na, const u32* __restrict__ slot,
                              const int64_t* __restrict__ diff, uint8_t* __restrict__ skip) {
  for (u32 j = blockIdx.x * blockDim.x + threadIdx.x; j < na; j += gridDim.x * blockDim.x)
    skip[j] = diff[slot[ans[j]]] == EVM_DIFF_RANGE_ERROR ? 1 : 0;
}

// evm_sync_log_read: per id its segment row -> the 46-B timestamp and the
// content's span (pass 1), then the contents (pass 2)
struct LSeg {
  u64 base;
  u64 n;
  const uint8_t* ts;
  const u64* coff;
  const uint8_t* content;
};
__device__ __forceinline__ int lseg_of(const LSeg* s, u32 ns, u64 id) {
  int lo = 0, hi = (int)ns;  // last segment with base <= id
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid].base <= id) lo = mid + 1;
    else hi = mid;
  }
  return lo - 1;
}
__global__ void k_log_spans(const LSeg* __restrict__ sg, u32 ns, const u64* __restrict__ ids, u64 n, char* __restrict__ ts,
                            u64* __restrict__ clen, u32* __restrict__ bad) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const int s = lseg_of(sg, ns, ids[i]);
    if (s < 0 || ids[i] - sg[s].base >= sg[s].n) {
      atomicOr(bad, 1u);
      clen[i] = 0;
      continue;
    }
    const u64 k = ids[i] - sg[s].base;
    for (int j = 0; j < 46; ++j) ts[i * 46 + j] = (char)sg[s].ts[k * 48 + j];
    clen[i] = sg[s].coff[k + 1] - sg[s].coff[k];
  }
}
__global__ void k_log_content(const LSeg* __restrict__ sg, u32 ns, const u64* __restrict__ ids, u64 n,
                              const u64* __restrict__ cpos, uint8_t* __restrict__ out) {
  for (u64 i = blockIdx.x; i < n; i += gridDim.x) {
    const int s = lseg_of(sg, ns, ids[i]);
    if (s < 0 || ids[i] - sg[s].base >= sg[s].n) continue;
    const u64 k = ids[i] - sg[s].base;
    const u64 a = sg[s].coff[k], b = sg[s].coff[k + 1];
    for (u64 j = a + threadIdx.x; j < b; j += blockDim.x) out[cpos[i] + j - a] = sg[s].content[j];
  }
}

template <typename F>
void host_parallel(size_t n, int threads, F f) {  // f(begin, end) over disjoint runs of [0, n)
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, n / ((size_t)1 << 20) + 1));
  if (T <= 1) {
    f((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k) th.emplace_back([=]() { f(n * k / T, n * (k + 1) / T); });
  for (auto& x : th) x.join();
}

int stage_threads() {
  int t = (int)std::thread::hardware_concurrency();
  if (const char* e = getenv("EVM_HOST_THREADS")) t = atoi(e);
  return std::max(1, std::min(t, 16));
}

int stage_get(evm_ctx* ctx, HostStage** out) {
  if (!ctx->stage) {
    HostStage* h = new HostStage;
    bool ok = hipStreamCreateWithFlags(&h->cs, hipStreamNonBlocking) == hipSuccess;
    for (int b = 0; ok && b < HostStage::NB; ++b)
      ok = hipHostMalloc(reinterpret_cast<void**>(&h->pin[b]), HostStage::CHUNK, hipHostMallocDefault) == hipSuccess &&
           hipEventCreateWithFlags(&h->ev[b], hipEventDisableTiming) == hipSuccess;
    h->ok = ok;
    ctx->stage = h;
  }
  *out = ctx->stage;
  return ctx->stage->ok ? EVM_OK : EVM_ENOMEM;
}

// host -> device through the pinned chunks: chunk k's copy-in on host threads
// while the copy engine still moves chunk k - 1 (and k - 2); ctx->stream waits
// for the last chunk
int stage_h2d(evm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  HostStage* h;
  int st = stage_get(ctx, &h);
  if (st) return st;
  const int T = stage_threads();
  size_t k = 0;
  for (size_t a = 0; a < bytes; a += HostStage::CHUNK, ++k) {
    const int b = (int)(k % HostStage::NB);
    const size_t m = std::min(HostStage::CHUNK, bytes - a);
    HIPR(hipEventSynchronize(h->ev[b]));  // (the chunk's previous transfer is done with it)
    const uint8_t* s = static_cast<const uint8_t*>(src) + a;
    uint8_t* p = h->pin[b];
    host_parallel(m, T, [&](size_t x, size_t y) { memcpy(p + x, s + x, y - x); });
    HIPR(hipMemcpyAsync(static_cast<uint8_t*>(dst) + a, p, m, hipMemcpyHostToDevice, h->cs));
    HIPR(hipEventRecord(h->ev[b], h->cs));
  }
  HIPR(hipEventRecord(h->ev[0], h->cs));
  HIPR(hipStreamWaitEvent(ctx->stream, h->ev[0], 0));
  return EVM_OK;
}

// device -> host the same way: the copy engine fills chunk k + 1 while host
// threads copy chunk k out
int stage_d2h(evm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  HostStage* h;
  int st = stage_get(ctx, &h);
  if (st) return st;
  HIPR(hipEventRecord(h->ev[0], ctx->stream));  // (src is written on ctx->stream)
  HIPR(hipStreamWaitEvent(h->cs, h->ev[0], 0));
  const int T = stage_threads();
  const size_t nk = (bytes + HostStage::CHUNK - 1) / HostStage::CHUNK;
  auto issue = [&](size_t k) -> int {
    const int b = (int)(k % HostStage::NB);
    const size_t a = k * HostStage::CHUNK, m = std::min(HostStage::CHUNK, bytes - a);
    HIPR(hipMemcpyAsync(h->pin[b], static_cast<const uint8_t*>(src) + a, m, hipMemcpyDeviceToHost, h->cs));
    HIPR(hipEventRecord(h->ev[b], h->cs));
    return EVM_OK;
  };
  for (size_t k = 0; k < nk && k < (size_t)HostStage::NB - 1; ++k)
    if ((st = issue(k))) return st;
  for (size_t k = 0; k < nk; ++k) {
    const int b = (int)(k % HostStage::NB);
    HIPR(hipEventSynchronize(h->ev[b]));
    const size_t a = k * HostStage::CHUNK, m = std::min(HostStage::CHUNK, bytes - a);
    const uint8_t* p = h->pin[b];
    uint8_t* d = static_cast<uint8_t*>(dst) + a;
    host_parallel(m, T, [&](size_t x, size_t y) { memcpy(d + x, p + x, y - x); });
    if (k + HostStage::NB - 1 < nk && (st = issue(k + HostStage::NB - 1))) return st;
  }
  return EVM_OK;
}

}  // namespace

void evm_host_stage_free(evm_ctx* ctx) {
  HostStage* h = ctx->stage;
  if (!h) return;
  if (h->cs) (void)hipStreamSynchronize(h->cs);
  for (int b = 0; b < HostStage::NB; ++b) {
    if (h->pin[b]) (void)hipHostFree(h->pin[b]);
    if (h->ev[b]) (void)hipEventDestroy(h->ev[b]);
  }
  if (h->cs) (void)hipStreamDestroy(h->cs);
  delete h;
  ctx->stage = nullptr;
}

// A message-log segment: rows [base, base + n), held in one device block.
struct SyncSeg {
  u64 base, n;
  uint8_t* ts;  // n x 48
  u64* coff;    // n + 1
  uint8_t* content;
  void* block;
  size_t bytes;
};

struct evm_sync_server {
  evm_ctx* ctx;
  evm_store* store;
  u32 cap = 0;  // owner slots (the store's owners)
  // the directory
  u32* table = nullptr;
  u32 mask = 0;
  u64* koff = nullptr;
  u32* klen = nullptr;
  u32* claim = nullptr;
  uint8_t* flag = nullptr;
  uint8_t* kbytes = nullptr;
  u64 kcap = 0, kused = 0;
  u32 users = 0;
  u32 epoch = 0;
  // the message log
  std::vector<SyncSeg> segs;
  u64 next_id = 0;
  // the last round's responses (device) and the host round's bodies (device)
  uint8_t* resp = nullptr;
  size_t resp_bytes = 0, resp_used = 0;
  uint8_t* din = nullptr;
  size_t din_bytes = 0;
  // pinned host scratch for the round's small arrays
  uint8_t* hbuf = nullptr;
  size_t hbuf_bytes = 0;
  // the last round's wall time by part (ms): h2d, decode, users, ingest, trees, select, encode, d2h
  double part_ms[8] = {};
  // the round's second stream: the client trees are parsed there while the
  // messages are split and ingested on the context's stream
  hipStream_t ps = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int hbuf_need(evm_sync_server* s, size_t bytes) {
  if (s->hbuf_bytes >= bytes) return EVM_OK;
  if (s->hbuf) (void)hipHostFree(s->hbuf);
  s->hbuf = nullptr;
  s->hbuf_bytes = 0;
  const size_t want = bytes + bytes / 4 + 4096;
  if (hipHostMalloc(reinterpret_cast<void**>(&s->hbuf), want, hipHostMallocDefault) != hipSuccess) return EVM_ENOMEM;
  s->hbuf_bytes = want;
  return EVM_OK;
}

int kbytes_need(evm_sync_server* s, u64 more) {
  evm_ctx* ctx = s->ctx;
  if (s->kused + more <= s->kcap) return EVM_OK;
  u64 want = std::max<u64>(s->kcap * 2, s->kused + more + 4096);
  uint8_t* nb = nullptr;
  HIPR(hipMallocAsync(reinterpret_cast<void**>(&nb), want, ctx->stream));
  if (s->kused) HIPR(hipMemcpyAsync(nb, s->kbytes, s->kused, hipMemcpyDeviceToDevice, ctx->stream));
  if (s->kbytes) HIPR(hipFreeAsync(s->kbytes, ctx->stream));
  s->kbytes = nb;
  s->kcap = want;
  return EVM_OK;
}

inline u64 align256(u64 x) { return (x + 255) & ~(u64)255; }

// a new log segment of n rows and cb content bytes (one device block)
int seg_alloc(evm_sync_server* s, u64 n, u64 cb, SyncSeg* g) {
  const u64 a = align256(n * 48 + 16), b = align256((n + 1) * 8), c = align256(cb + 16);
  size_t bytes = a + b + c;
  void* p = block_alloc(s->ctx, &bytes);
  if (!p) return EVM_ENOMEM;
  g->base = s->next_id;
  g->n = n;
  g->ts = static_cast<uint8_t*>(p);
  g->coff = reinterpret_cast<u64*>(static_cast<uint8_t*>(p) + a);
  g->content = static_cast<uint8_t*>(p) + a + b;
  g->block = p;
  g->bytes = bytes;
  return EVM_OK;
}

// users looked up / entered: keys src[soff[r] .. + slen[r]) (device), rf
// from k_sync_req or RQ_USE; outputs slot (device [n]) and the landed flags
int dir_resolve(evm_sync_server* s, Scratch& S, const uint8_t* src, const u64* soff, const u32* slen, u32 n,
                uint8_t* rf, u32* slot, u64 key_bytes, int insert, uint8_t* rf_host_out) {
  evm_ctx* ctx = s->ctx;
  int st;
  if ((st = kbytes_need(s, key_bytes))) return st;
  u32* tpos = S.alloc<u32>(n);
  u32* isnew = S.alloc<u32>(n);
  u64* nlen = S.alloc<u64>(n);
  u32* rank = S.alloc<u32>(n);
  u64* kpos = S.alloc<u64>(n);
  u32* cnt = S.alloc<u32>(4);
  u32* nnew = S.alloc<u32>(1);
  u64* ktot = S.alloc<u64>(1);
  if (!tpos || !isnew || !nlen || !rank || !kpos || !cnt || !nnew || !ktot) return EVM_ENOMEM;
  HIPR(hipMemsetAsync(cnt, 0, 4 * sizeof(u32), ctx->stream));
  if (++s->epoch == 0) s->epoch = 1;  // (claims start at 0: never an epoch)
  Dir d{s->table, s->mask, s->koff, s->klen, s->kbytes, s->claim, s->epoch, s->flag};
  KLAUNCH(k_dir_find, dim3(grid_for(n, 256)), dim3(256), d, src, soff, slen, n, rf, slot, tpos, isnew, nlen, cnt);
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, isnew, n, rank, nnew))) return st;
  if ((st = scan_exclusive<u64, OpAdd>(ctx, S, nlen, n, kpos, ktot))) return st;
  u32 hc[4] = {0, 0, 0, 0};
  u64 hk = 0;
  {
    LandList l;
    l.add(cnt, hc, 3 * sizeof(u32));
    l.add(nnew, &hc[3], sizeof(u32));
    l.add(ktot, &hk, sizeof(u64));
    if ((st = land_words(ctx, l))) return st;
  }
  const u32 n_new = hc[3];
  int ret = EVM_OK;
  if (hc[1]) ret = EVM_EROUNDS;
  else if (hc[2] || (u64)s->users + n_new > s->cap || (!insert && n_new)) ret = insert ? EVM_ECAPACITY : EVM_OK;
  const int rollback = (ret != EVM_OK || !insert) ? 1 : 0;
  KLAUNCH(k_dir_commit, dim3(grid_for(n, 256)), dim3(256), s->table, n, rf, tpos, rank, kpos, s->users, s->kused, src,
          soff, slen, s->koff, s->klen, s->kbytes, slot, s->flag, s->claim, s->epoch, rollback);
  if (rf_host_out) HIPR(hipMemcpyAsync(rf_host_out, rf, n, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (ret) return ret;
  if (insert) {
    s->kused += hk;
    s->users += n_new;
  }
  return EVM_OK;
}

int round_dev(evm_sync_server* sv, const uint8_t* arena, const u64* off_h, u32 n, int32_t* result, u64* resp_off,
              u64* resp_total) {
  evm_ctx* ctx = sv->ctx;
  int st;
  *resp_total = 0;
  sv->resp_used = 0;
  for (u32 k = 0; k <= n; ++k) resp_off[k] = 0;
  if (n == 0) return EVM_OK;
  const u32 O = sv->cap;
  double t0 = now_ms(), t1;
  for (int k = 1; k < 7; ++k) sv->part_ms[k] = 0;
  auto stamp = [&](int part) {
    t1 = now_ms();
    sv->part_ms[part] += t1 - t0;
    t0 = t1;
  };
  Scratch S(ctx);
  // ---- parseBody: scan every body (sizes, the string fields, each message's place)
  u64* off_d = S.alloc<u64>((size_t)n + 1);
  evm_pb_sync* info_d = S.alloc<evm_pb_sync>(n);
  int32_t* st_d = S.alloc<int32_t>(n);
  u64* mslot = S.alloc<u64>(off_h[n] / 50 + 1);
  u64* koff_r = S.alloc<u64>(n);
  u32* klen_r = S.alloc<u32>(n);
  uint8_t* rf = S.alloc<uint8_t>(n);
  u32* slot_d = S.alloc<u32>(n);
  if (!off_d || !info_d || !st_d || !mslot || !koff_r || !klen_r || !rf || !slot_d) return EVM_ENOMEM;
  HIPR(hipMemcpyAsync(off_d, off_h, sizeof(u64) * ((size_t)n + 1), hipMemcpyHostToDevice, ctx->stream));
  if ((st = evm_pb_scan_index_dev(ctx, EVM_PB_SYNC_REQUEST, arena, U64C(off_d), n, info_d, st_d, U64P(mslot)))) return st;
  KLAUNCH(k_sync_req, dim3(grid_for(n, 256)), dim3(256), arena, off_d, info_d, st_d, n, koff_r, klen_r, rf);
  // the scan's result to the host (pinned): sizes and statuses
  const size_t hb_info = sizeof(evm_pb_sync) * n, hb_st = sizeof(int32_t) * n;
  if ((st = hbuf_need(sv, hb_info + hb_st + 2 * (size_t)n + 64))) return st;
  evm_pb_sync* info = reinterpret_cast<evm_pb_sync*>(sv->hbuf);
  int32_t* pst = reinterpret_cast<int32_t*>(sv->hbuf + hb_info);
  uint8_t* hrf = sv->hbuf + hb_info + hb_st;
  uint8_t* hrc = hrf + n;
  HIPR(hipMemcpyAsync(info, info_d, hb_info, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(pst, st_d, hb_st, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  u64 key_bytes = 0;
  for (u32 r = 0; r < n; ++r)
    if (pst[r] == 0) key_bytes += info[r].user_len;
  stamp(1);
  // ---- the owners: userId -> slot (new users in request order)
  if ((st = dir_resolve(sv, S, arena, koff_r, klen_r, n, rf, slot_d, key_bytes, 1, hrf))) return st;
  stamp(2);
  // ---- which requests the round applies
  std::vector<uint8_t> incl(n, 0);
  std::vector<int32_t> st_mod(n);
  std::vector<u64> mb(n + 1, 0), cbase(n + 1, 0);
  for (u32 r = 0; r < n; ++r) {
    int32_t code = EVM_OK;
    if (pst[r]) code = EVM_EINVAL;  // SyncRequest.fromBinary threw: 500
    else if (hrf[r] & (RQ_NODEBAD | RQ_HANDED | RQ_NONASCII)) code = EVM_EHANDOVER;
    else if (info[r].nonstd_ts) code = EVM_ENONCANON;  // (a timestamp that is not 46 bytes: outside the domain)
    result[r] = code;
    incl[r] = code == EVM_OK;
    st_mod[r] = incl[r] ? 0 : 1;
    mb[r + 1] = mb[r] + (incl[r] ? info[r].n_messages : 0);
    cbase[r + 1] = cbase[r] + (incl[r] ? info[r].content_bytes : 0);
  }
  const u64 N = mb[n], CB = cbase[n];
  int32_t* stm_d = S.alloc<int32_t>(n);
  u64* mb_d = S.alloc<u64>((size_t)n + 1);
  u64* cb_d = S.alloc<u64>((size_t)n + 1);
  uint8_t* incl_d = S.alloc<uint8_t>(n);
  u32* owner = S.alloc<u32>(N);
  uint8_t* flags = S.alloc<uint8_t>(N);
  uint8_t* ostat = S.alloc<uint8_t>(O);
  if (!stm_d || !mb_d || !cb_d || !incl_d || !owner || !flags || !ostat) return EVM_ENOMEM;
  HIPR(hipMemcpyAsync(stm_d, st_mod.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(mb_d, mb.data(), sizeof(u64) * ((size_t)n + 1), hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(cb_d, cbase.data(), sizeof(u64) * ((size_t)n + 1), hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(incl_d, incl.data(), n, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemsetAsync(ostat, 0, O, ctx->stream));
  // ---- getMerkleTree's client side, forked: the requests' trees parsed where
  // they lie, on the round's second stream (its scratch from S, the tree sized
  // on the host from the texts' lengths: nothing on it waits for the host)
  u64* at = S.alloc<u64>(O);
  u64* ln = S.alloc<u64>(O);
  int32_t* tst = S.alloc<int32_t>(O);
  uint8_t* rc = S.alloc<uint8_t>(n);
  uint8_t* node = S.alloc<uint8_t>((size_t)O * 16);
  uint8_t* active = S.alloc<uint8_t>(O);
  u64* nl = S.alloc<u64>(1);
  if (!at || !ln || !tst || !rc || !node || !active || !nl) return EVM_ENOMEM;
  u64 tcap = 2ull * O;  // (json_slot_bound summed over the owners: an owner without a text takes 2)
  for (u32 r = 0; r < n; ++r)
    if (incl[r]) tcap += json_slot_bound(info[r].tree_len) - 2;
  evm_tree* client = nullptr;
  struct Fork {  // the parse stream joined (and the tree freed on a failure) on every path out
    evm_sync_server* sv;
    evm_tree** client;
    bool open = false, keep = false;
    void join() {
      if (open) (void)hipStreamWaitEvent(sv->ctx->stream, sv->ev_join, 0);
      open = false;
    }
    ~Fork() {
      if (open) (void)hipStreamSynchronize(sv->ps);
      join();
      if (!keep && *client) {
        (void)hipStreamSynchronize(sv->ctx->stream);
        evm_tree_free(sv->ctx, *client);
        *client = nullptr;
      }
    }
  } fork{sv, &client};
  {
    HIPR(hipEventRecord(sv->ev_fork, ctx->stream));
    HIPR(hipStreamWaitEvent(sv->ps, sv->ev_fork, 0));
    fork.open = true;
    const hipStream_t main = ctx->stream;
    ctx->stream = sv->ps;  // (launches only until it is restored: no host sync on either stream)
    u64* slots = nullptr;
    int pst2 = hip_ok(hipMemsetAsync(at, 0, sizeof(u64) * O, ctx->stream));
    if (!pst2) pst2 = hip_ok(hipMemsetAsync(ln, 0, sizeof(u64) * O, ctx->stream));
    if (!pst2) pst2 = hip_ok(hipMemsetAsync(node, '0', (size_t)O * 16, ctx->stream));
    if (!pst2) pst2 = hip_ok(hipMemsetAsync(active, 0, O, ctx->stream));
    if (!pst2) {
      KLAUNCH(k_sync_trees, dim3(grid_for(n, 256)), dim3(256), off_d, info_d, n, incl_d, slot_d, at, ln, rc);
      pst2 = json_tree_slots(ctx, S, O, ln, &slots);
    }
    if (!pst2) pst2 = tree_alloc_gapped(ctx, O, std::max<u64>(tcap, 1), &client);
    if (!pst2) pst2 = json_tree_parse(ctx, O, arena, at, ln, slots, tst, client, nl);
    if (!pst2) pst2 = hip_ok(hipEventRecord(sv->ev_join, ctx->stream));
    ctx->stream = main;
    if (pst2) return pst2;
  }
  // ---- the rows and contents of the round (a new log segment) + addMessages
  if (N) {
    SyncSeg g;
    if ((st = seg_alloc(sv, N, CB, &g))) return st;
    st = evm_pb_split_index_dev(ctx, EVM_PB_SYNC_REQUEST, arena, U64C(off_d), n, stm_d, U64C(mb_d), U64C(cb_d),
                                slot_d, reinterpret_cast<char*>(g.ts), 48, U64P(g.coff), g.content, owner,
                                U64C(mslot));
    if (!st) {
      st = evm_server_ingest_ex(ctx, sv->store, reinterpret_cast<const char*>(g.ts), 48, N, owner, sv->next_id, flags,
                                ostat);
      if (st == EVM_ENONCANON) st = EVM_OK;  // (those owners committed nothing: their requests say so below)
    }
    if (st) {
      block_free(ctx, g.block, g.bytes);
      return st;
    }
    sv->segs.push_back(g);
    sv->next_id += N;
  }
  stamp(3);
  // ---- the parse joined: the ingest's rejections, the parse's verdicts
  fork.join();
  KLAUNCH(k_sync_reject, dim3(grid_for(n, 256)), dim3(256), n, incl_d, slot_d, ostat, rc);
  KLAUNCH(k_sync_active, dim3(grid_for(n, 256)), dim3(256), arena, off_d, info_d, n, slot_d, tst, rc, node, active);
  HIPR(hipMemcpyAsync(hrc, rc, n, hipMemcpyDeviceToHost, ctx->stream));
  u64 hnl = 0;
  HIPR(hipMemcpyAsync(&hnl, nl, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  client->n_leaves = hnl;
  auto free_client = [&]() {
    if (client) evm_tree_free(ctx, client);
    client = nullptr;
  };
  // texts whose keys are out of order (valid JSON JSON.stringify never
  // writes): the host parser reads them, merged into the device's trees
  std::vector<u32> uns;
  for (u32 r = 0; r < n; ++r)
    if (hrc[r] == RC_UNSORTED) uns.push_back(r);
  if (!uns.empty()) {
    std::vector<u32> hslot(n);
    HIPR(hipMemcpy(hslot.data(), slot_d, sizeof(u32) * n, hipMemcpyDeviceToHost));
    std::vector<std::string> texts(uns.size());
    for (size_t j = 0; j < uns.size(); ++j) {
      const u32 r = uns[j];
      texts[j].resize(info[r].tree_len);
      HIPR(hipMemcpy(&texts[j][0], arena + off_h[r] + info[r].tree_off, info[r].tree_len, hipMemcpyDeviceToHost));
    }
    static const char empty[] = "{}";
    std::vector<const char*> ptr(O, empty);
    std::vector<size_t> lens(O, 2);
    std::vector<uint8_t> good(uns.size(), 0);
    for (size_t j = 0; j < uns.size(); ++j) {  // (one by one: a text the host rejects fails alone)
      std::vector<const char*> one(1, texts[j].data());
      std::vector<size_t> l1(1, texts[j].size());
      evm_tree* t1 = nullptr;
      if (evm_tree_from_json(ctx, 1, one.data(), l1.data(), &t1) == EVM_OK) {
        good[j] = 1;
        evm_tree_free(ctx, t1);
        ptr[hslot[uns[j]]] = texts[j].data();
        lens[hslot[uns[j]]] = texts[j].size();
      }
    }
    evm_tree* ht = nullptr;
    if ((st = evm_tree_from_json(ctx, O, ptr.data(), lens.data(), &ht))) {
      free_client();
      return st;
    }
    evm_tree* merged = nullptr;
    st = evm_tree_merge(ctx, client, ht, &merged);
    evm_tree_free(ctx, ht);
    free_client();
    if (st) return st;
    client = merged;
    for (size_t j = 0; j < uns.size(); ++j) {
      const u32 r = uns[j];
      if (!good[j]) {
        hrc[r] = RC_ETREE;
        continue;
      }
      hrc[r] = RC_ACTIVE;
      const u32 s = hslot[r];
      HIPR(hipMemcpyAsync(node + (size_t)s * 16, arena + off_h[r] + info[r].node_off, 16, hipMemcpyDeviceToDevice,
                          ctx->stream));
      KLAUNCH(k_set_u8, dim3(1), dim3(1), active, s, (uint8_t)1);
    }
  }
  stamp(4);
  // ---- getMessages for every answered request
  std::vector<u32> ans;
  for (u32 r = 0; r < n; ++r) {
    if (!incl[r]) continue;
    switch (hrc[r]) {
      case RC_ACTIVE: ans.push_back(r); break;
      case RC_REJECTED: result[r] = EVM_ENONCANON; break;
      case RC_ETREE: result[r] = EVM_ETREE; break;
      default: result[r] = EVM_ETREE; break;
    }
  }
  const u32 na = (u32)ans.size();
  uint64_t nst = 0;
  evm_store_info(sv->store, nullptr, &nst);
  int64_t* diff = S.alloc<int64_t>(O);
  u64* sel_off = S.alloc<u64>((size_t)O + 1);
  u64* sel_id = S.alloc<u64>(nst + 1);
  u32* ans_d = S.alloc<u32>(na);
  u32* owners = S.alloc<u32>(na);
  uint8_t* skip = S.alloc<uint8_t>(na);
  u64* rout = S.alloc<u64>((size_t)na + 1);
  u64* jlen = S.alloc<u64>((size_t)na + 1);
  u32* jbad = S.alloc<u32>(1);
  if (!diff || !sel_off || !sel_id || !ans_d || !owners || !skip || !rout || !jlen || !jbad) {
    free_client();
    return EVM_ENOMEM;
  }
  const evm_tree* tree = evm_store_tree(sv->store);
  // the answered owners, then their tree texts' lengths (k_jp_len) on the
  // second stream while getMessages runs: both only read the store's tree
  JsonPlan jplan;
  if (na) {
    HIPR(hipMemcpyAsync(ans_d, ans.data(), sizeof(u32) * na, hipMemcpyHostToDevice, ctx->stream));
    KLAUNCH(k_sync_owners, dim3(grid_for(na, 256)), dim3(256), ans_d, na, slot_d, owners);
    HIPR(hipMemsetAsync(jbad, 0, sizeof(u32), ctx->stream));
    HIPR(hipEventRecord(sv->ev_fork, ctx->stream));
    HIPR(hipStreamWaitEvent(sv->ps, sv->ev_fork, 0));
    fork.open = true;
    const hipStream_t main = ctx->stream;
    ctx->stream = sv->ps;  // (launches only)
    int pst2 = json_plan(ctx, S, tree, owners, na, reinterpret_cast<uint64_t*>(jlen), jbad, &jplan);
    if (!pst2) pst2 = hip_ok(hipEventRecord(sv->ev_join, ctx->stream));
    ctx->stream = main;
    if (pst2) {
      free_client();
      return pst2;
    }
  }
  uint64_t n_sel = 0;
  st = evm_server_select(ctx, sv->store, client, reinterpret_cast<const char*>(node), active, diff, U64P(sel_off),
                         U64P(sel_id), nst + 1, &n_sel);
  free_client();
  if (st) return st;
  HIPR(hipStreamSynchronize(ctx->stream));
  stamp(5);
  if (!na) return EVM_OK;
  fork.join();
  KLAUNCH(k_sync_answer, dim3(grid_for(na, 256)), dim3(256), ans_d, na, slot_d, diff, skip);
  // ---- SyncResponse.toBinary: sizes, then the bytes into the round's arena
  const u32 ns = (u32)sv->segs.size();
  std::vector<uint64_t> sbase(ns);
  std::vector<const uint64_t*> srow(ns, nullptr), scoff(ns);
  std::vector<const char*> sts(ns);
  std::vector<const uint8_t*> scon(ns);
  for (u32 k = 0; k < ns; ++k) {
    sbase[k] = sv->segs[k].base;
    sts[k] = reinterpret_cast<const char*>(sv->segs[k].ts);
    scoff[k] = U64C(sv->segs[k].coff);
    scon[k] = sv->segs[k].content;
  }
  uint64_t total = 0;
  int ast = EVM_OK;
  st = encode_responses_dev(
      ctx, na, tree, owners, U64C(sel_off), U64C(sel_id), skip, ns, sbase.data(), srow.data(), sts.data(), 48,
      scoff.data(), scon.data(),
      [&](uint64_t need) -> uint8_t* {  // (the round's response arena, from the context's block cache)
        if (need + 16 > sv->resp_bytes) {
          if (sv->resp) block_free(ctx, sv->resp, sv->resp_bytes);
          size_t bytes = need + 16;
          sv->resp = static_cast<uint8_t*>(block_alloc(ctx, &bytes));
          sv->resp_bytes = sv->resp ? bytes : 0;
          if (!sv->resp) ast = EVM_ENOMEM;
        }
        return sv->resp;
      },
      U64P(rout), &total, &jplan, reinterpret_cast<const uint64_t*>(jlen), jbad);
  if (!st) st = ast;
  if (st) return st;
  std::vector<u64> ro((size_t)na + 1);
  std::vector<uint8_t> hskip(na);
  HIPR(hipMemcpyAsync(ro.data(), rout, sizeof(u64) * ((size_t)na + 1), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(hskip.data(), skip, na, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  // (the responses lie back to back in request order; a RangeError's bytes stay unused)
  std::vector<u64> rlen(n, 0);
  for (u32 j = 0; j < na; ++j) {
    rlen[ans[j]] = ro[j + 1] - ro[j];
    if (hskip[j]) result[ans[j]] = EVM_ERANGE;
  }
  for (u32 r = 0; r < n; ++r) resp_off[r + 1] = resp_off[r] + rlen[r];
  *resp_total = total;
  sv->resp_used = total;
  stamp(6);
  return EVM_OK;
}

}  // namespace

extern "C" {

int evm_sync_create(evm_ctx* ctx, evm_store* store, evm_sync_server** out) {
  if (!ctx || !store || !out) return EVM_EINVAL;
  *out = nullptr;
  uint32_t O = 0;
  uint64_t nm = 0;
  if (evm_store_info(store, &O, &nm)) return EVM_EINVAL;
  evm_sync_server* s = new evm_sync_server;
  s->ctx = ctx;
  s->store = store;
  s->cap = O;
  u32 tsz = 64;
  while (tsz < 2u * std::max<u32>(O, 1)) tsz <<= 1;
  s->mask = tsz - 1;
  bool ok = hipMalloc(reinterpret_cast<void**>(&s->table), sizeof(u32) * tsz) == hipSuccess &&
            hipMalloc(reinterpret_cast<void**>(&s->koff), sizeof(u64) * std::max<u32>(O, 1)) == hipSuccess &&
            hipMalloc(reinterpret_cast<void**>(&s->klen), sizeof(u32) * std::max<u32>(O, 1)) == hipSuccess &&
            hipMalloc(reinterpret_cast<void**>(&s->claim), sizeof(u32) * std::max<u32>(O, 1)) == hipSuccess &&
            hipMalloc(reinterpret_cast<void**>(&s->flag), std::max<u32>(O, 1)) == hipSuccess &&
            hipStreamCreateWithFlags(&s->ps, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming) == hipSuccess;
  if (ok) {
    hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(tsz, 256)), dim3(256), 0, ctx->stream, s->table, (size_t)tsz,
                       DIR_EMPTY);
    ok = hipMemsetAsync(s->claim, 0, sizeof(u32) * std::max<u32>(O, 1), ctx->stream) == hipSuccess &&
         hipMemsetAsync(s->flag, 0, std::max<u32>(O, 1), ctx->stream) == hipSuccess &&
         hipStreamSynchronize(ctx->stream) == hipSuccess;
  }
  if (!ok) {
    evm_sync_destroy(s);
    return EVM_ENOMEM;
  }
  *out = s;
  return EVM_OK;
}

int evm_sync_destroy(evm_sync_server* s) {
  if (!s) return EVM_EINVAL;
  evm_ctx* ctx = s->ctx;
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& g : s->segs) block_free(ctx, g.block, g.bytes);
  if (s->resp) block_free(ctx, s->resp, s->resp_bytes);
  if (s->din) block_free(ctx, s->din, s->din_bytes);
  (void)hipFree(s->table);
  (void)hipFree(s->koff);
  (void)hipFree(s->klen);
  (void)hipFree(s->claim);
  (void)hipFree(s->flag);
  if (s->kbytes) (void)hipFree(s->kbytes);
  if (s->hbuf) (void)hipHostFree(s->hbuf);
  (void)hipStreamSynchronize(ctx->stream);
  if (s->ps) (void)hipStreamDestroy(s->ps);
  if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  delete s;
  return EVM_OK;
}

int evm_sync_round(evm_sync_server* s, const uint8_t* arena, const uint64_t* off, uint32_t n, int where,
                   int32_t* result, uint64_t* resp_off, uint64_t* resp_bytes) {
  if (!s || !off || !result || !resp_off || !resp_bytes || (n && !arena) ||
      (where != EVM_SYNC_HOST && where != EVM_SYNC_DEVICE))
    return EVM_EINVAL;
  for (uint32_t k = 0; k < n; ++k)
    if (off[k + 1] < off[k]) return EVM_EINVAL;
  evm_ctx* ctx = s->ctx;
  const u64* off_h = reinterpret_cast<const u64*>(off);
  s->part_ms[0] = s->part_ms[7] = 0;
  if (where == EVM_SYNC_DEVICE) return round_dev(s, arena, off_h, n, result, reinterpret_cast<u64*>(resp_off),
                                                 reinterpret_cast<u64*>(resp_bytes));
  // host bodies: staged into a device arena of the context's block cache
  // (16 B of slack: the kernels read whole 16-B chunks)
  const size_t bytes = off[n] - off[0];
  if (bytes + 64 > s->din_bytes) {
    if (s->din) block_free(ctx, s->din, s->din_bytes);
    size_t want = bytes + 64;
    s->din = static_cast<uint8_t*>(block_alloc(ctx, &want));
    s->din_bytes = s->din ? want : 0;
    if (!s->din) return EVM_ENOMEM;
  }
  const double h0 = now_ms();
  int st = stage_h2d(ctx, s->din, arena + off[0], bytes);
  if (!st) st = hip_ok(hipStreamSynchronize(ctx->stream));
  s->part_ms[0] = now_ms() - h0;
  if (st) return st;
  std::vector<u64> o((size_t)n + 1);
  for (uint32_t k = 0; k <= n; ++k) o[k] = off[k] - off[0];
  st = round_dev(s, s->din, o.data(), n, result, reinterpret_cast<u64*>(resp_off), reinterpret_cast<u64*>(resp_bytes));
  block_free(ctx, s->din, s->din_bytes);  // (back to the context's cache: the next round reuses it)
  s->din = nullptr;
  s->din_bytes = 0;
  return st;
}

int evm_sync_fetch(evm_sync_server* s, uint8_t* out) {
  if (!s || (s->resp_used && !out)) return EVM_EINVAL;
  if (!s->resp_used) return EVM_OK;
  const double h0 = now_ms();
  const int st = stage_d2h(s->ctx, out, s->resp, s->resp_used);
  s->part_ms[7] = now_ms() - h0;
  return st;
}

int evm_sync_timing(const evm_sync_server* s, double* ms) {
  if (!s || !ms) return EVM_EINVAL;
  for (int k = 0; k < 8; ++k) ms[k] = s->part_ms[k];
  return EVM_OK;
}

const uint8_t* evm_sync_responses_dev(const evm_sync_server* s) { return s ? s->resp : nullptr; }

int evm_sync_users(evm_sync_server* s, const uint8_t* ids, const uint64_t* id_off, uint32_t n, int insert,
                   uint32_t* slots) {
  if (!s || !id_off || !slots || (n && !ids)) return EVM_EINVAL;
  if (!n) return EVM_OK;
  for (uint32_t k = 0; k < n; ++k)
    if (id_off[k + 1] < id_off[k]) return EVM_EINVAL;
  evm_ctx* ctx = s->ctx;
  Scratch S(ctx);
  const u64 kb = id_off[n] - id_off[0];
  uint8_t* src = S.alloc<uint8_t>(kb + 16);
  u64* soff = S.alloc<u64>(n);
  u32* slen = S.alloc<u32>(n);
  uint8_t* rf = S.alloc<uint8_t>(n);
  u32* slot = S.alloc<u32>(n);
  if (!src || !soff || !slen || !rf || !slot) return EVM_ENOMEM;
  std::vector<u64> so(n);
  std::vector<u32> sl(n);
  std::vector<uint8_t> f(n, RQ_USE);
  for (uint32_t k = 0; k < n; ++k) {
    so[k] = id_off[k] - id_off[0];
    sl[k] = (u32)(id_off[k + 1] - id_off[k]);
  }
  if (kb) HIPR(hipMemcpyAsync(src, ids + id_off[0], kb, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(soff, so.data(), sizeof(u64) * n, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(slen, sl.data(), sizeof(u32) * n, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(rf, f.data(), n, hipMemcpyHostToDevice, ctx->stream));
  int st = dir_resolve(s, S, src, soff, slen, n, rf, slot, kb, insert, nullptr);
  if (st) return st;
  HIPR(hipMemcpyAsync(slots, slot, sizeof(u32) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  return EVM_OK;
}

int evm_sync_user_flag(evm_sync_server* s, uint32_t slot, int flag) {
  if (!s || slot >= s->users || flag < 0 || flag > 1) return EVM_EINVAL;
  evm_ctx* ctx = s->ctx;
  KLAUNCH(k_set_u8, dim3(1), dim3(1), s->flag, slot, (uint8_t)flag);
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

int evm_sync_user_count(const evm_sync_server* s, uint32_t* n_users, uint64_t* key_bytes) {
  if (!s) return EVM_EINVAL;
  if (n_users) *n_users = s->users;
  if (key_bytes) *key_bytes = s->kused;
  return EVM_OK;
}

int evm_sync_user_keys(evm_sync_server* s, uint8_t* keys, uint64_t* key_off) {
  if (!s || !key_off || (s->kused && !keys)) return EVM_EINVAL;
  evm_ctx* ctx = s->ctx;
  std::vector<u64> ko(s->users);
  std::vector<u32> kl(s->users);
  if (s->users) {
    HIPR(hipMemcpyAsync(ko.data(), s->koff, sizeof(u64) * s->users, hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipMemcpyAsync(kl.data(), s->klen, sizeof(u32) * s->users, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (s->kused) HIPR(hipMemcpyAsync(keys, s->kbytes, s->kused, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  // (slots are in key order: slot s's key starts where slot s - 1's ends)
  key_off[0] = 0;
  for (u32 k = 0; k < s->users; ++k) {
    if (ko[k] != key_off[k]) return EVM_ESTATE;
    key_off[k + 1] = ko[k] + kl[k];
  }
  return EVM_OK;
}

int evm_sync_log_add(evm_sync_server* s, const char* ts, size_t stride, uint64_t n, const uint64_t* content_off,
                     const uint8_t* content, uint64_t* first_id) {
  if (!s || !first_id || stride < 46 || (n && (!ts || !content_off)) || (n && content_off[0] != 0)) return EVM_EINVAL;
  *first_id = s->next_id;
  if (!n) return EVM_OK;
  evm_ctx* ctx = s->ctx;
  const u64 cb = content_off[n];
  if (cb && !content) return EVM_EINVAL;
  SyncSeg g;
  int st = seg_alloc(s, n, cb, &g);
  if (st) return st;
  std::vector<uint8_t> rows((size_t)n * 48, 0);
  for (u64 i = 0; i < n; ++i) memcpy(&rows[i * 48], ts + i * stride, 46);
  st = hip_ok(hipMemcpyAsync(g.ts, rows.data(), rows.size(), hipMemcpyHostToDevice, ctx->stream));
  if (!st) st = hip_ok(hipMemcpyAsync(g.coff, content_off, sizeof(u64) * (n + 1), hipMemcpyHostToDevice, ctx->stream));
  if (!st && cb) st = hip_ok(hipMemcpyAsync(g.content, content, cb, hipMemcpyHostToDevice, ctx->stream));
  if (!st) st = hip_ok(hipStreamSynchronize(ctx->stream));
  if (st) {
    block_free(ctx, g.block, g.bytes);
    return st;
  }
  s->segs.push_back(g);
  s->next_id += n;
  return EVM_OK;
}

int evm_sync_log_read(evm_sync_server* s, const uint64_t* ids, uint64_t n, char* ts, uint64_t* content_off,
                      uint8_t* content) {
  if (!s || !content_off || (n && (!ids || !ts))) return EVM_EINVAL;
  content_off[0] = 0;
  if (!n) return EVM_OK;
  evm_ctx* ctx = s->ctx;
  Scratch S(ctx);
  const u32 ns = (u32)s->segs.size();
  std::vector<LSeg> hs(ns);
  for (u32 k = 0; k < ns; ++k)
    hs[k] = LSeg{s->segs[k].base, s->segs[k].n, s->segs[k].ts, s->segs[k].coff, s->segs[k].content};
  LSeg* sg = S.alloc<LSeg>(std::max<u32>(ns, 1));
  u64* ids_d = S.alloc<u64>(n);
  char* ts_d = S.alloc<char>(n * 46);
  u64* clen = S.alloc<u64>(n);
  u64* cpos = S.alloc<u64>(n + 1);
  u32* bad = S.alloc<u32>(1);
  if (!sg || !ids_d || !ts_d || !clen || !cpos || !bad) return EVM_ENOMEM;
  if (ns) HIPR(hipMemcpyAsync(sg, hs.data(), sizeof(LSeg) * ns, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemcpyAsync(ids_d, ids, sizeof(u64) * n, hipMemcpyHostToDevice, ctx->stream));
  HIPR(hipMemsetAsync(bad, 0, sizeof(u32), ctx->stream));
  KLAUNCH(k_log_spans, dim3(grid_for(n, 256)), dim3(256), sg, ns, ids_d, n, ts_d, clen, bad);
  int st = scan_exclusive<u64, OpAdd>(ctx, S, clen, n, cpos, cpos + n);
  if (st) return st;
  u32 hb = 0;
  HIPR(hipMemcpyAsync(&hb, bad, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(ts, ts_d, n * 46, hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipMemcpyAsync(content_off, cpos, sizeof(u64) * (n + 1), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  if (hb) return EVM_EINVAL;  // (an id in no segment)
  if (!content || !content_off[n]) return EVM_OK;
  uint8_t* c_d = S.alloc<uint8_t>(content_off[n]);
  if (!c_d) return EVM_ENOMEM;
  KLAUNCH(k_log_content, dim3(grid_for(n, 1, 1 << 16)), dim3(64), sg, ns, ids_d, n, cpos, c_d);
  HIPR(hipMemcpyAsync(content, c_d, content_off[n], hipMemcpyDeviceToHost, ctx->stream));
  return hip_ok(hipStreamSynchronize(ctx->stream));
}

uint64_t evm_sync_next_id(const evm_sync_server* s) { return s ? s->next_id : 0; }

}  // extern "C"
