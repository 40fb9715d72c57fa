// receiveMessages (packages/evolu/src/receive.ts:45-66) as a data-parallel scan.
//
// The reference folds every received timestamp into the local HLC with
// receiveTimestamp (timestamp.ts:125-165), `now` fixed for the batch
// (db.worker.ts:71), and stops at the first error.  With T_i = max(m_i, now):
//   millis:  R_i = max(R_{i-1}, T_i), R_{-1} = local millis      (prefix max)
//   counter: C_i = max(C_{i-1}, d_i) + 1, d_i = c_i if m_i == R_i else -1,
//            restarting from C_{s-1} = -1 wherever R increases (s), and from
//            the local counter before the first increase.  Unrolled inside a
//            segment: C_i = i + 1 + max_{j in segment, j <= i} (d_j - j)
//            -> one prefix max over (segment id << 40 | d_j - j + bias).
//   errors at i (reference order): drift R_i - now > maxDrift; duplicate
//            node; counter overflow C_i > 65535.  The first i wins.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "evm_device.hpp"
#include "evm_internal.hpp"
#include "evm_prims.hpp"

using namespace evm;

namespace {

struct RfParams {
  u64 m0;       // local millis
  u32 c0;       // local counter
  u64 lnode;    // local node hex
  u32 lmask;    // local node case mask
  u64 now;
  u64 drift;    // config.maxDrift
  u64 bias;     // n + 2
};

struct RfOut {
  u64 first_err;  // (index << 2 | kind), ~0 = none
  u64 millis;
  u64 counter;
  u64 err_next;
};

__global__ void k_rf_t(const evm_rec* __restrict__ rec, size_t n, RfParams P, u64* __restrict__ T) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u64 m = rec[i].tc >> 16;
    T[i] = m > P.now ? m : P.now;
  }
}

__global__ void k_rf_inc(const u64* __restrict__ T, const u64* __restrict__ E, size_t n, RfParams P,
                         u32* __restrict__ inc) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u64 prev = max(P.m0, E[i]);  // E = exclusive prefix max of T (0 for i = 0)
    inc[i] = T[i] > prev ? 1u : 0u;
  }
}

__global__ void k_rf_v(const evm_rec* __restrict__ rec, const u64* __restrict__ T, const u64* __restrict__ E,
                       const u32* __restrict__ segx, const u32* __restrict__ inc, size_t n, RfParams P,
                       u64* __restrict__ v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u64 R = max(max(P.m0, E[i]), T[i]);
    const u64 m = rec[i].tc >> 16;
    const int64_t d = (m == R) ? (int64_t)(rec[i].tc & 0xffffu) : -1;
    const u64 seg = (u64)segx[i] + inc[i];
    v[i] = (seg << 40) | (u64)(d - (int64_t)i + (int64_t)P.bias);
  }
}

__global__ void k_rf_out(const evm_rec* __restrict__ rec, const u64* __restrict__ T, const u64* __restrict__ E,
                         const u64* __restrict__ V, const u64* __restrict__ Vx, size_t n, RfParams P,
                         RfOut* __restrict__ out) {
  const u64 init = (u64)P.c0 + P.bias;  // the local counter, segment 0 (j = -1 term)
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u64 R = max(max(P.m0, E[i]), T[i]);
    const u64 incl = max(max(Vx[i], V[i]), init);
    const int64_t C = (int64_t)i + 1 + ((int64_t)(incl & ((1ull << 40) - 1)) - (int64_t)P.bias);
    const evm_rec r = rec[i];
    u32 kind = 0;
    if (R - P.now > P.drift) kind = 1;  // TimestampDriftError (next = R)
    else if (r.node == P.lnode && (r.meta & EVM_META_CASEMASK) == P.lmask) kind = 2;  // TimestampDuplicateNodeError
    else if (C > 65535) kind = 3;  // TimestampCounterOverflowError
    if (kind) {
      atomicMin(&out->first_err, ((u64)i << 2) | kind);
    }
    if (i == n - 1) {
      out->millis = R;
      out->counter = (u64)C;
    }
  }
}

__global__ void k_rf_next(const u64* __restrict__ T, const u64* __restrict__ E, RfParams P, RfOut* __restrict__ out) {
  if (threadIdx.x == 0 && out->first_err != ~0ull) {
    const size_t i = out->first_err >> 2;
    out->err_next = max(max(P.m0, E[i]), T[i]);
  }
}

bool parse_node_host(const char* s, u64* v, u32* mask) {
  u64 x = 0;
  u32 m = 0;
  for (int i = 0; i < 16; ++i) {
    const char c = s[i];
    u32 d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') {
      d = c - 'A' + 10;
      m |= 1u << i;
    } else {
      return false;
    }
    x = (x << 4) | d;
  }
  *v = x;
  *mask = m;
  return true;
}

}  // namespace

extern "C" int evm_receive_fold(evm_ctx* ctx, const char* ts, size_t stride, size_t n, int64_t local_millis,
                                uint32_t local_counter, const char* local_node, int64_t now, int64_t max_drift,
                                evm_clock_result* res) {
  if (!ctx || !res || !local_node || stride < 46 || (n && !ts) || local_millis < 0 || now < 0 || max_drift < 0 ||
      local_counter > 65535)
    return EVM_EINVAL;
  RfParams P;
  if (!parse_node_host(local_node, &P.lnode, &P.lmask)) return EVM_EINVAL;
  P.m0 = (u64)local_millis;
  P.c0 = local_counter;
  P.now = (u64)now;
  P.drift = (u64)max_drift;
  P.bias = (u64)n + 2;
  res->error = 0;
  res->error_index = -1;
  res->next = 0;
  res->millis = local_millis;
  res->counter = local_counter;
  if (n == 0) return EVM_OK;
  if (n >= (1ull << 38)) return EVM_EINVAL;
  int st;
  Scratch S(ctx);
  Info* info = nullptr;
  if ((st = new_info(ctx, S, &info))) return st;
  evm_rec* rec = S.alloc<evm_rec>(n);
  u64* T = S.alloc<u64>(n);
  u64* E = S.alloc<u64>(n);
  u32* inc = S.alloc<u32>(n);
  u32* segx = S.alloc<u32>(n);
  u64* V = S.alloc<u64>(n);
  u64* Vx = S.alloc<u64>(n);
  RfOut* out = S.alloc<RfOut>(1);
  if (!rec || !T || !E || !inc || !segx || !V || !Vx || !out) return EVM_ENOMEM;
  if ((st = launch_pack(ctx, ts, stride, n, nullptr, 0, rec, info))) return st;
  RfOut init{~0ull, 0, 0, 0};
  HIPR(hipMemcpyAsync(out, &init, sizeof(init), hipMemcpyHostToDevice, ctx->stream));
  const int g = grid_for(n, 256);
  KLAUNCH(k_rf_t, dim3(g), dim3(256), rec, n, P, T);
  if ((st = scan_exclusive<u64, OpMax>(ctx, S, T, n, E, (u64*)nullptr))) return st;
  KLAUNCH(k_rf_inc, dim3(g), dim3(256), T, E, n, P, inc);
  if ((st = scan_exclusive<u32, OpAdd>(ctx, S, inc, n, segx, (u32*)nullptr))) return st;
  KLAUNCH(k_rf_v, dim3(g), dim3(256), rec, T, E, segx, inc, n, P, V);
  if ((st = scan_exclusive<u64, OpMax>(ctx, S, V, n, Vx, (u64*)nullptr))) return st;
  KLAUNCH(k_rf_out, dim3(g), dim3(256), rec, T, E, V, Vx, n, P, out);
  KLAUNCH(k_rf_next, dim3(1), dim3(64), T, E, P, out);
  Info hi;
  RfOut ho;
  HIPR(hipMemcpyAsync(&ho, out, sizeof(ho), hipMemcpyDeviceToHost, ctx->stream));
  if ((st = read_info(ctx, info, &hi))) return st;
  if (hi.bad) return EVM_ENONCANON;
  if (ho.first_err != ~0ull) {
    res->error = (int32_t)(ho.first_err & 3);
    res->error_index = (int64_t)(ho.first_err >> 2);
    res->next = (int64_t)ho.err_next;
  } else {
    res->millis = (int64_t)ho.millis;
    res->counter = (uint32_t)ho.counter;
  }
  return EVM_OK;
}
