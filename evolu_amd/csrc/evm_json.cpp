// MerkleTree JSON codec (types.ts:80-84) over the engine's leaf lists.
//
// JSON.stringify(tree) prints a node as {"0":..,"1":..,"2":..,"hash":h}: V8
// orders integer-like keys ascending before string keys, whatever the
// insertion order, and the root of an empty tree is `{}` (no hash).  The
// parser accepts exactly the trees insertIntoMerkleTree (merkleTree.ts:8-50)
// can produce -- every node carries an int32 hash, the root's hash is the XOR
// of its children -- and rebuilds the leaf list: a node's leaf XOR is its hash
// XOR its children's hashes (kept when non-zero or when the node has no
// children, which preserves node presence).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "evm_internal.hpp"

namespace {

constexpr int DIGITS = 20;

struct Emitter {
  const uint64_t* ck;
  const int32_t* pfx;  // host exclusive prefix XOR over the owner's leaves
  std::string out;

  size_t lower(size_t lo, size_t hi, uint64_t x) const {
    while (lo < hi) {
      const size_t m = (lo + hi) / 2;
      if (ck[m] < x) lo = m + 1;
      else hi = m;
    }
    return lo;
  }

  void node(size_t lo, size_t hi, uint64_t prefix, int depth, bool with_hash) {
    out.push_back('{');
    bool first = true;
    if (depth < DIGITS) {
      const int sh = 2 * (DIGITS - 1 - depth);
      size_t a = lower(lo, hi, prefix | (1ull << sh));
      for (int c = 0; c < 3; ++c) {
        const uint64_t beg = prefix | ((uint64_t)(c + 1) << sh);
        const size_t b = lower(a, hi, prefix + ((uint64_t)(c + 2) << sh));
        if (b > a) {
          if (!first) out.push_back(',');
          first = false;
          out += "\"";
          out.push_back((char)('0' + c));
          out += "\":";
          node(a, b, beg, depth + 1, true);
        }
        a = b;
      }
    }
    if (with_hash) {
      if (!first) out.push_back(',');
      out += "\"hash\":";
      out += std::to_string(pfx[hi] ^ pfx[lo]);
    }
    out.push_back('}');
  }
};

struct Parser {
  const char* p;
  const char* e;
  std::vector<uint64_t> codes;
  std::vector<int32_t> xors;

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  // key: returns 0,1,2 for digits, 3 for "hash", -1 otherwise
  int key() {
    ws();
    if (p >= e || *p != '"') return -1;
    const char* q = ++p;
    while (p < e && *p != '"') {
      if (*p == '\\') return -1;
      ++p;
    }
    if (p >= e) return -1;
    const size_t len = (size_t)(p - q);
    ++p;
    if (len == 1 && q[0] >= '0' && q[0] <= '2') return q[0] - '0';
    if (len == 4 && memcmp(q, "hash", 4) == 0) return 3;
    return -1;
  }
  bool integer(int32_t* v) {
    ws();
    bool neg = false;
    if (p < e && *p == '-') {
      neg = true;
      ++p;
    }
    if (p >= e || *p < '0' || *p > '9') return false;
    if (*p == '0' && p + 1 < e && p[1] >= '0' && p[1] <= '9') return false;  // no leading zeros
    int64_t x = 0;
    while (p < e && *p >= '0' && *p <= '9') {
      x = x * 10 + (*p - '0');
      if (x > 2147483648LL) return false;
      ++p;
    }
    if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) return false;
    if (neg) x = -x;
    if (x < INT32_MIN || x > INT32_MAX || (neg && x == 0)) return false;
    *v = (int32_t)x;
    return true;
  }
  // Parses one node, appending its leaves (any order; sorted by the caller).
  bool node(uint64_t prefix, int depth, bool root, int32_t* hash_out, bool* has_hash) {
    if (!lit('{')) return false;
    bool seen[4] = {false, false, false, false};
    int32_t h = 0, child_x = 0;
    bool any_child = false;
    if (!lit('}')) {
      do {
        const int k = key();
        if (k < 0 || seen[k] || !lit(':')) return false;
        seen[k] = true;
        if (k == 3) {
          if (!integer(&h)) return false;
        } else {
          if (depth >= DIGITS) return false;
          const int sh = 2 * (DIGITS - 1 - depth);
          int32_t ch = 0;
          bool chh = false;
          if (!node(prefix | ((uint64_t)(k + 1) << sh), depth + 1, false, &ch, &chh) || !chh) return false;
          child_x ^= ch;
          any_child = true;
        }
      } while (lit(','));
      if (!lit('}')) return false;
    }
    *has_hash = seen[3];
    *hash_out = h;
    if (root) {
      if (!seen[3]) return !any_child;                 // {} only
      return any_child && (h ^ child_x) == 0;          // no key of length 0
    }
    if (!seen[3]) return false;
    const int32_t t = h ^ child_x;
    if (!any_child || t != 0) {
      codes.push_back(prefix);
      xors.push_back(t);
    }
    return true;
  }
};

// f(begin, end) over disjoint runs of [0, n) on host threads (EVM_HOST_THREADS, at most 16)
template <typename F>
void run_parallel(size_t n, F f) {
  int T = (int)std::thread::hardware_concurrency();
  if (const char* e = getenv("EVM_HOST_THREADS")) T = atoi(e);
  T = (int)std::min<size_t>((size_t)std::max(1, std::min(T, 16)), std::max<size_t>(1, n / 16));
  if (T <= 1) {
    f((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k) th.emplace_back([=]() { f(n * k / T, n * (k + 1) / T); });
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" int evm_tree_to_json(evm_ctx* ctx, const evm_tree* t, uint32_t owner, char* buf, size_t cap, size_t* len) {
  if (!ctx || !t || !len || owner >= t->n_owners) return EVM_EINVAL;
  if (int e = evm::tree_compact(ctx, t)) return e;
  uint64_t ab[2];
  HIPR(hipMemcpyAsync(ab, t->off + owner, sizeof(ab), hipMemcpyDeviceToHost, ctx->stream));
  HIPR(hipStreamSynchronize(ctx->stream));
  const size_t L = (size_t)(ab[1] - ab[0]);
  std::vector<uint64_t> ck(L);
  std::vector<int32_t> xr(L), pfx(L + 1);
  if (L) {
    HIPR(hipMemcpyAsync(ck.data(), t->ck + ab[0], sizeof(uint64_t) * L, hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipMemcpyAsync(xr.data(), t->xr + ab[0], sizeof(int32_t) * L, hipMemcpyDeviceToHost, ctx->stream));
    HIPR(hipStreamSynchronize(ctx->stream));
  }
  pfx[0] = 0;
  for (size_t i = 0; i < L; ++i) {
    pfx[i + 1] = pfx[i] ^ xr[i];
    ck[i] &= (1ull << 40) - 1;
  }
  Emitter em{ck.data(), pfx.data(), std::string()};
  if (L == 0) em.out = "{}";
  else em.node(0, L, 0, 0, true);
  *len = em.out.size();
  if (buf) {
    if (cap < em.out.size()) return EVM_ECAPACITY;
    memcpy(buf, em.out.data(), em.out.size());
  }
  return EVM_OK;
}

extern "C" int evm_tree_from_json(evm_ctx* ctx, uint32_t n_owners, const char* const* json, const size_t* lens,
                                  evm_tree** out) {
  if (!ctx || !out || (n_owners && (!json || !lens))) return EVM_EINVAL;
  // owners parse independently: runs of them on host threads (a round's
  // client trees, index.ts:187), then one copy into the leaf arrays
  std::vector<std::vector<std::pair<uint64_t, int32_t>>> per(n_owners);
  std::atomic<int> bad{0};
  auto work = [&](size_t a, size_t b) {
    for (size_t o = a; o < b && !bad.load(std::memory_order_relaxed); ++o) {
      Parser ps{json[o], json[o] + lens[o], {}, {}};
      int32_t h = 0;
      bool hh = false;
      if (!ps.node(0, 0, true, &h, &hh)) {
        bad = 1;
        return;
      }
      ps.ws();
      if (ps.p != ps.e) {
        bad = 1;
        return;
      }
      auto& v = per[o];
      v.resize(ps.codes.size());
      for (size_t i = 0; i < v.size(); ++i) v[i] = {ps.codes[i], ps.xors[i]};
      std::sort(v.begin(), v.end());
    }
  };
  run_parallel(n_owners, work);
  if (bad) return EVM_ETREE;
  std::vector<uint64_t> off(n_owners + 1, 0);
  for (uint32_t o = 0; o < n_owners; ++o) off[o + 1] = off[o] + per[o].size();
  std::vector<uint64_t> codes(off[n_owners]);
  std::vector<int32_t> xors(off[n_owners]);
  run_parallel(n_owners, [&](size_t a, size_t b) {
    for (size_t o = a; o < b; ++o)
      for (size_t i = 0; i < per[o].size(); ++i) {
        codes[off[o] + i] = per[o][i].first;
        xors[off[o] + i] = per[o][i].second;
      }
  });
  return evm_tree_from_leaves(ctx, n_owners, off.data(), codes.data(), xors.data(), out);
}
