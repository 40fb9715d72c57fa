// Wire codec for the sync messages (packages/evolu/protos/protobuf.proto,
// generated code protobuf.ts:60-171, protobuf-ts 2.8.1 runtime -- absent here,
// so this restates the proto3 wire format it implements):
//
//   EncryptedCrdtMessage { string timestamp = 1; bytes content = 2; }
//   SyncRequest  { repeated EncryptedCrdtMessage messages = 1; string userId = 2;
//                  string nodeId = 3; string merkleTree = 4; }
//   SyncResponse { repeated EncryptedCrdtMessage messages = 1; string merkleTree = 2; }
//
// Encoding writes fields in field-number order and omits proto3 defaults
// (empty strings / bytes), as protobuf-ts' toBinary does.  Decoding accepts
// any field order, keeps the last value of a singular field, skips unknown
// fields by wire type and rejects truncation, wrong wire types and groups.
//
// Host code: it turns a request body into the engine's timestamp arena (one
// pass over the record headers) and a response back into bytes.  It is the
// server's `SyncRequest.fromBinary(body)` (apps/server/src/index.ts:115) and
// `SyncResponse.toBinary(...)` (index.ts:239), and the client's
// `SyncRequest.toBinary` / `SyncResponse.fromBinary` (sync.worker.ts:102,131).
#include <stdint.h>
#include <string.h>

#include "../../include/evm.h"

namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool more() const { return ok && p < e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int sh = 0; sh < 70; sh += 7) {
      if (p >= e) {
        ok = false;
        return 0;
      }
      const uint8_t b = *p++;
      if (sh == 63 && b > 1) {  // more than 64 bits
        ok = false;
        return 0;
      }
      v |= (uint64_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  // length-delimited payload -> [*q, *q + *n)
  bool bytes(const uint8_t** q, uint64_t* n) {
    const uint64_t len = varint();
    if (!ok || len > (uint64_t)(e - p)) return ok = false;
    *q = p;
    *n = len;
    p += len;
    return true;
  }
  bool skip(uint32_t wt) {
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
        uint64_t n;
        return bytes(&q, &n);
      }
      case 5:
        if (e - p < 4) return ok = false;
        p += 4;
        return true;
      default:  // groups (3, 4) and reserved wire types
        return ok = false;
    }
  }
};

struct Msg {
  const uint8_t* ts = nullptr;
  uint64_t ts_len = 0;
  const uint8_t* content = nullptr;
  uint64_t content_len = 0;
};

bool read_msg(const uint8_t* q, uint64_t n, Msg* m) {
  Reader r{q, q + n};
  *m = Msg{};
  while (r.more()) {
    const uint64_t tag = r.varint();
    if (!r.ok) return false;
    const uint32_t field = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
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

// Walks a SyncRequest / SyncResponse; calls on_msg(index, Msg) per message.
template <typename F>
int walk(int kind, const uint8_t* buf, size_t len, evm_pb_sync* info, F on_msg) {
  if (kind != EVM_PB_SYNC_REQUEST && kind != EVM_PB_SYNC_RESPONSE) return EVM_EINVAL;
  if (!buf && len) return EVM_EINVAL;
  Reader r{buf, buf + len};
  evm_pb_sync s;
  memset(&s, 0, sizeof(s));
  // string fields: field number -> (offset, length) slot
  const uint32_t tree_field = kind == EVM_PB_SYNC_REQUEST ? 4u : 2u;
  while (r.more()) {
    const uint64_t tag = r.varint();
    if (!r.ok) return EVM_EINVAL;
    const uint32_t field = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
    if (field == 0) return EVM_EINVAL;
    const bool is_str = field == 1 || field == tree_field || (kind == EVM_PB_SYNC_REQUEST && (field == 2 || field == 3));
    if (!is_str) {
      if (!r.skip(wt)) return EVM_EINVAL;
      continue;
    }
    if (wt != 2) return EVM_EINVAL;
    const uint8_t* q;
    uint64_t n;
    if (!r.bytes(&q, &n)) return EVM_EINVAL;
    const uint64_t off = (uint64_t)(q - buf);
    if (field == 1) {
      Msg m;
      if (!read_msg(q, n, &m)) return EVM_EINVAL;
      if (m.ts_len != 46) ++s.nonstd_ts;
      s.content_bytes += m.content_len;
      on_msg(s.n_messages, m);
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
  }
  if (!r.ok) return EVM_EINVAL;
  if (info) *info = s;
  return EVM_OK;
}

size_t varint_len(uint64_t v) {
  size_t k = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++k;
  }
  return k;
}

struct Writer {
  uint8_t* p;
  size_t cap;
  size_t n = 0;
  void byte(uint8_t b) {
    if (p && n < cap) p[n] = b;
    ++n;
  }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      byte((uint8_t)(v | 0x80));
      v >>= 7;
    }
    byte((uint8_t)v);
  }
  void raw(const void* s, size_t len) {
    if (p && n + len <= cap && len) memcpy(p + n, s, len);
    n += len;
  }
  void str(uint32_t field, const void* s, size_t len) {  // proto3: empty = omitted
    if (!len) return;
    varint((uint64_t)field << 3 | 2);
    varint(len);
    raw(s, len);
  }
};

}  // namespace

extern "C" {

int evm_pb_scan(int kind, const uint8_t* buf, size_t len, evm_pb_sync* info) {
  if (!info) return EVM_EINVAL;
  return walk(kind, buf, len, info, [](uint64_t, const Msg&) {});
}

int evm_pb_split(int kind, const uint8_t* buf, size_t len, char* ts, size_t stride, uint32_t* ts_len,
                 uint64_t* ts_off, uint64_t* content_off, uint8_t* content) {
  if (stride < 46 || !ts || !content_off) return EVM_EINVAL;
  uint64_t coff = 0;
  content_off[0] = 0;
  int st = walk(kind, buf, len, nullptr, [&](uint64_t i, const Msg& m) {
    char* row = ts + i * stride;
    // a non-46-byte timestamp cannot be canonical: 0xFF bytes, flagged by the engine
    if (m.ts_len == 46) memcpy(row, m.ts, 46);
    else memset(row, 0xff, 46);
    memset(row + 46, 0, stride - 46);
    if (ts_len) ts_len[i] = (uint32_t)(m.ts_len > 0xffffffffu ? 0xffffffffu : m.ts_len);
    if (ts_off) ts_off[i] = m.ts ? (uint64_t)(m.ts - buf) : 0;
    if (content && m.content_len) memcpy(content + coff, m.content, m.content_len);
    coff += m.content_len;
    content_off[i + 1] = coff;
  });
  return st;
}

int evm_pb_encode(int kind, const char* ts, size_t stride, const uint32_t* ts_len, size_t n,
                  const uint64_t* content_off, const uint8_t* content, const char* user, size_t user_len,
                  const char* node, size_t node_len, const char* tree, size_t tree_len, uint8_t* out, size_t cap,
                  size_t* out_len) {
  if (kind != EVM_PB_SYNC_REQUEST && kind != EVM_PB_SYNC_RESPONSE) return EVM_EINVAL;
  if (!out_len || (n && (!ts || stride < 46 || !content_off)) || (user_len && !user) || (node_len && !node) ||
      (tree_len && !tree))
    return EVM_EINVAL;
  Writer w{out, out ? cap : 0};
  for (size_t i = 0; i < n; ++i) {
    const size_t tl = ts_len ? ts_len[i] : 46;
    if (tl > stride) return EVM_EINVAL;
    const uint64_t cl = content_off[i + 1] - content_off[i];
    if (cl && !content) return EVM_EINVAL;
    const size_t body = (tl ? 1 + varint_len(tl) + tl : 0) + (cl ? 1 + varint_len(cl) + cl : 0);
    w.varint(1u << 3 | 2);  // messages: an empty message is still written (length 0)
    w.varint(body);
    w.str(1, ts + i * stride, tl);
    w.str(2, cl ? content + content_off[i] : nullptr, cl);
  }
  if (kind == EVM_PB_SYNC_REQUEST) {
    w.str(2, user, user_len);
    w.str(3, node, node_len);
    w.str(4, tree, tree_len);
  } else {
    w.str(2, tree, tree_len);
  }
  *out_len = w.n;
  return (out && w.n > cap) ? EVM_ECAPACITY : EVM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Batches of bodies (a server round: index.ts:224-248 per request), on host
// threads.  Bodies are independent, so each thread takes a contiguous run of
// them; EVM_HOST_THREADS caps the threads (default: the machine's, at most 16).
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace {

int host_threads(size_t items) {
  int t = (int)std::thread::hardware_concurrency();
  if (const char* e = getenv("EVM_HOST_THREADS")) t = atoi(e);
  t = std::max(1, std::min(t, 16));
  return (int)std::min<size_t>((size_t)t, std::max<size_t>(1, items / 32));
}

template <typename F>
void parallel_for(size_t n, F f) {  // f(begin, end) over disjoint runs of [0, n)
  const int T = host_threads(n);
  if (T <= 1) {
    f((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k) {
    const size_t a = n * k / T, b = n * (k + 1) / T;
    th.emplace_back([=]() { f(a, b); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

int evm_pb_scan_batch(int kind, const uint8_t* arena, const uint64_t* off, uint32_t n, evm_pb_sync* info,
                      int32_t* status) {
  if ((n && (!arena || !off || !info || !status)) || (kind != EVM_PB_SYNC_REQUEST && kind != EVM_PB_SYNC_RESPONSE))
    return EVM_EINVAL;
  parallel_for(n, [&](size_t a, size_t b) {
    for (size_t k = a; k < b; ++k) {
      status[k] = off[k + 1] < off[k] ? EVM_EINVAL : evm_pb_scan(kind, arena + off[k], off[k + 1] - off[k], &info[k]);
      if (status[k]) memset(&info[k], 0, sizeof(evm_pb_sync));
    }
  });
  return EVM_OK;
}

int evm_pb_split_batch(int kind, const uint8_t* arena, const uint64_t* off, uint32_t n, const int32_t* status,
                       const uint64_t* msg_base, const uint64_t* content_base, char* ts, size_t stride,
                       uint32_t* ts_len, uint64_t* ts_off, uint64_t* content_off, uint8_t* content) {
  if (n && (!arena || !off || !status || !msg_base || !content_base || !ts || !content_off)) return EVM_EINVAL;
  if (stride < 46) return EVM_EINVAL;
  std::atomic<int> err{EVM_OK};  // the first error any thread meets
  parallel_for(n, [&](size_t a, size_t b) {
    std::vector<uint64_t> co;
    for (size_t k = a; k < b; ++k) {
      if (status[k]) continue;
      const uint64_t m0 = msg_base[k], c0 = content_base[k];
      const uint8_t* body = arena + off[k];
      const size_t len = off[k + 1] - off[k];
      evm_pb_sync s;
      if (evm_pb_scan(kind, body, len, &s)) continue;  // (scanned fine before: unchanged bytes)
      co.assign(s.n_messages + 1, 0);
      const int st = evm_pb_split(kind, body, len, ts + m0 * stride, stride, ts_len ? ts_len + m0 : nullptr,
                                  ts_off ? ts_off + m0 : nullptr, co.data(), content ? content + c0 : nullptr);
      if (st) {
        int none = EVM_OK;
        err.compare_exchange_strong(none, st);  // (a body that changed between the passes)
        continue;
      }
      for (uint64_t i = 0; i < s.n_messages; ++i) {
        content_off[m0 + i] = c0 + co[i];
        if (ts_off) ts_off[m0 + i] += off[k];
      }
      // the entry after a body's last message is the next body's first (or
      // the end): written once, by whoever holds the total
      content_off[m0 + s.n_messages] = c0 + co[s.n_messages];
    }
  });
  return err.load();
}

// SyncResponse bodies (index.ts:235-245) for n requests: request r's
// messages are the ids sel_id[sel_off[r] .. sel_off[r + 1]); a message id
// lies in log segment s = the last with seg_base[s] <= id (row k = id -
// seg_base[s], or seg_row[s][k] when a segment indexes shared arrays): its
// 46-B timestamp at seg_ts[s] + row * stride, its content
// seg_content[s][seg_coff[s][row] ..  seg_coff[s][row + 1]); the merkleTree
// text json[json_off[r] .. json_off[r + 1]).  out == NULL: out_off[0..n]
// only (the sizes' exclusive prefix, out_off[n] = the total).
int evm_pb_encode_responses(uint32_t n, const uint64_t* sel_off, const uint64_t* sel_id, uint32_t n_seg,
                            const uint64_t* seg_base, const uint64_t* const* seg_row, const char* const* seg_ts,
                            size_t stride, const uint64_t* const* seg_coff, const uint8_t* const* seg_content,
                            const char* json, const uint64_t* json_off, uint8_t* out, uint64_t* out_off) {
  if (n && (!sel_off || !json_off || !out_off || (n_seg && (!seg_base || !seg_ts || !seg_coff || !seg_content))))
    return EVM_EINVAL;
  if (stride < 46) return EVM_EINVAL;
  std::vector<int> bad((size_t)host_threads(n) + 1, 0);
  auto locate = [&](uint64_t id, const char** t, const uint8_t** c, uint64_t* cl) -> bool {
    const uint32_t s = (uint32_t)(std::upper_bound(seg_base, seg_base + n_seg, id) - seg_base);
    if (s == 0) return false;
    const uint64_t k = id - seg_base[s - 1];
    const uint64_t row = seg_row && seg_row[s - 1] ? seg_row[s - 1][k] : k;
    *t = seg_ts[s - 1] + row * stride;
    const uint64_t a = seg_coff[s - 1][row], b = seg_coff[s - 1][row + 1];
    *c = seg_content[s - 1] + a;
    *cl = b - a;
    return true;
  };
  auto encode = [&](size_t r, uint8_t* dst, size_t cap) -> size_t {
    Writer w{dst, cap};
    for (uint64_t j = sel_off[r]; j < sel_off[r + 1]; ++j) {
      const char* t;
      const uint8_t* c;
      uint64_t cl;
      if (!locate(sel_id[j], &t, &c, &cl)) {
        bad[0] = 1;
        continue;
      }
      w.varint(1u << 3 | 2);
      w.varint(1 + varint_len(46) + 46 + (cl ? 1 + varint_len(cl) + cl : 0));
      w.str(1, t, 46);
      w.str(2, c, cl);
    }
    w.str(2, json + json_off[r], json_off[r + 1] - json_off[r]);
    return w.n;
  };
  std::vector<uint64_t> size(n);
  parallel_for(n, [&](size_t a, size_t b) {
    for (size_t r = a; r < b; ++r) size[r] = encode(r, nullptr, 0);
  });
  if (bad[0]) return EVM_EINVAL;  // (an id in no segment)
  uint64_t acc = 0;
  for (uint32_t r = 0; r < n; ++r) {
    out_off[r] = acc;
    acc += size[r];
  }
  out_off[n] = acc;
  if (!out) return EVM_OK;
  parallel_for(n, [&](size_t a, size_t b) {
    for (size_t r = a; r < b; ++r) encode(r, out + out_off[r], size[r]);
  });
  return EVM_OK;
}

}  // extern "C"

extern "C" {

// SyncRequest bodies for n requests (a client fleet's round: sync.worker.ts
// SyncRequest.toBinary), on host threads: request r's messages are rows
// [msg_off[r], msg_off[r + 1]) of ts (46-B timestamps at `stride`) with
// contents content[content_off[row] .. content_off[row + 1]); its userId,
// nodeId and merkleTree are the strings [x_off[r], x_off[r + 1]) of the
// user / node / tree arenas.  out == NULL: out_off only (sizes' prefix).
int evm_pb_encode_requests(uint32_t n, const uint64_t* msg_off, const char* ts, size_t stride,
                           const uint64_t* content_off, const uint8_t* content, const char* user,
                           const uint64_t* user_off, const char* node, const uint64_t* node_off, const char* tree,
                           const uint64_t* tree_off, uint8_t* out, uint64_t* out_off) {
  if (n && (!msg_off || !out_off || !user_off || !node_off || !tree_off)) return EVM_EINVAL;
  if (stride < 46) return EVM_EINVAL;
  auto encode = [&](size_t r, uint8_t* dst, size_t cap) -> size_t {
    Writer w{dst, cap};
    for (uint64_t i = msg_off[r]; i < msg_off[r + 1]; ++i) {
      const uint64_t cl = content_off[i + 1] - content_off[i];
      w.varint(1u << 3 | 2);
      w.varint(1 + varint_len(46) + 46 + (cl ? 1 + varint_len(cl) + cl : 0));
      w.str(1, ts + i * stride, 46);
      w.str(2, content + content_off[i], cl);
    }
    w.str(2, user + user_off[r], user_off[r + 1] - user_off[r]);
    w.str(3, node + node_off[r], node_off[r + 1] - node_off[r]);
    w.str(4, tree + tree_off[r], tree_off[r + 1] - tree_off[r]);
    return w.n;
  };
  std::vector<uint64_t> size(n);
  parallel_for(n, [&](size_t a, size_t b) {
    for (size_t r = a; r < b; ++r) size[r] = encode(r, nullptr, 0);
  });
  uint64_t acc = 0;
  for (uint32_t r = 0; r < n; ++r) {
    out_off[r] = acc;
    acc += size[r];
  }
  out_off[n] = acc;
  if (!out) return EVM_OK;
  parallel_for(n, [&](size_t a, size_t b) {
    for (size_t r = a; r < b; ++r) encode(r, out + out_off[r], size[r]);
  });
  return EVM_OK;
}

}  // extern "C"
