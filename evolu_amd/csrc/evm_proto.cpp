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
