// N-API addon: the reference-side binding of the C ABI (include/evm.h).
//
// This is the binding a maintainer would add to packages/evolu (client worker)
// and apps/server: plain N-API (ABI-stable, version 8), zero-copy views of the
// caller's typed arrays, host buffers staged to the device with evm_copy_*.
// Handles (context, tree set, store) are napi_external values; freeing is
// explicit (treeFree / storeFree / destroy) so GPU memory never waits for GC.
#include <node_api.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "evm.h"

namespace {

#define NAPI_OK(env, call)                                         \
  do {                                                             \
    if ((call) != napi_ok) {                                       \
      napi_throw_error((env), nullptr, "N-API call failed: " #call); \
      return nullptr;                                              \
    }                                                              \
  } while (0)

napi_value throw_status(napi_env env, int st, const char* where) {
  std::string m = std::string(where) + ": " + evm_strerror(st);
  napi_throw_error(env, std::to_string(st).c_str(), m.c_str());
  return nullptr;
}

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
  size_t argc = want;
  if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < want) {
    napi_throw_type_error(env, nullptr, "missing arguments");
    return false;
  }
  return true;
}

void* ext(napi_env env, napi_value v) {
  void* p = nullptr;
  napi_get_value_external(env, v, &p);
  return p;
}

napi_value make_ext(napi_env env, void* p) {
  napi_value v;
  napi_create_external(env, p, nullptr, nullptr, &v);
  return v;
}

// a typed array's bytes (zero-copy view)
bool bytes_of(napi_env env, napi_value v, void** data, size_t* len) {
  napi_typedarray_type t;
  size_t n;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &n, data, &ab, &off) != napi_ok) {
    napi_throw_type_error(env, nullptr, "expected a typed array");
    return false;
  }
  size_t el = 1;
  switch (t) {
    case napi_int32_array:
    case napi_uint32_array:
    case napi_float32_array: el = 4; break;
    case napi_float64_array:
    case napi_bigint64_array:
    case napi_biguint64_array: el = 8; break;
    case napi_int16_array:
    case napi_uint16_array: el = 2; break;
    default: el = 1;
  }
  *len = n * el;
  return true;
}

// device buffer holding a copy of host bytes (freed by the destructor)
struct Dev {
  evm_ctx* ctx;
  void* p = nullptr;
  Dev(evm_ctx* c, size_t bytes, const void* host = nullptr) : ctx(c) {
    if (evm_dev_alloc(ctx, bytes ? bytes : 1, &p) != EVM_OK) p = nullptr;
    if (p && host && bytes) evm_copy_h2d(ctx, p, host, bytes);
  }
  ~Dev() {
    if (p) evm_dev_free(ctx, p);
  }
};

napi_value typed(napi_env env, napi_typedarray_type t, size_t n, size_t el, void** data) {
  napi_value ab, arr;
  napi_create_arraybuffer(env, n * el, data, &ab);
  napi_create_typedarray(env, t, n, ab, 0, &arr);
  return arr;
}

uint32_t u32(napi_env env, napi_value v) {
  uint32_t x = 0;
  napi_get_value_uint32(env, v, &x);
  return x;
}

// ---------------------------------------------------------------- context
napi_value Create(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  evm_ctx* ctx = nullptr;
  const int st = evm_create((int)u32(env, a[0]), &ctx);
  if (st) return throw_status(env, st, "evm_create");
  return make_ext(env, ctx);
}

napi_value Destroy(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  evm_destroy((evm_ctx*)ext(env, a[0]));
  return nullptr;
}

// ---------------------------------------------------------------- trees (types.ts:80-84)
napi_value TreeFromJson(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  uint32_t n = 0;
  NAPI_OK(env, napi_get_array_length(env, a[1], &n));
  std::vector<std::string> s(n);
  std::vector<const char*> p(n);
  std::vector<size_t> l(n);
  for (uint32_t i = 0; i < n; ++i) {
    napi_value e;
    NAPI_OK(env, napi_get_element(env, a[1], i, &e));
    size_t len = 0;
    NAPI_OK(env, napi_get_value_string_utf8(env, e, nullptr, 0, &len));
    s[i].resize(len + 1);
    NAPI_OK(env, napi_get_value_string_utf8(env, e, &s[i][0], len + 1, &len));
    s[i].resize(len);
    p[i] = s[i].data();
    l[i] = len;
  }
  evm_tree* t = nullptr;
  const int st = evm_tree_from_json(ctx, n, p.data(), l.data(), &t);
  if (st) return throw_status(env, st, "evm_tree_from_json");
  return make_ext(env, t);
}

napi_value TreeToJson(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!get_args(env, info, 3, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  const evm_tree* t = (const evm_tree*)ext(env, a[1]);
  size_t len = 0;
  int st = evm_tree_to_json(ctx, t, u32(env, a[2]), nullptr, 0, &len);
  if (st) return throw_status(env, st, "evm_tree_to_json");
  std::string out(len, '\0');
  st = evm_tree_to_json(ctx, t, u32(env, a[2]), &out[0], len, &len);
  if (st) return throw_status(env, st, "evm_tree_to_json");
  napi_value v;
  napi_create_string_utf8(env, out.data(), len, &v);
  return v;
}

napi_value TreeFree(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  evm_tree_free((evm_ctx*)ext(env, a[0]), (evm_tree*)ext(env, a[1]));
  return nullptr;
}

// merkleTree.ts:63-91 per owner -> Float64Array (millis; -1 none; -2 RangeError)
napi_value Diff(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!get_args(env, info, 3, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  const evm_tree* x = (const evm_tree*)ext(env, a[1]);
  const evm_tree* y = (const evm_tree*)ext(env, a[2]);
  uint32_t no = 0;
  evm_tree_info(x, &no, nullptr);
  Dev d(ctx, sizeof(int64_t) * (no ? no : 1));
  int st = evm_merkle_diff(ctx, x, y, (int64_t*)d.p);
  if (st) return throw_status(env, st, "evm_merkle_diff");
  std::vector<int64_t> h(no);
  evm_copy_d2h(ctx, h.data(), d.p, sizeof(int64_t) * no);
  double* out;
  napi_value arr = typed(env, napi_float64_array, no, 8, (void**)&out);
  for (uint32_t i = 0; i < no; ++i) out[i] = (double)h[i];
  return arr;
}

// merkleTree.ts:31-50 batched: insert(ctx, tree, ts Uint8Array, stride, owner Uint32Array|null)
napi_value Insert(napi_env env, napi_callback_info info) {
  napi_value a[5];
  if (!get_args(env, info, 5, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  const evm_tree* t = (const evm_tree*)ext(env, a[1]);
  void* ts;
  size_t tl;
  if (!bytes_of(env, a[2], &ts, &tl)) return nullptr;
  const size_t stride = u32(env, a[3]);
  const size_t n = stride ? tl / stride : 0;
  napi_valuetype vt;
  napi_typeof(env, a[4], &vt);
  void* ow = nullptr;
  size_t ol = 0;
  if (vt != napi_null && vt != napi_undefined && !bytes_of(env, a[4], &ow, &ol)) return nullptr;
  Dev dts(ctx, tl, ts), dow(ctx, ol, ow);
  evm_tree* out = nullptr;
  const int st = evm_merkle_insert(ctx, t, (const char*)dts.p, stride, n, ow ? (const uint32_t*)dow.p : nullptr, &out);
  if (st) return throw_status(env, st, "evm_merkle_insert");
  return make_ext(env, out);
}

// ---------------------------------------------------------------- applyMessages.ts:26-131
// applyBatch(ctx, tree, ts Uint8Array, stride, cell Uint32Array, nCells, priorTs|null, priorPresent|null)
//   -> { status, flags: Uint8Array, winner: Int32Array, tree }
napi_value ApplyBatch(napi_env env, napi_callback_info info) {
  napi_value a[8];
  if (!get_args(env, info, 8, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  const evm_tree* t = (const evm_tree*)ext(env, a[1]);
  void *ts, *cell, *pts = nullptr, *pp = nullptr;
  size_t tl, cl, ptl = 0, ppl = 0;
  if (!bytes_of(env, a[2], &ts, &tl) || !bytes_of(env, a[4], &cell, &cl)) return nullptr;
  const size_t stride = u32(env, a[3]);
  const uint32_t nc = u32(env, a[5]);
  napi_valuetype vt;
  napi_typeof(env, a[6], &vt);
  if (vt != napi_null && vt != napi_undefined) {
    if (!bytes_of(env, a[6], &pts, &ptl) || !bytes_of(env, a[7], &pp, &ppl)) return nullptr;
  }
  const size_t n = stride ? tl / stride : 0;
  Dev dts(ctx, tl, ts), dcell(ctx, cl, cell), dpts(ctx, ptl, pts), dpp(ctx, ppl, pp);
  Dev dflags(ctx, n), dwin(ctx, sizeof(int32_t) * (nc ? nc : 1));
  evm_tree* out = nullptr;
  const int st = evm_apply_batch(ctx, t, (const char*)dts.p, stride, n, (const uint32_t*)dcell.p, nc, nullptr,
                                 pts ? (const char*)dpts.p : nullptr, nc ? ptl / nc : 48,
                                 pp ? (const uint8_t*)dpp.p : nullptr, (uint8_t*)dflags.p, (int32_t*)dwin.p, &out);
  napi_value res, v;
  napi_create_object(env, &res);
  napi_create_int32(env, st, &v);
  napi_set_named_property(env, res, "status", v);
  if (st != EVM_OK && st != EVM_ENONCANON && st != EVM_ECOLLISION) return throw_status(env, st, "evm_apply_batch");
  void* fh;
  napi_value flags = typed(env, napi_uint8_array, n, 1, &fh);
  evm_copy_d2h(ctx, fh, dflags.p, n);
  napi_set_named_property(env, res, "flags", flags);
  void* wh;
  napi_value win = typed(env, napi_int32_array, nc, 4, &wh);
  evm_copy_d2h(ctx, wh, dwin.p, sizeof(int32_t) * nc);
  napi_set_named_property(env, res, "winner", win);
  if (out) napi_set_named_property(env, res, "tree", make_ext(env, out));
  return res;
}

// ---------------------------------------------------------------- server (index.ts)
napi_value StoreNew(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  evm_store* s = nullptr;
  const int st = evm_store_new((evm_ctx*)ext(env, a[0]), u32(env, a[1]), &s);
  if (st) return throw_status(env, st, "evm_store_new");
  return make_ext(env, s);
}

napi_value StoreFree(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  evm_store_free((evm_ctx*)ext(env, a[0]), (evm_store*)ext(env, a[1]));
  return nullptr;
}

napi_value StoreTree(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  return make_ext(env, (void*)evm_store_tree((evm_store*)ext(env, a[0])));
}

// serverIngest(ctx, store, ts Uint8Array, stride, owner Uint32Array, idBase) -> { status, flags }
napi_value ServerIngest(napi_env env, napi_callback_info info) {
  napi_value a[6];
  if (!get_args(env, info, 6, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  evm_store* s = (evm_store*)ext(env, a[1]);
  void *ts, *ow;
  size_t tl, ol;
  if (!bytes_of(env, a[2], &ts, &tl) || !bytes_of(env, a[4], &ow, &ol)) return nullptr;
  const size_t stride = u32(env, a[3]);
  const size_t n = stride ? tl / stride : 0;
  double base = 0;
  napi_get_value_double(env, a[5], &base);
  Dev dts(ctx, tl, ts), dow(ctx, ol, ow), dfl(ctx, n);
  const int st = evm_server_ingest(ctx, s, (const char*)dts.p, stride, n, (const uint32_t*)dow.p, (uint64_t)base,
                                   (uint8_t*)dfl.p);
  if (st != EVM_OK && st != EVM_ENONCANON) return throw_status(env, st, "evm_server_ingest");
  napi_value res, v;
  napi_create_object(env, &res);
  napi_create_int32(env, st, &v);
  napi_set_named_property(env, res, "status", v);
  void* fh;
  napi_value flags = typed(env, napi_uint8_array, n, 1, &fh);
  evm_copy_d2h(ctx, fh, dfl.p, n);
  napi_set_named_property(env, res, "flags", flags);
  return res;
}

// serverSelect(ctx, store, clientTree, node Uint8Array(16 * nOwners)) -> { diff, off, ids } (Float64Arrays)
napi_value ServerSelect(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  const evm_store* s = (const evm_store*)ext(env, a[1]);
  const evm_tree* c = (const evm_tree*)ext(env, a[2]);
  void* node;
  size_t nl;
  if (!bytes_of(env, a[3], &node, &nl)) return nullptr;
  uint32_t no = 0;
  uint64_t nm = 0;
  evm_store_info(s, &no, &nm);
  Dev dn(ctx, nl, node), dd(ctx, 8 * (no ? no : 1)), doff(ctx, 8 * (no + 1)), dids(ctx, 8 * (nm ? nm : 1));
  uint64_t nsel = 0;
  const int st = evm_server_select(ctx, s, c, (const char*)dn.p, nullptr, (int64_t*)dd.p, (uint64_t*)doff.p,
                                   (uint64_t*)dids.p, nm, &nsel);
  if (st) return throw_status(env, st, "evm_server_select");
  std::vector<int64_t> hd(no);
  std::vector<uint64_t> ho(no + 1), hi(nsel);
  evm_copy_d2h(ctx, hd.data(), dd.p, 8 * no);
  evm_copy_d2h(ctx, ho.data(), doff.p, 8 * (no + 1));
  evm_copy_d2h(ctx, hi.data(), dids.p, 8 * nsel);
  napi_value res;
  napi_create_object(env, &res);
  double* p;
  napi_value x = typed(env, napi_float64_array, no, 8, (void**)&p);
  for (uint32_t i = 0; i < no; ++i) p[i] = (double)hd[i];
  napi_set_named_property(env, res, "diff", x);
  x = typed(env, napi_float64_array, no + 1, 8, (void**)&p);
  for (uint32_t i = 0; i <= no; ++i) p[i] = (double)ho[i];
  napi_set_named_property(env, res, "off", x);
  x = typed(env, napi_float64_array, nsel, 8, (void**)&p);
  for (uint64_t i = 0; i < nsel; ++i) p[i] = (double)hi[i];
  napi_set_named_property(env, res, "ids", x);
  return res;
}

// storeSince(ctx, store, since Float64Array(nOwners), -1 = none) -> { off, ids } (Float64Arrays)
// receive.ts:118-124 resend range over a store that mirrors "__message"
napi_value StoreSince(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!get_args(env, info, 3, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  const evm_store* s = (const evm_store*)ext(env, a[1]);
  void* sv;
  size_t sl;
  if (!bytes_of(env, a[2], &sv, &sl)) return nullptr;
  uint32_t no = 0;
  uint64_t nm = 0;
  evm_store_info(s, &no, &nm);
  if (sl != 8ull * no) return throw_status(env, EVM_EINVAL, "storeSince: one since per owner");
  std::vector<int64_t> since(no);
  for (uint32_t i = 0; i < no; ++i) since[i] = (int64_t)((const double*)sv)[i];
  Dev ds(ctx, 8 * (no ? no : 1), since.data()), doff(ctx, 8 * (no + 1)), dids(ctx, 8 * (nm ? nm : 1));
  uint64_t nsel = 0;
  const int st = evm_store_since(ctx, s, (const int64_t*)ds.p, (uint64_t*)doff.p, (uint64_t*)dids.p, nm, &nsel);
  if (st) return throw_status(env, st, "evm_store_since");
  std::vector<uint64_t> ho(no + 1), hi(nsel);
  evm_copy_d2h(ctx, ho.data(), doff.p, 8 * (no + 1));
  evm_copy_d2h(ctx, hi.data(), dids.p, 8 * nsel);
  napi_value res;
  napi_create_object(env, &res);
  double* p;
  napi_value x = typed(env, napi_float64_array, no + 1, 8, (void**)&p);
  for (uint32_t i = 0; i <= no; ++i) p[i] = (double)ho[i];
  napi_set_named_property(env, res, "off", x);
  x = typed(env, napi_float64_array, nsel, 8, (void**)&p);
  for (uint64_t i = 0; i < nsel; ++i) p[i] = (double)hi[i];
  napi_set_named_property(env, res, "ids", x);
  return res;
}

// receiveFold(ctx, ts Uint8Array, stride, millis, counter, node string, now, maxDrift)
//   -> { error, index, next, millis, counter }     (receive.ts:45-66)
napi_value ReceiveFold(napi_env env, napi_callback_info info) {
  napi_value a[8];
  if (!get_args(env, info, 8, a)) return nullptr;
  evm_ctx* ctx = (evm_ctx*)ext(env, a[0]);
  void* ts;
  size_t tl;
  if (!bytes_of(env, a[1], &ts, &tl)) return nullptr;
  const size_t stride = u32(env, a[2]);
  double millis = 0, now = 0, drift = 0;
  napi_get_value_double(env, a[3], &millis);
  napi_get_value_double(env, a[6], &now);
  napi_get_value_double(env, a[7], &drift);
  char node[17] = {0};
  size_t nl = 0;
  NAPI_OK(env, napi_get_value_string_latin1(env, a[5], node, sizeof node, &nl));
  if (nl != 16) return throw_status(env, EVM_EINVAL, "receiveFold: nodeId must be 16 chars");
  Dev dts(ctx, tl, ts);
  evm_clock_result r;
  const int st = evm_receive_fold(ctx, (const char*)dts.p, stride, stride ? tl / stride : 0, (int64_t)millis,
                                  u32(env, a[4]), node, (int64_t)now, (int64_t)drift, &r);
  if (st) return throw_status(env, st, "evm_receive_fold");
  napi_value res, v;
  napi_create_object(env, &res);
  const double vals[5] = {(double)r.error, (double)r.error_index, (double)r.next, (double)r.millis,
                          (double)r.counter};
  const char* names[5] = {"error", "index", "next", "millis", "counter"};
  for (int k = 0; k < 5; ++k) {
    napi_create_double(env, vals[k], &v);
    napi_set_named_property(env, res, names[k], v);
  }
  return res;
}

// pbDecode(kind, body Uint8Array) -> { ts Uint8Array(n * 48), tsLen, contentOff (Float64Array), content,
//   userId, nodeId, merkleTree }      (SyncRequest / SyncResponse fromBinary)
napi_value PbDecode(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  const int kind = (int)u32(env, a[0]);
  void* body;
  size_t bl;
  if (!bytes_of(env, a[1], &body, &bl)) return nullptr;
  evm_pb_sync si;
  int st = evm_pb_scan(kind, (const uint8_t*)body, bl, &si);
  if (st) return throw_status(env, st, "evm_pb_scan");
  const size_t n = si.n_messages;
  void *tsp, *tlp, *cp;
  napi_value ts = typed(env, napi_uint8_array, n * 48, 1, &tsp);
  napi_value tl = typed(env, napi_uint32_array, n, 4, &tlp);
  napi_value content = typed(env, napi_uint8_array, si.content_bytes, 1, &cp);
  std::vector<uint64_t> off(n + 1), toff(n);
  st = evm_pb_split(kind, (const uint8_t*)body, bl, (char*)tsp, 48, (uint32_t*)tlp, toff.data(), off.data(),
                    (uint8_t*)cp);
  if (st) return throw_status(env, st, "evm_pb_split");
  double* op;
  napi_value co = typed(env, napi_float64_array, n + 1, 8, (void**)&op);
  for (size_t i = 0; i <= n; ++i) op[i] = (double)off[i];
  napi_value res, v;
  napi_create_object(env, &res);
  napi_set_named_property(env, res, "ts", ts);
  napi_set_named_property(env, res, "tsLen", tl);
  napi_set_named_property(env, res, "contentOff", co);
  {
    double* tp;
    napi_value to = typed(env, napi_float64_array, n, 8, (void**)&tp);
    for (size_t i = 0; i < n; ++i) tp[i] = (double)toff[i];
    napi_set_named_property(env, res, "tsOff", to);
  }
  napi_set_named_property(env, res, "content", content);
  const char* b = (const char*)body;
  napi_create_string_utf8(env, b + si.tree_off, si.tree_len, &v);
  napi_set_named_property(env, res, "merkleTree", v);
  if (kind == EVM_PB_SYNC_REQUEST) {
    napi_create_string_utf8(env, b + si.user_off, si.user_len, &v);
    napi_set_named_property(env, res, "userId", v);
    napi_create_string_utf8(env, b + si.node_off, si.node_len, &v);
    napi_set_named_property(env, res, "nodeId", v);
  }
  return res;
}

std::string str_of(napi_env env, napi_value v) {
  size_t n = 0;
  napi_get_value_string_utf8(env, v, nullptr, 0, &n);
  std::string s(n, '\0');
  if (n) napi_get_value_string_utf8(env, v, &s[0], n + 1, &n);
  return s;
}

// pbEncode(kind, ts Uint8Array(n * 48), content Uint8Array, contentOff Float64Array(n + 1),
//          userId, nodeId, merkleTree) -> Uint8Array   (toBinary; 46-byte timestamps)
napi_value PbEncode(napi_env env, napi_callback_info info) {
  napi_value a[7];
  if (!get_args(env, info, 7, a)) return nullptr;
  const int kind = (int)u32(env, a[0]);
  void *ts, *content, *offv;
  size_t tl, cl, ol;
  if (!bytes_of(env, a[1], &ts, &tl) || !bytes_of(env, a[2], &content, &cl) || !bytes_of(env, a[3], &offv, &ol))
    return nullptr;
  const size_t n = tl / 48;
  if (ol != 8 * (n + 1)) return throw_status(env, EVM_EINVAL, "pbEncode: contentOff must have n + 1 entries");
  std::vector<uint64_t> off(n + 1);
  for (size_t i = 0; i <= n; ++i) off[i] = (uint64_t)((const double*)offv)[i];
  const std::string user = str_of(env, a[4]), node = str_of(env, a[5]), tree = str_of(env, a[6]);
  size_t need = 0;
  int st = evm_pb_encode(kind, (const char*)ts, 48, nullptr, n, off.data(), (const uint8_t*)content, user.data(),
                         user.size(), node.data(), node.size(), tree.data(), tree.size(), nullptr, 0, &need);
  if (st) return throw_status(env, st, "evm_pb_encode");
  void* out;
  napi_value arr = typed(env, napi_uint8_array, need, 1, &out);
  st = evm_pb_encode(kind, (const char*)ts, 48, nullptr, n, off.data(), (const uint8_t*)content, user.data(),
                     user.size(), node.data(), node.size(), tree.data(), tree.size(), (uint8_t*)out, need, &need);
  if (st) return throw_status(env, st, "evm_pb_encode");
  return arr;
}

napi_value Init(napi_env env, napi_value exports) {
  const struct {
    const char* name;
    napi_callback fn;
  } fns[] = {{"create", Create},         {"destroy", Destroy},       {"treeFromJson", TreeFromJson},
             {"treeToJson", TreeToJson}, {"treeFree", TreeFree},     {"diff", Diff},
             {"insert", Insert},         {"applyBatch", ApplyBatch}, {"storeNew", StoreNew},
             {"storeFree", StoreFree},   {"storeTree", StoreTree},   {"serverIngest", ServerIngest},
             {"serverSelect", ServerSelect}, {"storeSince", StoreSince}, {"receiveFold", ReceiveFold},
             {"pbDecode", PbDecode},         {"pbEncode", PbEncode}};
  for (const auto& f : fns) {
    napi_value v;
    napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.fn, nullptr, &v);
    napi_set_named_property(env, exports, f.name, v);
  }
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
