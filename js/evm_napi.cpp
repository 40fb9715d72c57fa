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

#include <functional>
#include <mutex>
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

// A context handle: the engine context plus a mutex, so calls from the JS
// thread and async work on libuv's pool never drive the context at once (one
// context per thread at a time, include/evm.h).
struct Ctx {
  evm_ctx* c;
  std::mutex m;
};
Ctx* ctx_of(napi_env env, napi_value v) { return static_cast<Ctx*>(ext(env, v)); }

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
  Ctx* c = new Ctx();
  c->c = ctx;
  return make_ext(env, c);
}

napi_value Destroy(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  Ctx* c = ctx_of(env, a[0]);
  {
    std::lock_guard<std::mutex> g(c->m);
    evm_destroy(c->c);
  }
  delete c;
  return nullptr;
}

// ---------------------------------------------------------------- trees (types.ts:80-84)
napi_value TreeFromJson(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
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
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
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
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_tree_free(cx->c, (evm_tree*)ext(env, a[1]));
  return nullptr;
}

// merkleTree.ts:63-91 per owner -> Float64Array (millis; -1 none; -2 RangeError)
napi_value Diff(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!get_args(env, info, 3, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
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
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
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

// ---------------------------------------------------------------- async work
// applyMessages is a ReaderTaskEither (applyMessages.ts:26-31): the *Async
// entry points run the batch on libuv's pool (napi_create_async_work) and
// return a Promise of an fp-ts Either -- { _tag: "Right", right } or
// { _tag: "Left", left: UnknownError } (types.ts:358-372) -- so the worker's
// event loop is never blocked on the GPU.  The caller's typed arrays are
// held by references until the work completes.
struct Async {
  Ctx* cx;
  napi_deferred deferred = nullptr;
  napi_async_work work = nullptr;
  std::vector<napi_ref> refs;
  std::function<int()> exec;                    // on the pool thread, context locked and bound
  std::function<napi_value(napi_env, int)> done;  // on the JS thread: the Right value for a status
  int status = EVM_OK;
};

napi_value either(napi_env env, bool right, napi_value v) {
  napi_value o, tag;
  napi_create_object(env, &o);
  napi_create_string_utf8(env, right ? "Right" : "Left", NAPI_AUTO_LENGTH, &tag);
  napi_set_named_property(env, o, "_tag", tag);
  napi_set_named_property(env, o, right ? "right" : "left", v);
  return o;
}

// UnknownError { type, error: { message, stack } } (types.ts:358-372)
napi_value unknown_error(napi_env env, int st, const char* where) {
  napi_value err, inner, v;
  napi_create_object(env, &err);
  napi_create_string_utf8(env, "UnknownError", NAPI_AUTO_LENGTH, &v);
  napi_set_named_property(env, err, "type", v);
  napi_create_object(env, &inner);
  const std::string m = std::string(where) + ": " + evm_strerror(st);
  napi_create_string_utf8(env, m.c_str(), m.size(), &v);
  napi_set_named_property(env, inner, "message", v);
  napi_get_undefined(env, &v);
  napi_set_named_property(env, inner, "stack", v);
  napi_set_named_property(env, err, "error", inner);
  return err;
}

void async_execute(napi_env, void* data) {
  Async* a = static_cast<Async*>(data);
  std::lock_guard<std::mutex> lock(a->cx->m);
  a->status = evm_bind_thread(a->cx->c);
  if (!a->status) a->status = a->exec();
}

void async_complete(napi_env env, napi_status, void* data) {
  Async* a = static_cast<Async*>(data);
  napi_value v = a->done(env, a->status);  // null: a device error
  if (v) napi_resolve_deferred(env, a->deferred, either(env, true, v));
  else napi_resolve_deferred(env, a->deferred, either(env, false, unknown_error(env, a->status, "evolu_evm")));
  for (napi_ref r : a->refs) napi_delete_reference(env, r);
  napi_delete_async_work(env, a->work);
  delete a;
}

// queues `a`, keeping the given values alive; -> the Promise
napi_value queue(napi_env env, Async* a, napi_value* keep, size_t nkeep) {
  for (size_t i = 0; i < nkeep; ++i) {
    napi_valuetype t;
    napi_typeof(env, keep[i], &t);
    if (t != napi_object) continue;
    napi_ref r;
    if (napi_create_reference(env, keep[i], 1, &r) == napi_ok) a->refs.push_back(r);
  }
  napi_value promise, name;
  napi_create_promise(env, &a->deferred, &promise);
  napi_create_string_utf8(env, "evolu_evm", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, nullptr, name, async_execute, async_complete, a, &a->work);
  napi_queue_async_work(env, a->work);
  return promise;
}

bool is_null(napi_env env, napi_value v) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  return t == napi_null || t == napi_undefined;
}

// ---------------------------------------------------------------- applyMessages.ts:26-131
// applyBatch(ctx, tree, ts Uint8Array, stride, cell Uint32Array, nCells, priorTs|null, priorPresent|null
//            [, storedTs|null, storedCell|null])
//   -> { status, flags: Uint8Array, winner: Int32Array, tree }
// storedTs / storedCell: the __message rows holding a batch timestamp
// (SELECT ... WHERE "timestamp" IN (...)), evm_apply_batch_ex.
struct ApplyJob {
  evm_ctx* ctx = nullptr;
  const evm_tree* t = nullptr;
  void *ts = nullptr, *cell = nullptr, *pts = nullptr, *pp = nullptr, *sts = nullptr, *sc = nullptr;
  size_t tl = 0, cl = 0, ptl = 0, ppl = 0, stl = 0, scl = 0, stride = 48;
  uint32_t nc = 0;
  std::vector<uint8_t> flags;
  std::vector<int32_t> winner;
  evm_tree* out = nullptr;

  bool parse(napi_env env, napi_value* a, size_t argc) {
    if (!bytes_of(env, a[2], &ts, &tl) || !bytes_of(env, a[4], &cell, &cl)) return false;
    stride = u32(env, a[3]);
    nc = u32(env, a[5]);
    if (!is_null(env, a[6]) && (!bytes_of(env, a[6], &pts, &ptl) || !bytes_of(env, a[7], &pp, &ppl))) return false;
    if (argc >= 10 && !is_null(env, a[8]) && (!bytes_of(env, a[8], &sts, &stl) || !bytes_of(env, a[9], &sc, &scl)))
      return false;
    return true;
  }
  // H2D, the batch, D2H -- on the calling thread, context locked
  int run() {
    const size_t n = stride ? tl / stride : 0;
    const size_t ns = scl / 4;
    Dev dts(ctx, tl, ts), dcell(ctx, cl, cell), dpts(ctx, ptl, pts), dpp(ctx, ppl, pp), dsts(ctx, stl, sts),
        dsc(ctx, scl, sc);
    Dev dflags(ctx, n), dwin(ctx, sizeof(int32_t) * (nc ? nc : 1));
    const int st = evm_apply_batch_ex(ctx, t, (const char*)dts.p, stride, n, (const uint32_t*)dcell.p, nc, nullptr,
                                      pts ? (const char*)dpts.p : nullptr, nc ? ptl / nc : 48,
                                      pp ? (const uint8_t*)dpp.p : nullptr, ns ? (const char*)dsts.p : nullptr,
                                      ns ? stl / ns : 48, ns, ns ? (const uint32_t*)dsc.p : nullptr,
                                      (uint8_t*)dflags.p, (int32_t*)dwin.p, &out);
    if (st != EVM_OK && st != EVM_ENONCANON && st != EVM_ECOLLISION) return st;
    flags.resize(n);
    winner.resize(nc);
    evm_copy_d2h(ctx, flags.data(), dflags.p, n);
    evm_copy_d2h(ctx, winner.data(), dwin.p, sizeof(int32_t) * nc);
    return st;
  }
  napi_value result(napi_env env, int st) {
    napi_value res, v;
    napi_create_object(env, &res);
    napi_create_int32(env, st, &v);
    napi_set_named_property(env, res, "status", v);
    void* fh;
    napi_value fl = typed(env, napi_uint8_array, flags.size(), 1, &fh);
    if (!flags.empty()) memcpy(fh, flags.data(), flags.size());
    napi_set_named_property(env, res, "flags", fl);
    void* wh;
    napi_value win = typed(env, napi_int32_array, winner.size(), 4, &wh);
    if (!winner.empty()) memcpy(wh, winner.data(), 4 * winner.size());
    napi_set_named_property(env, res, "winner", win);
    if (out) napi_set_named_property(env, res, "tree", make_ext(env, out));
    return res;
  }
};

napi_value ApplyBatch(napi_env env, napi_callback_info info) {
  napi_value a[10];
  size_t argc = 10;
  if (napi_get_cb_info(env, info, &argc, a, nullptr, nullptr) != napi_ok || argc < 8) {
    napi_throw_type_error(env, nullptr, "missing arguments");
    return nullptr;
  }
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  ApplyJob j;
  j.ctx = cx->c;
  j.t = (const evm_tree*)ext(env, a[1]);
  if (!j.parse(env, a, argc)) return nullptr;
  const int st = j.run();
  if (st != EVM_OK && st != EVM_ENONCANON && st != EVM_ECOLLISION) return throw_status(env, st, "evm_apply_batch");
  return j.result(env, st);
}

// applyBatchAsync(same arguments) -> Promise<Either<UnknownError, { status, flags, winner, tree }>>
napi_value ApplyBatchAsync(napi_env env, napi_callback_info info) {
  napi_value a[10];
  size_t argc = 10;
  if (napi_get_cb_info(env, info, &argc, a, nullptr, nullptr) != napi_ok || argc < 8) {
    napi_throw_type_error(env, nullptr, "missing arguments");
    return nullptr;
  }
  auto* j = new ApplyJob();
  Async* as = new Async();
  as->cx = ctx_of(env, a[0]);
  j->ctx = as->cx->c;
  j->t = (const evm_tree*)ext(env, a[1]);
  if (!j->parse(env, a, argc)) {
    delete j;
    delete as;
    return nullptr;
  }
  as->exec = [j]() {
    const int st = j->run();
    return st;
  };
  as->done = [j](napi_env e, int st) -> napi_value {
    napi_value v = nullptr;
    if (st == EVM_OK || st == EVM_ENONCANON || st == EVM_ECOLLISION) v = j->result(e, st);
    delete j;
    return v;
  };
  return queue(env, as, a + 1, argc - 1);
}

// ---------------------------------------------------------------- server (index.ts)
napi_value StoreNew(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  evm_store* s = nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  const int st = evm_store_new(cx->c, u32(env, a[1]), &s);
  if (st) return throw_status(env, st, "evm_store_new");
  return make_ext(env, s);
}

napi_value StoreFree(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_store_free(cx->c, (evm_store*)ext(env, a[1]));
  return nullptr;
}

napi_value StoreTree(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  return make_ext(env, (void*)evm_store_tree((evm_store*)ext(env, a[0])));
}

// serverIngest(ctx, store, ts Uint8Array, stride, owner Uint32Array, idBase) -> { status, flags }
struct IngestJob {
  evm_ctx* ctx = nullptr;
  evm_store* s = nullptr;
  void *ts = nullptr, *ow = nullptr;
  size_t tl = 0, ol = 0, stride = 48;
  double base = 0;
  std::vector<uint8_t> flags;
  bool parse(napi_env env, napi_value* a) {
    s = (evm_store*)ext(env, a[1]);
    if (!bytes_of(env, a[2], &ts, &tl) || !bytes_of(env, a[4], &ow, &ol)) return false;
    stride = u32(env, a[3]);
    napi_get_value_double(env, a[5], &base);
    return true;
  }
  int run() {
    const size_t n = stride ? tl / stride : 0;
    Dev dts(ctx, tl, ts), dow(ctx, ol, ow), dfl(ctx, n);
    const int st = evm_server_ingest(ctx, s, (const char*)dts.p, stride, n, (const uint32_t*)dow.p, (uint64_t)base,
                                     (uint8_t*)dfl.p);
    if (st != EVM_OK && st != EVM_ENONCANON) return st;
    flags.resize(n);
    evm_copy_d2h(ctx, flags.data(), dfl.p, n);
    return st;
  }
  napi_value result(napi_env env, int st) {
    napi_value res, v;
    napi_create_object(env, &res);
    napi_create_int32(env, st, &v);
    napi_set_named_property(env, res, "status", v);
    void* fh;
    napi_value fl = typed(env, napi_uint8_array, flags.size(), 1, &fh);
    if (!flags.empty()) memcpy(fh, flags.data(), flags.size());
    napi_set_named_property(env, res, "flags", fl);
    return res;
  }
};

napi_value ServerIngest(napi_env env, napi_callback_info info) {
  napi_value a[6];
  if (!get_args(env, info, 6, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  IngestJob j;
  j.ctx = cx->c;
  if (!j.parse(env, a)) return nullptr;
  const int st = j.run();
  if (st != EVM_OK && st != EVM_ENONCANON) return throw_status(env, st, "evm_server_ingest");
  return j.result(env, st);
}

napi_value ServerIngestAsync(napi_env env, napi_callback_info info) {
  napi_value a[6];
  if (!get_args(env, info, 6, a)) return nullptr;
  auto* j = new IngestJob();
  Async* as = new Async();
  as->cx = ctx_of(env, a[0]);
  j->ctx = as->cx->c;
  if (!j->parse(env, a)) {
    delete j;
    delete as;
    return nullptr;
  }
  as->exec = [j]() { return j->run(); };
  as->done = [j](napi_env e, int st) -> napi_value {
    napi_value v = (st == EVM_OK || st == EVM_ENONCANON) ? j->result(e, st) : nullptr;
    delete j;
    return v;
  };
  return queue(env, as, a + 1, 5);
}

// serverSelect(ctx, store, clientTree, node Uint8Array(16 * nOwners)) -> { diff, off, ids } (Float64Arrays)
struct SelectJob {
  evm_ctx* ctx = nullptr;
  const evm_store* s = nullptr;
  const evm_tree* c = nullptr;
  void* node = nullptr;
  size_t nl = 0;
  std::vector<int64_t> hd;
  std::vector<uint64_t> ho, hi;
  bool parse(napi_env env, napi_value* a) {
    s = (const evm_store*)ext(env, a[1]);
    c = (const evm_tree*)ext(env, a[2]);
    return bytes_of(env, a[3], &node, &nl);
  }
  int run() {
    uint32_t no = 0;
    uint64_t nm = 0;
    evm_store_info(s, &no, &nm);
    Dev dn(ctx, nl, node), dd(ctx, 8 * (no ? no : 1)), doff(ctx, 8 * (no + 1)), dids(ctx, 8 * (nm ? nm : 1));
    uint64_t nsel = 0;
    const int st = evm_server_select(ctx, s, c, (const char*)dn.p, nullptr, (int64_t*)dd.p, (uint64_t*)doff.p,
                                     (uint64_t*)dids.p, nm, &nsel);
    if (st) return st;
    hd.resize(no);
    ho.resize(no + 1);
    hi.resize(nsel);
    evm_copy_d2h(ctx, hd.data(), dd.p, 8 * no);
    evm_copy_d2h(ctx, ho.data(), doff.p, 8 * (no + 1));
    evm_copy_d2h(ctx, hi.data(), dids.p, 8 * nsel);
    return EVM_OK;
  }
  napi_value result(napi_env env) {
    napi_value res;
    napi_create_object(env, &res);
    double* p;
    napi_value x = typed(env, napi_float64_array, hd.size(), 8, (void**)&p);
    for (size_t i = 0; i < hd.size(); ++i) p[i] = (double)hd[i];
    napi_set_named_property(env, res, "diff", x);
    x = typed(env, napi_float64_array, ho.size(), 8, (void**)&p);
    for (size_t i = 0; i < ho.size(); ++i) p[i] = (double)ho[i];
    napi_set_named_property(env, res, "off", x);
    x = typed(env, napi_float64_array, hi.size(), 8, (void**)&p);
    for (size_t i = 0; i < hi.size(); ++i) p[i] = (double)hi[i];
    napi_set_named_property(env, res, "ids", x);
    return res;
  }
};

napi_value ServerSelect(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  SelectJob j;
  j.ctx = cx->c;
  if (!j.parse(env, a)) return nullptr;
  const int st = j.run();
  if (st) return throw_status(env, st, "evm_server_select");
  return j.result(env);
}

napi_value ServerSelectAsync(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  auto* j = new SelectJob();
  Async* as = new Async();
  as->cx = ctx_of(env, a[0]);
  j->ctx = as->cx->c;
  if (!j->parse(env, a)) {
    delete j;
    delete as;
    return nullptr;
  }
  as->exec = [j]() { return j->run(); };
  as->done = [j](napi_env e, int st) -> napi_value {
    napi_value v = st == EVM_OK ? j->result(e) : nullptr;
    delete j;
    return v;
  };
  return queue(env, as, a + 1, 3);
}

// storeSince(ctx, store, since Float64Array(nOwners), -1 = none) -> { off, ids } (Float64Arrays)
// receive.ts:118-124 resend range over a store that mirrors "__message"
napi_value StoreSince(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!get_args(env, info, 3, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
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
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
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
  char none[48];  // (a body without messages: a zero-length typed array may have no data pointer)
  st = evm_pb_split(kind, (const uint8_t*)body, bl, n ? (char*)tsp : none, 48, (uint32_t*)tlp, toff.data(), off.data(),
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

// ---------------------------------------------------------------- multi-GPU (evm_dist_*)
// One addon instance per GPU process; rank 0 makes the id and hands it to the others.
// distUniqueId() -> Uint8Array(128)
napi_value DistUniqueId(napi_env env, napi_callback_info) {
  void* p;
  napi_value arr = typed(env, napi_uint8_array, EVM_DIST_ID_BYTES, 1, &p);
  const int st = evm_dist_unique_id((uint8_t*)p);
  if (st) return throw_status(env, st, "evm_dist_unique_id");
  return arr;
}

// distInit(ctx, id, rank, world) -> handle   (collective, blocks until every rank joined)
napi_value DistInit(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  void* id;
  size_t il;
  if (!bytes_of(env, a[1], &id, &il)) return nullptr;
  if (il != EVM_DIST_ID_BYTES) return throw_status(env, EVM_EINVAL, "distInit: id must be 128 bytes");
  evm_dist* d = nullptr;
  const int st = evm_dist_init(cx->c, (const uint8_t*)id, (int)u32(env, a[2]), (int)u32(env, a[3]), &d);
  if (st) return throw_status(env, st, "evm_dist_init");
  return make_ext(env, d);
}

napi_value DistFree(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_dist_free(cx->c, (evm_dist*)ext(env, a[1]));
  return nullptr;
}

// distRoute(ctx, d, ts Uint8Array(n * stride), stride, owner Uint32Array, aux Uint32Array | null)
//   -> { ts, owner, aux, src (Float64Array: source rank * 2^32 + index) }   (collective)
napi_value DistRoute(napi_env env, napi_callback_info info) {
  napi_value a[7];
  size_t argc = 7;
  napi_get_undefined(env, &a[6]);
  if (napi_get_cb_info(env, info, &argc, a, nullptr, nullptr) != napi_ok || argc < 6) {
    napi_throw_type_error(env, nullptr, "missing arguments");
    return nullptr;
  }
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  evm_dist* d = (evm_dist*)ext(env, a[1]);
  void *ts, *ow, *ax = nullptr;
  size_t tl, ol, al = 0;
  if (!bytes_of(env, a[2], &ts, &tl) || !bytes_of(env, a[4], &ow, &ol)) return nullptr;
  if (!is_null(env, a[5]) && !bytes_of(env, a[5], &ax, &al)) return nullptr;
  const size_t stride = u32(env, a[3]);
  const size_t n = ol / 4;
  if (!stride || tl != n * stride || (ax && al != ol)) return throw_status(env, EVM_EINVAL, "distRoute: sizes");
  void* de = nullptr;
  size_t dl = 0;
  napi_valuetype t6;
  napi_typeof(env, a[6], &t6);
  if (argc >= 7 && t6 != napi_undefined && !is_null(env, a[6]) && !bytes_of(env, a[6], &de, &dl)) return nullptr;
  if (de && dl != n) return throw_status(env, EVM_EINVAL, "distRoute: dest must have one rank per row");
  Dev dts(ctx, tl, ts), dow(ctx, ol, ow), dax(ctx, ax ? al : 1, ax), dde(ctx, de ? dl : 1, de);
  uint64_t nr = 0;
  int st = evm_dist_route(ctx, d, (const char*)dts.p, stride, n, (const uint32_t*)dow.p,
                          ax ? (const uint32_t*)dax.p : nullptr, de ? (const uint8_t*)dde.p : nullptr, &nr);
  if (st) return throw_status(env, st, "evm_dist_route");
  Dev rts(ctx, nr * stride), row(ctx, nr * 4), rax(ctx, nr * 4), rsrc(ctx, nr * 8);
  st = evm_dist_take(ctx, d, 0, (char*)rts.p, stride, (uint32_t*)row.p, (uint32_t*)rax.p, (uint64_t*)rsrc.p, nr,
                     nullptr);
  if (st) return throw_status(env, st, "evm_dist_take");
  void *hts, *how, *hax;
  napi_value vts = typed(env, napi_uint8_array, nr * stride, 1, &hts);
  napi_value vow = typed(env, napi_uint32_array, nr, 4, &how);
  napi_value vax = typed(env, napi_uint32_array, nr, 4, &hax);
  std::vector<uint64_t> src(nr);
  evm_copy_d2h(ctx, hts, rts.p, nr * stride);
  evm_copy_d2h(ctx, how, row.p, nr * 4);
  evm_copy_d2h(ctx, hax, rax.p, nr * 4);
  evm_copy_d2h(ctx, src.data(), rsrc.p, nr * 8);
  double* sp;
  napi_value vsrc = typed(env, napi_float64_array, nr, 8, (void**)&sp);
  for (uint64_t i = 0; i < nr; ++i) sp[i] = (double)(src[i] >> 32) * 4294967296.0 + (double)(uint32_t)src[i];
  napi_value res;
  napi_create_object(env, &res);
  napi_set_named_property(env, res, "ts", vts);
  napi_set_named_property(env, res, "owner", vow);
  napi_set_named_property(env, res, "aux", vax);
  napi_set_named_property(env, res, "src", vsrc);
  return res;
}

// distIngest(ctx, d, store, idBase) -> { status, flags Uint8Array(nRecv) }   (local)
// addMessages of the last distRoute's rows into this rank's store, read from
// the received records (evm_dist_ingest); row i (receive order, as distRoute
// returned it) has id idBase + i
napi_value DistIngest(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  evm_dist* d = (evm_dist*)ext(env, a[1]);
  evm_store* s = (evm_store*)ext(env, a[2]);
  double base = 0;
  napi_get_value_double(env, a[3], &base);
  const uint64_t n = evm_dist_received(d);
  Dev dfl(ctx, n ? n : 1);
  const int st = evm_dist_ingest(ctx, d, s, (uint64_t)base, (uint8_t*)dfl.p);
  if (st != EVM_OK && st != EVM_ENONCANON) return throw_status(env, st, "evm_dist_ingest");
  void* fh;
  napi_value fl = typed(env, napi_uint8_array, n, 1, &fh);
  if (n) evm_copy_d2h(ctx, fh, dfl.p, n);
  napi_value res, v;
  napi_create_object(env, &res);
  napi_create_int32(env, st, &v);
  napi_set_named_property(env, res, "status", v);
  napi_set_named_property(env, res, "flags", fl);
  return res;
}

// distGatherRoots(ctx, d, tree, nOwnersGlobal) -> { root Int32Array, present Uint8Array }   (collective)
napi_value DistGatherRoots(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  const uint32_t ng = u32(env, a[3]);
  Dev dr(ctx, 4 * (ng ? ng : 1)), dp(ctx, ng ? ng : 1);
  const evm_tree* t = (const evm_tree*)ext(env, a[2]);
  const int st = evm_dist_gather_roots(ctx, (evm_dist*)ext(env, a[1]), &t, 1, ng, (int32_t*)dr.p, (uint8_t*)dp.p);
  if (st) return throw_status(env, st, "evm_dist_gather_roots");
  void *hr, *hp;
  napi_value vr = typed(env, napi_int32_array, ng, 4, &hr);
  napi_value vp = typed(env, napi_uint8_array, ng, 1, &hp);
  evm_copy_d2h(ctx, hr, dr.p, 4ull * ng);
  evm_copy_d2h(ctx, hp, dp.p, ng);
  napi_value res;
  napi_create_object(env, &res);
  napi_set_named_property(env, res, "root", vr);
  napi_set_named_property(env, res, "present", vp);
  return res;
}

// ---- loopback ranks (worker threads of one process, one GPU): the hub travels as a BigInt address
napi_value DistHubNew(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  evm_dist_hub* h = nullptr;
  const int st = evm_dist_hub_new((int)u32(env, a[0]), &h);
  if (st) return throw_status(env, st, "evm_dist_hub_new");
  napi_value v;
  napi_create_bigint_uint64(env, (uint64_t)(uintptr_t)h, &v);
  return v;
}

evm_dist_hub* hub_of(napi_env env, napi_value v) {
  uint64_t x = 0;
  bool lossless = false;
  napi_get_value_bigint_uint64(env, v, &x, &lossless);
  return (evm_dist_hub*)(uintptr_t)x;
}

napi_value DistHubFree(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  evm_dist_hub_free(hub_of(env, a[0]));
  return nullptr;
}

napi_value DistHubAbort(napi_env env, napi_callback_info info) {
  napi_value a[1];
  if (!get_args(env, info, 1, a)) return nullptr;
  evm_dist_hub_abort(hub_of(env, a[0]));
  return nullptr;
}

// distInitLoopback(ctx, hub BigInt, rank) -> handle   (collectives block until every rank's thread joins)
napi_value DistInitLoopback(napi_env env, napi_callback_info info) {
  napi_value a[3];
  if (!get_args(env, info, 3, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_dist* d = nullptr;
  const int st = evm_dist_init_loopback(cx->c, hub_of(env, a[1]), (int)u32(env, a[2]), &d);
  if (st) return throw_status(env, st, "evm_dist_init_loopback");
  return make_ext(env, d);
}

// distDirectory(ctx, d, ids Uint8Array(n * stride), stride, idLen) -> { dest Uint8Array, local Uint32Array, nLocal }
napi_value DistDirectory(napi_env env, napi_callback_info info) {
  napi_value a[5];
  if (!get_args(env, info, 5, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  void* ids;
  size_t il;
  if (!bytes_of(env, a[2], &ids, &il)) return nullptr;
  const size_t stride = u32(env, a[3]), id_len = u32(env, a[4]);
  if (!stride || il % stride) return throw_status(env, EVM_EINVAL, "distDirectory: sizes");
  const uint32_t n = (uint32_t)(il / stride);
  Dev dids(ctx, il, ids), ddest(ctx, n), dloc(ctx, 4ull * n);
  uint32_t nl = 0;
  const int st = evm_dist_directory(ctx, (evm_dist*)ext(env, a[1]), (const char*)dids.p, stride, id_len, n,
                                    (uint8_t*)ddest.p, (uint32_t*)dloc.p, &nl);
  if (st) return throw_status(env, st, "evm_dist_directory");
  void *hd, *hl;
  napi_value vd = typed(env, napi_uint8_array, n, 1, &hd);
  napi_value vl = typed(env, napi_uint32_array, n, 4, &hl);
  evm_copy_d2h(ctx, hd, ddest.p, n);
  evm_copy_d2h(ctx, hl, dloc.p, 4ull * n);
  napi_value res, v;
  napi_create_object(env, &res);
  napi_set_named_property(env, res, "dest", vd);
  napi_set_named_property(env, res, "local", vl);
  napi_create_uint32(env, nl, &v);
  napi_set_named_property(env, res, "nLocal", v);
  return res;
}

// distHotOwners(ctx, d, owner Uint32Array, nGlobal, share) -> Uint32Array (sorted)   (collective)
napi_value DistHotOwners(napi_env env, napi_callback_info info) {
  napi_value a[5];
  if (!get_args(env, info, 5, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  void* ow;
  size_t ol;
  if (!bytes_of(env, a[2], &ow, &ol)) return nullptr;
  double share = 0.25;
  napi_get_value_double(env, a[4], &share);
  const uint32_t ng = u32(env, a[3]);
  Dev dow(ctx, ol, ow);
  std::vector<uint32_t> hot(4096);
  uint32_t nh = 0;
  const int st = evm_dist_hot_owners(ctx, (evm_dist*)ext(env, a[1]), (const uint32_t*)dow.p, ol / 4, ng, share,
                                     hot.data(), (uint32_t)hot.size(), &nh);
  if (st) return throw_status(env, st, "evm_dist_hot_owners");
  void* hp;
  napi_value vh = typed(env, napi_uint32_array, nh, 4, &hp);
  if (nh) memcpy(hp, hot.data(), 4ull * nh);
  return vh;
}

// distSplit(ctx, d, hot Uint32Array, nGlobal) -> hotBase
napi_value DistSplit(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  void* hot;
  size_t hl;
  if (!bytes_of(env, a[2], &hot, &hl)) return nullptr;
  uint32_t base = 0;
  const int st = evm_dist_split(cx->c, (evm_dist*)ext(env, a[1]), (const uint32_t*)hot, (uint32_t)(hl / 4),
                                u32(env, a[3]), &base);
  if (st) return throw_status(env, st, "evm_dist_split");
  napi_value v;
  napi_create_uint32(env, base, &v);
  return v;
}

napi_value f64_array(napi_env env, const std::vector<uint64_t>& x) {
  double* p;
  napi_value v = typed(env, napi_float64_array, x.size(), 8, (void**)&p);
  for (size_t i = 0; i < x.size(); ++i) p[i] = (double)x[i];
  return v;
}

// distSelectSplit(ctx, d, store, clientTree, node Uint8Array(nLocal * 16), hotBase, nHot)
//   -> { diff Float64Array(nLocal), off, ids (this rank's rows per local id),
//        hotOff, hotIds (every rank's rows of the split owners, timestamp order) }   (collective)
// getMessages (index.ts:173-202) with split owners: their diffs are those of their FULL trees
napi_value DistSelectSplit(napi_env env, napi_callback_info info) {
  napi_value a[7];
  if (!get_args(env, info, 7, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  evm_dist* d = (evm_dist*)ext(env, a[1]);
  const evm_store* s = (const evm_store*)ext(env, a[2]);
  const evm_tree* client = (const evm_tree*)ext(env, a[3]);
  void* node;
  size_t nl;
  if (!bytes_of(env, a[4], &node, &nl)) return nullptr;
  const uint32_t base = u32(env, a[5]), nh = u32(env, a[6]);
  uint32_t n_local = 0;
  uint64_t n_msg = 0;
  evm_store_info(s, &n_local, &n_msg);
  if (nl != 16ull * n_local || base + (uint64_t)nh != n_local)
    return throw_status(env, EVM_EINVAL, "distSelectSplit: sizes");
  const evm_tree* tree = evm_store_tree(s);
  Dev ddiff(ctx, 8ull * n_local), dnode(ctx, nl, node), doff(ctx, 8ull * (n_local + 1)),
      dids(ctx, 8 * (n_msg ? n_msg : 1)), dkey(ctx, 24 * (n_msg ? n_msg : 1)), dhoff(ctx, 8ull * (nh + 1));
  // (a local failure still joins every collective, flagged: no peer is left waiting)
  int st = evm_merkle_diff(ctx, tree, client, (int64_t*)ddiff.p);
  evm_tree *full = nullptr, *sub = nullptr;
  const int st_m = evm_dist_merge_trees(ctx, d, st ? nullptr : tree, base, nh, &full);
  if (!st) st = st_m;
  // the client's trees of the split owners: its hot slots
  uint64_t L = 0;
  Dev dso(ctx, 8ull * (nh + 1));
  if (!st) st = evm_tree_slice(ctx, client, base, nh, (uint64_t*)dso.p, nullptr, nullptr, 0, &L);
  if (st == EVM_ECAPACITY) st = EVM_OK;
  Dev dsc(ctx, 8 * (L ? L : 1)), dsx(ctx, 4 * (L ? L : 1));
  if (!st) st = evm_tree_slice(ctx, client, base, nh, (uint64_t*)dso.p, (uint64_t*)dsc.p, (int32_t*)dsx.p, L, &L);
  if (!st) st = evm_tree_from_device_leaves(ctx, nh, (const uint64_t*)dso.p, (const uint64_t*)dsc.p,
                                            (const int32_t*)dsx.p, &sub);
  if (!st && nh) st = evm_merkle_diff(ctx, full, sub, (int64_t*)ddiff.p + base);
  if (full) evm_tree_free(ctx, full);
  if (sub) evm_tree_free(ctx, sub);
  uint64_t nsel = 0, nhot = 0;
  if (!st)
    st = evm_store_select_after(ctx, s, (const int64_t*)ddiff.p, (const char*)dnode.p, nullptr, (uint64_t*)doff.p,
                                (uint64_t*)dids.p, (uint64_t*)dkey.p, n_msg, &nsel);
  Dev dhids(ctx, 8);
  {
    const int st_s = evm_dist_merge_select(ctx, d, nh, st ? nullptr : (const uint64_t*)doff.p + base,
                                           (const uint64_t*)dids.p, (const uint64_t*)dkey.p, (uint64_t*)dhoff.p,
                                           nullptr, 0, &nhot);
    if (!st) st = st_s;
    if (st == EVM_ECAPACITY) {  // (every rank: the same total)
      Dev big(ctx, 8 * nhot);
      st = evm_dist_merge_select(ctx, d, nh, (const uint64_t*)doff.p + base, (const uint64_t*)dids.p,
                                 (const uint64_t*)dkey.p, (uint64_t*)dhoff.p, (uint64_t*)big.p, nhot, &nhot);
      std::swap(dhids.p, big.p);
    }
  }
  if (st) return throw_status(env, st, "distSelectSplit");
  std::vector<int64_t> diff(n_local);
  std::vector<uint64_t> off(n_local + 1), ids(nsel), hoff(nh + 1), hids(nhot);
  evm_copy_d2h(ctx, diff.data(), ddiff.p, 8ull * n_local);
  evm_copy_d2h(ctx, off.data(), doff.p, 8ull * (n_local + 1));
  if (nsel) evm_copy_d2h(ctx, ids.data(), dids.p, 8 * nsel);
  evm_copy_d2h(ctx, hoff.data(), dhoff.p, 8ull * (nh + 1));
  if (nhot) evm_copy_d2h(ctx, hids.data(), dhids.p, 8 * nhot);
  double* dp;
  napi_value vdiff = typed(env, napi_float64_array, n_local, 8, (void**)&dp);
  for (uint32_t i = 0; i < n_local; ++i) dp[i] = (double)diff[i];
  napi_value res;
  napi_create_object(env, &res);
  napi_set_named_property(env, res, "diff", vdiff);
  napi_set_named_property(env, res, "off", f64_array(env, off));
  napi_set_named_property(env, res, "ids", f64_array(env, ids));
  napi_set_named_property(env, res, "hotOff", f64_array(env, hoff));
  napi_set_named_property(env, res, "hotIds", f64_array(env, hids));
  return res;
}

// distSplitApply(ctx, d, ts Uint8Array(n * 48), cell Uint32Array, nCells, treeIn
//                [, priorTs Uint8Array(nCells * 48), priorPresent Uint8Array(nCells)
//                 [, storedTs Uint8Array(k * 48), storedCell Uint32Array(k)]])
//   -> { status, flags Uint8Array(n), winner Float64Array(nCells) (global batch index, -1), tree | null }
// applyMessages of ONE owner's batch split over the ranks by cell (collective): each rank passes its
// slice (the batch = the slices in rank order); winner and tree are the same on every rank.  The owner's
// DB state is the single-rank applyMessages' (evolu_evm.js _applyArgs): every cell's current max
// (applyMessages.ts:34-40) and the __message rows holding a batch timestamp (:42-45), the SAME arrays on
// every rank -- each rank decides its own cells against them with evm_apply_batch_ex
napi_value DistSplitApply(napi_env env, napi_callback_info info) {
  napi_value a[10];
  size_t argc = 10;
  if (napi_get_cb_info(env, info, &argc, a, nullptr, nullptr) != napi_ok || argc < 6) {
    napi_throw_type_error(env, nullptr, "missing arguments");
    return nullptr;
  }
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_ctx* ctx = cx->c;
  evm_dist* d = (evm_dist*)ext(env, a[1]);
  void *ts, *cell, *pts = nullptr, *pp = nullptr, *sts = nullptr, *sc = nullptr;
  size_t tl, cl, ptl = 0, ppl = 0, stl = 0, scl = 0;
  if (!bytes_of(env, a[2], &ts, &tl) || !bytes_of(env, a[3], &cell, &cl)) return nullptr;
  const uint32_t nc = u32(env, a[4]);
  const evm_tree* tree_in = (const evm_tree*)ext(env, a[5]);
  if (argc >= 8 && !is_null(env, a[6]) && (!bytes_of(env, a[6], &pts, &ptl) || !bytes_of(env, a[7], &pp, &ppl)))
    return nullptr;
  if (argc >= 10 && !is_null(env, a[8]) && (!bytes_of(env, a[8], &sts, &stl) || !bytes_of(env, a[9], &sc, &scl)))
    return nullptr;
  const size_t n = cl / 4;
  const size_t ns = scl / 4;
  if (tl != n * 48 || (pts && (ptl != 48ull * nc || ppl != nc)) || (sts && stl != ns * 48))
    return throw_status(env, EVM_EINVAL, "distSplitApply: sizes");
  Dev dts(ctx, tl, ts), dcell(ctx, cl, cell), dzero(ctx, 4 * (n ? n : 1)), ddest(ctx, n ? n : 1),
      dpts(ctx, ptl, pts), dpp(ctx, ppl, pp), dsts(ctx, stl, sts), dsc(ctx, scl, sc);
  std::vector<uint32_t> zero(n, 0u);
  if (n) evm_copy_h2d(ctx, dzero.p, zero.data(), 4 * n);
  uint64_t nr = 0;
  int local = EVM_OK;
  // the global PK check (applyMessages.ts:42-45): every copy of a timestamp meets on one rank.  A rank
  // whose destinations failed still joins the route (with no rows) and reports in the agreement
  int st = evm_dist_ts_dest(ctx, d, (const char*)dts.p, 48, n, (uint8_t*)ddest.p);
  if (st) local = st;
  st = evm_dist_route(ctx, d, (const char*)dts.p, 48, local ? 0 : n, (const uint32_t*)dzero.p,
                      (const uint32_t*)dcell.p, (const uint8_t*)ddest.p, &nr);
  if (st) return throw_status(env, st, "distSplitApply: route");  // (every rank fails a route together)
  {
    Dev rts(ctx, 48 * (nr ? nr : 1)), row(ctx, 4 * (nr ? nr : 1)), rax(ctx, 4 * (nr ? nr : 1));
    st = evm_dist_take(ctx, d, 0, (char*)rts.p, 48, (uint32_t*)row.p, (uint32_t*)rax.p, nullptr, nr, nullptr);
    int32_t found = 0;
    if (!st && nr) st = evm_cross_cell_check(ctx, (const char*)rts.p, 48, nr, (const uint32_t*)rax.p, nc, &found);
    if (st && !local) local = st;
    else if (found && !local) local = EVM_ECOLLISION;
    st = EVM_OK;
  }
  // the LWW decisions (applyMessages.ts:78-124) are per cell: every row of a cell on the cell's rank
  st = evm_dist_cell_dest(ctx, d, (const uint32_t*)dcell.p, n, (uint8_t*)ddest.p);
  if (st && !local) local = st;
  st = evm_dist_route(ctx, d, (const char*)dts.p, 48, local ? 0 : n, (const uint32_t*)dzero.p,
                      (const uint32_t*)dcell.p, (const uint8_t*)ddest.p, &nr);
  if (st) return throw_status(env, st, "distSplitApply: route");  // (every rank fails a route together)
  Dev rts(ctx, 48 * (nr ? nr : 1)), row(ctx, 4 * (nr ? nr : 1)), rax(ctx, 4 * (nr ? nr : 1)),
      fl(ctx, nr ? nr : 1), win(ctx, 4ull * (nc ? nc : 1)), dflags(ctx, n ? n : 1), dwin(ctx, 8ull * (nc ? nc : 1));
  // (local failures from here on go into `local`: every rank still reaches the status agreement)
  st = evm_dist_take(ctx, d, 0, (char*)rts.p, 48, (uint32_t*)row.p, (uint32_t*)rax.p, nullptr, nr, nullptr);
  if (st && !local) local = st;
  evm_tree *empty = nullptr, *part = nullptr;
  st = evm_tree_new(ctx, 1, &empty);
  if (st && !local) local = st;
  st = EVM_OK;
  if (!local) {
    if (nr) {
      const int a_st = evm_apply_batch_ex(ctx, empty, (const char*)rts.p, 48, nr, (const uint32_t*)rax.p, nc,
                                          nullptr, pts ? (const char*)dpts.p : nullptr, 48,
                                          pp ? (const uint8_t*)dpp.p : nullptr, ns ? (const char*)dsts.p : nullptr,
                                          48, ns, ns ? (const uint32_t*)dsc.p : nullptr, (uint8_t*)fl.p,
                                          (int32_t*)win.p, &part);
      if (a_st) local = a_st;
    } else {
      std::vector<int32_t> none(nc ? nc : 1, -1);
      st = evm_copy_h2d(ctx, win.p, none.data(), 4ull * (nc ? nc : 1));
      part = empty;
      empty = nullptr;
    }
  }
  if (st && !local) local = st;
  int32_t status = 0;
  st = evm_dist_agree_status(ctx, d, local, &status);
  napi_value res, v;
  napi_create_object(env, &res);
  if (!st && status == EVM_OK) st = evm_dist_return(ctx, d, fl.p, 1, dflags.p, n);
  if (!st && status == EVM_OK) st = evm_dist_split_winners(ctx, d, (const int32_t*)win.p, nc, (int64_t*)dwin.p);
  evm_tree *merged = nullptr, *out = nullptr;
  if (!st && status == EVM_OK) st = evm_dist_merge_trees(ctx, d, part, 0, 1, &merged);
  if (!st && status == EVM_OK) st = evm_tree_merge(ctx, tree_in, merged, &out);
  if (empty) evm_tree_free(ctx, empty);
  if (part) evm_tree_free(ctx, part);
  if (merged) evm_tree_free(ctx, merged);
  if (st) return throw_status(env, st, "distSplitApply");
  napi_create_int32(env, status, &v);
  napi_set_named_property(env, res, "status", v);
  void* hf;
  napi_value vf = typed(env, napi_uint8_array, n, 1, &hf);
  double* wp;
  napi_value vw = typed(env, napi_float64_array, nc, 8, (void**)&wp);
  if (status == EVM_OK) {
    if (n) evm_copy_d2h(ctx, hf, dflags.p, n);
    std::vector<int64_t> w(nc);
    if (nc) evm_copy_d2h(ctx, w.data(), dwin.p, 8ull * nc);
    for (uint32_t c = 0; c < nc; ++c) wp[c] = (double)w[c];
  } else {
    if (n) memset(hf, 0, n);
    for (uint32_t c = 0; c < nc; ++c) wp[c] = -1;
  }
  napi_set_named_property(env, res, "flags", vf);
  napi_set_named_property(env, res, "winner", vw);
  if (out) napi_set_named_property(env, res, "tree", make_ext(env, out));
  else {
    napi_get_null(env, &v);
    napi_set_named_property(env, res, "tree", v);
  }
  return res;
}

// ---------------------------------------------------------------- sync server (index.ts:204-251)
// syncCreate(ctx, store) -> server handle (the user directory + message log over the store)
napi_value SyncCreate(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_sync_server* s = nullptr;
  const int st = evm_sync_create(cx->c, (evm_store*)ext(env, a[1]), &s);
  if (st) return throw_status(env, st, "evm_sync_create");
  return make_ext(env, s);
}

napi_value SyncDestroy(napi_env env, napi_callback_info info) {
  napi_value a[2];
  if (!get_args(env, info, 2, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_sync_destroy((evm_sync_server*)ext(env, a[1]));
  return nullptr;
}

// syncRound(ctx, server, bodies Uint8Array, offsets Float64Array(n + 1))
//   -> { status, results: Int32Array(n), offsets: Float64Array(n + 1), responses: Uint8Array }
// status EVM_EROUNDS (a userId twice: nothing applied) leaves the rest empty.
napi_value SyncRound(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_sync_server* srv = (evm_sync_server*)ext(env, a[1]);
  void *body, *offd;
  size_t bl, ol;
  if (!bytes_of(env, a[2], &body, &bl) || !bytes_of(env, a[3], &offd, &ol)) return nullptr;
  const size_t n1 = ol / 8;
  if (n1 < 1) return throw_status(env, EVM_EINVAL, "syncRound: offsets");
  const uint32_t n = (uint32_t)(n1 - 1);
  std::vector<uint64_t> off(n1);
  for (size_t k = 0; k < n1; ++k) off[k] = (uint64_t)static_cast<const double*>(offd)[k];
  if (off[n] > bl) return throw_status(env, EVM_EINVAL, "syncRound: offsets past the bodies");
  std::vector<int32_t> res(n);
  std::vector<uint64_t> roff(n1);
  uint64_t total = 0;
  const int st = evm_sync_round(srv, (const uint8_t*)body, off.data(), n, EVM_SYNC_HOST, res.data(), roff.data(),
                                &total);
  if (st != EVM_OK && st != EVM_EROUNDS) return throw_status(env, st, "evm_sync_round");
  napi_value out, v;
  napi_create_object(env, &out);
  napi_create_int32(env, st, &v);
  napi_set_named_property(env, out, "status", v);
  if (st == EVM_EROUNDS) return out;
  void* p;
  napi_value vr = typed(env, napi_int32_array, n, 4, &p);
  if (n) memcpy(p, res.data(), 4 * (size_t)n);
  napi_set_named_property(env, out, "results", vr);
  napi_value vo = typed(env, napi_float64_array, n1, 8, &p);
  for (size_t k = 0; k < n1; ++k) static_cast<double*>(p)[k] = (double)roff[k];
  napi_set_named_property(env, out, "offsets", vo);
  napi_value vb = typed(env, napi_uint8_array, (size_t)total, 1, &p);
  if (total) {
    const int fs = evm_sync_fetch(srv, (uint8_t*)p);
    if (fs) return throw_status(env, fs, "evm_sync_fetch");
  }
  napi_set_named_property(env, out, "responses", vb);
  return out;
}

// syncUserFlag(ctx, server, userId string, flag): hand a user to the caller's path (1) or back (0)
napi_value SyncUserFlag(napi_env env, napi_callback_info info) {
  napi_value a[4];
  if (!get_args(env, info, 4, a)) return nullptr;
  Ctx* cx = ctx_of(env, a[0]);
  std::lock_guard<std::mutex> lock(cx->m);
  evm_sync_server* srv = (evm_sync_server*)ext(env, a[1]);
  size_t len = 0;
  napi_get_value_string_utf8(env, a[2], nullptr, 0, &len);
  std::string u(len + 1, '\0');
  napi_get_value_string_utf8(env, a[2], &u[0], len + 1, &len);
  const uint64_t uo[2] = {0, (uint64_t)len};
  uint32_t slot = 0;
  int st = evm_sync_users(srv, (const uint8_t*)u.data(), uo, 1, 1, &slot);
  if (!st) st = evm_sync_user_flag(srv, slot, (int)u32(env, a[3]));
  if (st) return throw_status(env, st, "syncUserFlag");
  return nullptr;
}

napi_value Init(napi_env env, napi_value exports) {
  const struct {
    const char* name;
    napi_callback fn;
  } fns[] = {{"create", Create},         {"destroy", Destroy},       {"treeFromJson", TreeFromJson},
             {"treeToJson", TreeToJson}, {"treeFree", TreeFree},     {"diff", Diff},
             {"insert", Insert},         {"applyBatch", ApplyBatch}, {"storeNew", StoreNew},
             {"applyBatchAsync", ApplyBatchAsync}, {"serverIngestAsync", ServerIngestAsync},
             {"serverSelectAsync", ServerSelectAsync},
             {"storeFree", StoreFree},   {"storeTree", StoreTree},   {"serverIngest", ServerIngest},
             {"serverSelect", ServerSelect}, {"storeSince", StoreSince}, {"receiveFold", ReceiveFold},
             {"pbDecode", PbDecode},         {"pbEncode", PbEncode},
             {"distUniqueId", DistUniqueId}, {"distInit", DistInit},     {"distFree", DistFree},
             {"distRoute", DistRoute},       {"distGatherRoots", DistGatherRoots}, {"distIngest", DistIngest},
             {"distHubNew", DistHubNew},     {"distHubFree", DistHubFree},   {"distHubAbort", DistHubAbort},
             {"distInitLoopback", DistInitLoopback}, {"distDirectory", DistDirectory},
             {"distHotOwners", DistHotOwners}, {"distSplit", DistSplit},   {"distSelectSplit", DistSelectSplit},
             {"distSplitApply", DistSplitApply}, {"syncCreate", SyncCreate}, {"syncDestroy", SyncDestroy},
             {"syncRound", SyncRound},       {"syncUserFlag", SyncUserFlag}};
  for (const auto& f : fns) {
    napi_value v;
    napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.fn, nullptr, &v);
    napi_set_named_property(env, exports, f.name, v);
  }
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
