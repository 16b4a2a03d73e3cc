// ymerge N-API addon: binds libymerge.so's C ABI (include/ymerge.h) for Node.js.
// Each call takes one packed batch (arena + offsets) in host memory and returns
// { arena, offsets, lengths, status } -- the JS module (js/index.js) turns that into per-document
// Uint8Arrays and yjs-shaped exceptions.
//   run(op, format, arena, updOff, docUpd[, svArena, svOff])       synchronous
//   runAsync(op, format, arena, updOff, docUpd[, svArena, svOff])  -> Promise (napi_async_work: the
//        library call runs on a libuv worker thread; the inputs are pinned by references until it ends)
//   strerror(status)                                              ym_strerror (yjs's exception text)
// The output arena comes uninitialised from the library's page-locked pool (ym_host_alloc: the device-to-host
// copies land in it directly; the library writes every byte it reports) and is handed to JS as an external
// ArrayBuffer whose finalizer returns it to the pool: no zero-fill, no second copy.
#include <node_api.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/ymerge.h"

#define NAPI_CALL(env, call)                                           \
  do {                                                                 \
    if ((call) != napi_ok) {                                           \
      napi_throw_error(env, "YMERGE_NAPI", "N-API call failed: " #call); \
      return nullptr;                                                  \
    }                                                                  \
  } while (0)

static bool get_u8(napi_env env, napi_value v, const uint8_t **p, size_t *n) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return false;
  napi_typedarray_type t;
  size_t len;
  void *data;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok || t != napi_uint8_array) return false;
  *p = (const uint8_t *)data;
  *n = len;
  return true;
}

// u64 offsets from a BigUint64Array (used in place), a Float64Array (exact below 2^53) or a Uint32Array
// (converted; update offsets in a Uint32Array are passed as they are instead, with YM_OFF32: see parse)
static bool get_u64(napi_env env, napi_value v, const uint64_t **p, size_t *n, std::vector<uint64_t> &conv) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return false;
  napi_typedarray_type t;
  size_t len;
  void *data;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok) return false;
  *n = len;
  if (t == napi_biguint64_array) { *p = (const uint64_t *)data; return true; }
  conv.resize(len);
  if (t == napi_float64_array) for (size_t i = 0; i < len; i++) conv[i] = (uint64_t)((double *)data)[i];
  else if (t == napi_uint32_array) for (size_t i = 0; i < len; i++) conv[i] = ((uint32_t *)data)[i];
  else return false;
  *p = conv.data();
  return true;
}

static bool get_u32(napi_env env, napi_value v, const uint32_t **p, size_t *n) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return false;
  napi_typedarray_type t;
  size_t len;
  void *data;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok || t != napi_uint32_array) return false;
  *p = (const uint32_t *)data;
  *n = len;
  return true;
}

// One library call: inputs (borrowed from the JS typed arrays), outputs (owned until handed to JS).
struct Job {
  int32_t op = 0;
  ym_batch b;
  std::vector<uint64_t> upd_conv, sv_conv;
  uint8_t *arena = nullptr;  // from the library's page-locked pool (ym_host_alloc), uninitialised
  uint64_t cap = 0;          // ... the bytes asked for it
  uint64_t used = 0;
  // per-document results, also from the pool: with every output array page-locked the library's packing
  // kernels write them straight into host memory (no copy op)
  uint64_t *out_off = nullptr, *out_len = nullptr;
  int32_t *status = nullptr;
  int rc = 0;
  // async only
  napi_ref refs[7] = {};
  size_t nrefs = 0;
  napi_deferred deferred = nullptr;
  napi_async_work work = nullptr;
  ~Job() {
    ym_host_free(arena);
    ym_host_free(out_off);
    ym_host_free(out_len);
    ym_host_free(status);
  }
};

// parses run()'s arguments into job (throws and returns false on a bad argument)
static bool parse(napi_env env, napi_callback_info info, Job &j, napi_value *argv, size_t &argc) {
  argc = 7;
  if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok) return false;
  if (argc < 5) { napi_throw_type_error(env, nullptr, "run(op, format, arena, updOff, docUpd[, svArena, svOff])"); return false; }
  int32_t fmt = 1;
  if (napi_get_value_int32(env, argv[0], &j.op) != napi_ok || napi_get_value_int32(env, argv[1], &fmt) != napi_ok) {
    napi_throw_type_error(env, nullptr, "op and format must be integers");
    return false;
  }
  const uint8_t *arena = nullptr, *sva = nullptr;
  const uint64_t *upd_off = nullptr, *sv_off = nullptr;
  size_t alen = 0, svlen = 0, ndocs1 = 0, nupd1 = 0, nsv1 = 0;
  const uint32_t *doc_upd = nullptr, *upd_off32 = nullptr;
  // update offsets: a Uint32Array goes to the library as it is (YM_OFF32: half the bytes to copy in, and host
  // merges of many documents run pipelined); BigUint64Array / Float64Array as u64
  const bool off32 = get_u32(env, argv[3], &upd_off32, &nupd1);
  if (!get_u8(env, argv[2], &arena, &alen) || (!off32 && !get_u64(env, argv[3], &upd_off, &nupd1, j.upd_conv)) ||
      !get_u32(env, argv[4], &doc_upd, &ndocs1) || nupd1 == 0 || ndocs1 == 0) {
    napi_throw_type_error(env, nullptr, "arena must be a Uint8Array, updOff a Uint32Array/BigUint64Array/Float64Array, docUpd a Uint32Array");
    return false;
  }
  const uint64_t off_end = off32 ? upd_off32[nupd1 - 1] : upd_off[nupd1 - 1];
  if (off_end > alen || doc_upd[ndocs1 - 1] > nupd1 - 1) {
    napi_throw_range_error(env, nullptr, "updOff / docUpd exceed the arena");
    return false;
  }
  // state vectors: ym_diff's (required), ym_compact's target vectors (optional)
  napi_valuetype t5 = napi_undefined;
  if (argc >= 7) napi_typeof(env, argv[5], &t5);
  const bool want_sv = j.op == 1 || (j.op == 7 && t5 != napi_undefined && t5 != napi_null);
  if (want_sv && (argc < 7 || !get_u8(env, argv[5], &sva, &svlen) || !get_u64(env, argv[6], &sv_off, &nsv1, j.sv_conv) ||
                  nsv1 != ndocs1 || sv_off[nsv1 - 1] > svlen)) {
    napi_throw_type_error(env, nullptr, "diff / compact need svArena (Uint8Array) and svOff (one more entry than documents)");
    return false;
  }
  static const uint8_t no_bytes[1] = {0};
  if (want_sv && !sva) sva = no_bytes;  // every vector empty: still a batch with targets (NULL: none)
  memset(&j.b, 0, sizeof(j.b));
  j.b.arena = arena;
  j.b.upd_off = off32 ? reinterpret_cast<const uint64_t *>(upd_off32) : upd_off;
  j.b.doc_upd = doc_upd;
  j.b.n_docs = (uint32_t)(ndocs1 - 1);
  j.b.n_upd = (uint32_t)(nupd1 - 1);
  j.b.format = fmt | (off32 ? YM_OFF32 : 0);
  j.b.mem = YM_MEM_HOST;
  j.b.sv_arena = want_sv ? sva : nullptr;
  j.b.sv_off = want_sv ? sv_off : nullptr;
  return true;
}

// the library call (no N-API use: runs on the main thread or a worker)
static void execute(Job &j) {
  const size_t nd = j.b.n_docs ? j.b.n_docs : 1;
  j.out_off = (uint64_t *)ym_host_alloc(nd * 8);
  j.out_len = (uint64_t *)ym_host_alloc(nd * 8);
  j.status = (int32_t *)ym_host_alloc(nd * 4);
  if (!j.out_off || !j.out_len || !j.status) { j.rc = YM_ERR_CAPACITY; return; }
  uint64_t cap = ym_out_bound(&j.b);
  for (int attempt = 0; attempt < 4; attempt++) {
    ym_host_free(j.arena);
    j.arena = (uint8_t *)ym_host_alloc(cap ? cap : 1);
    j.cap = cap;
    if (!j.arena) {
      if (getenv("YMERGE_TRACE_CAP")) fprintf(stderr, "addon: no pool buffer of %llu bytes\n", (unsigned long long)cap);
      j.rc = YM_ERR_CAPACITY;
      return;
    }
    ym_out o = {j.arena, cap, j.out_off, j.out_len, j.status, 0};
    j.rc = j.op == 0   ? ym_merge(&j.b, &o, nullptr, nullptr)
           : j.op == 1 ? ym_diff(&j.b, &o, nullptr, nullptr)
           : j.op == 3 ? ym_convert(&j.b, &o, nullptr, nullptr)
           : j.op == 4 ? ym_meta(&j.b, &o, nullptr, nullptr)
           : j.op == 5 ? ym_ds_merge(&j.b, &o, nullptr, nullptr)
           : j.op == 6 ? ym_snapshot(&j.b, &o, nullptr, nullptr)
           : j.op == 7 ? ym_compact(&j.b, &o, nullptr, nullptr)
                       : ym_sv(&j.b, &o, nullptr, nullptr);
    j.used = o.used;
    if (getenv("YMERGE_TRACE_CAP")) fprintf(stderr, "addon op %d attempt %d cap %llu rc %d used %llu\n", j.op, attempt, (unsigned long long)cap, j.rc, (unsigned long long)o.used);
    if (j.rc == YM_ERR_CAPACITY) { cap = o.used + 4096; continue; }
    break;
  }
}

// A pool buffer handed to JS is reported to V8 as external memory (its whole page-locked size class, >= 64 KiB),
// so the collector runs as such buffers pile up: unreported, a few thousand small results (each a 64 KiB pinned
// buffer) waited for a collection V8 saw no reason to start, and the pool's hipHostMalloc failed.
static size_t pool_bytes(size_t n) {
  size_t c = 1ull << 16;  // ym_host_alloc's smallest class
  while (c < n) c <<= 1;
  return c;
}
static void free_arena(napi_env env, void *data, void *hint) {  // back to the pool
  ym_host_free(data);
  int64_t now = 0;
  napi_adjust_external_memory(env, -(int64_t)(uintptr_t)hint, &now);
}
// data (from ym_host_alloc, `bytes` asked for) as an external ArrayBuffer
static napi_status pool_arraybuffer(napi_env env, void *data, size_t n, size_t bytes, napi_value *ab) {
  const size_t c = pool_bytes(bytes ? bytes : 1);
  napi_status s = napi_create_external_arraybuffer(env, data, n, free_arena, (void *)(uintptr_t)c, ab);
  if (s != napi_ok) return s;
  int64_t now = 0;
  napi_adjust_external_memory(env, (int64_t)c, &now);
  return napi_ok;
}

static napi_value make_f64(napi_env env, const uint64_t *src, size_t n) {
  void *data = nullptr;
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, n * 8, &data, &ab) != napi_ok) return nullptr;
  for (size_t i = 0; i < n; i++) ((double *)data)[i] = (double)src[i];
  if (napi_create_typedarray(env, napi_float64_array, n, ab, 0, &ta) != napi_ok) return nullptr;
  return ta;
}
static napi_value make_i32(napi_env env, const int32_t *src, size_t n) {
  void *data = nullptr;
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, n * 4, &data, &ab) != napi_ok) return nullptr;
  if (n) memcpy(data, src, n * 4);
  if (napi_create_typedarray(env, napi_int32_array, n, ab, 0, &ta) != napi_ok) return nullptr;
  return ta;
}

// the result object, or nullptr with *err set to the exception to throw / reject with
static napi_value result(napi_env env, Job &j, napi_value *err) {
  *err = nullptr;
  if (j.rc != 0) {
    napi_value code, msg;
    napi_create_string_utf8(env, "YMERGE_DEVICE", NAPI_AUTO_LENGTH, &code);
    napi_create_string_utf8(env, ym_strerror(j.rc), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, code, msg, err);
    return nullptr;
  }
  // host batches: the outputs are packed back to back, `used` bytes in all
  const uint64_t n = j.used;
  napi_value ab, ta, res;
  if (n > 0) {
    if (pool_arraybuffer(env, j.arena, n, j.cap, &ab) != napi_ok) return nullptr;
    j.arena = nullptr;  // owned by the ArrayBuffer now
  } else if (napi_create_arraybuffer(env, 0, nullptr, &ab) != napi_ok) {
    return nullptr;
  }
  if (napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta) != napi_ok) return nullptr;
  if (napi_create_object(env, &res) != napi_ok) return nullptr;
  napi_set_named_property(env, res, "arena", ta);
  napi_set_named_property(env, res, "offsets", make_f64(env, j.out_off, j.b.n_docs));
  napi_set_named_property(env, res, "lengths", make_f64(env, j.out_len, j.b.n_docs));
  napi_set_named_property(env, res, "status", make_i32(env, j.status, j.b.n_docs));
  return res;
}

static napi_value Run(napi_env env, napi_callback_info info) {
  Job j;
  napi_value argv[7];
  size_t argc;
  if (!parse(env, info, j, argv, argc)) return nullptr;
  execute(j);
  napi_value err, res = result(env, j, &err);
  if (err) napi_throw(env, err);
  return res;
}

static void async_execute(napi_env, void *data) { execute(*static_cast<Job *>(data)); }
static void async_complete(napi_env env, napi_status status, void *data) {
  Job *j = static_cast<Job *>(data);
  napi_value err = nullptr, res = nullptr;
  if (status != napi_ok) {
    napi_value msg;
    napi_create_string_utf8(env, "ymerge: async work cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, nullptr, msg, &err);
  } else {
    res = result(env, *j, &err);
    if (!res && !err) {
      napi_value msg;
      napi_create_string_utf8(env, "ymerge: could not build the result", NAPI_AUTO_LENGTH, &msg);
      napi_create_error(env, nullptr, msg, &err);
    }
  }
  if (err) napi_reject_deferred(env, j->deferred, err);
  else napi_resolve_deferred(env, j->deferred, res);
  for (size_t i = 0; i < j->nrefs; i++) napi_delete_reference(env, j->refs[i]);
  napi_delete_async_work(env, j->work);
  delete j;
}

static napi_value RunAsync(napi_env env, napi_callback_info info) {
  Job *j = new Job();
  napi_value argv[7];
  size_t argc;
  if (!parse(env, info, *j, argv, argc)) { delete j; return nullptr; }
  // the typed arrays stay alive (and their memory in place) until the work completes
  for (size_t i = 2; i < argc; i++) napi_create_reference(env, argv[i], 1, &j->refs[j->nrefs++]);
  // failure paths: release the references, the work and the Job; a created promise is rejected
  auto release = [&](napi_value err) {
    if (j->deferred) napi_reject_deferred(env, j->deferred, err);
    if (j->work) napi_delete_async_work(env, j->work);
    for (size_t i = 0; i < j->nrefs; i++) napi_delete_reference(env, j->refs[i]);
    delete j;
  };
  napi_value promise, name, msg, err;
  if (napi_create_promise(env, &j->deferred, &promise) != napi_ok) {
    j->deferred = nullptr;
    release(nullptr);
    napi_throw_error(env, "YMERGE_NAPI", "could not create the promise");
    return nullptr;
  }
  napi_create_string_utf8(env, "ymerge", NAPI_AUTO_LENGTH, &name);
  if (napi_create_async_work(env, nullptr, name, async_execute, async_complete, j, &j->work) != napi_ok ||
      napi_queue_async_work(env, j->work) != napi_ok) {
    napi_create_string_utf8(env, "ymerge: could not queue the async work", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, nullptr, msg, &err);
    release(err);  // the promise is rejected: callers awaiting it see the failure
    return promise;
  }
  return promise;
}

// hostBuffer(n) -> Uint8Array over n bytes of page-locked memory from the library's pool (ym_host_alloc), given
// back to the pool when the buffer is garbage collected; undefined when none can be had (no HIP runtime).  The
// JS module packs large batches into it, so the library's copies to the GPU are DMA transfers of that memory.
static napi_value HostBuffer(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  double n = 0;
  if (argc < 1 || napi_get_value_double(env, argv[0], &n) != napi_ok || !(n >= 0) || n > 9007199254740991.0) {
    napi_throw_type_error(env, nullptr, "hostBuffer(bytes)");
    return nullptr;
  }
  napi_value undef;
  napi_get_undefined(env, &undef);
  const size_t bytes = (size_t)n;
  void *p = ym_host_alloc(bytes ? bytes : 1);
  if (!p) return undef;
  napi_value ab, ta;
  if (pool_arraybuffer(env, p, bytes, bytes, &ab) != napi_ok) {
    ym_host_free(p);
    return undef;
  }
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, bytes, ab, 0, &ta));
  return ta;
}

static napi_value StrError(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int32_t st = 0;
  if (argc > 0) NAPI_CALL(env, napi_get_value_int32(env, argv[0], &st));
  napi_value r;
  NAPI_CALL(env, napi_create_string_utf8(env, ym_strerror(st), NAPI_AUTO_LENGTH, &r));
  return r;
}

static napi_value Init(napi_env env, napi_value exports) {
  int32_t dev = 0;
  const char *e = getenv("YMERGE_DEVICE");
  if (e) dev = atoi(e);
  struct { const char *name; napi_callback cb; } fns[] = {{"run", Run}, {"runAsync", RunAsync}, {"strerror", StrError}, {"hostBuffer", HostBuffer}};
  for (auto &f : fns) {
    napi_value fn;
    if (napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.cb, nullptr, &fn) != napi_ok) return nullptr;
    napi_set_named_property(env, exports, f.name, fn);
  }
  napi_value d;
  napi_create_int32(env, dev, &d);
  napi_set_named_property(env, exports, "device", d);
  // the library selects the device lazily (ym_init is called by the JS module on first use)
  napi_value initfn;
  napi_create_function(env, "init", NAPI_AUTO_LENGTH, [](napi_env env, napi_callback_info info) -> napi_value {
    size_t argc = 1;
    napi_value argv[1];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    int32_t dv = 0;
    if (argc > 0) napi_get_value_int32(env, argv[0], &dv);
    napi_value r;
    napi_create_int32(env, ym_init(dv), &r);
    return r;
  }, nullptr, &initfn);
  napi_set_named_property(env, exports, "init", initfn);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
