// ymerge N-API addon: binds libymerge.so's C ABI (include/ymerge.h) for Node.js.
// Each call takes one packed batch (arena + offsets) in host memory and returns
// { arena, offsets, lengths, status } -- the JS module (js/index.js) turns that into per-document
// Uint8Arrays and yjs-shaped exceptions.
#include <node_api.h>

#include <stdint.h>
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

// u64 offsets from a BigUint64Array or a Float64Array (exact below 2^53)
static bool get_u64(napi_env env, napi_value v, std::vector<uint64_t> &out) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return false;
  napi_typedarray_type t;
  size_t len;
  void *data;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok) return false;
  out.resize(len);
  if (t == napi_biguint64_array) memcpy(out.data(), data, len * 8);
  else if (t == napi_float64_array) for (size_t i = 0; i < len; i++) out[i] = (uint64_t)((double *)data)[i];
  else if (t == napi_uint32_array) for (size_t i = 0; i < len; i++) out[i] = ((uint32_t *)data)[i];
  else return false;
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

static napi_value make_u8(napi_env env, const uint8_t *src, size_t n) {
  void *data = nullptr;
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, n, &data, &ab) != napi_ok) return nullptr;
  if (n) memcpy(data, src, n);
  if (napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta) != napi_ok) return nullptr;
  return ta;
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

// run(op, format, arena, updOff, docUpd[, svArena, svOff])
static napi_value Run(napi_env env, napi_callback_info info) {
  size_t argc = 7;
  napi_value argv[7];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  if (argc < 5) { napi_throw_type_error(env, nullptr, "run(op, format, arena, updOff, docUpd[, svArena, svOff])"); return nullptr; }
  int32_t op = 0, fmt = 1;
  NAPI_CALL(env, napi_get_value_int32(env, argv[0], &op));
  NAPI_CALL(env, napi_get_value_int32(env, argv[1], &fmt));
  const uint8_t *arena = nullptr, *sva = nullptr;
  size_t alen = 0, svlen = 0, ndocs1 = 0;
  const uint32_t *doc_upd = nullptr;
  std::vector<uint64_t> upd_off, sv_off;
  if (!get_u8(env, argv[2], &arena, &alen) || !get_u64(env, argv[3], upd_off) || !get_u32(env, argv[4], &doc_upd, &ndocs1) ||
      upd_off.empty() || ndocs1 == 0) {
    napi_throw_type_error(env, nullptr, "arena must be a Uint8Array, updOff a BigUint64Array/Float64Array, docUpd a Uint32Array");
    return nullptr;
  }
  if (op == 1 && (argc < 7 || !get_u8(env, argv[5], &sva, &svlen) || !get_u64(env, argv[6], sv_off))) {
    napi_throw_type_error(env, nullptr, "diff needs svArena (Uint8Array) and svOff");
    return nullptr;
  }
  ym_batch b;
  memset(&b, 0, sizeof(b));
  b.arena = arena;
  b.upd_off = upd_off.data();
  b.doc_upd = doc_upd;
  b.n_docs = (uint32_t)(ndocs1 - 1);
  b.n_upd = (uint32_t)(upd_off.size() - 1);
  b.format = fmt;
  b.mem = YM_MEM_HOST;
  b.sv_arena = sva;
  b.sv_off = op == 1 ? sv_off.data() : nullptr;
  uint64_t cap = ym_out_bound(&b);
  std::vector<uint8_t> out_arena;
  std::vector<uint64_t> out_off(b.n_docs ? b.n_docs : 1), out_len(b.n_docs ? b.n_docs : 1);
  std::vector<int32_t> status(b.n_docs ? b.n_docs : 1);
  int rc = 0;
  for (int attempt = 0; attempt < 4; attempt++) {
    out_arena.assign(cap ? cap : 1, 0);
    ym_out o = {out_arena.data(), cap, out_off.data(), out_len.data(), status.data(), 0};
    rc = op == 0   ? ym_merge(&b, &o, nullptr, nullptr)
         : op == 1 ? ym_diff(&b, &o, nullptr, nullptr)
         : op == 3 ? ym_convert(&b, &o, nullptr, nullptr)
         : op == 4 ? ym_meta(&b, &o, nullptr, nullptr)
         : op == 5 ? ym_ds_merge(&b, &o, nullptr, nullptr)
                   : ym_sv(&b, &o, nullptr, nullptr);
    if (rc == YM_ERR_CAPACITY) { cap = o.used + 4096; continue; }
    break;
  }
  if (rc != 0) {
    napi_throw_error(env, "YMERGE_DEVICE", ym_strerror(rc));
    return nullptr;
  }
  napi_value res;
  NAPI_CALL(env, napi_create_object(env, &res));
  NAPI_CALL(env, napi_set_named_property(env, res, "arena", make_u8(env, out_arena.data(), out_arena.size())));
  NAPI_CALL(env, napi_set_named_property(env, res, "offsets", make_f64(env, out_off.data(), b.n_docs)));
  NAPI_CALL(env, napi_set_named_property(env, res, "lengths", make_f64(env, out_len.data(), b.n_docs)));
  NAPI_CALL(env, napi_set_named_property(env, res, "status", make_i32(env, status.data(), b.n_docs)));
  return res;
}

static napi_value Init(napi_env env, napi_value exports) {
  int32_t dev = 0;
  const char *e = getenv("YMERGE_DEVICE");
  if (e) dev = atoi(e);
  napi_value fn;
  if (napi_create_function(env, "run", NAPI_AUTO_LENGTH, Run, nullptr, &fn) != napi_ok) return nullptr;
  napi_set_named_property(env, exports, "run", fn);
  napi_value d;
  napi_create_int32(env, dev, &d);
  napi_set_named_property(env, exports, "device", d);
  (void)ym_init;  // the library selects the device lazily (ym_init is called by the JS module on first use)
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
