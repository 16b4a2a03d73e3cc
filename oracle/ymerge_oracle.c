/*
 * ymerge_oracle.c -- CPU restatement of yjs's binary update layer.  TEST INFRASTRUCTURE ONLY: this file
 * is the parity checker and the cpu_baseline "port"; it is never linked into the product library.
 *
 * Follows, function by function (citations into /root/reference = gaberogan/yjs@v0 = yjs 13.4.9, and
 * into the yjs 13.5.16 JupyterLab bundle 3502.fbe0c610be82ba1360db.js "@offset", lib0 0.2.42 bundle
 * 8086.1dfabaac37d971e2cc4c.js "lib0@offset"):
 *   lib0 readVarUint/readVarInt/readVarString/readAny ........ lib0@2950-4300 (module 64485 U,T,E,B)
 *   lib0 writeVarUint/writeVarInt/writeVarString/writeAny .... lib0@7400-9300 (module 29194 x,I,j,G)
 *   lib0 Rle/UintOptRle/IntDiffOptRle/String en-/decoders .... lib0@4300-5600, 9300-10300
 *   UpdateDecoderV1/V2, DSDecoderV1/V2 ....................... src/utils/UpdateDecoder.js:127-392
 *   UpdateEncoderV1/V2, DSEncoderV1/V2 ....................... src/utils/UpdateEncoder.js:110-408
 *   Item.write / GC.write / Content*.write / read*  .......... src/structs/Item.js:625-683, GC.js:45-48,
 *                                                              Content{String,Deleted,JSON,Binary,Any,
 *                                                              Embed,Format,Type,Doc}.js; 13.5.16 @78000+
 *   ContentString.splice (U+FFFD rule) ....................... src/structs/ContentString.js:51-66
 *   readDeleteSet / writeDeleteSet / mergeDeleteSets ......... src/utils/DeleteSet.js:141-256; 13.5.16
 *                                                              le@10242 he@10482 fe@11101 ge@11342
 *   LazyStructReader (ts/es) ................................. 13.5.16 @36560, @37148
 *   sliceStruct (as) ......................................... 13.5.16 @38661
 *   mergeUpdatesV2 (ds) ...................................... 13.5.16 @39007
 *   diffUpdateV2 (us) ........................................ 13.5.16 @40707
 *   LazyStructWriter write/flush/finish (ps/gs/ws) ........... 13.5.16 @41236-41700
 *   encodeStateVectorFromUpdateV2 (os) ....................... 13.5.16 @37724
 *   decodeStateVector (Fe/Ve) ................................ src/utils/encoding.js:536-565
 * The per-iteration reader sort of mergeUpdates restates V8's Array.prototype.sort (TimSort with
 * galloping merges) operation by operation: the comparator is inconsistent when a GC and an Item tie
 * on (client, clock), so the output order depends on exactly which pairs V8 compares.
 * JS values: numbers are IEEE doubles, strings are UTF-16 code-unit arrays, object property order
 * follows OrdinaryOwnPropertyKeys (array-index keys ascending, then insertion order).
 */
#define _GNU_SOURCE
#include "ymerge_oracle.h"
#include <math.h>
#include <pthread.h>
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------------ */
/* arena + error context                                                                           */
/* ------------------------------------------------------------------------------------------------ */
typedef struct Chunk { struct Chunk *next; size_t cap, used; } Chunk;
typedef struct Ctx {
  jmp_buf jb;
  Chunk *chunks;
  int v2;
  int inconsistent_cmp; /* a GC/Item tie was compared during a reader sort */
} Ctx;

static void ctx_free(Ctx *c) {
  Chunk *k = c->chunks;
  while (k) { Chunk *n = k->next; free(k); k = n; }
  c->chunks = NULL;
}

static void __attribute__((noreturn)) fail(Ctx *c, int code) { longjmp(c->jb, code); }

static void *aalloc(Ctx *c, size_t n) {
  n = (n + 15) & ~(size_t)15;
  Chunk *k = c->chunks;
  if (!k || k->cap - k->used < n) {
    size_t cap = n + sizeof(Chunk) + 15 > (1u << 16) ? n + sizeof(Chunk) + 16 : (1u << 16);
    Chunk *nk = (Chunk *)malloc(cap);
    if (!nk) fail(c, YMO_ERR_UNSUPPORTED);
    nk->cap = cap;
    nk->used = (sizeof(Chunk) + 15) & ~(size_t)15;
    nk->next = c->chunks;
    c->chunks = nk;
    k = nk;
  }
  void *p = (char *)k + k->used;
  k->used += n;
  return p;
}

/* growable byte buffer (lib0 Encoder) */
typedef struct { uint8_t *p; size_t n, cap; } Buf;
static Buf *buf_new(Ctx *c) {
  Buf *b = (Buf *)aalloc(c, sizeof(Buf));
  b->cap = 64; b->n = 0; b->p = (uint8_t *)aalloc(c, b->cap);
  return b;
}
static void buf_reserve(Ctx *c, Buf *b, size_t extra) {
  if (b->n + extra <= b->cap) return;
  size_t cap = b->cap * 2;
  while (cap < b->n + extra) cap *= 2;
  uint8_t *np = (uint8_t *)aalloc(c, cap);
  memcpy(np, b->p, b->n);
  b->p = np; b->cap = cap;
}
static void put8(Ctx *c, Buf *b, unsigned v) { buf_reserve(c, b, 1); b->p[b->n++] = (uint8_t)v; }
static void putraw(Ctx *c, Buf *b, const uint8_t *p, size_t n) {
  if (!n) return;
  buf_reserve(c, b, n); memcpy(b->p + b->n, p, n); b->n += n;
}

/* JS strings: UTF-16 code units */
typedef struct { const uint16_t *u; size_t n; } Str;
static int str_eq(Str a, Str b) { return a.n == b.n && (a.n == 0 || memcmp(a.u, b.u, a.n * 2) == 0); }
static Str str_slice(Str s, int64_t a, int64_t b) { /* String.prototype.slice with non-negative args */
  if (a > (int64_t)s.n) a = (int64_t)s.n;
  if (b > (int64_t)s.n) b = (int64_t)s.n;
  if (b < a) b = a;
  Str r = {s.u + a, (size_t)(b - a)};
  return r;
}

/* ------------------------------------------------------------------------------------------------ */
/* JS number helpers                                                                               */
/* ------------------------------------------------------------------------------------------------ */
static uint32_t js_touint32(double v) {
  if (!isfinite(v) || v == 0) return 0;
  double t = trunc(v);
  double m = fmod(t, 4294967296.0);
  if (m < 0) m += 4294967296.0;
  return (uint32_t)m;
}
static int32_t js_toint32(double v) { return (int32_t)js_touint32(v); }
static int js_is_negzero_or_neg(double v) { return v != 0 ? v < 0 : signbit(v) != 0; } /* math.isNegativeZero */

/* ------------------------------------------------------------------------------------------------ */
/* UTF-8 <-> UTF-16 (decodeURIComponent(escape(..)) / unescape(encodeURIComponent(..)))             */
/* ------------------------------------------------------------------------------------------------ */
static Str utf8_decode_strict(Ctx *c, const uint8_t *p, size_t n) {
  uint16_t *u = (uint16_t *)aalloc(c, n * 2 + 2);
  size_t k = 0, i = 0;
  while (i < n) {
    uint32_t b = p[i];
    if (b < 0x80) { u[k++] = (uint16_t)b; i++; continue; }
    int len;
    uint32_t cp, min;
    if ((b & 0xE0) == 0xC0) { len = 2; cp = b & 0x1F; min = 0x80; }
    else if ((b & 0xF0) == 0xE0) { len = 3; cp = b & 0x0F; min = 0x800; }
    else if ((b & 0xF8) == 0xF0) { len = 4; cp = b & 0x07; min = 0x10000; }
    else fail(c, YMO_ERR_URI);
    if (i + len > n) fail(c, YMO_ERR_URI);
    for (int j = 1; j < len; j++) {
      uint32_t cb = p[i + j];
      if ((cb & 0xC0) != 0x80) fail(c, YMO_ERR_URI);
      cp = (cp << 6) | (cb & 0x3F);
    }
    if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) fail(c, YMO_ERR_URI);
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u[k++] = (uint16_t)(0xD800 + (cp >> 10));
      u[k++] = (uint16_t)(0xDC00 + (cp & 0x3FF));
    } else {
      u[k++] = (uint16_t)cp;
    }
    i += len;
  }
  Str r = {u, k};
  return r;
}

/* UTF-16 -> UTF-8 into b; URIError on lone surrogates */
static void utf8_encode(Ctx *c, Buf *b, Str s) {
  buf_reserve(c, b, s.n * 3 + 4);
  for (size_t i = 0; i < s.n; i++) {
    uint32_t cu = s.u[i];
    if (cu < 0x80) { b->p[b->n++] = (uint8_t)cu; continue; }
    if (cu < 0x800) { b->p[b->n++] = (uint8_t)(0xC0 | (cu >> 6)); b->p[b->n++] = (uint8_t)(0x80 | (cu & 0x3F)); continue; }
    if (cu >= 0xD800 && cu <= 0xDBFF) {
      if (i + 1 >= s.n || s.u[i + 1] < 0xDC00 || s.u[i + 1] > 0xDFFF) fail(c, YMO_ERR_URI);
      uint32_t cp = 0x10000 + ((cu - 0xD800) << 10) + (s.u[i + 1] - 0xDC00);
      i++;
      buf_reserve(c, b, 4 + (s.n - i) * 3);
      b->p[b->n++] = (uint8_t)(0xF0 | (cp >> 18));
      b->p[b->n++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
      b->p[b->n++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
      b->p[b->n++] = (uint8_t)(0x80 | (cp & 0x3F));
      continue;
    }
    if (cu >= 0xDC00 && cu <= 0xDFFF) fail(c, YMO_ERR_URI);
    b->p[b->n++] = (uint8_t)(0xE0 | (cu >> 12));
    b->p[b->n++] = (uint8_t)(0x80 | ((cu >> 6) & 0x3F));
    b->p[b->n++] = (uint8_t)(0x80 | (cu & 0x3F));
  }
}

/* ------------------------------------------------------------------------------------------------ */
/* lib0 decoding (module 64485)                                                                    */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { const uint8_t *a; size_t len; size_t pos; } Dec;
/* readUint8: t.arr[t.pos++]; -1 stands for `undefined` past the end */
static inline int dbyte(Dec *d) { size_t p = d->pos++; return p < d->len ? d->a[p] : -1; }
static inline int dhas(Dec *d) { return d->pos != d->len; } /* hasContent */

static uint32_t rd_vu(Ctx *c, Dec *d) { /* readVarUint (U) */
  uint32_t s = 0;
  unsigned n = 0;
  for (;;) {
    int e = dbyte(d);
    uint32_t bits = e < 0 ? 0u : (uint32_t)(e & 127);
    s |= bits << (n & 31);
    n += 7;
    if (e >= 0 && e < 128) return s;
    if (n > 35) fail(c, YMO_ERR_INT_RANGE);
  }
}

static double rd_vi(Ctx *c, Dec *d) { /* readVarInt (T), returns a JS number incl. -0 */
  int s = dbyte(d);
  uint32_t sb = s < 0 ? 0u : (uint32_t)s;
  uint32_t n = sb & 63;
  unsigned e = 6;
  double sign = (sb & 64) ? -1.0 : 1.0;
  if ((sb & 128) == 0) return sign * (double)n;
  for (;;) {
    s = dbyte(d);
    sb = s < 0 ? 0u : (uint32_t)s;
    n |= (sb & 127) << (e & 31);
    e += 7;
    if (s >= 0 && s < 128) return sign * (double)n;
    if (e > 41) fail(c, YMO_ERR_INT_RANGE);
  }
}

static Str rd_vstr(Ctx *c, Dec *d) { /* readVarString (E) */
  uint32_t L = rd_vu(c, d);
  Str empty = {NULL, 0};
  if (L == 0) return empty;
  size_t avail = d->pos < d->len ? d->len - d->pos : 0;
  uint8_t *tmp = (uint8_t *)aalloc(c, ((size_t)L < avail ? (size_t)L : avail) + 2);
  size_t k = 0;
  int b = dbyte(d);
  if (b < 0) fail(c, YMO_ERR_RANGE); /* String.fromCodePoint(undefined) */
  tmp[k++] = (uint8_t)b;
  uint32_t s = L - 1;
  if (s < 100) {
    while (s--) {
      b = dbyte(d);
      if (b < 0) fail(c, YMO_ERR_RANGE);
      tmp[k++] = (uint8_t)b;
    }
  } else {
    while (s > 0) {
      uint32_t e = s < 10000 ? s : 10000;
      size_t a0 = d->pos, a1 = d->pos + e;
      if (a0 > d->len) a0 = d->len;
      if (a1 > d->len) a1 = d->len;
      if (a1 > a0) { memcpy(tmp + k, d->a + a0, a1 - a0); k += a1 - a0; }
      d->pos += e;
      s -= e;
    }
  }
  return utf8_decode_strict(c, tmp, k);
}

typedef struct { const uint8_t *p; size_t n; } Span;
static Span rd_vbytes(Ctx *c, Dec *d) { /* readVarUint8Array: new Uint8Array(buffer, pos, len) */
  uint32_t L = rd_vu(c, d);
  if (d->pos > d->len || (size_t)L > d->len - d->pos) fail(c, YMO_ERR_RANGE);
  Span s = {d->a + d->pos, L};
  d->pos += L;
  return s;
}

/* ------------------------------------------------------------------------------------------------ */
/* JS values produced by readAny / JSON.parse                                                      */
/* ------------------------------------------------------------------------------------------------ */
enum { V_UNDEF, V_NULL, V_BOOL, V_NUM, V_BIGINT, V_STR, V_ARR, V_OBJ, V_BYTES };
typedef struct Val {
  int t;
  int b;
  double num;
  uint8_t big[8];
  Str s;
  struct Val **items; /* ARR / OBJ values */
  Str *keys;          /* OBJ keys */
  size_t n, cap;
  Span bytes;
  struct Val *proto;  /* OBJ built by readAny: NULL = Object.prototype, else the value assigned to
                         "__proto__" (an object, array, Uint8Array or null) */
} Val;

static Val *val_new(Ctx *c, int t) {
  Val *v = (Val *)aalloc(c, sizeof(Val));
  memset(v, 0, sizeof(Val));
  v->t = t;
  return v;
}
/* canonical array index ("0" .. "4294967294"); returns 1 and the index */
static int key_array_index(Str k, uint32_t *idx) {
  if (k.n == 0 || k.n > 10) return 0;
  if (k.n > 1 && k.u[0] == '0') return 0;
  uint64_t v = 0;
  for (size_t i = 0; i < k.n; i++) {
    if (k.u[i] < '0' || k.u[i] > '9') return 0;
    v = v * 10 + (k.u[i] - '0');
  }
  if (v >= 4294967295ull) return 0;
  *idx = (uint32_t)v;
  return 1;
}
static int str_is(Str k, const char *t) {
  size_t i = 0;
  for (; t[i]; i++) if (i >= k.n || k.u[i] != (uint8_t)t[i]) return 0;
  return i == k.n;
}
static void js_num_to_string(double x, char *out);
/* CanonicalNumericIndexString (ES2019 7.1.16): 1 when numeric; *idx = integer index or -1 */
static int key_canonical_numeric(Str k, int64_t *idx) {
  char buf[64];
  *idx = -1;
  if (k.n == 0 || k.n >= sizeof buf) return 0;
  for (size_t i = 0; i < k.n; i++) { if (k.u[i] > 127) return 0; buf[i] = (char)k.u[i]; }
  buf[k.n] = 0;
  if (!strcmp(buf, "-0")) return 1;
  char *end;
  double x = strtod(buf, &end);
  if (!strcmp(buf, "NaN")) x = NAN;
  else if (*end) return 0;
  char t[64];
  js_num_to_string(x, t);
  if (strcmp(t, buf)) return 0;
  if (isfinite(x) && floor(x) == x && x >= 0 && !signbit(x)) *idx = (int64_t)x;
  return 1;
}
static int obj_find(const Val *o, Str k) {
  for (size_t i = 0; i < o->n; i++) if (str_eq(o->keys[i], k)) return (int)i;
  return -1;
}
static void obj_append(Ctx *c, Val *o, Str k, Val *v) {
  if (o->n == o->cap) {
    size_t cap = o->cap ? o->cap * 2 : 4;
    Val **ni = (Val **)aalloc(c, cap * sizeof(Val *));
    Str *nk = (Str *)aalloc(c, cap * sizeof(Str));
    if (o->n) { memcpy(ni, o->items, o->n * sizeof(Val *)); memcpy(nk, o->keys, o->n * sizeof(Str)); }
    o->items = ni; o->keys = nk; o->cap = cap;
  }
  /* position: array-index keys ascending before all string keys */
  uint32_t idx;
  size_t pos = o->n;
  if (key_array_index(k, &idx)) {
    pos = 0;
    while (pos < o->n) {
      uint32_t j;
      if (!key_array_index(o->keys[pos], &j) || j > idx) break;
      pos++;
    }
  }
  memmove(o->items + pos + 1, o->items + pos, (o->n - pos) * sizeof(Val *));
  memmove(o->keys + pos + 1, o->keys + pos, (o->n - pos) * sizeof(Str));
  o->items[pos] = v; o->keys[pos] = k; o->n++;
}
/* [[Set]] / CreateDataProperty on a plain object, keeping OrdinaryOwnPropertyKeys order.
 * is_json: JSON.parse (CreateDataProperty: "__proto__" is an ordinary key).  Else readAny's
 * `obj[key] = v` in strict code: OrdinarySet walks the prototype chain -- Object.prototype's __proto__
 * setter replaces the prototype with an object / array / Uint8Array / null (a primitive is ignored);
 * a null prototype, or a prototype object owning the key as data, creates an own property; a Uint8Array
 * in the chain throws TypeError on its getters (length, byteLength, byteOffset, buffer) and read-only
 * BYTES_PER_ELEMENT and, in the reference's V8, creates a canonical numeric key only when it indexes
 * the array (else ignores it). */
static void obj_set(Ctx *c, Val *o, Str k, Val *v, int is_json) {
  int at = obj_find(o, k);
  if (at >= 0) { o->items[at] = v; return; }
  if (!is_json) {
    int dunder = str_is(k, "__proto__");
    int setter = v->t == V_OBJ || v->t == V_ARR || v->t == V_BYTES || v->t == V_NULL;
    for (Val *P = o->proto;; P = P->proto) {
      if (!P) {  /* Object.prototype */
        if (dunder) { if (setter) o->proto = v; return; }
        break;
      }
      if (P->t == V_NULL) break;
      if (P->t == V_ARR) {
        if (dunder) { if (setter) o->proto = v; return; }
        break;
      }
      if (P->t == V_BYTES) {
        if (str_is(k, "length") || str_is(k, "byteLength") || str_is(k, "byteOffset") || str_is(k, "buffer") ||
            str_is(k, "BYTES_PER_ELEMENT"))
          fail(c, YMO_ERR_TYPE);
        int64_t idx;
        if (key_canonical_numeric(k, &idx)) {
          if (idx < 0 || (size_t)idx >= P->bytes.n) return;  /* ignored */
          break;
        }
        if (dunder) { if (setter) o->proto = v; return; }
        break;
      }
      if (obj_find(P, k) >= 0) break;  /* an inherited writable data property: created on the receiver */
    }
  }
  obj_append(c, o, k, v);
}
/* the end of a readAny object's prototype chain: V_ARR / V_BYTES / 0 (Object.prototype or null) */
static int proto_end(const Val *o) {
  for (const Val *P = o->proto; P; P = P->proto)
    if (P->t != V_OBJ) return P->t == V_NULL ? 0 : P->t;
  return 0;
}
/* [[Get]](o, k) along the chain of an object whose chain ends in an Array */
static const Val *chain_get(const Val *o, Str k, const Val **arr) {
  for (const Val *P = o; P; P = P->proto) {
    if (P->t == V_ARR) { *arr = P; return NULL; }
    int at = obj_find(P, k);
    if (at >= 0) return P->items[at];
  }
  return NULL;
}
static void arr_push(Ctx *c, Val *a, Val *v) {
  if (a->n == a->cap) {
    size_t cap = a->cap ? a->cap * 2 : 4;
    Val **ni = (Val **)aalloc(c, cap * sizeof(Val *));
    if (a->n) memcpy(ni, a->items, a->n * sizeof(Val *));
    a->items = ni; a->cap = cap;
  }
  a->items[a->n++] = v;
}

static double rd_be_f32(const uint8_t *p) {
  uint32_t u = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  float f; memcpy(&f, &u, 4); return (double)f;
}
static double rd_be_f64(const uint8_t *p) {
  uint64_t u = 0;
  for (int i = 0; i < 8; i++) u = (u << 8) | p[i];
  double f; memcpy(&f, &u, 8); return f;
}

static Val *rd_any(Ctx *c, Dec *d) { /* readAny (B) */
  int tag = dbyte(d);
  if (tag < 116 || tag > 127) fail(c, YMO_ERR_TYPE); /* k[127 - tag] is not a function */
  Val *v;
  switch (tag) {
    case 127: return val_new(c, V_UNDEF);
    case 126: return val_new(c, V_NULL);
    case 125: v = val_new(c, V_NUM); v->num = rd_vi(c, d); return v;
    case 124:
      if (d->pos > d->len || d->len - d->pos < 4) fail(c, YMO_ERR_RANGE);
      v = val_new(c, V_NUM); v->num = rd_be_f32(d->a + d->pos); d->pos += 4; return v;
    case 123:
      if (d->pos > d->len || d->len - d->pos < 8) fail(c, YMO_ERR_RANGE);
      v = val_new(c, V_NUM); v->num = rd_be_f64(d->a + d->pos); d->pos += 8; return v;
    case 122:
      if (d->pos > d->len || d->len - d->pos < 8) fail(c, YMO_ERR_RANGE);
      v = val_new(c, V_BIGINT); memcpy(v->big, d->a + d->pos, 8); d->pos += 8; return v;
    case 121: v = val_new(c, V_BOOL); v->b = 0; return v;
    case 120: v = val_new(c, V_BOOL); v->b = 1; return v;
    case 119: v = val_new(c, V_STR); v->s = rd_vstr(c, d); return v;
    case 118: {
      uint32_t n = rd_vu(c, d);
      v = val_new(c, V_OBJ);
      for (uint32_t i = 0; i < n; i++) {
        Str k = rd_vstr(c, d);
        Val *x = rd_any(c, d);
        obj_set(c, v, k, x, 0);
      }
      return v;
    }
    case 117: {
      uint32_t n = rd_vu(c, d);
      v = val_new(c, V_ARR);
      for (uint32_t i = 0; i < n; i++) arr_push(c, v, rd_any(c, d));
      return v;
    }
    default: /* 116 */
      v = val_new(c, V_BYTES); v->bytes = rd_vbytes(c, d); return v;
  }
}

/* ------------------------------------------------------------------------------------------------ */
/* lib0 encoding (module 29194)                                                                    */
/* ------------------------------------------------------------------------------------------------ */
/* writeVarUint on a JS integer (int64 domain): `while (num > 127) { .. num >>>= 7 }` */
static void wr_vu(Ctx *c, Buf *b, int64_t num) {
  while (num > 127) {
    put8(c, b, 0x80 | (unsigned)(num & 127));
    num = (int64_t)((uint32_t)num >> 7);
  }
  put8(c, b, (unsigned)(num & 127));
}
/* writeVarInt on a JS number (integral, possibly -0) */
static void wr_vi(Ctx *c, Buf *b, double num) {
  int neg = js_is_negzero_or_neg(num);
  if (neg) num = -num;
  put8(c, b, (num > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (unsigned)(js_toint32(num) & 63));
  uint32_t s = js_touint32(num) >> 6;
  while (s > 0) {
    put8(c, b, (s > 127 ? 0x80 : 0) | (s & 127));
    s >>= 7;
  }
}
static void wr_vstr(Ctx *c, Buf *b, Str s) { /* writeVarString */
  Buf *t = buf_new(c);
  utf8_encode(c, t, s);
  wr_vu(c, b, (int64_t)t->n);
  putraw(c, b, t->p, t->n);
}
static void wr_vbytes(Ctx *c, Buf *b, const uint8_t *p, size_t n) { wr_vu(c, b, (int64_t)n); putraw(c, b, p, n); }

static int js_is_integer(double v) { return isfinite(v) && floor(v) == v; }
static int js_f32_exact(double v) { return (double)(float)v == v; } /* setFloat32 / getFloat32 === v */

static void wr_any(Ctx *c, Buf *b, const Val *v) { /* writeAny (G) */
  switch (v->t) {
    case V_UNDEF: put8(c, b, 127); return;
    case V_NULL: put8(c, b, 126); return;
    case V_BOOL: put8(c, b, v->b ? 120 : 121); return;
    case V_NUM: {
      double x = v->num;
      if (js_is_integer(x) && x <= 2147483647.0) { put8(c, b, 125); wr_vi(c, b, x); }
      else if (js_f32_exact(x)) {
        float f = (float)x; uint32_t u; memcpy(&u, &f, 4);
        put8(c, b, 124); put8(c, b, u >> 24); put8(c, b, (u >> 16) & 255); put8(c, b, (u >> 8) & 255); put8(c, b, u & 255);
      } else {
        uint64_t u; memcpy(&u, &x, 8);
        put8(c, b, 123);
        for (int i = 7; i >= 0; i--) put8(c, b, (unsigned)((u >> (8 * i)) & 255));
      }
      return;
    }
    case V_BIGINT: put8(c, b, 122); putraw(c, b, v->big, 8); return;
    case V_STR: put8(c, b, 119); wr_vstr(c, b, v->s); return;
    case V_ARR:
      put8(c, b, 117); wr_vu(c, b, (int64_t)v->n);
      for (size_t i = 0; i < v->n; i++) wr_any(c, b, v->items[i]);
      return;
    case V_BYTES: put8(c, b, 116); wr_vbytes(c, b, v->bytes.p, v->bytes.n); return;
    default: {
      /* writeAny: `data instanceof Array` / `instanceof Uint8Array` see the prototype chain */
      int end = proto_end(v);
      if (end == V_BYTES) fail(c, YMO_ERR_TYPE); /* writeVarUint8Array reads byteLength: incompatible receiver */
      if (end == V_ARR) {
        static const uint16_t lk[] = {'l', 'e', 'n', 'g', 't', 'h'};
        Str ls = {lk, 6};
        const Val *arr = NULL;
        if (chain_get(v, ls, &arr)) fail(c, YMO_ERR_UNSUPPORTED); /* an own "length" on the chain */
        put8(c, b, 117); wr_vu(c, b, (int64_t)arr->n);
        for (size_t i = 0; i < arr->n; i++) {
          char nb[32];
          snprintf(nb, sizeof nb, "%zu", i);
          uint16_t ku[32];
          size_t kn = strlen(nb);
          for (size_t j = 0; j < kn; j++) ku[j] = (uint8_t)nb[j];
          Str ks = {ku, kn};
          const Val *a2 = NULL;
          const Val *x = chain_get(v, ks, &a2);
          wr_any(c, b, x ? x : arr->items[i]);
        }
        return;
      }
      put8(c, b, 118); wr_vu(c, b, (int64_t)v->n);
      for (size_t i = 0; i < v->n; i++) { wr_vstr(c, b, v->keys[i]); wr_any(c, b, v->items[i]); }
      return;
    }
  }
}

/* ------------------------------------------------------------------------------------------------ */
/* JSON.parse / JSON.stringify (V1 writeJSON/readJSON, ContentJSON in both formats)                */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { const uint16_t *u; size_t n, i; } JP;
static void jws(JP *p) { while (p->i < p->n && (p->u[p->i] == ' ' || p->u[p->i] == '\t' || p->u[p->i] == '\n' || p->u[p->i] == '\r')) p->i++; }
static int jhex(int ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}
static Str jstr(Ctx *c, JP *p) {
  p->i++; /* opening quote */
  uint16_t *out = (uint16_t *)aalloc(c, (p->n - p->i) * 2 + 2);
  size_t k = 0;
  for (;;) {
    if (p->i >= p->n) fail(c, YMO_ERR_SYNTAX);
    uint16_t ch = p->u[p->i++];
    if (ch == '"') break;
    if (ch < 0x20) fail(c, YMO_ERR_SYNTAX);
    if (ch != '\\') { out[k++] = ch; continue; }
    if (p->i >= p->n) fail(c, YMO_ERR_SYNTAX);
    ch = p->u[p->i++];
    switch (ch) {
      case '"': out[k++] = '"'; break;
      case '\\': out[k++] = '\\'; break;
      case '/': out[k++] = '/'; break;
      case 'b': out[k++] = 8; break;
      case 'f': out[k++] = 12; break;
      case 'n': out[k++] = 10; break;
      case 'r': out[k++] = 13; break;
      case 't': out[k++] = 9; break;
      case 'u': {
        if (p->i + 4 > p->n) fail(c, YMO_ERR_SYNTAX);
        unsigned v = 0;
        for (int j = 0; j < 4; j++) {
          int h = jhex(p->u[p->i + j]);
          if (h < 0) fail(c, YMO_ERR_SYNTAX);
          v = v * 16 + (unsigned)h;
        }
        p->i += 4;
        out[k++] = (uint16_t)v;
        break;
      }
      default: fail(c, YMO_ERR_SYNTAX);
    }
  }
  Str r = {out, k};
  return r;
}
static Val *jval(Ctx *c, JP *p, int depth) {
  if (depth > 10000) fail(c, YMO_ERR_RANGE);
  jws(p);
  if (p->i >= p->n) fail(c, YMO_ERR_SYNTAX);
  uint16_t ch = p->u[p->i];
  if (ch == '{') {
    p->i++;
    Val *o = val_new(c, V_OBJ);
    jws(p);
    if (p->i < p->n && p->u[p->i] == '}') { p->i++; return o; }
    for (;;) {
      jws(p);
      if (p->i >= p->n || p->u[p->i] != '"') fail(c, YMO_ERR_SYNTAX);
      Str k = jstr(c, p);
      jws(p);
      if (p->i >= p->n || p->u[p->i] != ':') fail(c, YMO_ERR_SYNTAX);
      p->i++;
      Val *v = jval(c, p, depth + 1);
      obj_set(c, o, k, v, 1);
      jws(p);
      if (p->i >= p->n) fail(c, YMO_ERR_SYNTAX);
      if (p->u[p->i] == ',') { p->i++; continue; }
      if (p->u[p->i] == '}') { p->i++; return o; }
      fail(c, YMO_ERR_SYNTAX);
    }
  }
  if (ch == '[') {
    p->i++;
    Val *a = val_new(c, V_ARR);
    jws(p);
    if (p->i < p->n && p->u[p->i] == ']') { p->i++; return a; }
    for (;;) {
      arr_push(c, a, jval(c, p, depth + 1));
      jws(p);
      if (p->i >= p->n) fail(c, YMO_ERR_SYNTAX);
      if (p->u[p->i] == ',') { p->i++; continue; }
      if (p->u[p->i] == ']') { p->i++; return a; }
      fail(c, YMO_ERR_SYNTAX);
    }
  }
  if (ch == '"') { Val *v = val_new(c, V_STR); v->s = jstr(c, p); return v; }
  static const char *lits[3] = {"true", "false", "null"};
  for (int l = 0; l < 3; l++) {
    size_t ln = strlen(lits[l]);
    if (p->i + ln <= p->n) {
      int ok = 1;
      for (size_t j = 0; j < ln; j++) if (p->u[p->i + j] != (uint16_t)lits[l][j]) { ok = 0; break; }
      if (ok) {
        p->i += ln;
        if (l == 2) return val_new(c, V_NULL);
        Val *v = val_new(c, V_BOOL); v->b = (l == 0); return v;
      }
    }
  }
  /* number: -?(0|[1-9]\d*)(\.\d+)?([eE][+-]?\d+)? */
  size_t st = p->i;
  if (p->i < p->n && p->u[p->i] == '-') p->i++;
  if (p->i >= p->n) fail(c, YMO_ERR_SYNTAX);
  if (p->u[p->i] == '0') p->i++;
  else if (p->u[p->i] >= '1' && p->u[p->i] <= '9') { while (p->i < p->n && p->u[p->i] >= '0' && p->u[p->i] <= '9') p->i++; }
  else fail(c, YMO_ERR_SYNTAX);
  if (p->i < p->n && p->u[p->i] == '.') {
    p->i++;
    if (p->i >= p->n || p->u[p->i] < '0' || p->u[p->i] > '9') fail(c, YMO_ERR_SYNTAX);
    while (p->i < p->n && p->u[p->i] >= '0' && p->u[p->i] <= '9') p->i++;
  }
  if (p->i < p->n && (p->u[p->i] == 'e' || p->u[p->i] == 'E')) {
    p->i++;
    if (p->i < p->n && (p->u[p->i] == '+' || p->u[p->i] == '-')) p->i++;
    if (p->i >= p->n || p->u[p->i] < '0' || p->u[p->i] > '9') fail(c, YMO_ERR_SYNTAX);
    while (p->i < p->n && p->u[p->i] >= '0' && p->u[p->i] <= '9') p->i++;
  }
  size_t ln = p->i - st;
  char *tmp = (char *)aalloc(c, ln + 1);
  for (size_t j = 0; j < ln; j++) tmp[j] = (char)p->u[st + j];
  tmp[ln] = 0;
  Val *v = val_new(c, V_NUM);
  v->num = strtod(tmp, NULL);
  return v;
}
static Val *json_parse(Ctx *c, Str s) {
  JP p = {s.u, s.n, 0};
  Val *v = jval(c, &p, 0);
  jws(&p);
  if (p.i != p.n) fail(c, YMO_ERR_SYNTAX);
  return v;
}

/* Number::toString(x) for finite x (ECMA-262 7.1.12.1), shortest round-trip digits */
static void js_num_to_string(double x, char *out) {
  if (x == 0) { strcpy(out, "0"); return; }
  if (isnan(x)) { strcpy(out, "NaN"); return; }
  char *o = out;
  if (x < 0) { *o++ = '-'; x = -x; }
  if (isinf(x)) { strcpy(o, "Infinity"); return; }
  char buf[64];
  int p;
  for (p = 1; p <= 17; p++) {
    snprintf(buf, sizeof buf, "%.*e", p - 1, x);
    if (strtod(buf, NULL) == x) break;
  }
  char digits[32];
  int k = 0;
  char *e = strchr(buf, 'e');
  for (char *q = buf; q < e; q++) if (*q >= '0' && *q <= '9') digits[k++] = *q;
  while (k > 1 && digits[k - 1] == '0') k--;
  digits[k] = 0;
  int n = atoi(e + 1) + 1;
  if (k <= n && n <= 21) {
    memcpy(o, digits, k); o += k;
    for (int i = 0; i < n - k; i++) *o++ = '0';
    *o = 0;
  } else if (0 < n && n <= 21) {
    memcpy(o, digits, n); o += n; *o++ = '.';
    memcpy(o, digits + n, k - n); o += k - n; *o = 0;
  } else if (-6 < n && n <= 0) {
    *o++ = '0'; *o++ = '.';
    for (int i = 0; i < -n; i++) *o++ = '0';
    memcpy(o, digits, k); o += k; *o = 0;
  } else {
    *o++ = digits[0];
    if (k > 1) { *o++ = '.'; memcpy(o, digits + 1, k - 1); o += k - 1; }
    sprintf(o, "e%c%d", n - 1 >= 0 ? '+' : '-', abs(n - 1));
  }
}

typedef struct { uint16_t *u; size_t n, cap; } WStr;
static void ws_put(Ctx *c, WStr *w, uint16_t ch) {
  if (w->n == w->cap) {
    size_t cap = w->cap ? w->cap * 2 : 32;
    uint16_t *nu = (uint16_t *)aalloc(c, cap * 2);
    if (w->n) memcpy(nu, w->u, w->n * 2);
    w->u = nu; w->cap = cap;
  }
  w->u[w->n++] = ch;
}
static void ws_ascii(Ctx *c, WStr *w, const char *s) { while (*s) ws_put(c, w, (uint8_t)*s++); }
static void json_quote(Ctx *c, WStr *w, Str s) {
  static const char *hexd = "0123456789abcdef";
  ws_put(c, w, '"');
  for (size_t i = 0; i < s.n; i++) {
    uint16_t ch = s.u[i];
    switch (ch) {
      case 8: ws_ascii(c, w, "\\b"); continue;
      case 9: ws_ascii(c, w, "\\t"); continue;
      case 10: ws_ascii(c, w, "\\n"); continue;
      case 12: ws_ascii(c, w, "\\f"); continue;
      case 13: ws_ascii(c, w, "\\r"); continue;
      case '"': ws_ascii(c, w, "\\\""); continue;
      case '\\': ws_ascii(c, w, "\\\\"); continue;
    }
    int lone = 0;
    if (ch >= 0xD800 && ch <= 0xDBFF) {
      if (i + 1 < s.n && s.u[i + 1] >= 0xDC00 && s.u[i + 1] <= 0xDFFF) { ws_put(c, w, ch); ws_put(c, w, s.u[++i]); continue; }
      lone = 1;
    } else if (ch >= 0xDC00 && ch <= 0xDFFF) lone = 1;
    if (ch < 0x20 || lone) {
      ws_ascii(c, w, "\\u");
      ws_put(c, w, hexd[(ch >> 12) & 15]); ws_put(c, w, hexd[(ch >> 8) & 15]);
      ws_put(c, w, hexd[(ch >> 4) & 15]); ws_put(c, w, hexd[ch & 15]);
      continue;
    }
    ws_put(c, w, ch);
  }
  ws_put(c, w, '"');
}
static void json_stringify_into(Ctx *c, WStr *w, const Val *v) {
  switch (v->t) {
    case V_NULL: case V_UNDEF: ws_ascii(c, w, "null"); return;
    case V_BOOL: ws_ascii(c, w, v->b ? "true" : "false"); return;
    case V_NUM: {
      if (!isfinite(v->num)) { ws_ascii(c, w, "null"); return; }
      char buf[64]; js_num_to_string(v->num, buf); ws_ascii(c, w, buf); return;
    }
    case V_STR: json_quote(c, w, v->s); return;
    case V_ARR:
      ws_put(c, w, '[');
      for (size_t i = 0; i < v->n; i++) { if (i) ws_put(c, w, ','); json_stringify_into(c, w, v->items[i]); }
      ws_put(c, w, ']');
      return;
    case V_OBJ:
      ws_put(c, w, '{');
      for (size_t i = 0; i < v->n; i++) {
        if (i) ws_put(c, w, ',');
        json_quote(c, w, v->keys[i]); ws_put(c, w, ':'); json_stringify_into(c, w, v->items[i]);
      }
      ws_put(c, w, '}');
      return;
    default: fail(c, YMO_ERR_UNSUPPORTED); /* not producible by JSON.parse */
  }
}
static Str json_stringify(Ctx *c, const Val *v) {
  WStr w = {NULL, 0, 0};
  json_stringify_into(c, &w, v);
  Str r = {w.u, w.n};
  return r;
}
/* JSON.stringify over any readAny value (V2 -> V1 conversion of embeds / formats): undefined members of
   objects are omitted, undefined array elements become null, a Uint8Array is an object with index
   keys, a bigint throws TypeError; a top-level undefined gives JS `undefined`, which writeVarString
   encodes as the text "undefined" (encodeURIComponent(undefined)). */
static void json_any_into(Ctx *c, WStr *w, const Val *v) {
  switch (v->t) {
    case V_BIGINT: fail(c, YMO_ERR_TYPE); return;
    case V_BYTES: {
      ws_put(c, w, '{');
      for (size_t i = 0; i < v->bytes.n; i++) {
        char buf[32];
        if (i) ws_put(c, w, ',');
        snprintf(buf, sizeof buf, "\"%zu\":%u", i, (unsigned)v->bytes.p[i]);
        ws_ascii(c, w, buf);
      }
      ws_put(c, w, '}');
      return;
    }
    case V_ARR:
      ws_put(c, w, '[');
      for (size_t i = 0; i < v->n; i++) { if (i) ws_put(c, w, ','); json_any_into(c, w, v->items[i]); }
      ws_put(c, w, ']');
      return;
    case V_OBJ: {
      ws_put(c, w, '{');
      int first = 1;
      for (size_t i = 0; i < v->n; i++) {
        if (v->items[i]->t == V_UNDEF) continue;
        if (!first) ws_put(c, w, ',');
        first = 0;
        json_quote(c, w, v->keys[i]); ws_put(c, w, ':'); json_any_into(c, w, v->items[i]);
      }
      ws_put(c, w, '}');
      return;
    }
    default: json_stringify_into(c, w, v); return;
  }
}
static Str json_text_of_any(Ctx *c, const Val *v) {
  WStr w = {NULL, 0, 0};
  if (v->t == V_UNDEF) ws_ascii(c, &w, "undefined");
  else json_any_into(c, &w, v);
  Str r = {w.u, w.n};
  return r;
}

/* ------------------------------------------------------------------------------------------------ */
/* lib0 RLE column decoders (V2)                                                                   */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { Dec d; int s; int64_t count; } RleDec;            /* RleDecoder<readUint8> (N) */
typedef struct { Dec d; double s; int64_t count; } UintOptDec;     /* UintOptRleDecoder (P)     */
typedef struct { Dec d; int64_t s; int64_t count; int64_t diff; } IntDiffDec; /* (G)          */
typedef struct { UintOptDec lens; Str str; int64_t spos; } StrDec; /* StringDecoder ($)         */

static int rle_read(Ctx *c, RleDec *r) {
  if (r->count == 0) {
    r->s = dbyte(&r->d);
    if (dhas(&r->d)) r->count = (int64_t)rd_vu(c, &r->d) + 1;
    else r->count = -1;
  }
  r->count--;
  return r->s;
}
static int64_t uopt_read(Ctx *c, UintOptDec *r) {
  if (r->count == 0) {
    r->s = rd_vi(c, &r->d);
    int neg = js_is_negzero_or_neg(r->s);
    r->count = 1;
    if (neg) { r->s = -r->s; r->count = (int64_t)rd_vu(c, &r->d) + 2; }
  }
  r->count--;
  return (int64_t)r->s;
}
static int64_t idiff_read(Ctx *c, IntDiffDec *r) {
  if (r->count == 0) {
    double t = rd_vi(c, &r->d);
    int32_t ti = js_toint32(t);
    int sb = ti & 1;
    r->diff = ti >> 1;
    r->count = 1;
    if (sb) r->count = (int64_t)rd_vu(c, &r->d) + 2;
  }
  r->s += r->diff;
  r->count--;
  return r->s;
}
static Str sdec_read(Ctx *c, StrDec *r) {
  int64_t t = r->spos + uopt_read(c, &r->lens);
  Str s = str_slice(r->str, r->spos, t);
  r->spos = t;
  return s;
}

/* ------------------------------------------------------------------------------------------------ */
/* lib0 RLE column encoders (V2)                                                                   */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { Buf *b; int s; int64_t count; } RleEnc;             /* RleEncoder<writeUint8> ($) */
typedef struct { Buf *b; double s; int64_t count; } UintOptEnc;      /* UintOptRleEncoder (K)       */
typedef struct { Buf *b; int64_t s, count, diff; } IntDiffEnc;        /* IntDiffOptRleEncoder (H)    */
typedef struct { WStr s; UintOptEnc lens; } StrEnc;                   /* StringEncoder (W)           */

static void rle_write(Ctx *c, RleEnc *e, int v) {
  if (e->s == v) { e->count++; return; }
  if (e->count > 0) wr_vu(c, e->b, e->count - 1);
  e->count = 1;
  put8(c, e->b, (unsigned)v & 255);
  e->s = v;
}
static void uopt_flush(Ctx *c, UintOptEnc *e) {
  if (e->count > 0) {
    wr_vi(c, e->b, e->count == 1 ? e->s : -e->s);
    if (e->count > 1) wr_vu(c, e->b, e->count - 2);
  }
}
static void uopt_write(Ctx *c, UintOptEnc *e, double v) {
  if (e->s == v) { e->count++; return; } /* JS ===: 0 === -0 */
  uopt_flush(c, e);
  e->count = 1;
  e->s = v;
}
static void idiff_flush(Ctx *c, IntDiffEnc *e) {
  if (e->count > 0) {
    int32_t d = (int32_t)((uint32_t)js_toint32((double)e->diff) << 1) | (e->count == 1 ? 0 : 1);
    wr_vi(c, e->b, (double)d);
    if (e->count > 1) wr_vu(c, e->b, e->count - 2);
  }
}
static void idiff_write(Ctx *c, IntDiffEnc *e, int64_t v) {
  if (e->diff == v - e->s) { e->s = v; e->count++; return; }
  idiff_flush(c, e);
  e->count = 1;
  e->diff = v - e->s;
  e->s = v;
}
static void senc_write(Ctx *c, StrEnc *e, Str s) {
  for (size_t i = 0; i < s.n; i++) ws_put(c, &e->s, s.u[i]);
  uopt_write(c, &e->lens, (double)s.n);
}

/* ------------------------------------------------------------------------------------------------ */
/* UpdateDecoderV1 / UpdateDecoderV2 (src/utils/UpdateDecoder.js:154-243, 270-392)                 */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
  int v2;
  Dec rest;
  IntDiffDec keyClock, leftClock, rightClock;
  UintOptDec client, typeRef, len;
  RleDec info, parentInfo;
  StrDec str;
  Str *keys;
  size_t nkeys, capkeys;
  int64_t dsCurr;
} UDec;

static Dec col_dec(Ctx *c, Dec *rest) {
  Span s = rd_vbytes(c, rest);
  Dec d = {s.p, s.n, 0};
  return d;
}
static void udec_init(Ctx *c, UDec *u, const uint8_t *p, size_t n, int v2) {
  memset(u, 0, sizeof(*u));
  u->v2 = v2;
  u->rest.a = p; u->rest.len = n; u->rest.pos = 0;
  if (!v2) return;
  rd_vu(c, &u->rest); /* feature flag (13.5.16 reads it with readVarUint) */
  u->keyClock.d = col_dec(c, &u->rest);
  u->client.d = col_dec(c, &u->rest);
  u->leftClock.d = col_dec(c, &u->rest);
  u->rightClock.d = col_dec(c, &u->rest);
  u->info.d = col_dec(c, &u->rest);
  u->str.lens.d = col_dec(c, &u->rest);
  u->str.str = rd_vstr(c, &u->str.lens.d); /* StringDecoder decodes the whole column up front */
  u->parentInfo.d = col_dec(c, &u->rest);
  u->typeRef.d = col_dec(c, &u->rest);
  u->len.d = col_dec(c, &u->rest);
}
typedef struct { int64_t client, clock; } JID;
static JID ud_left(Ctx *c, UDec *u) {
  JID r;
  if (u->v2) { r.client = uopt_read(c, &u->client); r.clock = idiff_read(c, &u->leftClock); }
  else { r.client = rd_vu(c, &u->rest); r.clock = rd_vu(c, &u->rest); }
  return r;
}
static JID ud_right(Ctx *c, UDec *u) {
  JID r;
  if (u->v2) { r.client = uopt_read(c, &u->client); r.clock = idiff_read(c, &u->rightClock); }
  else { r.client = rd_vu(c, &u->rest); r.clock = rd_vu(c, &u->rest); }
  return r;
}
static int64_t ud_client(Ctx *c, UDec *u) { return u->v2 ? uopt_read(c, &u->client) : (int64_t)rd_vu(c, &u->rest); }
static int ud_info(Ctx *c, UDec *u) { return u->v2 ? rle_read(c, &u->info) : dbyte(&u->rest); }
static Str ud_string(Ctx *c, UDec *u) { return u->v2 ? sdec_read(c, &u->str) : rd_vstr(c, &u->rest); }
static int ud_parent_info(Ctx *c, UDec *u) { return u->v2 ? rle_read(c, &u->parentInfo) == 1 : rd_vu(c, &u->rest) == 1; }
static int64_t ud_typeref(Ctx *c, UDec *u) { return u->v2 ? uopt_read(c, &u->typeRef) : (int64_t)rd_vu(c, &u->rest); }
static int64_t ud_len(Ctx *c, UDec *u) { return u->v2 ? uopt_read(c, &u->len) : (int64_t)rd_vu(c, &u->rest); }
/* readKey (UpdateDecoder.js:382-391): `keyClock < this.keys.length ? this.keys[keyClock] : read` -- a
   negative keyClock indexes nothing: the key is `undefined` (K_UNDEF_KEY) */
static const uint16_t K_UNDEF_KEY[1] = {0};
static Str ud_key(Ctx *c, UDec *u) {
  if (!u->v2) return rd_vstr(c, &u->rest);
  int64_t kc = idiff_read(c, &u->keyClock);
  if (kc < 0) { Str un = {K_UNDEF_KEY, 0}; return un; }
  if ((size_t)kc < u->nkeys) return u->keys[kc];
  Str s = sdec_read(c, &u->str);
  if (u->nkeys == u->capkeys) {
    size_t cap = u->capkeys ? u->capkeys * 2 : 8;
    Str *nk = (Str *)aalloc(c, cap * sizeof(Str));
    if (u->nkeys) memcpy(nk, u->keys, u->nkeys * sizeof(Str));
    u->keys = nk; u->capkeys = cap;
  }
  u->keys[u->nkeys++] = s;
  return s;
}
static void ud_reset_ds(UDec *u) { u->dsCurr = 0; }
static int64_t ud_ds_clock(Ctx *c, UDec *u) {
  if (!u->v2) return rd_vu(c, &u->rest);
  u->dsCurr += rd_vu(c, &u->rest);
  return u->dsCurr;
}
static int64_t ud_ds_len(Ctx *c, UDec *u) {
  if (!u->v2) return rd_vu(c, &u->rest);
  int64_t d = (int64_t)rd_vu(c, &u->rest) + 1;
  u->dsCurr += d;
  return d;
}

/* ------------------------------------------------------------------------------------------------ */
/* UpdateEncoderV1 / UpdateEncoderV2 (src/utils/UpdateEncoder.js:138-227, 264-408)                  */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
  int v2;
  Buf *rest;
  IntDiffEnc keyClock, leftClock, rightClock;
  UintOptEnc client, typeRef, len;
  RleEnc info, parentInfo;
  StrEnc str;
  int64_t keyClockCounter;
  int64_t dsCurr;
} UEnc;

static void uenc_init(Ctx *c, UEnc *e, int v2) {
  memset(e, 0, sizeof(*e));
  e->v2 = v2;
  e->rest = buf_new(c);
  if (!v2) return;
  e->keyClock.b = buf_new(c); e->leftClock.b = buf_new(c); e->rightClock.b = buf_new(c);
  e->client.b = buf_new(c); e->typeRef.b = buf_new(c); e->len.b = buf_new(c);
  e->info.b = buf_new(c); e->info.s = -1000; /* RleEncoder starts with s = null */
  e->parentInfo.b = buf_new(c); e->parentInfo.s = -1000;
  e->str.lens.b = buf_new(c);
}
static void ue_left(Ctx *c, UEnc *e, JID id) {
  if (e->v2) { uopt_write(c, &e->client, (double)id.client); idiff_write(c, &e->leftClock, id.clock); }
  else { wr_vu(c, e->rest, id.client); wr_vu(c, e->rest, id.clock); }
}
static void ue_right(Ctx *c, UEnc *e, JID id) {
  if (e->v2) { uopt_write(c, &e->client, (double)id.client); idiff_write(c, &e->rightClock, id.clock); }
  else { wr_vu(c, e->rest, id.client); wr_vu(c, e->rest, id.clock); }
}
static void ue_client(Ctx *c, UEnc *e, int64_t client) {
  if (e->v2) uopt_write(c, &e->client, (double)client);
  else wr_vu(c, e->rest, client);
}
static void ue_info(Ctx *c, UEnc *e, int info) {
  if (e->v2) rle_write(c, &e->info, info);
  else put8(c, e->rest, (unsigned)info & 255);
}
static void ue_string(Ctx *c, UEnc *e, Str s) {
  if (e->v2) senc_write(c, &e->str, s);
  else wr_vstr(c, e->rest, s);
}
static void ue_parent_info(Ctx *c, UEnc *e, int isykey) {
  if (e->v2) rle_write(c, &e->parentInfo, isykey ? 1 : 0);
  else wr_vu(c, e->rest, isykey ? 1 : 0);
}
static void ue_typeref(Ctx *c, UEnc *e, int64_t t) {
  if (e->v2) uopt_write(c, &e->typeRef, (double)t);
  else wr_vu(c, e->rest, t);
}
static void ue_len(Ctx *c, UEnc *e, int64_t l) {
  if (e->v2) uopt_write(c, &e->len, (double)l);
  else wr_vu(c, e->rest, l);
}
static void ue_key(Ctx *c, UEnc *e, Str k) {
  if (k.u == K_UNDEF_KEY) {  /* writeKey(undefined): V2 StringEncoder reads undefined.length (TypeError);
                                V1 writeVarString(undefined) writes encodeURIComponent(undefined) = "undefined" */
    if (e->v2) fail(c, YMO_ERR_TYPE);
    static const uint16_t und[] = {'u', 'n', 'd', 'e', 'f', 'i', 'n', 'e', 'd'};
    Str us = {und, 9};
    wr_vstr(c, e->rest, us);
    return;
  }
  if (e->v2) { idiff_write(c, &e->keyClock, e->keyClockCounter++); senc_write(c, &e->str, k); }
  else wr_vstr(c, e->rest, k);
}
static void ue_reset_ds(UEnc *e) { e->dsCurr = 0; }
static void ue_ds_clock(Ctx *c, UEnc *e, int64_t clock) {
  if (!e->v2) { wr_vu(c, e->rest, clock); return; }
  int64_t d = clock - e->dsCurr;
  e->dsCurr = clock;
  wr_vu(c, e->rest, d);
}
static void ue_ds_len(Ctx *c, UEnc *e, int64_t len) {
  if (!e->v2) { wr_vu(c, e->rest, len); return; }
  if (len == 0) fail(c, YMO_ERR_UNEXPECTED);
  wr_vu(c, e->rest, len - 1);
  e->dsCurr += len;
}
static Buf *uenc_finish(Ctx *c, UEnc *e) {
  if (!e->v2) return e->rest;
  Buf *o = buf_new(c);
  wr_vu(c, o, 0); /* feature flag */
  idiff_flush(c, &e->keyClock); wr_vbytes(c, o, e->keyClock.b->p, e->keyClock.b->n);
  uopt_flush(c, &e->client); wr_vbytes(c, o, e->client.b->p, e->client.b->n);
  idiff_flush(c, &e->leftClock); wr_vbytes(c, o, e->leftClock.b->p, e->leftClock.b->n);
  idiff_flush(c, &e->rightClock); wr_vbytes(c, o, e->rightClock.b->p, e->rightClock.b->n);
  wr_vbytes(c, o, e->info.b->p, e->info.b->n);
  {
    Buf *sb = buf_new(c);
    Str all = {e->str.s.u, e->str.s.n};
    wr_vstr(c, sb, all);
    uopt_flush(c, &e->str.lens);
    putraw(c, sb, e->str.lens.b->p, e->str.lens.b->n);
    wr_vbytes(c, o, sb->p, sb->n);
  }
  wr_vbytes(c, o, e->parentInfo.b->p, e->parentInfo.b->n);
  uopt_flush(c, &e->typeRef); wr_vbytes(c, o, e->typeRef.b->p, e->typeRef.b->n);
  uopt_flush(c, &e->len); wr_vbytes(c, o, e->len.b->p, e->len.b->n);
  putraw(c, o, e->rest->p, e->rest->n);
  return o;
}

/* ------------------------------------------------------------------------------------------------ */
/* Structs and contents                                                                            */
/* ------------------------------------------------------------------------------------------------ */
enum { K_GC = 0, K_SKIP = 1, K_ITEM = 2 };
typedef struct {
  int ref;      /* 1..9 */
  int64_t dlen; /* ContentDeleted */
  Str str;      /* ContentString */
  Span bin;     /* ContentBinary */
  /* JSON (ref 2): elements are canonical JSON texts, `undef` marks the literal 'undefined' */
  Str *jstrs; uint8_t *jundef;
  /* Any (ref 8): values */
  Val **anys;
  size_t n;     /* JSON / Any element count */
  /* Embed (5) / Format value (6): V1 canonical JSON text; V2 any value */
  Str jtext; Val *jval;
  Str key;      /* Format key */
  int64_t typeRef; Str typeName; /* ContentType */
  Str guid; Val *docOpts;        /* ContentDoc */
} Content;

typedef struct Struct {
  int kind;
  int64_t client, clock, len;
  int has_origin, has_right;
  JID origin, right;
  int parent_kind; /* 0 none, 1 ykey, 2 ID */
  Str pkey; JID pid;
  int has_psub; Str psub;
  Content *content;
} Struct;

static int js_truthy(const Val *v) {
  switch (v->t) {
    case V_UNDEF: case V_NULL: return 0;
    case V_BOOL: return v->b;
    case V_NUM: return !(v->num == 0 || isnan(v->num));
    case V_STR: return v->s.n != 0;
    case V_BIGINT: { for (int i = 0; i < 8; i++) if (v->big[i]) return 1; return 0; }
    default: return 1;
  }
}

/* ContentDoc (13.5.16 Pr/Rr; ContentDoc.js:116-135): new Doc({guid, ...opts}) then opts re-derived */
static void content_doc_canon(Ctx *c, Content *ct, Str guid, Val *o) {
  static const uint16_t kg[] = {'g', 'u', 'i', 'd'}, kgc[] = {'g', 'c'},
                        kal[] = {'a', 'u', 't', 'o', 'L', 'o', 'a', 'd'}, km[] = {'m', 'e', 't', 'a'};
  Str sg = {kg, 4}, sgc = {kgc, 2}, sal = {kal, 8}, sm = {km, 4};
  Val *vguid = NULL, *vgc = NULL, *val = NULL, *vmeta = NULL;
  if (o->t == V_OBJ) {
    for (size_t i = 0; i < o->n; i++) {
      if (str_eq(o->keys[i], sg)) vguid = o->items[i];
      else if (str_eq(o->keys[i], sgc)) vgc = o->items[i];
      else if (str_eq(o->keys[i], sal)) val = o->items[i];
      else if (str_eq(o->keys[i], sm)) vmeta = o->items[i];
    }
  }
  if (vguid) {
    if (vguid->t == V_UNDEF || vguid->t != V_STR) fail(c, YMO_ERR_UNSUPPORTED); /* random / non-string guid */
    guid = vguid->s;
  }
  Val *opts = val_new(c, V_OBJ);
  int gc = (vgc == NULL || vgc->t == V_UNDEF) ? 1 : js_truthy(vgc);
  int autoload = (val == NULL || val->t == V_UNDEF) ? 0 : js_truthy(val);
  Val *meta = (vmeta == NULL || vmeta->t == V_UNDEF) ? NULL : vmeta;
  if (!gc) { Val *f = val_new(c, V_BOOL); f->b = 0; obj_set(c, opts, sgc, f, 1); }
  if (autoload) { Val *t = val_new(c, V_BOOL); t->b = 1; obj_set(c, opts, sal, t, 1); }
  if (meta && meta->t != V_NULL) obj_set(c, opts, sm, meta, 1);
  ct->guid = guid;
  ct->docOpts = opts;
}

static int64_t content_len(const Content *ct) {
  switch (ct->ref) {
    case 1: return ct->dlen;
    case 2: case 8: return (int64_t)ct->n;
    case 4: return (int64_t)ct->str.n;
    default: return 1;
  }
}

static Content *read_content(Ctx *c, UDec *u, int info) { /* readItemContent / contentRefs (Item.js:665-683) */
  int ref = info & 31;
  Content *ct = (Content *)aalloc(c, sizeof(Content));
  memset(ct, 0, sizeof(*ct));
  ct->ref = ref;
  switch (ref) {
    case 1: ct->dlen = ud_len(c, u); break;
    case 2: {
      int64_t n = ud_len(c, u);
      static const uint16_t und[] = {'u', 'n', 'd', 'e', 'f', 'i', 'n', 'e', 'd'};
      Str us = {und, 9};
      size_t cap = 0;
      for (int64_t i = 0; i < n; i++) {
        Str s = ud_string(c, u);
        if (ct->n == cap) {
          cap = cap ? cap * 2 : 4;
          Str *nj = (Str *)aalloc(c, cap * sizeof(Str));
          uint8_t *nu = (uint8_t *)aalloc(c, cap);
          if (ct->n) { memcpy(nj, ct->jstrs, ct->n * sizeof(Str)); memcpy(nu, ct->jundef, ct->n); }
          ct->jstrs = nj; ct->jundef = nu;
        }
        if (str_eq(s, us)) { ct->jundef[ct->n] = 1; ct->jstrs[ct->n] = us; }
        else { ct->jundef[ct->n] = 0; ct->jstrs[ct->n] = json_stringify(c, json_parse(c, s)); }
        ct->n++;
      }
      break;
    }
    case 3: {
      Span s = rd_vbytes(c, &u->rest);
      ct->bin = s;
      break;
    }
    case 4: ct->str = ud_string(c, u); break;
    case 5:  /* readJSON: V1 JSON.parse(readVarString), V2 readAny; both forms kept for either writer */
      if (u->v2) ct->jval = rd_any(c, &u->rest);
      else { ct->jval = json_parse(c, rd_vstr(c, &u->rest)); ct->jtext = json_stringify(c, ct->jval); }
      break;
    case 6:
      ct->key = ud_string(c, u);
      if (u->v2) ct->jval = rd_any(c, &u->rest);
      else { ct->jval = json_parse(c, rd_vstr(c, &u->rest)); ct->jtext = json_stringify(c, ct->jval); }
      break;
    case 7: {
      int64_t tr = ud_typeref(c, u);
      if (tr < 0 || tr > 6) fail(c, YMO_ERR_TYPE);
      ct->typeRef = tr;
      if (tr == 3 || tr == 5) {
        ct->typeName = ud_key(c, u);
        if (tr == 3 && ct->typeName.u == K_UNDEF_KEY) { /* new YXmlElement(undefined): nodeName = 'UNDEFINED' */
          static const uint16_t un[] = {'U', 'N', 'D', 'E', 'F', 'I', 'N', 'E', 'D'};
          Str us = {un, 9};
          ct->typeName = us;
        }
      }
      break;
    }
    case 8: {
      int64_t n = ud_len(c, u);
      size_t cap = 0;
      for (int64_t i = 0; i < n; i++) {
        Val *v = rd_any(c, &u->rest);
        if (ct->n == cap) {
          cap = cap ? cap * 2 : 4;
          Val **na = (Val **)aalloc(c, cap * sizeof(Val *));
          if (ct->n) memcpy(na, ct->anys, ct->n * sizeof(Val *));
          ct->anys = na;
        }
        ct->anys[ct->n++] = v;
      }
      break;
    }
    case 9: {
      Str guid = ud_string(c, u);
      Val *o = rd_any(c, &u->rest);
      content_doc_canon(c, ct, guid, o);
      break;
    }
    case 0: case 10: fail(c, YMO_ERR_UNEXPECTED);
    default: fail(c, YMO_ERR_TYPE);
  }
  return ct;
}

/* ContentX.splice(offset): returns the right part (13.5.16 @70000-75900) */
static Content *content_splice(Ctx *c, const Content *src, int64_t off) {
  Content *r = (Content *)aalloc(c, sizeof(Content));
  *r = *src;
  switch (src->ref) {
    case 1: r->dlen = src->dlen - off; break;
    case 2:
      r->n = off < (int64_t)src->n ? src->n - (size_t)off : 0;
      r->jstrs = src->jstrs + (off < (int64_t)src->n ? off : (int64_t)src->n);
      r->jundef = src->jundef + (off < (int64_t)src->n ? off : (int64_t)src->n);
      break;
    case 8:
      r->n = off < (int64_t)src->n ? src->n - (size_t)off : 0;
      r->anys = src->anys + (off < (int64_t)src->n ? off : (int64_t)src->n);
      break;
    case 4: {
      Str right = str_slice(src->str, off, (int64_t)src->str.n);
      if (off >= 1 && off <= (int64_t)src->str.n) { /* charCodeAt(t - 1) of the left part */
        uint16_t ch = src->str.u[off - 1];
        if (ch >= 0xD800 && ch <= 0xDBFF) { /* ContentString.js:55-64: replace both halves by U+FFFD */
          uint16_t *nu = (uint16_t *)aalloc(c, (right.n + 1) * 2);
          nu[0] = 0xFFFD;
          if (right.n > 1) memcpy(nu + 1, right.u + 1, (right.n - 1) * 2);
          Str ns = {nu, right.n ? right.n : 1};
          right = ns;
        }
      }
      r->str = right;
      break;
    }
    default: fail(c, YMO_ERR_METHOD);
  }
  return r;
}

static void content_write(Ctx *c, UEnc *e, const Content *ct, int64_t off) {
  switch (ct->ref) {
    case 1: ue_len(c, e, ct->dlen - off); break;
    case 2:
      ue_len(c, e, (int64_t)ct->n - off);
      for (int64_t i = off; i < (int64_t)ct->n; i++) ue_string(c, e, ct->jstrs[i]);
      break;
    case 3: wr_vbytes(c, e->rest, ct->bin.p, ct->bin.n); break;
    case 4: ue_string(c, e, off == 0 ? ct->str : str_slice(ct->str, off, (int64_t)ct->str.n)); break;
    case 5:
      if (e->v2) wr_any(c, e->rest, ct->jval);
      else wr_vstr(c, e->rest, ct->jtext.u ? ct->jtext : json_text_of_any(c, ct->jval));
      break;
    case 6:
      ue_key(c, e, ct->key);
      if (e->v2) wr_any(c, e->rest, ct->jval);
      else wr_vstr(c, e->rest, ct->jtext.u ? ct->jtext : json_text_of_any(c, ct->jval));
      break;
    case 7:
      ue_typeref(c, e, ct->typeRef);
      if (ct->typeRef == 3 || ct->typeRef == 5) ue_key(c, e, ct->typeName);
      break;
    case 8:
      ue_len(c, e, (int64_t)ct->n - off);
      for (int64_t i = off; i < (int64_t)ct->n; i++) wr_any(c, e->rest, ct->anys[i]);
      break;
    case 9: ue_string(c, e, ct->guid); wr_any(c, e->rest, ct->docOpts); break;
    default: fail(c, YMO_ERR_UNEXPECTED);
  }
}

/* Item.write / GC.write / Skip.write with offset (Item.js:625-658, GC.js:45-48, 13.5.16 ui.write) */
static void struct_write(Ctx *c, UEnc *e, const Struct *s, int64_t off) {
  if (s->kind == K_GC) { ue_info(c, e, 0); ue_len(c, e, s->len - off); return; }
  if (s->kind == K_SKIP) { ue_info(c, e, 10); wr_vu(c, e->rest, s->len - off); return; }
  int has_origin = off > 0 ? 1 : s->has_origin;
  JID origin = s->origin;
  if (off > 0) { origin.client = s->client; origin.clock = s->clock + off - 1; }
  int info = (s->content->ref & 31) | (has_origin ? 0x80 : 0) | (s->has_right ? 0x40 : 0) | (s->has_psub ? 0x20 : 0);
  ue_info(c, e, info);
  if (has_origin) ue_left(c, e, origin);
  if (s->has_right) ue_right(c, e, s->right);
  if (!has_origin && !s->has_right) {
    if (s->parent_kind == 1) { ue_parent_info(c, e, 1); ue_string(c, e, s->pkey); }
    else if (s->parent_kind == 2) { ue_parent_info(c, e, 0); ue_left(c, e, s->pid); }
    else fail(c, YMO_ERR_UNEXPECTED);
    if (s->has_psub) ue_string(c, e, s->psub);
  }
  content_write(c, e, s->content, off);
}

/* sliceStruct (13.5.16 as@38661) */
static Struct *slice_struct(Ctx *c, const Struct *s, int64_t diff) {
  Struct *r = (Struct *)aalloc(c, sizeof(Struct));
  *r = *s;
  r->clock = s->clock + diff;
  r->len = s->len - diff;
  if (s->kind == K_ITEM) {
    r->has_origin = 1;
    r->origin.client = s->client; r->origin.clock = s->clock + diff - 1;
    r->content = content_splice(c, s->content, diff);
    r->len = content_len(r->content);
  }
  return r;
}

/* ------------------------------------------------------------------------------------------------ */
/* LazyStructReader (13.5.16 ts@36560 generator + es@37148)                                         */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
  UDec *u;
  int filter_skips;
  int64_t nclients, ci;  /* outer loop */
  int64_t nstructs, si;  /* inner loop */
  int64_t client, clock;
  int started, done;
  Struct *curr;
} LReader;

static Struct *gen_next(Ctx *c, LReader *r) {
  UDec *u = r->u;
  if (r->done) return NULL;
  if (!r->started) {
    r->started = 1;
    r->nclients = rd_vu(c, &u->rest);
    r->ci = 0;
    r->si = 0; r->nstructs = 0;
  }
  for (;;) {
    if (r->si < r->nstructs) break;
    if (r->ci >= r->nclients) { r->done = 1; return NULL; }
    r->ci++;
    r->nstructs = rd_vu(c, &u->rest);
    r->client = ud_client(c, u);
    r->clock = rd_vu(c, &u->rest);
    r->si = 0;
  }
  r->si++;
  Struct *s = (Struct *)aalloc(c, sizeof(Struct));
  memset(s, 0, sizeof(*s));
  s->client = r->client;
  s->clock = r->clock;
  int info = ud_info(c, u);
  if (info == 10) {
    s->kind = K_SKIP;
    s->len = rd_vu(c, &u->rest);
  } else if (info >= 0 && (info & 31) != 0) {
    s->kind = K_ITEM;
    int noorig = (info & (0x40 | 0x80)) == 0;
    if (info & 0x80) { s->has_origin = 1; s->origin = ud_left(c, u); }
    if (info & 0x40) { s->has_right = 1; s->right = ud_right(c, u); }
    if (noorig) {
      if (ud_parent_info(c, u)) { s->parent_kind = 1; s->pkey = ud_string(c, u); }
      else { s->parent_kind = 2; s->pid = ud_left(c, u); }
      if (info & 0x20) { s->has_psub = 1; s->psub = ud_string(c, u); }
    }
    s->content = read_content(c, u, info);
    s->len = content_len(s->content);
  } else {
    s->kind = K_GC;
    s->len = ud_len(c, u);
  }
  r->clock += s->len;
  return s;
}
static Struct *lr_next(Ctx *c, LReader *r) {
  do { r->curr = gen_next(c, r); } while (r->filter_skips && r->curr && r->curr->kind == K_SKIP);
  return r->curr;
}
static void lr_init(Ctx *c, LReader *r, UDec *u, int filter_skips) {
  memset(r, 0, sizeof(*r));
  r->u = u;
  r->filter_skips = filter_skips;
  lr_next(c, r);
}

/* ------------------------------------------------------------------------------------------------ */
/* LazyStructWriter (13.5.16 rs / ps / gs / ws)                                                     */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { int64_t written; Buf *rest; } Part;
typedef struct {
  int64_t currClient, written;
  UEnc *enc;
  Part *parts;
  size_t nparts, cap;
} LWriter;

static void lw_flush(Ctx *c, LWriter *w) {
  if (w->written > 0) {
    if (w->nparts == w->cap) {
      size_t cap = w->cap ? w->cap * 2 : 16;
      Part *np = (Part *)aalloc(c, cap * sizeof(Part));
      if (w->nparts) memcpy(np, w->parts, w->nparts * sizeof(Part));
      w->parts = np; w->cap = cap;
    }
    w->parts[w->nparts].written = w->written;
    w->parts[w->nparts].rest = w->enc->rest;
    w->nparts++;
    w->enc->rest = buf_new(c);
    w->written = 0;
  }
}
static void lw_write(Ctx *c, LWriter *w, const Struct *s, int64_t off) {
  if (w->written > 0 && w->currClient != s->client) lw_flush(c, w);
  if (w->written == 0) {
    w->currClient = s->client;
    ue_client(c, w->enc, s->client);
    wr_vu(c, w->enc->rest, s->clock + off);
  }
  struct_write(c, w->enc, s, off);
  w->written++;
}
static void lw_finish(Ctx *c, LWriter *w) {
  lw_flush(c, w);
  Buf *r = w->enc->rest;
  wr_vu(c, r, (int64_t)w->nparts);
  for (size_t i = 0; i < w->nparts; i++) {
    wr_vu(c, r, w->parts[i].written);
    putraw(c, r, w->parts[i].rest->p, w->parts[i].rest->n);
  }
}

/* ------------------------------------------------------------------------------------------------ */
/* DeleteSet (DeleteSet.js:113-256; 13.5.16 le/he/fe/ge)                                            */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { int64_t clock, len; } DItem;
typedef struct { int64_t client; DItem *items; size_t n, cap; } DClient;
typedef struct { DClient *cl; size_t n, cap; } DSet;

static DClient *ds_get_or_add(Ctx *c, DSet *ds, int64_t client) {
  for (size_t i = 0; i < ds->n; i++) if (ds->cl[i].client == client) return &ds->cl[i];
  if (ds->n == ds->cap) {
    size_t cap = ds->cap ? ds->cap * 2 : 8;
    DClient *nc = (DClient *)aalloc(c, cap * sizeof(DClient));
    if (ds->n) memcpy(nc, ds->cl, ds->n * sizeof(DClient));
    ds->cl = nc; ds->cap = cap;
  }
  DClient *d = &ds->cl[ds->n++];
  memset(d, 0, sizeof(*d));
  d->client = client;
  return d;
}
static void dc_push(Ctx *c, DClient *d, int64_t clock, int64_t len) {
  if (d->n == d->cap) {
    size_t cap = d->cap ? d->cap * 2 : 8;
    DItem *ni = (DItem *)aalloc(c, cap * sizeof(DItem));
    if (d->n) memcpy(ni, d->items, d->n * sizeof(DItem));
    d->items = ni; d->cap = cap;
  }
  d->items[d->n].clock = clock; d->items[d->n].len = len; d->n++;
}
static void ds_read(Ctx *c, UDec *u, DSet *ds) { /* readDeleteSet (ge) */
  memset(ds, 0, sizeof(*ds));
  uint32_t n = rd_vu(c, &u->rest);
  for (uint32_t i = 0; i < n; i++) {
    ud_reset_ds(u);
    int64_t client = rd_vu(c, &u->rest);
    uint32_t m = rd_vu(c, &u->rest);
    if (m > 0) {
      DClient *d = ds_get_or_add(c, ds, client);
      for (uint32_t j = 0; j < m; j++) {
        int64_t clock = ud_ds_clock(c, u);
        int64_t len = ud_ds_len(c, u);
        dc_push(c, d, clock, len);
      }
    }
  }
}
static void ds_write(Ctx *c, UEnc *e, const DSet *ds) { /* writeDeleteSet (fe) */
  wr_vu(c, e->rest, (int64_t)ds->n);
  for (size_t i = 0; i < ds->n; i++) {
    ue_reset_ds(e);
    wr_vu(c, e->rest, ds->cl[i].client);
    wr_vu(c, e->rest, (int64_t)ds->cl[i].n);
    for (size_t j = 0; j < ds->cl[i].n; j++) {
      ue_ds_clock(c, e, ds->cl[i].items[j].clock);
      ue_ds_len(c, e, ds->cl[i].items[j].len);
    }
  }
}
static void ditem_msort(DItem *a, DItem *tmp, size_t n) { /* stable by clock */
  if (n < 2) return;
  size_t h = n / 2;
  ditem_msort(a, tmp, h);
  ditem_msort(a + h, tmp, n - h);
  size_t i = 0, j = h, k = 0;
  while (i < h && j < n) tmp[k++] = (a[j].clock < a[i].clock) ? a[j++] : a[i++];
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, n * sizeof(DItem));
}
/* sortAndMergeDeleteSet: 13.5.16 (le@10242) merges touching and overlapping ranges (>=, max of the ends);
   ref = the reference's own (gaberogan/yjs@v0 src/utils/DeleteSet.js:113-135) merges only exactly
   adjacent ranges (left.clock + left.len === right.clock, left.len += right.len) and keeps the rest */
static void ds_sort_and_merge_mode(Ctx *c, DSet *ds, int ref) {
  for (size_t ci = 0; ci < ds->n; ci++) {
    DClient *d = &ds->cl[ci];
    if (d->n > 1) {
      DItem *tmp = (DItem *)aalloc(c, d->n * sizeof(DItem));
      ditem_msort(d->items, tmp, d->n);
    }
    size_t i, j;
    for (i = 1, j = 1; i < d->n; i++) {
      DItem *left = &d->items[j - 1];
      DItem right = d->items[i];
      if (ref ? left->clock + left->len == right.clock : left->clock + left->len >= right.clock) {
        if (ref) left->len += right.len;
        else {
          int64_t m = right.clock + right.len - left->clock;
          if (m > left->len) left->len = m;
        }
      } else {
        if (j < i) d->items[j] = right;
        j++;
      }
    }
    if (d->n > 0) d->n = j;
  }
}
static void ds_merge_mode(Ctx *c, DSet *dss, size_t k, DSet *out, int ref) { /* mergeDeleteSets (he; DeleteSet.js:141-161) */
  memset(out, 0, sizeof(*out));
  for (size_t i = 0; i < k; i++) {
    for (size_t ci = 0; ci < dss[i].n; ci++) {
      int64_t client = dss[i].cl[ci].client;
      int have = 0;
      for (size_t q = 0; q < out->n; q++) if (out->cl[q].client == client) { have = 1; break; }
      if (have) continue;
      DClient *d = ds_get_or_add(c, out, client);
      for (size_t j = i; j < k; j++) {
        for (size_t cj = 0; cj < dss[j].n; cj++) {
          if (dss[j].cl[cj].client != client) continue;
          for (size_t t = 0; t < dss[j].cl[cj].n; t++) dc_push(c, d, dss[j].cl[cj].items[t].clock, dss[j].cl[cj].items[t].len);
        }
      }
    }
  }
  ds_sort_and_merge_mode(c, out, ref);
}
static void ds_merge(Ctx *c, DSet *dss, size_t k, DSet *out) { ds_merge_mode(c, dss, k, out, 0); }

/* ------------------------------------------------------------------------------------------------ */
/* mergeUpdatesV2 (13.5.16 ds@39007)                                                                */
/* ------------------------------------------------------------------------------------------------ */
/* reader comparator (dec1, dec2) */
static int reader_cmp(Ctx *c, const LReader *a, const LReader *b) {
  const Struct *x = a->curr, *y = b->curr;
  if (x->client == y->client) {
    int64_t d = x->clock - y->clock;
    if (d == 0) {
      int cx = x->kind, cy = y->kind;
      if (cx == cy) return 0;
      if (cx != K_SKIP && cy != K_SKIP) c->inconsistent_cmp = 1;
      return cx == K_SKIP ? 1 : -1;
    }
    return d < 0 ? -1 : 1;
  }
  return y->client - x->client < 0 ? -1 : 1;
}

/* V8's Array.prototype.sort (TimSort, third_party/v8/builtins/array-sort.tq of the reference's Node):
 * runs found by CountAndMakeRun and extended to minrun by BinaryInsertionSort, a pending-run stack
 * collapsed by MergeCollapse, merges by MergeLow / MergeHigh with galloping (minGallop starts at 7).
 * Restated operation by operation because the reader comparator is inconsistent for a GC / Item tie
 * (compare(a, b) = compare(b, a) = -1): the order then depends on exactly which pairs are compared. */
typedef struct {
  Ctx *c;
  LReader **a, **tmp;
  size_t base[80], len[80];
  int nruns;
  long min_gallop;
} TS;
#define TS_CMP(x, y) reader_cmp(ts->c, (x), (y))
static long ts_gallop_left(TS *ts, LReader **arr, LReader *key, long base, long length, long hint) {
  long last = 0, ofs = 1;
  if (TS_CMP(arr[base + hint], key) < 0) {
    long maxo = length - hint;
    while (ofs < maxo) {
      if (TS_CMP(arr[base + hint + ofs], key) >= 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    last += hint;
    ofs += hint;
  } else {
    long maxo = hint + 1;
    while (ofs < maxo) {
      if (TS_CMP(arr[base + hint - ofs], key) < 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    long t = last;
    last = hint - ofs;
    ofs = hint - t;
  }
  last++;
  while (last < ofs) {
    long m = last + ((ofs - last) >> 1);
    if (TS_CMP(arr[base + m], key) < 0) last = m + 1; else ofs = m;
  }
  return ofs;
}
static long ts_gallop_right(TS *ts, LReader **arr, LReader *key, long base, long length, long hint) {
  long last = 0, ofs = 1;
  if (TS_CMP(key, arr[base + hint]) < 0) {
    long maxo = hint + 1;
    while (ofs < maxo) {
      if (TS_CMP(key, arr[base + hint - ofs]) >= 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    long t = last;
    last = hint - ofs;
    ofs = hint - t;
  } else {
    long maxo = length - hint;
    while (ofs < maxo) {
      if (TS_CMP(key, arr[base + hint + ofs]) < 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    last += hint;
    ofs += hint;
  }
  last++;
  while (last < ofs) {
    long m = last + ((ofs - last) >> 1);
    if (TS_CMP(key, arr[base + m]) < 0) ofs = m; else last = m + 1;
  }
  return ofs;
}
static void ts_merge_low(TS *ts, long baseA, long lenA, long baseB, long lenB) {
  LReader **a = ts->a, **t = ts->tmp;
  memcpy(t, a + baseA, lenA * sizeof(LReader *));
  long dest = baseA, ct = 0, cb = baseB;
  a[dest++] = a[cb++];
  if (--lenB == 0) goto succeed;
  if (lenA == 1) goto copy_b;
  for (;;) {
    long wa = 0, wb = 0;
    for (;;) {
      if (TS_CMP(a[cb], t[ct]) < 0) {
        a[dest++] = a[cb++]; wb++; lenB--; wa = 0;
        if (lenB == 0) goto succeed;
        if (wb >= ts->min_gallop) break;
      } else {
        a[dest++] = t[ct++]; wa++; lenA--; wb = 0;
        if (lenA == 1) goto copy_b;
        if (wa >= ts->min_gallop) break;
      }
    }
    ts->min_gallop++;
    int first = 1;
    while (wa >= 7 || wb >= 7 || first) {
      first = 0;
      ts->min_gallop = ts->min_gallop - 1 > 1 ? ts->min_gallop - 1 : 1;
      wa = ts_gallop_right(ts, t, a[cb], ct, lenA, 0);
      if (wa > 0) {
        memcpy(a + dest, t + ct, wa * sizeof(LReader *));
        dest += wa; ct += wa; lenA -= wa;
        if (lenA == 1) goto copy_b;
        if (lenA == 0) goto succeed;
      }
      a[dest++] = a[cb++];
      if (--lenB == 0) goto succeed;
      wb = ts_gallop_left(ts, a, t[ct], cb, lenB, 0);
      if (wb > 0) {
        memmove(a + dest, a + cb, wb * sizeof(LReader *));
        dest += wb; cb += wb; lenB -= wb;
        if (lenB == 0) goto succeed;
      }
      a[dest++] = t[ct++];
      if (--lenA == 1) goto copy_b;
    }
    ts->min_gallop++;
  }
succeed:
  if (lenA > 0) memcpy(a + dest, t + ct, lenA * sizeof(LReader *));
  return;
copy_b:
  memmove(a + dest, a + cb, lenB * sizeof(LReader *));
  a[dest + lenB] = t[ct];
}
static void ts_merge_high(TS *ts, long baseA, long lenA, long baseB, long lenB) {
  LReader **a = ts->a, **t = ts->tmp;
  memcpy(t, a + baseB, lenB * sizeof(LReader *));
  long dest = baseB + lenB - 1, ct = lenB - 1, ca = baseA + lenA - 1;
  a[dest--] = a[ca--];
  if (--lenA == 0) goto succeed;
  if (lenB == 1) goto copy_a;
  for (;;) {
    long wa = 0, wb = 0;
    for (;;) {
      if (TS_CMP(t[ct], a[ca]) < 0) {
        a[dest--] = a[ca--]; wa++; lenA--; wb = 0;
        if (lenA == 0) goto succeed;
        if (wa >= ts->min_gallop) break;
      } else {
        a[dest--] = t[ct--]; wb++; lenB--; wa = 0;
        if (lenB == 1) goto copy_a;
        if (wb >= ts->min_gallop) break;
      }
    }
    ts->min_gallop++;
    int first = 1;
    while (wa >= 7 || wb >= 7 || first) {
      first = 0;
      ts->min_gallop = ts->min_gallop - 1 > 1 ? ts->min_gallop - 1 : 1;
      long k = ts_gallop_right(ts, a, t[ct], baseA, lenA, lenA - 1);
      wa = lenA - k;
      if (wa > 0) {
        dest -= wa; ca -= wa;
        memmove(a + dest + 1, a + ca + 1, wa * sizeof(LReader *));
        lenA -= wa;
        if (lenA == 0) goto succeed;
      }
      a[dest--] = t[ct--];
      if (--lenB == 1) goto copy_a;
      k = ts_gallop_left(ts, t, a[ca], 0, lenB, lenB - 1);
      wb = lenB - k;
      if (wb > 0) {
        dest -= wb; ct -= wb;
        memcpy(a + dest + 1, t + ct + 1, wb * sizeof(LReader *));
        lenB -= wb;
        if (lenB == 1) goto copy_a;
        if (lenB == 0) goto succeed;
      }
      a[dest--] = a[ca--];
      if (--lenA == 0) goto succeed;
    }
    ts->min_gallop++;
  }
succeed:
  if (lenB > 0) memcpy(a + dest - (lenB - 1), t, lenB * sizeof(LReader *));
  return;
copy_a:
  dest -= lenA; ca -= lenA;
  memmove(a + dest + 1, a + ca + 1, lenA * sizeof(LReader *));
  a[dest] = t[ct];
}
static void ts_merge_at(TS *ts, int i) {
  long baseA = (long)ts->base[i], lenA = (long)ts->len[i], baseB = (long)ts->base[i + 1], lenB = (long)ts->len[i + 1];
  ts->len[i] = lenA + lenB;
  if (i == ts->nruns - 3) { ts->base[i + 1] = ts->base[i + 2]; ts->len[i + 1] = ts->len[i + 2]; }
  ts->nruns--;
  long k = ts_gallop_right(ts, ts->a, ts->a[baseB], baseA, lenA, 0);
  baseA += k;
  lenA -= k;
  if (lenA == 0) return;
  lenB = ts_gallop_left(ts, ts->a, ts->a[baseA + lenA - 1], baseB, lenB, lenB - 1);
  if (lenB == 0) return;
  if (lenA <= lenB) ts_merge_low(ts, baseA, lenA, baseB, lenB);
  else ts_merge_high(ts, baseA, lenA, baseB, lenB);
}
static int ts_inv(TS *ts, int n) { return n < 2 || ts->len[n - 2] > ts->len[n - 1] + ts->len[n]; }
static void v8_sort(Ctx *c, LReader **a, size_t n, LReader **tmp) {
  if (n < 2) return;
  TS ts_;
  TS *ts = &ts_;
  ts->c = c; ts->a = a; ts->tmp = tmp; ts->nruns = 0; ts->min_gallop = 7;
  long remaining = (long)n, low = 0;
  long minrun = remaining, r = 0;
  while (minrun >= 64) { r |= minrun & 1; minrun >>= 1; }
  minrun += r;
  while (remaining != 0) {
    /* CountAndMakeRun(low, low + remaining) */
    long run;
    if (remaining == 1) run = 1;
    else {
      run = 2;
      int desc = TS_CMP(a[low + 1], a[low]) < 0;
      LReader *prev = a[low + 1];
      for (long i = low + 2; i < low + remaining; i++) {
        int o = TS_CMP(a[i], prev);
        if (desc ? o >= 0 : o < 0) break;
        prev = a[i];
        run++;
      }
      if (desc) for (long i = low, j = low + run - 1; i < j; i++, j--) { LReader *x = a[i]; a[i] = a[j]; a[j] = x; }
    }
    if (run < minrun) {
      long forced = minrun < remaining ? minrun : remaining;
      /* BinaryInsertionSort(low, low + run, low + forced) */
      for (long start = low + run; start < low + forced; start++) {
        LReader *pivot = a[start];
        long left = low, right = start;
        while (left < right) {
          long mid = left + ((right - left) >> 1);
          if (TS_CMP(pivot, a[mid]) < 0) right = mid; else left = mid + 1;
        }
        for (long p = start; p > left; p--) a[p] = a[p - 1];
        a[left] = pivot;
      }
      run = forced;
    }
    ts->base[ts->nruns] = (size_t)low;
    ts->len[ts->nruns] = (size_t)run;
    ts->nruns++;
    /* MergeCollapse */
    while (ts->nruns > 1) {
      int m = ts->nruns - 2;
      if (!ts_inv(ts, m + 1) || !ts_inv(ts, m)) {
        if (ts->len[m - 1] < ts->len[m + 1]) m--;
        ts_merge_at(ts, m);
      } else if (ts->len[m] <= ts->len[m + 1]) {
        ts_merge_at(ts, m);
      } else break;
    }
    low += run;
    remaining -= run;
  }
  while (ts->nruns > 1) { /* MergeForceCollapse */
    int m = ts->nruns - 2;
    if (m > 0 && ts->len[m - 1] < ts->len[m + 1]) m--;
    ts_merge_at(ts, m);
  }
}

static int struct_merge_with(Struct *cur, const Struct *s) { /* GC/Skip.mergeWith; Item never merges */
  if (cur->kind == K_ITEM) return 0;
  if (cur->kind != s->kind) return 0;
  cur->len += s->len;
  return 1;
}

static Buf *merge_impl(Ctx *c, const uint8_t *const *upds, const size_t *lens, size_t n, int v2) {
  UDec *decs = (UDec *)aalloc(c, (n + 1) * sizeof(UDec));
  for (size_t i = 0; i < n; i++) udec_init(c, &decs[i], upds[i], lens[i], v2);
  LReader *rs = (LReader *)aalloc(c, (n + 1) * sizeof(LReader));
  for (size_t i = 0; i < n; i++) lr_init(c, &rs[i], &decs[i], 1);
  LReader **arr = (LReader **)aalloc(c, (n + 1) * sizeof(LReader *));
  LReader **tmp = (LReader **)aalloc(c, (n + 1) * sizeof(LReader *));
  size_t na = n;
  for (size_t i = 0; i < n; i++) arr[i] = &rs[i];
  UEnc enc;
  uenc_init(c, &enc, v2);
  LWriter w;
  memset(&w, 0, sizeof(w));
  w.enc = &enc;
  Struct *cur = NULL;
  for (;;) {
    size_t k = 0;
    for (size_t i = 0; i < na; i++) if (arr[i]->curr) arr[k++] = arr[i];
    na = k;
    v8_sort(c, arr, na, tmp);
    if (na == 0) break;
    LReader *R = arr[0];
    int64_t first_client = R->curr->client;
    if (cur) {
      Struct *s = R->curr;
      int iterated = 0;
      while (s && s->clock + s->len <= cur->clock + cur->len && s->client >= cur->client) {
        s = lr_next(c, R);
        iterated = 1;
      }
      if (!s || s->client != first_client || (iterated && s->clock > cur->clock + cur->len)) continue;
      if (first_client != cur->client) {
        lw_write(c, &w, cur, 0);
        cur = s;
        lr_next(c, R);
      } else if (cur->clock + cur->len < s->clock) {
        if (cur->kind == K_SKIP) {
          cur->len = s->clock + s->len - cur->clock;
        } else {
          lw_write(c, &w, cur, 0);
          int64_t diff = s->clock - cur->clock - cur->len;
          Struct *sk = (Struct *)aalloc(c, sizeof(Struct));
          memset(sk, 0, sizeof(*sk));
          sk->kind = K_SKIP; sk->client = first_client; sk->clock = cur->clock + cur->len; sk->len = diff;
          cur = sk;
        }
      } else {
        int64_t d = cur->clock + cur->len - s->clock;
        if (d > 0) {
          if (cur->kind == K_SKIP) cur->len -= d;
          else s = slice_struct(c, s, d);
        }
        if (!struct_merge_with(cur, s)) {
          lw_write(c, &w, cur, 0);
          cur = s;
          lr_next(c, R);
        }
      }
    } else {
      cur = R->curr;
      lr_next(c, R);
    }
    for (Struct *nx = R->curr; nx && nx->client == first_client && nx->clock == cur->clock + cur->len && nx->kind != K_SKIP;
         nx = lr_next(c, R)) {
      lw_write(c, &w, cur, 0);
      cur = nx;
    }
  }
  if (cur) lw_write(c, &w, cur, 0);
  lw_finish(c, &w);
  DSet *dss = (DSet *)aalloc(c, (n + 1) * sizeof(DSet));
  for (size_t i = 0; i < n; i++) ds_read(c, &decs[i], &dss[i]);
  DSet merged;
  ds_merge(c, dss, n, &merged);
  ds_write(c, &enc, &merged);
  return uenc_finish(c, &enc);
}

/* decodeStateVector (encoding.js:536-565; 13.5.16 Fe/Ve) */
typedef struct { int64_t client, clock; } SVE;
typedef struct { SVE *e; size_t n; } SV;
static void sv_decode(Ctx *c, const uint8_t *p, size_t n, SV *sv) {
  Dec d = {p, n, 0};
  uint32_t cnt = rd_vu(c, &d);
  sv->e = (SVE *)aalloc(c, ((size_t)(cnt < 1u << 20 ? cnt : 1u << 20) + 1) * sizeof(SVE));
  sv->n = 0;
  size_t cap = (cnt < 1u << 20 ? cnt : 1u << 20) + 1;
  for (uint32_t i = 0; i < cnt; i++) {
    int64_t client = rd_vu(c, &d);
    int64_t clock = rd_vu(c, &d);
    size_t j;
    for (j = 0; j < sv->n; j++) if (sv->e[j].client == client) break;
    if (j == sv->n) {
      if (sv->n == cap) {
        SVE *ne = (SVE *)aalloc(c, cap * 2 * sizeof(SVE));
        memcpy(ne, sv->e, sv->n * sizeof(SVE));
        sv->e = ne; cap *= 2;
      }
      sv->e[sv->n].client = client; sv->n++;
    }
    sv->e[j].clock = clock;
  }
}
static int64_t sv_get(const SV *sv, int64_t client) {
  for (size_t j = 0; j < sv->n; j++) if (sv->e[j].client == client) return sv->e[j].clock;
  return 0;
}

/* diffUpdateV2 (13.5.16 us@40707) */
static Buf *diff_impl(Ctx *c, const uint8_t *upd, size_t len, const uint8_t *svb, size_t svlen, int v2) {
  SV sv;
  sv_decode(c, svb, svlen, &sv);
  UEnc enc;
  uenc_init(c, &enc, v2);
  LWriter w;
  memset(&w, 0, sizeof(w));
  w.enc = &enc;
  UDec dec;
  udec_init(c, &dec, upd, len, v2);
  LReader r;
  lr_init(c, &r, &dec, 0);
  while (r.curr) {
    Struct *t = r.curr;
    int64_t client = t->client;
    int64_t k = sv_get(&sv, client);
    if (t->kind == K_SKIP) { lr_next(c, &r); continue; }
    if (t->clock + t->len > k) {
      int64_t off = k - t->clock;
      if (off < 0) off = 0;
      lw_write(c, &w, t, off);
      lr_next(c, &r);
      while (r.curr && r.curr->client == client) { lw_write(c, &w, r.curr, 0); lr_next(c, &r); }
    } else {
      while (r.curr && r.curr->client == client && r.curr->clock + r.curr->len <= k) lr_next(c, &r);
    }
  }
  lw_finish(c, &w);
  DSet ds;
  ds_read(c, &dec, &ds);
  ds_write(c, &enc, &ds);
  return uenc_finish(c, &enc);
}

/* convertUpdateFormat (13.5.16 ms@41803; convertUpdateFormatV2ToV1 = ks@42002 = ms(u, UpdateDecoderV2,
   UpdateEncoderV1), V1ToV2 = ms(u, UpdateDecoderV1, UpdateEncoderV2)): a LazyStructReader that keeps
   Skips, every struct written with offset 0 through a LazyStructWriter of the other format, then
   readDeleteSet + writeDeleteSet. */
static Buf *conv_impl(Ctx *c, const uint8_t *upd, size_t len, int v2_in) {
  UEnc enc;
  uenc_init(c, &enc, !v2_in);
  LWriter w;
  memset(&w, 0, sizeof(w));
  w.enc = &enc;
  UDec dec;
  udec_init(c, &dec, upd, len, v2_in);
  LReader r;
  lr_init(c, &r, &dec, 0);
  for (; r.curr; lr_next(c, &r)) lw_write(c, &w, r.curr, 0);
  lw_finish(c, &w);
  DSet ds;
  ds_read(c, &dec, &ds);
  ds_write(c, &enc, &ds);
  return uenc_finish(c, &enc);
}

/* encodeStateVectorFromUpdateV2 (13.5.16 os@37724) */
static Buf *sv_impl(Ctx *c, const uint8_t *upd, size_t len, int v2) {
  Buf *rest = buf_new(c);
  UDec dec;
  udec_init(c, &dec, upd, len, v2);
  LReader r;
  lr_init(c, &r, &dec, 0);
  Struct *i = r.curr;
  Buf *out = buf_new(c);
  if (i) {
    int64_t cnt = 0;
    int64_t client = i->client;
    int stop = i->clock != 0;
    int64_t clock = stop ? 0 : i->clock + i->len;
    for (; i; i = lr_next(c, &r)) {
      if (client != i->client) {
        if (clock != 0) { cnt++; wr_vu(c, rest, client); wr_vu(c, rest, clock); }
        client = i->client;
        clock = 0;
        stop = i->clock != 0;
      }
      if (i->kind == K_SKIP) stop = 1;
      if (!stop) clock = i->clock + i->len;
    }
    if (clock != 0) { cnt++; wr_vu(c, rest, client); wr_vu(c, rest, clock); }
    wr_vu(c, out, cnt);
    putraw(c, out, rest->p, rest->n);
  } else {
    wr_vu(c, out, 0);
  }
  return out;
}

/* parseUpdateMetaV2 (13.5.16 parseUpdateMeta / parseUpdateMetaV2): a LazyStructReader that keeps Skips;
   `from` gets a client's first clock when its section starts, `to` the end (clock + length) of its last
   struct when the next section starts.  Both are JS Maps: a client met again keeps its first position and
   takes the new value.  Output (the engine's encoding of the two Maps): from then to, each as an encoded
   state vector, vu(count) | (client, clock)*, in Map order. */
static void meta_set(Ctx *c, int64_t **kv, size_t *n, size_t *cap, int64_t client, int64_t clock) {
  for (size_t i = 0; i < *n; i++) if ((*kv)[2 * i] == client) { (*kv)[2 * i + 1] = clock; return; }
  if (*n == *cap) {
    size_t nc = *cap ? *cap * 2 : 16;
    int64_t *p = (int64_t *)aalloc(c, nc * 2 * sizeof(int64_t));
    if (*n) memcpy(p, *kv, *n * 2 * sizeof(int64_t));
    *kv = p; *cap = nc;
  }
  (*kv)[2 * *n] = client; (*kv)[2 * *n + 1] = clock; (*n)++;
}
static Buf *meta_impl(Ctx *c, const uint8_t *upd, size_t len, int v2) {
  UDec dec;
  udec_init(c, &dec, upd, len, v2);
  LReader r;
  lr_init(c, &r, &dec, 0);
  int64_t *from = NULL, *to = NULL;
  size_t nf = 0, cf = 0, nt = 0, ct = 0;
  Struct *i = r.curr;
  if (i) {
    int64_t client = i->client, clock = i->clock;
    meta_set(c, &from, &nf, &cf, client, clock);
    for (; i; i = lr_next(c, &r)) {
      if (client != i->client) {
        meta_set(c, &to, &nt, &ct, client, clock);
        meta_set(c, &from, &nf, &cf, i->client, i->clock);
        client = i->client;
      }
      clock = i->clock + i->len;
    }
    meta_set(c, &to, &nt, &ct, client, clock);
  }
  Buf *out = buf_new(c);
  wr_vu(c, out, (int64_t)nf);
  for (size_t k = 0; k < nf; k++) { wr_vu(c, out, from[2 * k]); wr_vu(c, out, from[2 * k + 1]); }
  wr_vu(c, out, (int64_t)nt);
  for (size_t k = 0; k < nt; k++) { wr_vu(c, out, to[2 * k]); wr_vu(c, out, to[2 * k + 1]); }
  return out;
}

/* PermanentUserData's delete-set merge (PermanentUserData.js:49-54): every encoded delete set is read
   with readDeleteSet (DeleteSet.js:241-256; DSDecoderV1, or DSDecoderV2 for fmt 2), the k sets are
   merged by mergeDeleteSets (13.5.16 he@10482 + le@10242 union) and written by writeDeleteSet
   (DSEncoderV1 / DSEncoderV2 rest bytes, as encodeSnapshot[V2] writes them, Snapshot.js:84-101). */
static Buf *dsmerge_impl(Ctx *c, const uint8_t *const *dss_in, const size_t *lens, size_t k, int v2, int ref) {
  DSet *dss = (DSet *)aalloc(c, (k ? k : 1) * sizeof(DSet));
  for (size_t i = 0; i < k; i++) {
    UDec dec;
    udec_init(c, &dec, dss_in[i], lens[i], 0);
    dec.v2 = v2;
    ds_read(c, &dec, &dss[i]);
  }
  DSet m;
  ds_merge_mode(c, dss, k, &m, ref);
  UEnc enc;
  uenc_init(c, &enc, 0);
  enc.v2 = v2;
  ds_write(c, &enc, &m);
  return enc.rest;
}

/* Snapshot codec (gaberogan/yjs@v0 src/utils/Snapshot.js:84-124; 13.5.16 _n / En): the snapshot that
   decodeSnapshot[V2] reads -- readDeleteSet (DeleteSet.js:241-256) then readStateVector (encoding.js:
   536-545, a Map: a repeated client keeps its first position and takes the last clock) -- written back by
   encodeSnapshot[V2]: writeDeleteSet (DeleteSet.js:219-232) then writeStateVector (encoding.js:572-579). */
static Buf *snap_impl(Ctx *c, const uint8_t *p, size_t n, int v2in, int v2out) {
  UDec dec;
  udec_init(c, &dec, p, n, 0);
  dec.v2 = v2in;
  DSet ds;
  ds_read(c, &dec, &ds);
  uint32_t m = rd_vu(c, &dec.rest);
  size_t nsv = 0, cap = 0;
  int64_t *sv = NULL; /* (client, clock) pairs in Map order */
  for (uint32_t i = 0; i < m; i++) {
    int64_t client = rd_vu(c, &dec.rest);
    int64_t clock = rd_vu(c, &dec.rest);
    size_t k = 0;
    while (k < nsv && sv[2 * k] != client) k++;
    if (k == nsv) {
      if (nsv == cap) {
        cap = cap ? 2 * cap : 16;
        int64_t *ns = (int64_t *)aalloc(c, cap * 2 * sizeof(int64_t));
        if (nsv) memcpy(ns, sv, nsv * 2 * sizeof(int64_t));
        sv = ns;
      }
      sv[2 * nsv] = client;
      nsv++;
    }
    sv[2 * k + 1] = clock;
  }
  UEnc enc;
  uenc_init(c, &enc, 0);
  enc.v2 = v2out;
  ds_write(c, &enc, &ds);
  wr_vu(c, enc.rest, (int64_t)nsv);
  for (size_t k = 0; k < nsv; k++) { wr_vu(c, enc.rest, sv[2 * k]); wr_vu(c, enc.rest, sv[2 * k + 1]); }
  return enc.rest;
}

/* ------------------------------------------------------------------------------------------------ */
/* Doc round-trip compaction: gaberogan/yjs@v0 (yjs 13.4.9) itself --        */
/* new Doc() (gc: true, Doc.js:40), applyUpdate[V2] of every input in order (one transaction each,   */
/* encoding.js:462-473 readUpdateV2), encodeStateAsUpdate[V2] (encoding.js:490-526).                 */
/*   readStructs            encoding.js:415-436 (readClientsStructRefs :127-198,                     */
/*                          mergeReadStructsIntoPendingReads :354-372, resumeStructIntegration        */
/*                          :225-321, cleanupPendingStructs :377-388, tryResumePendingDeleteReaders)  */
/*   Item.getMissing / integrate / delete / gc / mergeWith   Item.js:355-517, 545-616                 */
/*   splitItem Item.js:85-125, getItemCleanStart / End StructStore.js:190-231, replaceStruct :241-244  */
/*   readAndApplyDeleteSet  DeleteSet.js:270-323, sortAndMergeDeleteSet :113-135                      */
/*   cleanupTransactions    Transaction.js:244-367 (tryGcDeleteSet :182-204, tryMergeDeleteSet        */
/*                          :210-227, tryToMergeWithLeft :165-176)                                    */
/*   ContentType.delete / gc ContentType.js:101-141; ContentString.splice ContentString.js:51-66      */
/*   writeClientsStructs / writeStructs encoding.js:71-116; createDeleteSetFromStructStore            */
/*                          DeleteSet.js:185-210; writeDeleteSet :219-232                              */
/* ------------------------------------------------------------------------------------------------ */
typedef struct CType CType;
typedef struct CIt {
  int gc;                       /* a GC struct */
  int64_t client, clock, len;
  int has_origin, has_right;
  JID origin, right;            /* origin / rightOrigin */
  struct CIt *left, *rightp;    /* left / right */
  CType *parent;                /* resolved parent type (NULL: none) */
  int pkind; Str pkey; JID pid; /* parent as read: 0 none (copied from a neighbour), 1 ykey, 2 ID */
  int has_psub; Str psub;
  int deleted;
  Content *ct;
  CType *type;                  /* ContentType: its type */
  uint32_t gen_before, gen_conf; /* Item.integrate's itemsBeforeOrigin / conflictingItems sets */
} CIt;
struct CType {
  CIt *start, *item;            /* _start, _item */
  int tref;                     /* typeRef of the ContentType (2 YText, 6 YXmlText ...); -1: a root (AbstractType) */
  Str key;                      /* a root type's key (doc.share) */
  Str *mk; CIt **mv; size_t mn, mcap; /* _map in insertion order */
};
typedef struct { int64_t client; CIt **a; size_t n, cap; } CCl;
typedef struct { int64_t client; CIt **refs; size_t n, i; int live; } CPend;
typedef struct {
  Ctx *c;
  CCl *cl; size_t ncl, capcl;        /* store.clients, Map insertion order */
  CPend *pend; size_t npend, cappend; /* store.pendingClientsStructRefs */
  CIt **stack; size_t nstack, capstack; /* store.pendingStack */
  DSet *pdel; size_t npdel, cappdel; /* store.pendingDeleteReaders */
  CType **roots; size_t nroots, caproots; /* doc.share */
  uint32_t gen;
  struct CTx *tx;                    /* doc._transaction */
  int64_t *hk; size_t *hv; size_t hcap; /* client -> index into cl (open addressing) */
} CDoc;
typedef struct CTx {                 /* Transaction (Transaction.js:57-140) */
  DSet ds;                           /* deleteSet */
  CIt **ms; size_t nms, capms;       /* _mergeStructs */
  int64_t *bc_client, *bc_clock; size_t nbc; /* beforeState */
  CType **chg; size_t nchg, capchg;  /* changed (Map insertion order; the parentSub sets are not needed) */
  int local;
} CTx;

#define CGROW(c, arr, n, cap, T)                                                   \
  do {                                                                             \
    if ((n) == (cap)) {                                                            \
      size_t nc_ = (cap) ? (cap) * 2 : 8;                                          \
      T *na_ = (T *)aalloc((c), nc_ * sizeof(T));                                  \
      if (n) memcpy(na_, (arr), (n) * sizeof(T));                                  \
      (arr) = na_; (cap) = nc_;                                                    \
    }                                                                              \
  } while (0)

static size_t cd_hslot(const CDoc *d, int64_t client) {
  size_t h = (size_t)((uint64_t)client * 0x9E3779B97F4A7C15ull >> 20) & (d->hcap - 1);
  while (d->hv[h] != 0 && d->hk[h] != client) h = (h + 1) & (d->hcap - 1);
  return h;
}
static CCl *cd_client(CDoc *d, int64_t client) {
  if (d->hcap == 0) return NULL;
  size_t h = cd_hslot(d, client);
  return d->hv[h] ? &d->cl[d->hv[h] - 1] : NULL;
}
static void cd_hput(CDoc *d, int64_t client, size_t idx) {
  if (2 * (d->ncl + 1) > d->hcap) {
    size_t nc = d->hcap ? d->hcap * 2 : 64;
    int64_t *ok = d->hk;
    size_t *ov = d->hv, oc = d->hcap;
    d->hk = (int64_t *)aalloc(d->c, nc * sizeof(int64_t));
    d->hv = (size_t *)aalloc(d->c, nc * sizeof(size_t));
    memset(d->hv, 0, nc * sizeof(size_t));
    d->hcap = nc;
    for (size_t i = 0; i < oc; i++)
      if (ov[i]) { size_t h = cd_hslot(d, ok[i]); d->hk[h] = ok[i]; d->hv[h] = ov[i]; }
  }
  size_t h = cd_hslot(d, client);
  d->hk[h] = client;
  d->hv[h] = idx + 1;
}
static int64_t cl_state(const CCl *s) {
  if (!s || s->n == 0) return 0;
  CIt *l = s->a[s->n - 1];
  return l->clock + l->len;
}
static int64_t cd_state(CDoc *d, int64_t client) { return cl_state(cd_client(d, client)); } /* getState */
static size_t cd_find_index(CDoc *d, CCl *s, int64_t clock) { /* findIndexSS (StructStore.js:123-151) */
  if (!s || s->n == 0) fail(d->c, YMO_ERR_UNEXPECTED);
  size_t lo = 0, hi = s->n;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    CIt *m = s->a[mid];
    if (m->clock <= clock) {
      if (clock < m->clock + m->len) return mid;
      lo = mid + 1;
    } else hi = mid;
  }
  fail(d->c, YMO_ERR_UNEXPECTED);
}
static CIt *cd_get(CDoc *d, JID id) { CCl *s = cd_client(d, id.client); return s->a[cd_find_index(d, s, id.clock)]; }
static void cl_insert(CDoc *d, CCl *s, size_t at, CIt *it) {
  CGROW(d->c, s->a, s->n, s->cap, CIt *);
  memmove(s->a + at + 1, s->a + at, (s->n - at) * sizeof(CIt *));
  s->a[at] = it;
  s->n++;
}
static void cl_remove(CCl *s, size_t at) { memmove(s->a + at, s->a + at + 1, (s->n - at - 1) * sizeof(CIt *)); s->n--; }
static void cd_add_struct(CDoc *d, CIt *it) { /* addStruct (StructStore.js:92-104) */
  CCl *s = cd_client(d, it->client);
  if (!s) {
    cd_hput(d, it->client, d->ncl);
    CGROW(d->c, d->cl, d->ncl, d->capcl, CCl);
    s = &d->cl[d->ncl++];
    memset(s, 0, sizeof(*s));
    s->client = it->client;
  } else {
    CIt *l = s->a[s->n - 1];
    if (l->clock + l->len != it->clock) fail(d->c, YMO_ERR_UNEXPECTED);
  }
  CGROW(d->c, s->a, s->n, s->cap, CIt *);
  s->a[s->n++] = it;
}
static CType *ct_new(CDoc *d) { CType *t = (CType *)aalloc(d->c, sizeof(CType)); memset(t, 0, sizeof(*t)); t->tref = -1; return t; }
/* beforeState.get(client) || 0: beforeState holds the store's clients in order, so the index of a client in
   the store is its index there */
static int64_t tx_before_at(const CTx *t, size_t idx) { return idx < t->nbc ? t->bc_clock[idx] : 0; }
static int64_t tx_before(CDoc *d, const CTx *t, int64_t client) {
  CCl *s = cd_client(d, client);
  return s ? tx_before_at(t, (size_t)(s - d->cl)) : 0;
}
static void changed_add(CDoc *d, CType *t) { /* addChangedTypeToTransaction (Transaction.js:154-159) */
  CTx *x = d->tx;
  if (t->item && !(t->item->clock < tx_before(d, x, t->item->client) && !t->item->deleted)) return;
  for (size_t i = 0; i < x->nchg; i++) if (x->chg[i] == t) return;
  CGROW(d->c, x->chg, x->nchg, x->capchg, CType *);
  x->chg[x->nchg++] = t;
}
static void changed_del(CDoc *d, CType *t) {
  CTx *x = d->tx;
  for (size_t i = 0; i < x->nchg; i++)
    if (x->chg[i] == t) { memmove(x->chg + i, x->chg + i + 1, (x->nchg - i - 1) * sizeof(CType *)); x->nchg--; return; }
}
static CType *cd_root(CDoc *d, Str key) { /* doc.get(key): the root type, created on first use */
  for (size_t i = 0; i < d->nroots; i++) if (str_eq(d->roots[i]->key, key)) return d->roots[i];
  CType *t = ct_new(d);
  t->key = key;
  CGROW(d->c, d->roots, d->nroots, d->caproots, CType *);
  d->roots[d->nroots++] = t;
  return t;
}
static CIt *map_get(CType *t, Str k) {
  for (size_t i = 0; i < t->mn; i++) if (str_eq(t->mk[i], k)) return t->mv[i];
  return NULL;
}
static void map_set(CDoc *d, CType *t, Str k, CIt *v) {
  for (size_t i = 0; i < t->mn; i++) if (str_eq(t->mk[i], k)) { t->mv[i] = v; return; }
  if (t->mn == t->mcap) {
    size_t nc = t->mcap ? t->mcap * 2 : 4;
    Str *nk = (Str *)aalloc(d->c, nc * sizeof(Str));
    CIt **nv = (CIt **)aalloc(d->c, nc * sizeof(CIt *));
    if (t->mn) { memcpy(nk, t->mk, t->mn * sizeof(Str)); memcpy(nv, t->mv, t->mn * sizeof(CIt *)); }
    t->mk = nk; t->mv = nv; t->mcap = nc;
  }
  t->mk[t->mn] = k; t->mv[t->mn] = v; t->mn++;
}
static void tds_add(CDoc *d, DSet *ds, int64_t client, int64_t clock, int64_t len) { /* addToDeleteSet */
  dc_push(d->c, ds_get_or_add(d->c, ds, client), clock, len);
}
static void ms_push(CDoc *d, CIt *it) { CTx *x = d->tx; CGROW(d->c, x->ms, x->nms, x->capms, CIt *); x->ms[x->nms++] = it; }
static JID it_last(const CIt *it) { JID r = {it->client, it->clock + it->len - 1}; return r; }
static int jid_eq(int ha, JID a, int hb, JID b) { return ha == hb && (!ha || (a.client == b.client && a.clock == b.clock)); }

/* the left part of content.splice(off) (ContentString.js:51-66 and the other contents' splice) */
static void content_truncate(Ctx *c, Content *ct, int64_t off) {
  switch (ct->ref) {
    case 1: ct->dlen = off; break;
    case 2: case 8: ct->n = (size_t)off; break;
    case 4: {
      Str l = str_slice(ct->str, 0, off);
      if (off >= 1 && l.n >= (size_t)off && l.u[off - 1] >= 0xD800 && l.u[off - 1] <= 0xDBFF) {
        uint16_t *nu = (uint16_t *)aalloc(c, (size_t)off * 2);
        memcpy(nu, l.u, ((size_t)off - 1) * 2);
        nu[off - 1] = 0xFFFD;
        Str ns = {nu, (size_t)off};
        l = ns;
      }
      ct->str = l;
      break;
    }
    default: fail(c, YMO_ERR_METHOD);
  }
}
static Content *content_copy(Ctx *c, const Content *src) {
  Content *r = (Content *)aalloc(c, sizeof(Content));
  *r = *src;
  return r;
}
static int content_merge(Ctx *c, Content *l, const Content *r) { /* AbstractContent.mergeWith */
  switch (l->ref) {
    case 1: l->dlen += r->dlen; return 1;
    case 4: {
      uint16_t *nu = (uint16_t *)aalloc(c, (l->str.n + r->str.n + 1) * 2);
      if (l->str.n) memcpy(nu, l->str.u, l->str.n * 2);
      if (r->str.n) memcpy(nu + l->str.n, r->str.u, r->str.n * 2);
      Str s = {nu, l->str.n + r->str.n};
      l->str = s;
      return 1;
    }
    case 8: {
      Val **na = (Val **)aalloc(c, (l->n + r->n + 1) * sizeof(Val *));
      if (l->n) memcpy(na, l->anys, l->n * sizeof(Val *));
      if (r->n) memcpy(na + l->n, r->anys, r->n * sizeof(Val *));
      l->anys = na; l->n += r->n;
      return 1;
    }
    case 2: {
      Str *nj = (Str *)aalloc(c, (l->n + r->n + 1) * sizeof(Str));
      uint8_t *nu = (uint8_t *)aalloc(c, l->n + r->n + 1);
      if (l->n) { memcpy(nj, l->jstrs, l->n * sizeof(Str)); memcpy(nu, l->jundef, l->n); }
      if (r->n) { memcpy(nj + l->n, r->jstrs, r->n * sizeof(Str)); memcpy(nu + l->n, r->jundef, r->n); }
      l->jstrs = nj; l->jundef = nu; l->n += r->n;
      return 1;
    }
    default: return 0;
  }
}

static CIt *split_item(CDoc *d, CIt *left, int64_t diff) { /* splitItem (Item.js:85-125) */
  CIt *r = (CIt *)aalloc(d->c, sizeof(CIt));
  *r = *left;
  r->clock = left->clock + diff;
  r->left = left;
  r->has_origin = 1;
  r->origin.client = left->client; r->origin.clock = left->clock + diff - 1;
  r->rightp = left->rightp;
  r->ct = content_splice(d->c, left->ct, diff);
  r->len = left->len - diff;
  r->gen_before = r->gen_conf = 0;
  r->type = NULL;
  Content *lc = content_copy(d->c, left->ct);
  content_truncate(d->c, lc, diff);
  left->ct = lc;
  left->rightp = r;
  if (r->rightp) r->rightp->left = r;
  ms_push(d, r);
  if (r->has_psub && r->rightp == NULL) map_set(d, r->parent, r->psub, r);
  left->len = diff;
  return r;
}
static CIt *get_clean_start(CDoc *d, JID id) { /* getItemCleanStart / findIndexCleanStart */
  CCl *s = cd_client(d, id.client);
  size_t idx = cd_find_index(d, s, id.clock);
  CIt *st = s->a[idx];
  if (st->clock < id.clock && !st->gc) {
    CIt *r = split_item(d, st, id.clock - st->clock);
    cl_insert(d, s, idx + 1, r);
    return r;
  }
  return st;
}
static CIt *get_clean_end(CDoc *d, JID id) { /* getItemCleanEnd */
  CCl *s = cd_client(d, id.client);
  size_t idx = cd_find_index(d, s, id.clock);
  CIt *st = s->a[idx];
  if (id.clock != st->clock + st->len - 1 && !st->gc) cl_insert(d, s, idx + 1, split_item(d, st, id.clock - st->clock + 1));
  return st;
}

static void it_delete(CDoc *d, CIt *it);
static void ctype_delete(CDoc *d, CType *t) { /* ContentType.delete */
  for (CIt *x = t->start; x; x = x->rightp) {
    if (!x->deleted) it_delete(d, x);
    else ms_push(d, x);
  }
  for (size_t i = 0; i < t->mn; i++) {
    CIt *x = t->mv[i];
    if (!x->deleted) it_delete(d, x);
    else ms_push(d, x);
  }
  changed_del(d, t);
}
static void it_delete(CDoc *d, CIt *it) { /* Item.delete */
  if (it->deleted) return;
  it->deleted = 1;
  tds_add(d, &d->tx->ds, it->client, it->clock, it->len);
  changed_add(d, it->parent);
  if (it->ct->ref == 7 && it->type) ctype_delete(d, it->type);
}
static void cd_replace(CDoc *d, CIt *old, CIt *nw) { /* replaceStruct */
  CCl *s = cd_client(d, old->client);
  s->a[cd_find_index(d, s, old->clock)] = nw;
}
static void it_gc(CDoc *d, CIt *it, int parent_gcd) { /* Item.gc */
  if (!it->deleted) fail(d->c, YMO_ERR_UNEXPECTED);
  if (it->ct->ref == 7 && it->type) { /* ContentType.gc */
    CType *t = it->type;
    for (CIt *x = t->start; x; x = x->rightp) it_gc(d, x, 1);
    t->start = NULL;
    for (size_t i = 0; i < t->mn; i++)
      for (CIt *x = t->mv[i]; x; x = x->left) it_gc(d, x, 1);
    t->mn = 0;
  }
  if (parent_gcd) {
    if (it->gc) return;
    CIt *g = (CIt *)aalloc(d->c, sizeof(CIt));
    memset(g, 0, sizeof(*g));
    g->gc = 1; g->client = it->client; g->clock = it->clock; g->len = it->len; g->deleted = 1;
    cd_replace(d, it, g);
  } else {
    Content *cd = (Content *)aalloc(d->c, sizeof(Content));
    memset(cd, 0, sizeof(*cd));
    cd->ref = 1; cd->dlen = it->len;
    it->ct = cd;
  }
}

/* Item.getMissing: the client of a missing dependency, or -1 (and left / right / parent resolved) */
static int64_t it_missing(CDoc *d, CIt *it) {
  if (it->gc) return -1;
  if (it->has_origin && it->origin.client != it->client && it->origin.clock >= cd_state(d, it->origin.client)) return it->origin.client;
  if (it->has_right && it->right.client != it->client && it->right.clock >= cd_state(d, it->right.client)) return it->right.client;
  if (it->pkind == 2 && it->client != it->pid.client && it->pid.clock >= cd_state(d, it->pid.client)) return it->pid.client;
  if (it->has_origin) {
    it->left = get_clean_end(d, it->origin);
    it->origin = it_last(it->left);
  }
  if (it->has_right) {
    it->rightp = get_clean_start(d, it->right);
    it->right.client = it->rightp->client; it->right.clock = it->rightp->clock;
  }
  int par_set = it->pkind != 0;  /* `this.parent` truthy before the neighbour rules */
  if ((it->left && it->left->gc) || (it->rightp && it->rightp->gc)) { par_set = 0; it->parent = NULL; it->pkind = 0; }
  if (!par_set) {
    if (it->left && !it->left->gc) { it->parent = it->left->parent; it->has_psub = it->left->has_psub; it->psub = it->left->psub; }
    if (it->rightp && !it->rightp->gc) { it->parent = it->rightp->parent; it->has_psub = it->rightp->has_psub; it->psub = it->rightp->psub; }
  } else if (it->pkind == 2) {
    CIt *p = cd_get(d, it->pid);
    it->parent = (!p->gc && p->ct->ref == 7) ? p->type : NULL;  /* a GC'd parent, or no type: GC */
  }
  return -1;
}
static void it_integrate(CDoc *d, CIt *it, int64_t off) {
  if (it->gc) { /* GC.integrate */
    if (off > 0) { it->clock += off; it->len -= off; }
    cd_add_struct(d, it);
    return;
  }
  if (off > 0) {
    it->clock += off;
    JID p = {it->client, it->clock - 1};
    it->left = get_clean_end(d, p);
    it->origin = it_last(it->left);
    it->has_origin = 1;
    it->ct = content_splice(d->c, it->ct, off);
    it->len -= off;
  }
  if (!it->parent) { /* parent is not defined: integrate a GC struct instead */
    CIt *g = (CIt *)aalloc(d->c, sizeof(CIt));
    memset(g, 0, sizeof(*g));
    g->gc = 1; g->client = it->client; g->clock = it->clock; g->len = it->len; g->deleted = 1;
    cd_add_struct(d, g);
    return;
  }
  CType *P = it->parent;
  /* 13.4.9 Item.js:413-450: a GC on the left has no `right`, so the conflict scan reads undefined.origin */
  if (it->left && it->left->gc) fail(d->c, YMO_ERR_TYPE);
  if ((!it->left && (!it->rightp || it->rightp->left != NULL)) || (it->left && it->left->rightp != it->rightp)) {
    CIt *left = it->left, *o;
    if (left) o = left->rightp;
    else if (it->has_psub) { o = map_get(P, it->psub); while (o && o->left) o = o->left; }
    else o = P->start;
    const uint32_t gb = ++d->gen;
    uint32_t gcf = ++d->gen;
    while (o && o != it->rightp) {
      o->gen_before = gb;
      o->gen_conf = gcf;
      if (jid_eq(it->has_origin, it->origin, o->has_origin, o->origin)) {
        if (o->client < it->client) { left = o; gcf = ++d->gen; }
        else if (jid_eq(it->has_right, it->right, o->has_right, o->right)) break;
      } else if (o->has_origin) {
        CIt *oo = cd_get(d, o->origin);
        if (oo->gen_before == gb) {
          if (oo->gen_conf != gcf) { left = o; gcf = ++d->gen; }
        } else break;
      } else break;
      o = o->rightp;
    }
    it->left = left;
  }
  if (it->left) {
    CIt *r = it->left->rightp;
    it->rightp = r;
    it->left->rightp = it;
  } else {
    CIt *r;
    if (it->has_psub) { r = map_get(P, it->psub); while (r && r->left) r = r->left; }
    else { r = P->start; P->start = it; }
    it->rightp = r;
  }
  if (it->rightp) it->rightp->left = it;
  else if (it->has_psub) {
    map_set(d, P, it->psub, it);
    if (it->left) it_delete(d, it->left);
  }
  cd_add_struct(d, it);
  if (it->ct->ref == 7) { it->type = ct_new(d); it->type->item = it; it->type->tref = (int)it->ct->typeRef; } /* type._integrate */
  if (it->ct->ref == 1) { /* ContentDeleted.integrate */
    tds_add(d, &d->tx->ds, it->client, it->clock, it->ct->dlen);
    it->deleted = 1;
  }
  changed_add(d, P);
  if ((P->item && P->item->deleted) || (it->has_psub && it->rightp)) it_delete(d, it);
}

static void cd_pend_clear(CDoc *d) { d->npend = 0; }
static CPend *cd_pend(CDoc *d, int64_t client) {
  for (size_t i = 0; i < d->npend; i++) if (d->pend[i].live && d->pend[i].client == client) return &d->pend[i];
  return NULL;
}
static void refs_sort(CIt **a, size_t n) { /* stable sort by clock (V8 TimSort is stable) */
  for (size_t i = 1; i < n; i++) {
    CIt *v = a[i];
    size_t j = i;
    while (j > 0 && a[j - 1]->clock > v->clock) { a[j] = a[j - 1]; j--; }
    a[j] = v;
  }
}
static int cmp_i64(const void *a, const void *b) { int64_t x = *(const int64_t *)a, y = *(const int64_t *)b; return x < y ? -1 : x > y; }
static void resume_integration(CDoc *d) { /* resumeStructIntegration (encoding.js:225-321) */
  Ctx *c = d->c;
  size_t nids = 0;
  int64_t *ids = (int64_t *)aalloc(c, (d->npend + 1) * sizeof(int64_t));
  for (size_t i = 0; i < d->npend; i++) if (d->pend[i].live) ids[nids++] = d->pend[i].client;
  qsort(ids, nids, sizeof(int64_t), cmp_i64); /* Array.from(keys).sort((a, b) => a - b): distinct keys */
  if (nids == 0) return;
  CPend *cur = NULL;
  #define NEXT_TARGET()                                                      \
    do {                                                                     \
      cur = cd_pend(d, ids[nids - 1]);                                       \
      while (cur->n == cur->i) {                                             \
        nids--;                                                              \
        if (nids > 0) cur = cd_pend(d, ids[nids - 1]);                       \
        else { cd_pend_clear(d); cur = NULL; break; }                        \
      }                                                                      \
    } while (0)
  NEXT_TARGET();
  if (cur == NULL && d->nstack == 0) return;
  CIt *head = d->nstack > 0 ? d->stack[--d->nstack] : cur->refs[cur->i++];
  /* the reference's state cache (encoding.js:257-260, 289) always equals getState: a client's state only
     changes when one of its structs integrates, and that updates the cache to the same value */
  while (1) {
    int64_t local = cd_state(d, head->client);
    int64_t off = head->clock < local ? local - head->clock : 0;
    if (head->clock + off != local) {
      CPend *sr = cd_pend(d, head->client);
      if (sr && sr->n != sr->i) {
        CIt *r = sr->refs[sr->i];
        if (r->clock < head->clock) {
          sr->refs[sr->i] = head;
          head = r;
          CIt **rest = sr->refs + sr->i;
          size_t rn = sr->n - sr->i;
          CIt **na = (CIt **)aalloc(c, (rn + 1) * sizeof(CIt *));
          memcpy(na, rest, rn * sizeof(CIt *));
          refs_sort(na, rn);
          sr->refs = na; sr->n = rn; sr->i = 0;
          continue;
        }
      }
      CGROW(c, d->stack, d->nstack, d->capstack, CIt *);
      d->stack[d->nstack++] = head;
      return;
    }
    int64_t missing = it_missing(d, head);
    if (missing < 0) {
      if (off == 0 || off < head->len) {
        it_integrate(d, head, off);
      }
      if (d->nstack > 0) head = d->stack[--d->nstack];
      else if (cur && cur->i < cur->n) head = cur->refs[cur->i++];
      else {
        NEXT_TARGET();
        if (cur == NULL) break;
        head = cur->refs[cur->i++];
      }
    } else {
      CPend *sr = cd_pend(d, missing);
      if (!sr || sr->n == sr->i) {
        CGROW(c, d->stack, d->nstack, d->capstack, CIt *);
        d->stack[d->nstack++] = head;
        return;
      }
      CGROW(c, d->stack, d->nstack, d->capstack, CIt *);
      d->stack[d->nstack++] = head;
      head = sr->refs[sr->i++];
    }
  }
  #undef NEXT_TARGET
  cd_pend_clear(d);
}

static void cd_split_into(CDoc *d, CCl *s, size_t at, CIt *it) { cl_insert(d, s, at, it); }
/* readAndApplyDeleteSet over a decoded delete set (DeleteSet.js:270-323); the unapplied ranges become a
   pending delete reader.  An unapplied range of length 0 (a V1 delete set may hold one) sets *zero: the
   reference's writeDeleteSet of the unapplied set throws at it (DSEncoderV2.writeDsLen, UpdateEncoder.js:
   255-258), after every client of the update's delete set has been read and applied */
static void apply_ds(CDoc *d, const DSet *ds, int kept, int *zero) {
  DSet un;
  memset(&un, 0, sizeof(un));
  if (kept) { /* a pending reader none of whose ranges applies comes back unchanged (it went through the
                 round trip below once already) */
    int any = 0;
    for (size_t ci = 0; ci < ds->n && !any; ci++) {
      int64_t state = cd_state(d, ds->cl[ci].client);
      for (size_t k = 0; k < ds->cl[ci].n && !any; k++) any = ds->cl[ci].items[k].clock < state;
    }
    if (!any) {
      CGROW(d->c, d->pdel, d->npdel, d->cappdel, DSet);
      d->pdel[d->npdel++] = *ds;
      return;
    }
  }
  for (size_t ci = 0; ci < ds->n; ci++) {
    int64_t client = ds->cl[ci].client;
    CCl *s = cd_client(d, client);
    int64_t state = cd_state(d, client);
    for (size_t k = 0; k < ds->cl[ci].n; k++) {
      int64_t clock = ds->cl[ci].items[k].clock, end = clock + ds->cl[ci].items[k].len;
      if (clock < state) {
        if (state < end) tds_add(d, &un, client, state, end - state);
        size_t idx = cd_find_index(d, s, clock);
        CIt *st = s->a[idx];
        if (!st->deleted && st->clock < clock) {
          cd_split_into(d, s, idx + 1, split_item(d, st, clock - st->clock));
          idx++;
        }
        while (idx < s->n) {
          st = s->a[idx++];
          if (st->clock < end) {
            if (!st->deleted) {
              if (end < st->clock + st->len) cd_split_into(d, s, idx, split_item(d, st, end - st->clock));
              it_delete(d, st);
            }
          } else break;
        }
      } else tds_add(d, &un, client, clock, end - clock);
    }
  }
  if (un.n > 0) {
    /* the pending reader is a DSDecoderV2 over writeDeleteSet(DSEncoderV2, unappliedDS) (:317-321): clock
       deltas to the previous range's end and len - 1 through writeVarUint (a negative value: its low 7 bits) */
    for (size_t ci = 0; ci < un.n; ci++) {
      int64_t enc = 0, dec = 0;
      for (size_t k = 0; k < un.cl[ci].n; k++) {
        DItem *r = &un.cl[ci].items[k];
        if (r->len == 0 && zero) *zero = 1;
        int64_t dc = r->clock - enc, dl = r->len - 1;
        enc = r->clock + r->len;
        dec += dc > 127 ? dc : (dc & 127);
        r->clock = dec;
        r->len = (dl > 127 ? dl : (dl & 127)) + 1;
        dec += r->len;
      }
    }
    CGROW(d->c, d->pdel, d->npdel, d->cappdel, DSet);
    d->pdel[d->npdel++] = un;
  }
}
/* readClientsStructRefs (encoding.js:127-198): per section a ref list (a repeated client replaces the
   earlier list: Map.set), GC for info & 31 == 0 */
static void read_refs(CDoc *d, UDec *u, CPend **out, size_t *nout) {
  Ctx *c = d->c;
  uint32_t nsec = rd_vu(c, &u->rest);
  CPend *lst = (CPend *)aalloc(c, (nsec + 1) * sizeof(CPend));
  size_t nl = 0;
  for (uint32_t si = 0; si < nsec; si++) {
    uint32_t ns = rd_vu(c, &u->rest);
    int64_t client = ud_client(c, u);
    int64_t clock = rd_vu(c, &u->rest);
    CIt **refs = (CIt **)aalloc(c, (ns + 1) * sizeof(CIt *));
    for (uint32_t k = 0; k < ns; k++) {
      int info = ud_info(c, u);
      CIt *it = (CIt *)aalloc(c, sizeof(CIt));
      memset(it, 0, sizeof(*it));
      it->client = client; it->clock = clock;
      if ((info & 31) != 0) {
        int cant_copy = (info & 0xC0) == 0;
        if (info & 0x80) { it->has_origin = 1; it->origin = ud_left(c, u); }
        if (info & 0x40) { it->has_right = 1; it->right = ud_right(c, u); }
        if (cant_copy) {
          if (ud_parent_info(c, u)) { it->pkind = 1; it->pkey = ud_string(c, u); it->parent = cd_root(d, it->pkey); }
          else { it->pkind = 2; it->pid = ud_left(c, u); }
          if (info & 0x20) { it->has_psub = 1; it->psub = ud_string(c, u); }
        }
        if ((info & 31) == 10) fail(c, YMO_ERR_TYPE);  /* contentRefs[10] is undefined (13.4.9) */
        it->ct = read_content(c, u, info);
        it->len = content_len(it->ct);
      } else {
        it->gc = 1;
        it->deleted = 1;
        it->len = ud_len(c, u);
      }
      refs[k] = it;
      clock += it->len;
    }
    size_t at = nl;
    for (size_t q = 0; q < nl; q++) if (lst[q].client == client) at = q;
    if (at == nl) nl++;
    lst[at].client = client; lst[at].refs = refs; lst[at].n = ns; lst[at].i = 0; lst[at].live = 1;
  }
  *out = lst;
  *nout = nl;
}
static void try_merge_left(CDoc *d, CCl *s, size_t pos) { /* tryToMergeWithLeft (Transaction.js:165-176) */
  CIt *l = s->a[pos - 1], *r = s->a[pos];
  if (l->deleted != r->deleted || l->gc != r->gc) return;
  int ok;
  if (l->gc) { l->len += r->len; ok = 1; }
  else {
    JID ll = it_last(l);
    ok = jid_eq(r->has_origin, r->origin, 1, ll) && l->rightp == r && jid_eq(l->has_right, l->right, r->has_right, r->right) &&
         l->client == r->client && l->clock + l->len == r->clock && l->deleted == r->deleted && l->ct->ref == r->ct->ref;
    if (ok) {
      Content *m = content_copy(d->c, l->ct);
      ok = content_merge(d->c, m, r->ct);
      if (ok) {
        l->ct = m;
        l->rightp = r->rightp;
        if (l->rightp) l->rightp->left = l;
        l->len += r->len;
      }
    }
  }
  if (ok) {
    cl_remove(s, pos);
    if (!r->gc && r->has_psub && r->parent && map_get(r->parent, r->psub) == r) map_set(d, r->parent, r->psub, l);
  }
}
static CTx *tx_new(CDoc *d, int local) { /* new Transaction: beforeState = getStateVector(store) */
  Ctx *c = d->c;
  CTx *t = (CTx *)aalloc(c, sizeof(CTx));
  memset(t, 0, sizeof(*t));
  t->local = local;
  t->nbc = d->ncl;
  t->bc_client = (int64_t *)aalloc(c, (d->ncl + 1) * sizeof(int64_t));
  t->bc_clock = (int64_t *)aalloc(c, (d->ncl + 1) * sizeof(int64_t));
  for (size_t i = 0; i < d->ncl; i++) { t->bc_client[i] = d->cl[i].client; t->bc_clock[i] = cl_state(&d->cl[i]); }
  return t;
}

/* ---- YText._callObserver's remote formatting cleanup (YText.js:803-856) ---- */
typedef struct { Str *k; Val **v; size_t n, cap; } AttrMap; /* Map<string, any> of current attributes */
static Val *am_get(const AttrMap *m, Str k) {
  for (size_t i = 0; i < m->n; i++) if (str_eq(m->k[i], k)) return m->v[i];
  return NULL;
}
static void am_set(Ctx *c, AttrMap *m, Str k, Val *v) {
  for (size_t i = 0; i < m->n; i++) if (str_eq(m->k[i], k)) { m->v[i] = v; return; }
  if (m->n == m->cap) {
    size_t nc = m->cap ? m->cap * 2 : 8;
    Str *nk = (Str *)aalloc(c, nc * sizeof(Str));
    Val **nv = (Val **)aalloc(c, nc * sizeof(Val *));
    if (m->n) { memcpy(nk, m->k, m->n * sizeof(Str)); memcpy(nv, m->v, m->n * sizeof(Val *)); }
    m->k = nk; m->v = nv; m->cap = nc;
  }
  m->k[m->n] = k; m->v[m->n] = v; m->n++;
}
static void am_del(AttrMap *m, Str k) {
  for (size_t i = 0; i < m->n; i++)
    if (str_eq(m->k[i], k)) { m->k[i] = m->k[m->n - 1]; m->v[i] = m->v[m->n - 1]; m->n--; return; }
}
static AttrMap am_copy(Ctx *c, const AttrMap *m) {
  AttrMap r = {0};
  for (size_t i = 0; i < m->n; i++) am_set(c, &r, m->k[i], m->v[i]);
  return r;
}
static void am_update(Ctx *c, AttrMap *m, const Content *f) { /* updateCurrentAttributes (YText.js:182-189) */
  if (f->jval->t == V_NULL) am_del(m, f->key);
  else am_set(c, m, f->key, f->jval);
}
/* (x || null) === v for an attribute value x (NULL: absent) and a ContentFormat value v: JS strict equality,
   objects / arrays / typed arrays by identity */
static int or_null_eq(const Val *x, const Val *v) {
  if (x == NULL || !js_truthy(x)) return v->t == V_NULL;
  if (x->t != v->t) return 0;
  switch (x->t) {
    case V_BOOL: return x->b == v->b;
    case V_NUM: return x->num == v->num;
    case V_STR: return str_eq(x->s, v->s);
    case V_BIGINT: return memcmp(x->big, v->big, 8) == 0;
    default: return x == v;
  }
}
static int is_text_content(const CIt *it) { return it->ct->ref == 4 || it->ct->ref == 5; }
/* cleanupFormattingGap (YText.js:348-374) */
static int cleanup_gap(CDoc *d, CIt *start, CIt *end, const AttrMap *sa, AttrMap *ea) {
  while (end && !is_text_content(end)) {
    if (!end->deleted && end->ct->ref == 6) am_update(d->c, ea, end->ct);
    end = end->rightp;
  }
  int n = 0;
  while (start != end) {
    if (!start->deleted && start->ct->ref == 6) {
      const Content *f = start->ct;
      if (!or_null_eq(am_get(ea, f->key), f->jval) || or_null_eq(am_get(sa, f->key), f->jval)) { it_delete(d, start); n++; }
    }
    start = start->rightp;
  }
  return n;
}
static void cleanup_ytext(CDoc *d, CType *t) { /* cleanupYTextFormatting (YText.js:412-437) */
  CIt *start = t->start, *end = t->start;
  AttrMap sa = {0}, cur = {0};
  while (end) {
    if (!end->deleted) {
      if (end->ct->ref == 6) am_update(d->c, &cur, end->ct);
      else if (is_text_content(end)) {
        cleanup_gap(d, start, end, &sa, &cur);
        sa = am_copy(d->c, &cur);
        start = end;
      }
    }
    end = end->rightp;
  }
}
static void cleanup_contextless(CDoc *d, CIt *it) { /* cleanupContextlessFormattingGap (YText.js:380-398) */
  while (it && it->rightp && (it->rightp->deleted || !is_text_content(it->rightp))) it = it->rightp;
  AttrMap seen = {0};
  while (it && (it->deleted || !is_text_content(it))) {
    if (!it->deleted && it->ct->ref == 6) {
      if (am_get(&seen, it->ct->key)) it_delete(d, it);
      else am_set(d->c, &seen, it->ct->key, it->ct->jval);
    }
    it = it->left;
  }
}
typedef struct { int kind; int found; CType *t; } ObsCb;
static void obs_visit(CDoc *d, ObsCb *cb, CIt *st) {
  switch (cb->kind) {
    case 0: if (!st->deleted && st->ct->ref == 6) cb->found = 1; break; /* a new non-deleted format item */
    case 1: if (!st->gc && !cb->found && st->parent == cb->t && st->ct->ref == 6) cb->found = 1; break;
    case 2: if (!st->gc && st->parent == cb->t) cleanup_contextless(d, st); break;
  }
}
static size_t find_clean_start(CDoc *d, CCl *s, int64_t clock) { /* findIndexCleanStart (StructStore.js:173-181) */
  size_t idx = cd_find_index(d, s, clock);
  CIt *st = s->a[idx];
  if (st->clock < clock && !st->gc) {
    cl_insert(d, s, idx + 1, split_item(d, st, clock - st->clock));
    return idx + 1;
  }
  return idx;
}
/* iterateStructs (StructStore.js:259-273), splitting at both ends under d->tx */
static void iterate_structs(CDoc *d, CCl *s, int64_t clock, int64_t len, ObsCb *cb) {
  if (len == 0) return;
  int64_t end = clock + len;
  size_t idx = find_clean_start(d, s, clock);
  do {
    CIt *st = s->a[idx++];
    if (end < st->clock + st->len) find_clean_start(d, s, end);
    obs_visit(d, cb, st);
  } while (idx < s->n && s->a[idx]->clock < end);
}
/* iterateDeletedStructs (DeleteSet.js:58-65): Map.forEach and the ranges loop both see entries appended
   while they run */
static void iterate_deleted(CDoc *d, DSet *ds, ObsCb *cb) {
  for (size_t ci = 0; ci < ds->n; ci++) {
    for (size_t k = 0; k < ds->cl[ci].n; k++) {
      DItem di = ds->cl[ci].items[k];
      iterate_structs(d, cd_client(d, ds->cl[ci].client), di.clock, di.len, cb);
    }
  }
}
static void ytext_observer(CDoc *d, CTx *x, CType *t, CTx **nested) {
  ObsCb cb = {0, 0, t};
  d->tx = x;
  for (size_t ci = 0; ci < d->ncl && !cb.found; ci++) { /* afterState entries (store.clients order) */
    int64_t before = tx_before_at(x, ci), after = cl_state(&d->cl[ci]);
    if (after == before) continue;
    iterate_structs(d, &d->cl[ci], before, after, &cb); /* (len = afterClock, as the reference passes it) */
  }
  if (!cb.found) { cb.kind = 1; iterate_deleted(d, &x->ds, &cb); }
  /* transact(doc, t => ...): the first observer opens a new local transaction; it stays doc._transaction
     (it is cleaned up after this one), so every later observer's transact joins it */
  if (!*nested) *nested = tx_new(d, 1);
  d->tx = *nested;
  if (cb.found) cleanup_ytext(d, t);
  else { ObsCb c2 = {2, 0, t}; iterate_deleted(d, &(*nested)->ds, &c2); }
  d->tx = x;
}
/* cleanupTransactions (Transaction.js:244-367) for one transaction; returns the transaction the observers
   opened (or NULL) */
static CTx *tx_cleanup(CDoc *d, CTx *x) {
  Ctx *c = d->c;
  d->tx = x;
  ds_sort_and_merge_mode(c, &x->ds, 1);
  CTx *nested = NULL;
  if (!x->local) { /* observers of the changed types, in Map order: only Y.Text / Y.XmlText act */
    size_t nchg = x->nchg;
    CType **chg = (CType **)aalloc(c, (nchg + 1) * sizeof(CType *));
    if (nchg) memcpy(chg, x->chg, nchg * sizeof(CType *));
    for (size_t i = 0; i < nchg; i++) {
      CType *t = chg[i];
      if (t->item && t->item->deleted) continue;
      if (t->tref == 2 || t->tref == 6) ytext_observer(d, x, t, &nested);
    }
  }
  d->tx = x;
  for (size_t ci = 0; ci < x->ds.n; ci++) { /* tryGcDeleteSet (doc.gc) */
    DClient *dc = &x->ds.cl[ci];
    CCl *s = cd_client(d, dc->client);
    for (size_t k = dc->n; k-- > 0;) {
      int64_t clock = dc->items[k].clock, end = clock + dc->items[k].len;
      for (size_t si = cd_find_index(d, s, clock); si < s->n && s->a[si]->clock < end; si++) {
        CIt *st = s->a[si];
        if (!st->gc && st->deleted) it_gc(d, st, 0);
      }
    }
  }
  for (size_t ci = 0; ci < x->ds.n; ci++) { /* tryMergeDeleteSet */
    DClient *dc = &x->ds.cl[ci];
    CCl *s = cd_client(d, dc->client);
    for (size_t k = dc->n; k-- > 0;) {
      int64_t clock = dc->items[k].clock, len = dc->items[k].len;
      size_t mr = cd_find_index(d, s, clock + len - 1) + 1;
      if (mr > s->n - 1) mr = s->n - 1;
      for (size_t si = mr; si > 0 && s->a[si]->clock >= clock; si--) try_merge_left(d, s, si);
    }
  }
  for (size_t ci = 0; ci < d->ncl; ci++) { /* the clients whose state changed (afterState) */
    CCl *s = &d->cl[ci];
    int64_t before = tx_before_at(x, ci);
    if (before == cl_state(s)) continue;
    size_t first = cd_find_index(d, s, before);
    if (first < 1) first = 1;
    for (size_t i = s->n - 1; i >= first && i > 0; i--) try_merge_left(d, s, i);
  }
  for (size_t q = 0; q < x->nms; q++) { /* _mergeStructs */
    CIt *m = x->ms[q];
    CCl *s = cd_client(d, m->client);
    size_t pos = cd_find_index(d, s, m->clock);
    if (pos + 1 < s->n) try_merge_left(d, s, pos + 1);
    if (pos > 0) try_merge_left(d, s, pos);
  }
  return nested;
}
static void cd_transact(CDoc *d, UDec *u) { /* transact(readUpdateV2, local = false) + cleanupTransactions */
  Ctx *c = d->c;
  CTx *x = tx_new(d, 0);
  d->tx = x;
  /* readStructs */
  CPend *refs;
  size_t nrefs;
  read_refs(d, u, &refs, &nrefs);
  for (size_t q = 0; q < nrefs; q++) { /* mergeReadStructsIntoPendingReads */
    CPend *p = cd_pend(d, refs[q].client);
    if (!p) {
      CGROW(c, d->pend, d->npend, d->cappend, CPend);
      d->pend[d->npend++] = refs[q];
    } else {
      size_t rn = p->n - p->i;
      CIt **na = (CIt **)aalloc(c, (rn + refs[q].n + 1) * sizeof(CIt *));
      memcpy(na, p->refs + p->i, rn * sizeof(CIt *));
      memcpy(na + rn, refs[q].refs, refs[q].n * sizeof(CIt *));
      refs_sort(na, rn + refs[q].n);
      p->refs = na; p->n = rn + refs[q].n; p->i = 0;
    }
  }
  resume_integration(d);
  { /* cleanupPendingStructs (the finished entries leave the Map; the rest keep their order) */
    size_t w = 0;
    for (size_t q = 0; q < d->npend; q++) {
      CPend *p = &d->pend[q];
      if (!p->live || p->i == p->n) continue;
      p->refs += p->i; p->n -= p->i; p->i = 0;
      d->pend[w++] = *p;
    }
    d->npend = w;
  }
  { /* tryResumePendingDeleteReaders */
    DSet *pr = d->pdel;
    size_t np = d->npdel;
    d->pdel = NULL; d->npdel = 0; d->cappdel = 0;
    for (size_t q = 0; q < np; q++) apply_ds(d, &pr[q], 1, NULL);
  }
  { /* readAndApplyDeleteSet: each client's ranges are applied as read (the clients are independent) */
    uint32_t n = rd_vu(c, &u->rest);
    int zero = 0;
    for (uint32_t i = 0; i < n; i++) {
      ud_reset_ds(u);
      int64_t client = rd_vu(c, &u->rest);
      uint32_t m = rd_vu(c, &u->rest);
      DSet one;
      memset(&one, 0, sizeof(one));
      DClient *dc = ds_get_or_add(c, &one, client);
      for (uint32_t j = 0; j < m; j++) {
        int64_t clock = ud_ds_clock(c, u);
        int64_t len = ud_ds_len(c, u);
        dc_push(c, dc, clock, len);
      }
      apply_ds(d, &one, 0, &zero);
    }
    if (zero) fail(c, YMO_ERR_UNEXPECTED);
  }
  /* cleanupTransactions: this one, then the one its observers opened (local: its observers do nothing) */
  CTx *nested = tx_cleanup(d, x);
  if (nested) tx_cleanup(d, nested);
  d->tx = NULL;
}
static void cit_write(CDoc *d, UEnc *e, const CIt *it) { /* Item.write / GC.write with offset 0 */
  Ctx *c = d->c;
  if (it->gc) { ue_info(c, e, 0); ue_len(c, e, it->len); return; }
  int info = (it->ct->ref & 31) | (it->has_origin ? 0x80 : 0) | (it->has_right ? 0x40 : 0) | (it->has_psub ? 0x20 : 0);
  ue_info(c, e, info);
  if (it->has_origin) ue_left(c, e, it->origin);
  if (it->has_right) ue_right(c, e, it->right);
  if (!it->has_origin && !it->has_right) {
    CType *p = it->parent;
    if (!p) fail(c, YMO_ERR_UNEXPECTED);
    if (!p->item) { ue_parent_info(c, e, 1); ue_string(c, e, p->key); }
    else { JID pid = {p->item->client, p->item->clock}; ue_parent_info(c, e, 0); ue_left(c, e, pid); }
    if (it->has_psub) ue_string(c, e, it->psub);
  }
  content_write(c, e, it->ct, 0);
}
static Buf *compact_impl(Ctx *c, const uint8_t *const *upds, const size_t *lens, size_t n, int v2) {
  CDoc d;
  memset(&d, 0, sizeof(d));
  d.c = c;
  for (size_t k = 0; k < n; k++) {
    UDec u;
    udec_init(c, &u, upds[k], lens[k], v2);
    cd_transact(&d, &u);
  }
  /* what is still pending (structs on the stack / in the pending refs, delete readers) is not written:
     encodeStateAsUpdate = the integrated store + its delete set (encoding.js:490-493) */
  UEnc e;
  uenc_init(c, &e, v2);
  /* writeClientsStructs: clients descending, every struct from clock 0 */
  size_t *ord = (size_t *)aalloc(c, (d.ncl + 1) * sizeof(size_t));
  for (size_t i = 0; i < d.ncl; i++) ord[i] = i;
  for (size_t i = 1; i < d.ncl; i++) { size_t v = ord[i], j = i; while (j > 0 && d.cl[ord[j - 1]].client < d.cl[v].client) { ord[j] = ord[j - 1]; j--; } ord[j] = v; }
  wr_vu(c, e.rest, (int64_t)d.ncl);
  for (size_t oi = 0; oi < d.ncl; oi++) {
    CCl *s = &d.cl[ord[oi]];
    wr_vu(c, e.rest, (int64_t)s->n);
    ue_client(c, &e, s->client);
    wr_vu(c, e.rest, 0);
    for (size_t i = 0; i < s->n; i++) cit_write(&d, &e, s->a[i]);
  }
  /* createDeleteSetFromStructStore (store.clients order) + writeDeleteSet */
  DSet ds;
  memset(&ds, 0, sizeof(ds));
  for (size_t ci = 0; ci < d.ncl; ci++) {
    CCl *s = &d.cl[ci];
    DClient *dc = NULL;
    for (size_t i = 0; i < s->n; i++) {
      CIt *st = s->a[i];
      if (!st->deleted) continue;
      int64_t clock = st->clock, len = st->len;
      while (i + 1 < s->n && s->a[i + 1]->clock == clock + len && s->a[i + 1]->deleted) len += s->a[++i]->len;
      if (!dc) dc = ds_get_or_add(c, &ds, s->client);
      dc_push(c, dc, clock, len);
    }
  }
  ds_write(c, &e, &ds);
  return uenc_finish(c, &e);
}

/* ------------------------------------------------------------------------------------------------ */
/* public API                                                                                      */
/* ------------------------------------------------------------------------------------------------ */
static int finish_out(Ctx *c, Buf *b, uint8_t **out, size_t *out_len) {
  *out = (uint8_t *)malloc(b->n ? b->n : 1);
  if (!*out) return YMO_ERR_UNSUPPORTED;
  memcpy(*out, b->p, b->n);
  *out_len = b->n;
  (void)c;
  return YMO_OK;
}

int ymo_merge(const uint8_t *const *upds, const size_t *lens, size_t n, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  if (n == 1) { /* identity: `if (updates.length === 1) return updates[0]` */
    *out = (uint8_t *)malloc(lens[0] ? lens[0] : 1);
    memcpy(*out, upds[0], lens[0]);
    *out_len = lens[0];
    return YMO_OK;
  }
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  Buf *b = merge_impl(&c, upds, lens, n, fmt == 2);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_compact(const uint8_t *const *upds, const size_t *lens, size_t n, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  Buf *b = compact_impl(&c, upds, lens, n, fmt == 2);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_diff(const uint8_t *upd, size_t len, const uint8_t *sv, size_t sv_len, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  Buf *b = diff_impl(&c, upd, len, sv, sv_len, fmt == 2);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_convert(const uint8_t *upd, size_t len, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  Buf *b = conv_impl(&c, upd, len, fmt == 2);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_sv_from_update(const uint8_t *upd, size_t len, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  Buf *b = sv_impl(&c, upd, len, fmt == 2);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_meta(const uint8_t *upd, size_t len, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  Buf *b = meta_impl(&c, upd, len, fmt == 2);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_ds_merge(const uint8_t *const *dss, const size_t *lens, size_t n, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  /* fmt: 1 DSEncoderV1 / 2 DSEncoderV2 blobs; | 0x100: the reference's adjacency-only coalescing */
  Buf *b = dsmerge_impl(&c, dss, lens, n, (fmt & 0xff) == 2, (fmt & 0x100) != 0);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

int ymo_snapshot(const uint8_t *buf, size_t len, int fmt, uint8_t **out, size_t *out_len) {
  *out = NULL; *out_len = 0;
  Ctx c;
  memset(&c, 0, sizeof(c));
  int code = setjmp(c.jb);
  if (code) { ctx_free(&c); return code; }
  /* fmt: 1 / 2 the input encoding; | 0x1000 V1 output, | 0x2000 V2 output (default: the input's) */
  const int v2in = (fmt & 0xff) == 2;
  const int v2out = (fmt & 0x2000) ? 1 : (fmt & 0x1000) ? 0 : v2in;
  Buf *b = snap_impl(&c, buf, len, v2in, v2out);
  int rc = finish_out(&c, b, out, out_len);
  ctx_free(&c);
  return rc;
}

void ymo_free(void *p) { free(p); }

/* ------------------------------------------------------------------------------------------------ */
/* batched host baseline (one worker thread per core, docs dealt round-robin)                       */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
  int op, fmt;
  const uint8_t *arena; const uint64_t *upd_off; const uint32_t *doc_upd; uint32_t n_docs;
  const uint8_t *sv_arena; const uint64_t *sv_off;
  uint8_t *out_arena; const uint64_t *out_cap_off; uint64_t *out_len; int32_t *status;
  int tid, nthreads;
  int nerr;
} BatchJob;

static void *batch_worker(void *arg) {
  BatchJob *j = (BatchJob *)arg;
  size_t cap_ptrs = 64;
  const uint8_t **ptrs = (const uint8_t **)malloc(cap_ptrs * sizeof(*ptrs));
  size_t *lens = (size_t *)malloc(cap_ptrs * sizeof(*lens));
  for (uint32_t d = (uint32_t)j->tid; d < j->n_docs; d += (uint32_t)j->nthreads) {
    uint32_t u0 = j->doc_upd[d], u1 = j->doc_upd[d + 1];
    size_t n = u1 - u0;
    if (n > cap_ptrs) {
      cap_ptrs = n * 2;
      ptrs = (const uint8_t **)realloc(ptrs, cap_ptrs * sizeof(*ptrs));
      lens = (size_t *)realloc(lens, cap_ptrs * sizeof(*lens));
    }
    for (size_t i = 0; i < n; i++) {
      ptrs[i] = j->arena + j->upd_off[u0 + i];
      lens[i] = (size_t)(j->upd_off[u0 + i + 1] - j->upd_off[u0 + i]);
    }
    uint8_t *out = NULL;
    size_t olen = 0;
    int st;
    if (j->op == 0) st = ymo_merge(ptrs, lens, n, j->fmt, &out, &olen);
    else if (j->op == 1) {
      const uint8_t *sv = j->sv_arena + j->sv_off[d];
      size_t svl = (size_t)(j->sv_off[d + 1] - j->sv_off[d]);
      st = n >= 1 ? ymo_diff(ptrs[0], lens[0], sv, svl, j->fmt, &out, &olen) : YMO_ERR_UNEXPECTED;
    } else if (j->op == 3) {
      st = n >= 1 ? ymo_convert(ptrs[0], lens[0], j->fmt, &out, &olen) : YMO_ERR_UNEXPECTED;
    } else if (j->op == 4) {
      st = n == 1 ? ymo_meta(ptrs[0], lens[0], j->fmt, &out, &olen) : YMO_ERR_UNEXPECTED;
    } else if (j->op == 5) {
      st = ymo_ds_merge(ptrs, lens, n, j->fmt, &out, &olen);
    } else if (j->op == 6) {
      st = n == 1 ? ymo_snapshot(ptrs[0], lens[0], j->fmt, &out, &olen) : YMO_ERR_UNEXPECTED;
    } else if (j->op == 7) {
      st = ymo_compact(ptrs, lens, n, j->fmt, &out, &olen);
    } else st = n >= 1 ? ymo_sv_from_update(ptrs[0], lens[0], j->fmt, &out, &olen) : YMO_ERR_UNEXPECTED;
    if (st == YMO_OK && j->out_arena) {
      uint64_t cap = j->out_cap_off[d + 1] - j->out_cap_off[d];
      if (olen > cap) st = YMO_ERR_CAPACITY;
      else memcpy(j->out_arena + j->out_cap_off[d], out, olen);
    }
    free(out);
    j->out_len[d] = olen;
    j->status[d] = st;
    if (st) j->nerr++;
  }
  free(ptrs);
  free(lens);
  return NULL;
}

int ymo_batch(int op, int fmt, const uint8_t *arena, const uint64_t *upd_off, const uint32_t *doc_upd,
              uint32_t n_docs, const uint8_t *sv_arena, const uint64_t *sv_off, int nthreads,
              uint8_t *out_arena, const uint64_t *out_cap_off, uint64_t *out_len, int32_t *status) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  BatchJob jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++) {
    BatchJob b = {op, fmt, arena, upd_off, doc_upd, n_docs, sv_arena, sv_off, out_arena, out_cap_off, out_len, status, t, nthreads, 0};
    jobs[t] = b;
  }
  if (nthreads == 1) batch_worker(&jobs[0]);
  else {
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  }
  int nerr = 0;
  for (int t = 0; t < nthreads; t++) nerr += jobs[t].nerr;
  return nerr;
}
