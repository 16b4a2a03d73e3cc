// ym_core.h -- sequential per-document core of the MI355X update engine ("general path").
//
// One GPU thread owns one document and runs the exact yjs 13.5.16 lazy algorithms over it:
//   mergeUpdatesV2      (13.5.16 bundle ds@39007)    -> merge_doc()
//   diffUpdateV2        (13.5.16 bundle us@40707)    -> diff_doc()
//   encodeStateVectorFromUpdateV2 (os@37724)         -> sv_doc()
// on the wire format of gaberogan/yjs@v0 (src/utils/UpdateDecoder.js:127-392, UpdateEncoder.js:110-408,
// DeleteSet.js:113-256, structs/Item.js:625-683) with lib0 0.2.42 codec semantics.  The code is written
// for the device: no allocation (caller-provided workspace), no recursion, errors as status codes,
// and two passes (pass 1 sizes every output stream, pass 2 writes each stream straight into its final
// place in the output arena).  It is used for documents the LDS fast path (ym_fast.hip) does not take:
// overlapping / duplicate / gapped inputs, GC-Item ties, very large documents, and all V2 encoding.
//
// Payload bytes (strings, any values, binaries, JSON texts) are copied, never re-encoded: the decoder
// verifies that they are in the canonical form yjs's re-encode would produce and reports
// YM_ERR_UNSUPPORTED otherwise (DESIGN.md "canonicalisation").  Structural fields (info, IDs, lengths,
// string length prefixes, RLE columns) are always re-encoded from decoded values.
#pragma once
#include <stdint.h>

#ifndef YM_HD
#define YM_HD __host__ __device__
#endif
#define YM_INL YM_HD inline
// big per-document routines stay out of line: inlining them into one kernel explodes code size and
// compile time, and the general path is latency- not call-bound
#ifdef __HIP_DEVICE_COMPILE__
#define YM_BIG YM_HD __attribute__((noinline))
#else
#define YM_BIG YM_HD inline
#endif

namespace ym {

enum : int {
  ST_OK = 0, ST_INT_RANGE = 1, ST_UNEXPECTED = 2, ST_URI = 3, ST_TYPE = 4, ST_RANGE = 5, ST_SYNTAX = 6,
  ST_UNSUPPORTED = 7, ST_METHOD = 8, ST_CAPACITY = 9,
  ST_RETRY = 100,  // internal: workspace too small for this doc, run again with more
};
// Which message the exception carries (yjs under V8, include/ymerge.h): status = class | detail << 8 |
// argument << 16 (argument 0x7fff: unknown).  Class tests use st & 0xff.
enum : int {
  D_CONTENT_REF = 1,    // TypeError  contentRefs[(info & binary.BITS5)] is not a function   (Item.js readItemContent)
  D_TYPE_REF = 2,       // TypeError  typeRefs[decoder.readTypeRef(...)] is not a function   (ContentType.js)
  D_ANY_TAG = 3,        // TypeError  readAnyLookupTable[(127 - readUint8(...))] is not a function (lib0 readAny)
  D_BIGINT_JSON = 4,    // TypeError  Do not know how to serialize a BigInt                   (JSON.stringify)
  D_BYTELENGTH = 5,     // TypeError  Method get TypedArray.prototype.byteLength called on incompatible receiver [object Object]
  D_SET_GETTER = 6,     // TypeError  Cannot set property <arg: length|byteLength|byteOffset|buffer> of [object Object] which has only a getter
  D_SET_RO = 7,         // TypeError  Cannot assign to read only property 'BYTES_PER_ELEMENT' of object '[object Object]'
  D_KEY_UNDEF = 8,      // TypeError  Cannot read property 'length' of undefined              (V2 writeKey(undefined))
  D_CODEPOINT_NAN = 9,  // RangeError Invalid code point NaN                                  (lib0 readVarString, short)
  D_DATAVIEW = 10,      // RangeError Offset is outside the bounds of the DataView            (readFloat32/64, readBigInt64)
  D_TA_LENGTH = 11,     // RangeError Invalid typed array length: <arg>                       (lib0 readUint8Array)
  D_ORIGIN_UNDEF = 12,  // TypeError  Cannot read property 'origin' of undefined              (13.4.9 Item.integrate, Item.js:450: left is a GC)
};
YM_INL int st_d(int cls, int detail, uint64_t arg = 0) {
  return cls | (detail << 8) | (int)((arg < 0x7fff ? arg : 0x7fff) << 16);
}

struct Ctx {
  int err;
  const uint8_t *A;  // arena base (all spans are absolute offsets into it)
};
YM_INL void seterr(Ctx &c, int e) {
  if (!c.err) c.err = e;
}

// ------------------------------------------------------------------------------------------------
// byte reader with lib0 semantics (reads past the end yield `undefined`, encoded as -1)
// ------------------------------------------------------------------------------------------------
struct Rd {
  uint64_t start;  // absolute offset of byte 0
  uint64_t len;
  uint64_t pos;    // relative position (may exceed len, as t.pos++ does)
};
YM_INL int rbyte(const Ctx &c, Rd &d) {
  uint64_t p = d.pos++;
  return p < d.len ? (int)c.A[d.start + p] : -1;
}
YM_INL bool rhas(const Rd &d) { return d.pos != d.len; }

// readVarUint (lib0 U): u32 with `<< n` shift-count wrap, throws past 35 bits
YM_INL uint32_t rd_vu(Ctx &c, Rd &d) {
  uint32_t s = 0;
  unsigned n = 0;
  for (;;) {
    int e = rbyte(c, d);
    uint32_t bits = e < 0 ? 0u : (uint32_t)(e & 127);
    s |= bits << (n & 31);
    n += 7;
    if (e >= 0 && e < 128) return s;
    if (n > 35) { seterr(c, ST_INT_RANGE); return 0; }
  }
}
// readVarInt (lib0 T): sign flag (includes -0) + u32 magnitude
struct VI { uint32_t mag; bool neg; };
YM_INL VI rd_vi(Ctx &c, Rd &d) {
  int s = rbyte(c, d);
  uint32_t sb = s < 0 ? 0u : (uint32_t)s;
  uint32_t n = sb & 63;
  unsigned e = 6;
  VI r;
  r.neg = (sb & 64) != 0;
  if ((sb & 128) == 0) { r.mag = n; return r; }
  for (;;) {
    s = rbyte(c, d);
    sb = s < 0 ? 0u : (uint32_t)s;
    n |= (sb & 127) << (e & 31);
    e += 7;
    if (s >= 0 && s < 128) { r.mag = n; return r; }
    if (e > 41) { seterr(c, ST_INT_RANGE); r.mag = 0; return r; }
  }
}

// ------------------------------------------------------------------------------------------------
// strings: spans of UTF-8 bytes; fffd = a U+FFFD prefix synthesised by ContentString.splice.  A V2
// string column is one UTF-8 string sliced by UTF-16 lengths (StringDecoder), so a slice can start with
// the low half (lo) or end with the high half (hi) of a surrogate pair whose 4 UTF-8 bytes sit just
// before off / just after off + n; those halves are not part of the n bytes.
// ------------------------------------------------------------------------------------------------
struct Span {
  uint64_t off;   // absolute
  uint32_t n;     // bytes (excluding the fffd prefix and the lo / hi halves)
  uint32_t n16;   // UTF-16 length (including the fffd prefix and the lo / hi halves)
  uint8_t fffd;   // 1: string starts with U+FFFD (3 extra UTF-8 bytes)
  uint8_t lo, hi; // starts with a lone low surrogate / ends with a lone high surrogate
  uint8_t pad;
};
YM_INL uint32_t span_bytes(const Span &s) { return s.n + (s.fffd ? 3u : 0u); }

// strict UTF-8 validation (decodeURIComponent(escape(..))); counts UTF-16 units
YM_INL int utf8_check(const Ctx &c, uint64_t off, uint64_t n, uint32_t *n16) {
  uint64_t i = 0;
  uint32_t u = 0;
  while (i < n) {
    uint32_t b = c.A[off + i];
    if (b < 0x80) { u++; i++; continue; }
    int len;
    uint32_t cp, mn;
    if ((b & 0xE0) == 0xC0) { len = 2; cp = b & 0x1F; mn = 0x80; }
    else if ((b & 0xF0) == 0xE0) { len = 3; cp = b & 0x0F; mn = 0x800; }
    else if ((b & 0xF8) == 0xF0) { len = 4; cp = b & 0x07; mn = 0x10000; }
    else return ST_URI;
    if (i + len > n) return ST_URI;
    for (int j = 1; j < len; j++) {
      uint32_t cb = c.A[off + i + j];
      if ((cb & 0xC0) != 0x80) return ST_URI;
      cp = (cp << 6) | (cb & 0x3F);
    }
    if (cp < mn || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return ST_URI;
    u += cp >= 0x10000 ? 2 : 1;
    i += len;
  }
  *n16 = u;
  return 0;
}
// byte offset of UTF-16 unit k inside a valid UTF-8 span; *split = 1 if k falls inside a surrogate pair
YM_INL uint64_t utf8_unit_offset(const Ctx &c, uint64_t off, uint64_t n, uint64_t k, int *split) {
  uint64_t i = 0, u = 0;
  *split = 0;
  while (i < n && u < k) {
    uint32_t b = c.A[off + i];
    int len = b < 0x80 ? 1 : (b & 0xE0) == 0xC0 ? 2 : (b & 0xF0) == 0xE0 ? 3 : 4;
    uint32_t w = len == 4 ? 2 : 1;
    if (u + w > k) { *split = 1; return i; }  // k points at the low surrogate of this char
    u += w;
    i += len;
  }
  return i;
}

// readVarString (lib0 E) -> span
YM_INL Span rd_vstr(Ctx &c, Rd &d) {
  Span s = {0, 0, 0, 0};
  uint32_t L = rd_vu(c, d);
  if (c.err || L == 0) return s;
  uint64_t p0 = d.pos;
  uint64_t take;
  if (L - 1 < 100) {
    if (d.pos > d.len || (uint64_t)L > d.len - d.pos) { seterr(c, st_d(ST_RANGE, D_CODEPOINT_NAN)); return s; }  // fromCodePoint(undefined)
    take = L;
  } else {
    take = d.pos >= d.len ? 0 : (d.len - d.pos < L ? d.len - d.pos : L);  // subarray clamps
  }
  d.pos += L;
  s.off = d.start + p0;
  s.n = (uint32_t)take;
  int e = utf8_check(c, s.off, take, &s.n16);
  if (e) seterr(c, e);
  return s;
}

// readVarUint8Array: bounds-checked view
YM_INL Span rd_vbytes(Ctx &c, Rd &d) {
  Span s = {0, 0, 0, 0};
  uint32_t L = rd_vu(c, d);
  if (c.err) return s;
  if (d.pos > d.len || (uint64_t)L > d.len - d.pos) { seterr(c, st_d(ST_RANGE, D_TA_LENGTH, L)); return s; }
  s.off = d.start + d.pos;
  s.n = L;
  d.pos += L;
  return s;
}

// ------------------------------------------------------------------------------------------------
// `any` values: skip + verify canonical (= what readAny -> writeAny would re-emit)
// ------------------------------------------------------------------------------------------------
YM_INL bool span_eq(const Ctx &c, const Span &a, const Span &b) {
  if (a.n != b.n) return false;
  for (uint32_t i = 0; i < a.n; i++)
    if (c.A[a.off + i] != c.A[b.off + i]) return false;
  return true;
}
YM_INL bool key_is_index(const Ctx &c, const Span &k) {  // canonical array index "0".."4294967294"
  if (k.n == 0 || k.n > 10) return false;
  if (k.n > 1 && c.A[k.off] == '0') return false;
  uint64_t v = 0;
  for (uint32_t i = 0; i < k.n; i++) {
    uint8_t ch = c.A[k.off + i];
    if (ch < '0' || ch > '9') return false;
    v = v * 10 + (ch - '0');
  }
  return v < 4294967295ull;
}
YM_INL int64_t key_index(const Ctx &c, const Span &k) {
  if (!key_is_index(c, k)) return -1;
  int64_t v = 0;
  for (uint32_t i = 0; i < k.n; i++) v = v * 10 + (c.A[k.off + i] - '0');
  return v;
}
YM_INL bool key_is_proto(const Ctx &c, const Span &k) {
  const char *p = "__proto__";
  if (k.n != 9) return false;
  for (int i = 0; i < 9; i++)
    if (c.A[k.off + i] != (uint8_t)p[i]) return false;
  return true;
}
YM_INL bool vu_minimal(const Ctx &c, uint64_t start, uint64_t end) {  // last byte of a multi-byte varuint != 0
  return end - start <= 1 || c.A[end - 1] != 0;
}
// is the varuint at d.pos minimally encoded (d is not advanced)
YM_INL bool vu_prefix_minimal(Ctx &c, const Rd &d) {
  Rd t = d;
  rd_vu(c, t);
  return vu_minimal(c, t.start + d.pos, t.start + (t.pos < t.len ? t.pos : t.len));
}
YM_INL uint32_t vu_size(uint64_t v) {
  uint32_t n = 1;
  while (v > 127) { v = (uint32_t)v >> 7; n++; }
  return n;
}
// canonical writeVarInt bytes of (neg, mag) compared with the input bytes
YM_INL bool vi_canonical(const Ctx &c, uint64_t start, uint64_t end, VI v) {
  uint8_t buf[8];
  int k = 0;
  uint32_t num = v.mag;
  buf[k++] = (uint8_t)((num > 63 ? 0x80 : 0) | (v.neg ? 0x40 : 0) | (num & 63));
  num >>= 6;
  while (num > 0) { buf[k++] = (uint8_t)((num > 127 ? 0x80 : 0) | (num & 127)); num >>= 7; }
  if ((uint64_t)k != end - start) return false;
  for (int i = 0; i < k; i++)
    if (c.A[start + i] != buf[i]) return false;
  return true;
}
YM_INL double be_f32(const Ctx &c, uint64_t o) {
  uint32_t u = ((uint32_t)c.A[o] << 24) | ((uint32_t)c.A[o + 1] << 16) | ((uint32_t)c.A[o + 2] << 8) | c.A[o + 3];
  float f;
  __builtin_memcpy(&f, &u, 4);
  return (double)f;
}
YM_INL double be_f64(const Ctx &c, uint64_t o) {
  uint64_t u = 0;
  for (int i = 0; i < 8; i++) u = (u << 8) | c.A[o + i];
  double f;
  __builtin_memcpy(&f, &u, 8);
  return f;
}
YM_INL bool num_is_int(double x) { return x == x && x - x == 0 && __builtin_floor(x) == x; }

// Skips one `any` value at d, setting *noncanon when writeAny(readAny(..)) would differ.
// Iterative: a stack of pending element counts (objects: per entry a key then a value).
#define YM_ANY_DEPTH 48
#define YM_ANY_KEYS 64
YM_BIG void any_skip(Ctx &c, Rd &d, int *noncanon) {
  uint32_t left[YM_ANY_DEPTH];
  uint8_t isobj[YM_ANY_DEPTH];
  uint16_t kbase[YM_ANY_DEPTH];
  int64_t lastidx[YM_ANY_DEPTH];  // last array-index key (-1 none); -2 once a string key was seen
  Span keys[YM_ANY_KEYS];
  int nkeys = 0;
  int sp = 0;
  for (;;) {
    // parse one value
    int tag = rbyte(c, d);
    if (tag < 116 || tag > 127) { seterr(c, st_d(ST_TYPE, D_ANY_TAG)); return; }
    switch (tag) {
      case 127: case 126: case 121: case 120: break;
      case 125: {
        uint64_t s0 = d.pos;
        VI v = rd_vi(c, d);
        if (c.err) return;
        // writeAny: integer <= 2^31-1 -> varInt; larger positive -> float
        if (!v.neg && v.mag > 2147483647u) *noncanon = 1;
        else if (!vi_canonical(c, d.start + s0, d.start + d.pos, v)) *noncanon = 1;
        break;
      }
      case 124: {
        if (d.pos > d.len || d.len - d.pos < 4) { seterr(c, st_d(ST_RANGE, D_DATAVIEW)); return; }
        double x = be_f32(c, d.start + d.pos);
        if (x != x || (num_is_int(x) && x <= 2147483647.0)) *noncanon = 1;
        d.pos += 4;
        break;
      }
      case 123: {
        if (d.pos > d.len || d.len - d.pos < 8) { seterr(c, st_d(ST_RANGE, D_DATAVIEW)); return; }
        double x = be_f64(c, d.start + d.pos);
        if (num_is_int(x) && x <= 2147483647.0) *noncanon = 1;
        else if (x == x && (double)(float)x == x) *noncanon = 1;
        d.pos += 8;
        break;
      }
      case 122:
        if (d.pos > d.len || d.len - d.pos < 8) { seterr(c, st_d(ST_RANGE, D_DATAVIEW)); return; }
        d.pos += 8;
        break;
      case 119: case 116: {  // writeVarString / writeVarUint8Array re-encode the length prefix
        if (!vu_prefix_minimal(c, d)) *noncanon = 1;
        if (tag == 119) rd_vstr(c, d); else rd_vbytes(c, d);
        if (c.err) return;
        break;
      }
      default: {  // 118 object / 117 array
        uint64_t s0 = d.pos;
        uint32_t n = rd_vu(c, d);
        if (c.err) return;
        if (!vu_minimal(c, d.start + s0, d.start + d.pos)) *noncanon = 1;
        if (n > 0) {
          if (sp >= YM_ANY_DEPTH) { seterr(c, ST_UNSUPPORTED); return; }
          left[sp] = n;
          isobj[sp] = tag == 118;
          kbase[sp] = (uint16_t)nkeys;
          lastidx[sp] = -1;
          sp++;
        }
        break;
      }
    }
    if (c.err) return;
    // advance the container stack; before each object value read its key
    for (;;) {
      if (sp == 0) return;
      if (left[sp - 1] == 0) { nkeys = kbase[sp - 1]; sp--; continue; }
      left[sp - 1]--;
      if (isobj[sp - 1]) {
        if (!vu_prefix_minimal(c, d)) *noncanon = 1;
        Span k = rd_vstr(c, d);
        if (c.err) return;
        int64_t ki = key_index(c, k);
        if (ki >= 0) {  // Object.keys puts array-index keys first, ascending
          if (lastidx[sp - 1] == -2 || ki <= lastidx[sp - 1]) *noncanon = 1;
          lastidx[sp - 1] = ki;
        } else lastidx[sp - 1] = -2;
        if (key_is_proto(c, k)) *noncanon = 1;
        else {
          if (nkeys >= YM_ANY_KEYS) { *noncanon = 1; }
          else {
            for (int i = kbase[sp - 1]; i < nkeys; i++)
              if (span_eq(c, keys[i], k)) *noncanon = 1;
            keys[nkeys++] = k;
          }
        }
      }
      break;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// JSON texts (V1 readJSON/writeJSON, ContentJSON): validate the grammar (SyntaxError) and check that
// JSON.stringify(JSON.parse(text)) == text; non-canonical texts are reported as *noncanon.
// Canonical numbers accepted here: integers without fraction/exponent, |v| < 2^53, not "-0".
// ------------------------------------------------------------------------------------------------
YM_BIG int json_check(const Ctx &c, uint64_t off, uint64_t n, int *noncanon) {
  uint64_t i = 0;
  uint32_t stk[YM_ANY_DEPTH];  // bit0: object, bit1: expect key
  int sp = 0;
  auto ws = [&]() {
    uint64_t j = i;
    while (i < n) {
      uint8_t ch = c.A[off + i];
      if (ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r') i++;
      else break;
    }
    if (i != j) *noncanon = 1;
  };
  auto str = [&](Span *out) -> int {  // at '"'
    i++;
    uint64_t s0 = i;
    for (;;) {
      if (i >= n) return ST_SYNTAX;
      uint8_t ch = c.A[off + i++];
      if (ch == '"') break;
      if (ch < 0x20) return ST_SYNTAX;
      if (ch != '\\') continue;
      if (i >= n) return ST_SYNTAX;
      ch = c.A[off + i++];
      switch (ch) {
        case '"': case '\\': case 'b': case 'f': case 'n': case 'r': case 't': break;
        case '/': *noncanon = 1; break;
        case 'u': {
          if (i + 4 > n) return ST_SYNTAX;
          uint32_t v = 0;
          bool lower = true;
          for (int j = 0; j < 4; j++) {
            uint8_t h = c.A[off + i + j];
            int hv = h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10 : h >= 'A' && h <= 'F' ? (lower = false, h - 'A' + 10) : -1;
            if (hv < 0) return ST_SYNTAX;
            v = v * 16 + (uint32_t)hv;
          }
          i += 4;
          // stringify escapes only control chars (other than \b\t\n\f\r) and lone surrogates
          if (v >= 0x20 || v == 8 || v == 9 || v == 10 || v == 12 || v == 13 || !lower) *noncanon = 1;
          break;
        }
        default: return ST_SYNTAX;
      }
    }
    if (out) { out->off = off + s0; out->n = (uint32_t)(i - 1 - s0); }
    return 0;
  };
  Span keys[YM_ANY_KEYS];
  uint16_t kbase[YM_ANY_DEPTH];
  int64_t lastidx[YM_ANY_DEPTH];
  int nkeys = 0;
  auto keyorder = [&](const Span &k) {
    int64_t ki = key_index(c, k);
    if (ki >= 0) {
      if (lastidx[sp - 1] == -2 || ki <= lastidx[sp - 1]) *noncanon = 1;
      lastidx[sp - 1] = ki;
    } else lastidx[sp - 1] = -2;
  };
  ws();
  for (;;) {
    // value
    if (i >= n) return ST_SYNTAX;
    uint8_t ch = c.A[off + i];
    bool scalar = true;
    if (ch == '{' || ch == '[') {
      i++;
      if (sp >= YM_ANY_DEPTH) return ST_UNSUPPORTED;
      stk[sp] = ch == '{' ? 1u : 0u;
      kbase[sp] = (uint16_t)nkeys;
      lastidx[sp] = -1;
      sp++;
      ws();
      if (i < n && c.A[off + i] == (ch == '{' ? '}' : ']')) { i++; nkeys = kbase[--sp]; }
      else {
        if (ch == '{') {  // first key
          if (i >= n || c.A[off + i] != '"') return ST_SYNTAX;
          Span k;
          int e = str(&k);
          if (e) return e;
          keyorder(k);
          if (nkeys < YM_ANY_KEYS) keys[nkeys++] = k; else *noncanon = 1;
          ws();
          if (i >= n || c.A[off + i] != ':') return ST_SYNTAX;
          i++;
          ws();
        }
        continue;  // parse first element / value
      }
      scalar = false;
    } else if (ch == '"') {
      int e = str(nullptr);
      if (e) return e;
    } else if (ch == 't' || ch == 'f' || ch == 'n') {
      const char *lit = ch == 't' ? "true" : ch == 'f' ? "false" : "null";
      uint64_t ln = ch == 'f' ? 5 : 4;
      if (i + ln > n) return ST_SYNTAX;
      for (uint64_t j = 0; j < ln; j++)
        if (c.A[off + i + j] != (uint8_t)lit[j]) return ST_SYNTAX;
      i += ln;
    } else {
      uint64_t s0 = i;
      bool neg = false;
      if (c.A[off + i] == '-') { neg = true; i++; }
      if (i >= n) return ST_SYNTAX;
      uint64_t d0 = i;
      if (c.A[off + i] == '0') i++;
      else if (c.A[off + i] >= '1' && c.A[off + i] <= '9') { while (i < n && c.A[off + i] >= '0' && c.A[off + i] <= '9') i++; }
      else return ST_SYNTAX;
      uint64_t nd = i - d0;
      bool frac = false;
      if (i < n && c.A[off + i] == '.') {
        i++;
        frac = true;
        if (i >= n || c.A[off + i] < '0' || c.A[off + i] > '9') return ST_SYNTAX;
        while (i < n && c.A[off + i] >= '0' && c.A[off + i] <= '9') i++;
      }
      if (i < n && (c.A[off + i] == 'e' || c.A[off + i] == 'E')) {
        i++;
        frac = true;
        if (i < n && (c.A[off + i] == '+' || c.A[off + i] == '-')) i++;
        if (i >= n || c.A[off + i] < '0' || c.A[off + i] > '9') return ST_SYNTAX;
        while (i < n && c.A[off + i] >= '0' && c.A[off + i] <= '9') i++;
      }
      if (frac || nd > 15 || (neg && nd == 1 && c.A[off + d0] == '0')) *noncanon = 1;
      (void)s0;
    }
    (void)scalar;
    // after a value: close containers / separators
    for (;;) {
      ws();
      if (sp == 0) {
        if (i != n) return ST_SYNTAX;
        return 0;
      }
      if (i >= n) return ST_SYNTAX;
      uint8_t t = c.A[off + i];
      bool obj = stk[sp - 1] & 1;
      if (t == ',') {
        i++;
        ws();
        if (obj) {
          if (i >= n || c.A[off + i] != '"') return ST_SYNTAX;
          Span k;
          int e = str(&k);
          if (e) return e;
          keyorder(k);
          for (int q = kbase[sp - 1]; q < nkeys; q++)
            if (span_eq(c, keys[q], k)) *noncanon = 1;
          if (nkeys < YM_ANY_KEYS) keys[nkeys++] = k; else *noncanon = 1;
          ws();
          if (i >= n || c.A[off + i] != ':') return ST_SYNTAX;
          i++;
          ws();
        }
        break;  // next value
      }
      if (t == (obj ? '}' : ']')) { i++; nkeys = kbase[--sp]; continue; }
      return ST_SYNTAX;
    }
  }
}

}  // namespace ym
#include "ym_canon.h"
namespace ym {

// ------------------------------------------------------------------------------------------------
// V2 RLE column decoders (lib0 RleDecoder / UintOptRleDecoder / IntDiffOptRleDecoder)
// ------------------------------------------------------------------------------------------------
struct RleCol { Rd d; int s; int64_t count; };
struct UOptCol { Rd d; uint32_t s; int64_t count; };
struct IDiffCol { Rd d; int64_t s; int64_t count; int32_t diff; };

YM_INL int rle_read(Ctx &c, RleCol &r) {
  if (r.count == 0) {
    r.s = rbyte(c, r.d);
    if (rhas(r.d)) r.count = (int64_t)rd_vu(c, r.d) + 1;
    else r.count = -1;
  }
  r.count--;
  return r.s;
}
YM_INL uint32_t uopt_read(Ctx &c, UOptCol &r) {
  if (r.count == 0) {
    VI v = rd_vi(c, r.d);
    r.s = v.mag;
    r.count = 1;
    if (v.neg) r.count = (int64_t)rd_vu(c, r.d) + 2;
  }
  r.count--;
  return r.s;
}
YM_INL int64_t idiff_read(Ctx &c, IDiffCol &r) {
  if (r.count == 0) {
    VI v = rd_vi(c, r.d);
    int32_t t = v.neg ? -(int32_t)v.mag : (int32_t)v.mag;  // ToInt32(sign * mag)
    r.diff = t >> 1;
    r.count = 1;
    if (t & 1) r.count = (int64_t)rd_vu(c, r.d) + 2;
  }
  r.s += r.diff;
  r.count--;
  return r.s;
}

// ------------------------------------------------------------------------------------------------
// decoded struct (Item | GC | Skip) of the lazy reader
// ------------------------------------------------------------------------------------------------
enum : uint8_t { K_GC = 0, K_SKIP = 1, K_ITEM = 2 };
struct SStruct {
  int64_t client, clock, len;
  int64_t oc, ok, rc, rk, pc, pk;
  Span pkey, psub;
  Span a, b;       // content payload (see read_content)
  int64_t cnt;     // Deleted length, JSON/Any element count, typeRef
  UOptCol lsnap;   // V2 ContentJSON: string-length decoder snapshot at the first element
  uint64_t lsb;    // V2 ContentJSON: byte offset (absolute) of the first element
  uint8_t kind, ref, has_origin, has_right, parent_kind, has_psub;
  uint8_t nca, ncb;  // payload a / b not in the form yjs re-encodes it to: written through ym_canon.h
  uint8_t keyundef;  // ContentType element / hook name read by readKey as `undefined` (negative keyClock)
};

// ------------------------------------------------------------------------------------------------
// update decoder (V1 row format or V2 columns) + LazyStructReader state, per input update
// ------------------------------------------------------------------------------------------------
struct Reader {
  Rd rest;
  uint32_t v2;
  uint8_t started, done, filter, has_curr;
  uint8_t lax;  // non-canonical JSON / any accepted (parseUpdateMeta never re-encodes content)
  uint32_t nclients, ci, nstructs, si;
  int64_t client, clock;
  // V2 columns
  IDiffCol kc, lc, rc;
  UOptCol cl, tr, ln, sl;
  RleCol in, pi;
  uint64_t str_off, str_n;  // decoded string column (UTF-8), absolute
  uint64_t spos_b;          // string decoder byte position (relative to str_off)
  uint32_t mid;             // ... inside a surrogate pair (the high half was sliced off)
  int64_t spos16;           // ... in UTF-16 units
  uint64_t str_n16;
  uint32_t nkeys;
  Span *keys;        // V2 readKey cache (the keys read so far), keys_cap entries of the doc's workspace
  uint32_t keys_cap;
  int64_t dsCurr;
  SStruct curr;
};

YM_INL Rd col_view(Ctx &c, Rd &rest) {
  Span s = rd_vbytes(c, rest);
  Rd d = {s.off, s.n, 0};
  return d;
}
YM_BIG void reader_open(Ctx &c, Reader &r, uint64_t off, uint64_t len, uint32_t v2) {
  __builtin_memset(&r, 0, sizeof(Reader));
  r.rest.start = off;
  r.rest.len = len;
  r.v2 = v2;
  if (!v2) return;
  rd_vu(c, r.rest);  // feature flag
  r.kc.d = col_view(c, r.rest);
  r.cl.d = col_view(c, r.rest);
  r.lc.d = col_view(c, r.rest);
  r.rc.d = col_view(c, r.rest);
  r.in.d = col_view(c, r.rest);
  r.sl.d = col_view(c, r.rest);
  if (c.err) return;
  {
    Span s = rd_vstr(c, r.sl.d);  // StringDecoder: whole column decoded (and validated) up front
    r.str_off = s.off;
    r.str_n = s.n;
    r.str_n16 = s.n16;
  }
  r.pi.d = col_view(c, r.rest);
  r.tr.d = col_view(c, r.rest);
  r.ln.d = col_view(c, r.rest);
}

// V2 StringDecoder.read: `str.slice(spos, spos + len)` of the decoded column; a slice boundary may fall
// inside a surrogate pair (r.mid: the column position is past the high half of the 4-byte character at
// spos_b), giving strings that start / end with a lone surrogate (Span lo / hi)
YM_BIG Span sdec_read(Ctx &c, Reader &r) {
  uint32_t L = uopt_read(c, r.sl);
  Span s = {r.str_off + r.spos_b, 0, 0, 0, 0, 0, 0};
  if (c.err) return s;
  int64_t t = r.spos16 + (int64_t)L;
  if (r.spos16 >= (int64_t)r.str_n16) { r.spos16 = t; return s; }  // slice past the end: ""
  int64_t take = t > (int64_t)r.str_n16 ? (int64_t)r.str_n16 - r.spos16 : (int64_t)L;
  int64_t units = take;
  uint64_t pb = r.spos_b;
  if (r.mid && units > 0) { s.lo = 1; pb += 4; units--; r.mid = 0; }
  int split = 0;
  uint64_t nb = utf8_unit_offset(c, r.str_off + pb, r.str_n - pb, (uint64_t)units, &split);
  s.off = r.str_off + pb;
  s.n = (uint32_t)nb;
  s.n16 = (uint32_t)take;
  if (split) { s.hi = 1; r.mid = 1; }  // the character at pb + nb: its low half starts the next slice
  r.spos_b = pb + nb;
  r.spos16 = t;
  return s;
}

YM_INL void rd_left(Ctx &c, Reader &r, int64_t &cl, int64_t &ck) {
  if (r.v2) { cl = uopt_read(c, r.cl); ck = idiff_read(c, r.lc); }
  else { cl = rd_vu(c, r.rest); ck = rd_vu(c, r.rest); }
}
YM_INL void rd_right(Ctx &c, Reader &r, int64_t &cl, int64_t &ck) {
  if (r.v2) { cl = uopt_read(c, r.cl); ck = idiff_read(c, r.rc); }
  else { cl = rd_vu(c, r.rest); ck = rd_vu(c, r.rest); }
}
YM_INL Span rd_string(Ctx &c, Reader &r) { return r.v2 ? sdec_read(c, r) : rd_vstr(c, r.rest); }
YM_INL int64_t rd_len(Ctx &c, Reader &r) { return r.v2 ? (int64_t)uopt_read(c, r.ln) : (int64_t)rd_vu(c, r.rest); }

// V1 JSON field (readJSON = JSON.parse(readVarString)): the text, validated; *nc = 1 when
// JSON.stringify(JSON.parse(text)) differs from it
YM_INL Span rd_json_text(Ctx &c, Reader &r, uint8_t *nc) {
  Span s = rd_vstr(c, r.rest);
  if (c.err) return s;
  int n = 0;
  int e = json_check(c, s.off, s.n, &n);
  if (e) seterr(c, e);
  else if (n && !r.lax) *nc = 1;
  return s;
}
// one `any` value in rest, validated; *nc = 1 when writeAny(readAny(..)) differs from it
YM_INL Span rd_any_span(Ctx &c, Reader &r, uint8_t *nc) {
  uint64_t p0 = r.rest.pos;
  int n = 0;
  any_skip(c, r.rest, &n);
  Span s = {r.rest.start + p0, (uint32_t)(r.rest.pos - p0), 0, 0};
  if (!c.err && n) {
    const int e = any_read_check(c.A, s.off, s.off + s.n);  // readAny itself can throw (prototype keys)
    if (e) seterr(c, e);
    else if (!r.lax) *nc = 1;
  }
  return s;
}

// ContentDoc options already in the form ContentDoc re-derives ({gc:false}?, {autoLoad:true}?, {meta}?,
// meta canonical)?  Otherwise they are re-derived on write (ym_canon.h doc_opts).
YM_BIG bool doc_opts_canonical(Ctx &c, const Span &o) {
  Ctx cc = {0, c.A};
  Rd d = {o.off, o.n, 0};
  int tag = rbyte(cc, d);
  if (tag != 118) return false;
  uint32_t n = rd_vu(cc, d);
  int stage = 0;
  for (uint32_t i = 0; i < n && !cc.err; i++) {
    Span k = rd_vstr(cc, d);
    const char *want[3] = {"gc", "autoLoad", "meta"};
    int which = -1;
    for (int w = stage; w < 3; w++) {
      uint32_t wl = w == 0 ? 2 : w == 1 ? 8 : 4;
      if (k.n != wl) continue;
      bool eq = true;
      for (uint32_t q = 0; q < wl; q++)
        if (c.A[k.off + q] != (uint8_t)want[w][q]) eq = false;
      if (eq) { which = w; break; }
    }
    if (which < 0) return false;
    stage = which + 1;
    uint64_t v0 = d.pos;
    int vt = rbyte(cc, d);
    d.pos = v0;
    if (which == 0 && vt != 121) return false;
    if (which == 1 && vt != 120) return false;
    if (which == 2 && (vt == 126 || vt == 127)) return false;
    int nc = 0;
    any_skip(cc, d, &nc);
    if (nc) return false;
  }
  return !cc.err;
}

// readItemContent (Item.js:665-683, 13.5.16 ai[] table)
YM_BIG void read_content(Ctx &c, Reader &r, SStruct &s, int info) {
  int ref = info & 31;
  s.ref = (uint8_t)ref;
  switch (ref) {
    case 1: s.cnt = rd_len(c, r); s.len = s.cnt; break;
    case 2: {  // ContentJSON: n strings, each 'undefined' or canonical JSON
      s.cnt = rd_len(c, r);
      if (r.v2) { s.lsnap = r.sl; s.lsb = r.str_off + r.spos_b; }
      uint64_t first = r.v2 ? r.str_off + r.spos_b : r.rest.start + r.rest.pos;
      for (int64_t i = 0; i < s.cnt && !c.err; i++) {
        Span t = rd_string(c, r);
        if (c.err) break;
        if (t.lo || t.hi) { seterr(c, ST_SYNTAX); break; }  // a lone surrogate at either end: not JSON
        bool und = t.n == 9;
        const char *u = "undefined";
        for (uint32_t q = 0; und && q < 9; q++)
          if (c.A[t.off + q] != (uint8_t)u[q]) und = false;
        if (!und) {
          int nc = 0;
          int e = json_check(c, t.off, t.n, &nc);
          if (e) seterr(c, e);
          else if (nc && !r.lax) s.nca = 1;
        }
      }
      uint64_t last = r.v2 ? r.str_off + r.spos_b : r.rest.start + r.rest.pos;
      s.a.off = first;
      s.a.n = (uint32_t)(last - first);
      s.len = s.cnt;
      break;
    }
    case 3: s.a = rd_vbytes(c, r.rest); s.len = 1; break;
    case 4: s.a = rd_string(c, r); s.len = s.a.n16; break;
    case 5: s.a = r.v2 ? rd_any_span(c, r, &s.nca) : rd_json_text(c, r, &s.nca); s.len = 1; break;
    case 6:
      s.a = rd_string(c, r);
      s.b = r.v2 ? rd_any_span(c, r, &s.ncb) : rd_json_text(c, r, &s.ncb);
      s.len = 1;
      break;
    case 7: {
      int64_t t = r.v2 ? (int64_t)uopt_read(c, r.tr) : (int64_t)rd_vu(c, r.rest);
      if (c.err) break;
      if (t < 0 || t > 6) { seterr(c, st_d(ST_TYPE, D_TYPE_REF)); break; }
      s.cnt = t;
      s.len = 1;
      if (t == 3 || t == 5) {  // readKey (UpdateDecoder.js:382-391)
        if (r.v2) {
          int64_t kc = idiff_read(c, r.kc);
          if (c.err) break;
          if (kc < 0) { s.keyundef = 1; break; }  // keys[negative]: undefined
          if ((uint64_t)kc < r.nkeys) { s.a = r.keys[kc]; break; }  // a cached key
          s.a = sdec_read(c, r);
          if (c.err) break;
          if (r.nkeys >= r.keys_cap) { seterr(c, ST_RETRY); break; }
          r.keys[r.nkeys++] = s.a;
        } else {
          s.a = rd_vstr(c, r.rest);
        }
      }
      s.len = 1;
      break;
    }
    case 8: {
      s.cnt = rd_len(c, r);
      uint64_t p0 = r.rest.pos;
      for (int64_t i = 0; i < s.cnt && !c.err; i++) {
        int nc = 0;
        const uint64_t v0 = r.rest.pos;
        any_skip(c, r.rest, &nc);
        if (!c.err && nc) {
          const int e = any_read_check(c.A, r.rest.start + v0, r.rest.start + r.rest.pos);
          if (e) seterr(c, e);
          else if (!r.lax) s.nca = 1;
        }
      }
      s.a.off = r.rest.start + p0;
      s.a.n = (uint32_t)(r.rest.pos - p0);
      s.len = s.cnt;
      break;
    }
    case 9:
      s.a = rd_string(c, r);
      s.b = rd_any_span(c, r, &s.ncb);
      if (!c.err && !r.lax && !doc_opts_canonical(c, s.b)) s.ncb = 1;
      s.len = 1;
      break;
    case 0: case 10: seterr(c, ST_UNEXPECTED); break;
    default: seterr(c, st_d(ST_TYPE, D_CONTENT_REF)); break;
  }
}

// LazyStructReader generator step (13.5.16 ts@36560)
YM_BIG bool gen_next(Ctx &c, Reader &r) {
  if (r.done || c.err) { r.has_curr = 0; return false; }
  if (!r.started) {
    r.started = 1;
    r.nclients = rd_vu(c, r.rest);
    r.ci = 0;
    r.si = 0;
    r.nstructs = 0;
  }
  while (r.si >= r.nstructs) {
    if (c.err) { r.has_curr = 0; return false; }
    if (r.ci >= r.nclients) { r.done = 1; r.has_curr = 0; return false; }
    r.ci++;
    r.nstructs = rd_vu(c, r.rest);
    r.client = r.v2 ? (int64_t)uopt_read(c, r.cl) : (int64_t)rd_vu(c, r.rest);
    r.clock = rd_vu(c, r.rest);
    r.si = 0;
  }
  if (c.err) { r.has_curr = 0; return false; }
  r.si++;
  SStruct &s = r.curr;
  __builtin_memset(&s, 0, sizeof(SStruct));
  s.client = r.client;
  s.clock = r.clock;
  int info = r.v2 ? rle_read(c, r.in) : rbyte(c, r.rest);
  if (info == 10) {
    s.kind = K_SKIP;
    s.len = rd_vu(c, r.rest);
  } else if (info >= 0 && (info & 31) != 0) {
    s.kind = K_ITEM;
    bool noorig = (info & 0xC0) == 0;
    if (info & 0x80) { s.has_origin = 1; rd_left(c, r, s.oc, s.ok); }
    if (info & 0x40) { s.has_right = 1; rd_right(c, r, s.rc, s.rk); }
    if (noorig) {
      bool ykey = r.v2 ? rle_read(c, r.pi) == 1 : rd_vu(c, r.rest) == 1;
      if (ykey) { s.parent_kind = 1; s.pkey = rd_string(c, r); }
      else { s.parent_kind = 2; rd_left(c, r, s.pc, s.pk); }
      if (info & 0x20) { s.has_psub = 1; s.psub = rd_string(c, r); }
    }
    read_content(c, r, s, info);
  } else {
    s.kind = K_GC;
    s.len = rd_len(c, r);
  }
  if (c.err) { r.has_curr = 0; return false; }
  r.clock += s.len;
  r.has_curr = 1;
  return true;
}
YM_INL bool reader_next(Ctx &c, Reader &r) {
  bool ok;
  do { ok = gen_next(c, r); } while (ok && r.filter && r.curr.kind == K_SKIP);
  return ok;
}

// ------------------------------------------------------------------------------------------------
// output streams.  Out with p == nullptr only counts (pass 1); pass 2 writes at exact positions.
// ------------------------------------------------------------------------------------------------
struct Out { uint8_t *p; uint64_t n; };
YM_INL void o8(Out &o, uint32_t v) { if (o.p) o.p[o.n] = (uint8_t)v; o.n++; }
YM_INL void ovu(Out &o, int64_t num) {  // writeVarUint on a JS integer
  while (num > 127) { o8(o, 0x80 | (uint32_t)(num & 127)); num = (int64_t)((uint32_t)num >> 7); }
  o8(o, (uint32_t)(num & 127));
}
YM_INL void ovi(Out &o, bool neg, uint32_t mag) {  // writeVarInt
  o8(o, (mag > 63 ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (mag & 63));
  mag >>= 6;
  while (mag > 0) { o8(o, (mag > 127 ? 0x80u : 0u) | (mag & 127)); mag >>= 7; }
}
YM_INL void ovi64(Out &o, int64_t v, bool negzero) {  // writeVarInt on a JS integer value
  bool neg = v < 0 || negzero;
  uint64_t m = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
  // first byte tests the full magnitude, later bytes use ToUint32 (>>>)
  o8(o, (m > 63 ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (uint32_t)(m & 63));
  uint32_t r = ((uint32_t)m) >> 6;
  while (r > 0) { o8(o, (r > 127 ? 0x80u : 0u) | (r & 127)); r >>= 7; }
}
YM_INL void ocopy(Out &o, const Ctx &c, uint64_t off, uint64_t n) {
  if (o.p)
    for (uint64_t i = 0; i < n; i++) o.p[o.n + i] = c.A[off + i];
  o.n += n;
}
YM_INL void ostr_bytes(Out &o, const Ctx &c, const Span &s) {
  if (s.fffd) { o8(o, 0xEF); o8(o, 0xBF); o8(o, 0xBD); }
  ocopy(o, c, s.off, s.n);
}

// V2 encoder state (UpdateEncoderV2, UpdateEncoder.js:264-408) + V1 (rest only)
struct Enc {
  uint32_t v2;
  uint32_t xfmt;  // convertUpdateFormat: the structs were read in the other format (JSON text <-> any)
  Out rest;
  Out kc, cl, lc, rc, in, sb, sl, pi, tr, ln;  // columns; sb = string bytes, sl = string lengths
  int64_t kc_s, kc_n, lc_s, lc_n, rc_s, rc_n;
  int32_t kc_d, lc_d, rc_d;
  uint32_t cl_s, tr_s, ln_s, sl_s;
  int64_t cl_n, tr_n, ln_n, sl_n;
  int in_s, pi_s;
  int64_t in_n, pi_n;
  int64_t keyClock;
  int64_t dsCurr;
  uint32_t pend_hi;  // V2 string column: a lone high surrogate ended the last string written (0: none)
};
YM_INL void enc_init(Enc &e, uint32_t v2) {
  __builtin_memset(&e, 0, sizeof(Enc));
  e.v2 = v2;
  e.in_s = -1000;
  e.pi_s = -1000;
}
YM_INL void rle_w(Out &o, int &s, int64_t &n, int v) {
  if (s == v) { n++; return; }
  if (n > 0) ovu(o, n - 1);
  n = 1;
  o8(o, (uint32_t)v & 255);
  s = v;
}
YM_INL void uopt_flush(Out &o, uint32_t s, int64_t n) {
  if (n > 0) {
    ovi(o, n != 1, s);  // count==1 ? s : -s  (-0 for s==0)
    if (n > 1) ovu(o, n - 2);
  }
}
YM_INL void uopt_w(Out &o, uint32_t &s, int64_t &n, uint32_t v) {
  if (s == v) { n++; return; }
  uopt_flush(o, s, n);
  n = 1;
  s = v;
}
YM_INL void idiff_flush(Out &o, int32_t d, int64_t n) {
  if (n > 0) {
    int32_t x = (int32_t)((uint32_t)d << 1) | (n == 1 ? 0 : 1);
    ovi64(o, x, false);
    if (n > 1) ovu(o, n - 2);
  }
}
YM_INL void idiff_w(Out &o, int64_t &s, int64_t &n, int32_t &d, int64_t v) {
  if ((int64_t)d == v - s && n > 0) { s = v; n++; return; }
  if ((int64_t)d == v - s && n == 0) { s = v; n++; return; }
  idiff_flush(o, d, n);
  n = 1;
  d = (int32_t)(v - s);
  s = v;
}
YM_INL void e_client(Enc &e, int64_t client) {
  if (e.v2) uopt_w(e.cl, e.cl_s, e.cl_n, (uint32_t)client);
  else ovu(e.rest, client);
}
YM_INL void e_left(Enc &e, int64_t cl, int64_t ck) {
  if (e.v2) { uopt_w(e.cl, e.cl_s, e.cl_n, (uint32_t)cl); idiff_w(e.lc, e.lc_s, e.lc_n, e.lc_d, ck); }
  else { ovu(e.rest, cl); ovu(e.rest, ck); }
}
YM_INL void e_right(Enc &e, int64_t cl, int64_t ck) {
  if (e.v2) { uopt_w(e.cl, e.cl_s, e.cl_n, (uint32_t)cl); idiff_w(e.rc, e.rc_s, e.rc_n, e.rc_d, ck); }
  else { ovu(e.rest, cl); ovu(e.rest, ck); }
}
YM_INL void e_info(Enc &e, int info) {
  if (e.v2) rle_w(e.in, e.in_s, e.in_n, info);
  else o8(e.rest, (uint32_t)info);
}
// the surrogate halves of the 4-byte UTF-8 character at A[o]
YM_INL uint32_t sur_hi(const Ctx &c, uint64_t o) {
  const uint32_t cp = ((c.A[o] & 7u) << 18) | ((c.A[o + 1] & 63u) << 12) | ((c.A[o + 2] & 63u) << 6) | (c.A[o + 3] & 63u);
  return 0xD800 + ((cp - 0x10000) >> 10);
}
YM_INL uint32_t sur_lo(const Ctx &c, uint64_t o) {
  const uint32_t cp = ((c.A[o] & 7u) << 18) | ((c.A[o + 1] & 63u) << 12) | ((c.A[o + 2] & 63u) << 6) | (c.A[o + 3] & 63u);
  return 0xDC00 + ((cp - 0x10000) & 0x3FF);
}
// writeString: V1 writeVarString (a lone surrogate throws URIError); V2 StringEncoder.write: the column
// is one string, so a string ending with a lone high surrogate pairs with the next one's leading lone
// low surrogate (any other lone half makes toUint8Array's writeVarString throw URIError)
YM_INL void e_str_bytes(Enc &e, Ctx &c, const Span &s) {
  if (s.lo) {
    if (!e.pend_hi) { seterr(c, ST_URI); return; }
    const uint32_t cp = 0x10000 + ((e.pend_hi - 0xD800) << 10) + (sur_lo(c, s.off - 4) - 0xDC00);
    o8(e.sb, 0xF0 | (cp >> 18)); o8(e.sb, 0x80 | ((cp >> 12) & 63)); o8(e.sb, 0x80 | ((cp >> 6) & 63)); o8(e.sb, 0x80 | (cp & 63));
    e.pend_hi = 0;
  }
  if (e.pend_hi && (s.fffd || s.n || s.hi)) { seterr(c, ST_URI); return; }
  ostr_bytes(e.sb, c, s);
  if (s.hi) e.pend_hi = sur_hi(c, s.off + s.n);
}
YM_INL void e_string(Enc &e, Ctx &c, const Span &s) {
  if (e.v2) { e_str_bytes(e, c, s); uopt_w(e.sl, e.sl_s, e.sl_n, s.n16); }
  else if (s.lo || s.hi) seterr(c, ST_URI);
  else { ovu(e.rest, span_bytes(s)); ostr_bytes(e.rest, c, s); }
}
YM_INL void e_parent_info(Enc &e, int ykey) {
  if (e.v2) rle_w(e.pi, e.pi_s, e.pi_n, ykey ? 1 : 0);
  else ovu(e.rest, ykey ? 1 : 0);
}
YM_INL void e_typeref(Enc &e, int64_t t) {
  if (e.v2) uopt_w(e.tr, e.tr_s, e.tr_n, (uint32_t)t);
  else ovu(e.rest, t);
}
YM_INL void e_len(Enc &e, int64_t l) {
  if (e.v2) uopt_w(e.ln, e.ln_s, e.ln_n, (uint32_t)l);
  else ovu(e.rest, l);
}
YM_INL void e_key(Enc &e, Ctx &c, const Span &k) {
  if (e.v2) { idiff_w(e.kc, e.kc_s, e.kc_n, e.kc_d, e.keyClock++); e_str_bytes(e, c, k); uopt_w(e.sl, e.sl_s, e.sl_n, k.n16); }
  else if (k.lo || k.hi) seterr(c, ST_URI);
  else { ovu(e.rest, span_bytes(k)); ostr_bytes(e.rest, c, k); }
}
YM_INL void e_flush_columns(Ctx &c, Enc &e) {
  if (!e.v2) return;
  if (e.pend_hi) seterr(c, ST_URI);  // the column ends with a lone high surrogate
  idiff_flush(e.kc, e.kc_d, e.kc_n);
  uopt_flush(e.cl, e.cl_s, e.cl_n);
  idiff_flush(e.lc, e.lc_d, e.lc_n);
  idiff_flush(e.rc, e.rc_d, e.rc_n);
  uopt_flush(e.sl, e.sl_s, e.sl_n);
  uopt_flush(e.tr, e.tr_s, e.tr_n);
  uopt_flush(e.ln, e.ln_s, e.ln_n);
}

struct SinkOut {
  Out *o;
  YM_INL void put(uint32_t b) { o8(*o, b); }
};
// canonical form of a value into an Out (counting when o.p == nullptr)
YM_INL void canon_out(Ctx &c, Out &o, const uint8_t *A, uint64_t p, uint64_t end, uint8_t g, uint8_t t) {
  SinkOut s = {&o};
  canon_value(c, s, A, p, end, g, t);
}
// byte / UTF-16 length of a canonical JSON text
YM_INL SinkLen canon_len(Ctx &c, const uint8_t *A, uint64_t p, uint64_t end, uint8_t g, uint8_t t) {
  SinkLen n = {0, 0};
  canon_value(c, n, A, p, end, g, t);
  return n;
}

// writeString of a canonical JSON text (ContentJSON element: JSON.stringify(JSON.parse(text)))
YM_BIG void e_json_string(Ctx &c, Enc &e, uint64_t off, uint64_t n) {
  if (e.v2 && e.pend_hi) { seterr(c, ST_URI); return; }  // a pending lone high surrogate stays unpaired
  const uint64_t p = js_ws(c.A, off, off + n);
  const SinkLen L = canon_len(c, c.A, p, off + n, G_JSON, T_JSON);
  if (c.err) return;
  if (e.v2) {
    canon_out(c, e.sb, c.A, p, off + n, G_JSON, T_JSON);
    uopt_w(e.sl, e.sl_s, e.sl_n, (uint32_t)L.u16);
  } else {
    ovu(e.rest, (int64_t)L.bytes);
    canon_out(c, e.rest, c.A, p, off + n, G_JSON, T_JSON);
  }
}
// writeJSON / writeAny of an embed or format value read as span s (V1: JSON text, V2: any), canonical.
// Same format: V1 writeVarString(JSON.stringify(JSON.parse(text))), V2 writeAny(readAny(..)).
// convertUpdateFormat (e.xfmt): V1 -> V2 writeAny(JSON.parse(text)); V2 -> V1
// writeVarString(JSON.stringify(readAny(..))) (undefined -> the text "undefined", encodeURIComponent).
YM_BIG void e_json_value(Ctx &c, Enc &e, const Span &s) {
  const bool src_json = e.xfmt ? e.v2 != 0 : !e.v2;
  if (src_json) {
    const uint64_t p = js_ws(c.A, s.off, s.off + s.n);
    if (e.v2) { canon_out(c, e.rest, c.A, p, s.off + s.n, G_JSON, T_ANY); return; }
    const SinkLen L = canon_len(c, c.A, p, s.off + s.n, G_JSON, T_JSON);
    if (c.err) return;
    ovu(e.rest, (int64_t)L.bytes);
    canon_out(c, e.rest, c.A, p, s.off + s.n, G_JSON, T_JSON);
    return;
  }
  if (!e.v2) {  // V2 any -> V1 JSON text
    if (c.A[s.off] == 127) { ovu(e.rest, 9); for (const char *t = "undefined"; *t; t++) o8(e.rest, (uint32_t)*t); return; }
    const SinkLen L = canon_len(c, c.A, s.off, s.off + s.n, G_ANY, T_JSONANY);
    if (c.err) return;
    ovu(e.rest, (int64_t)L.bytes);
    canon_out(c, e.rest, c.A, s.off, s.off + s.n, G_ANY, T_JSONANY);
    return;
  }
  canon_out(c, e.rest, c.A, s.off, s.off + s.n, G_ANY, T_ANY);
}

// skip k JSON element strings of a ContentJSON starting at its first element (returns new start)
YM_BIG Span json_elems_from(Ctx &c, const SStruct &s, int64_t k, UOptCol *lens_out) {
  Span out = s.a;
  if (s.ref != 2) return out;
  uint64_t p = s.a.off;
  if (s.lsb == 0 && s.a.n == 0) return out;
  UOptCol ls = s.lsnap;
  for (int64_t i = 0; i < k && i < s.cnt; i++) {
    if (s.lsb) {  // V2: the lengths come from the string-length column snapshot
      uint32_t L = uopt_read(c, ls);
      int split = 0;
      p += utf8_unit_offset(c, p, s.a.off + s.a.n - p, L, &split);
    } else {
      Rd d = {p, s.a.off + s.a.n - p, 0};
      uint32_t L = rd_vu(c, d);
      p += d.pos + L;
    }
  }
  out.n = (uint32_t)(s.a.off + s.a.n - p);
  out.off = p;
  if (lens_out) *lens_out = ls;
  return out;
}

// skip k `any` values (canonical, already validated)
YM_INL uint64_t any_skip_n(Ctx &c, uint64_t off, uint64_t n, int64_t k) {
  Rd d = {off, n, 0};
  for (int64_t i = 0; i < k && !c.err; i++) {
    int nc = 0;
    any_skip(c, d, &nc);
  }
  return off + d.pos;
}

// Content*.write(encoder, offset)
YM_BIG void content_write(Ctx &c, Enc &e, const SStruct &s, int64_t off) {
  switch (s.ref) {
    case 1: e_len(e, s.cnt - off); break;
    case 2: {
      e_len(e, s.cnt - off);
      UOptCol ls;
      Span from = json_elems_from(c, s, off, &ls);
      uint64_t p = from.off, end = from.off + from.n;
      for (int64_t i = off; i < s.cnt; i++) {
        Span t = {p, 0, 0, 0};
        if (s.lsb) {
          uint32_t L = uopt_read(c, ls);
          int split = 0;
          t.n = (uint32_t)utf8_unit_offset(c, p, end - p, L, &split);
          t.n16 = L;
        } else {
          Rd d = {p, end - p, 0};
          uint32_t L = rd_vu(c, d);
          t.off = p + d.pos;
          t.n = L;
          uint32_t n16 = 0;
          utf8_check(c, t.off, t.n, &n16);
          t.n16 = n16;
        }
        // JSON.stringify(JSON.parse(text)) unless the element is 'undefined' (ContentJSON.js:83-90)
        const bool und = t.n == 9 && c.A[t.off] == 'u' && c.A[t.off + 1] == 'n' && c.A[t.off + 2] == 'd' &&
                         c.A[t.off + 3] == 'e' && c.A[t.off + 8] == 'd';
        if (s.nca && !und) e_json_string(c, e, t.off, t.n);
        else e_string(e, c, t);
        p = t.off + t.n;
      }
      break;
    }
    case 3: ovu(e.rest, s.a.n); ocopy(e.rest, c, s.a.off, s.a.n); break;
    case 4: {
      if (off == 0) { e_string(e, c, s.a); break; }
      // str.slice(offset) without the U+FFFD rule: a cut inside a surrogate pair leaves a lone
      // surrogate that writeVarString / the V2 StringEncoder reject (URIError)
      Span t = s.a;
      int64_t k = off;
      if (t.fffd && k >= 1) { t.fffd = 0; k--; t.n16--; }
      if (t.lo && k >= 1) { t.lo = 0; k--; t.n16--; }
      int split = 0;
      uint64_t b = utf8_unit_offset(c, t.off, t.n, (uint64_t)k, &split);
      t.n16 -= (uint32_t)k;
      if (split) {  // the cut leaves the low half of the pair at byte b: a lone surrogate (e_string decides)
        t.lo = 1;
        b += 4;
      }
      t.off += b;
      t.n -= (uint32_t)b;
      e_string(e, c, t);
      break;
    }
    case 5:
      if (e.xfmt || s.nca) e_json_value(c, e, s.a);
      else if (e.v2) ocopy(e.rest, c, s.a.off, s.a.n);
      else { ovu(e.rest, s.a.n); ocopy(e.rest, c, s.a.off, s.a.n); }
      break;
    case 6:
      e_key(e, c, s.a);
      if (e.xfmt || s.ncb) e_json_value(c, e, s.b);
      else if (e.v2) ocopy(e.rest, c, s.b.off, s.b.n);
      else { ovu(e.rest, s.b.n); ocopy(e.rest, c, s.b.off, s.b.n); }
      break;
    case 7:
      e_typeref(e, s.cnt);
      if (s.cnt == 3 || s.cnt == 5) {
        if (!s.keyundef) { e_key(e, c, s.a); break; }
        // an undefined name: YXmlElement's constructor defaults it to 'UNDEFINED' (YXmlElement.js:22);
        // YXmlHook keeps undefined, so writeKey(undefined): the V2 StringEncoder reads undefined.length
        // (TypeError), V1 writeVarString writes encodeURIComponent(undefined) = "undefined"
        const char *lit = s.cnt == 3 ? "UNDEFINED" : "undefined";
        if (e.v2) {
          if (s.cnt == 5) { seterr(c, st_d(ST_TYPE, D_KEY_UNDEF)); break; }
          idiff_w(e.kc, e.kc_s, e.kc_n, e.kc_d, e.keyClock++);
          if (e.pend_hi) { seterr(c, ST_URI); break; }
          for (const char *t = lit; *t; t++) o8(e.sb, (uint32_t)*t);
          uopt_w(e.sl, e.sl_s, e.sl_n, 9);
        } else {
          ovu(e.rest, 9);
          for (const char *t = lit; *t; t++) o8(e.rest, (uint32_t)*t);
        }
      }
      break;
    case 8: {
      e_len(e, s.cnt - off);
      uint64_t p = off ? any_skip_n(c, s.a.off, s.a.n, off) : s.a.off;
      if (!s.nca) { ocopy(e.rest, c, p, s.a.off + s.a.n - p); break; }
      for (int64_t i = off; i < s.cnt && !c.err; i++) {  // writeAny(readAny(..)) element by element
        canon_out(c, e.rest, c.A, p, s.a.off + s.a.n, G_ANY, T_ANY);
        p = any_end(c.A, p);
      }
      break;
    }
    case 9: {
      if (!s.ncb) { e_string(e, c, s.a); ocopy(e.rest, c, s.b.off, s.b.n); break; }
      // new ContentDoc(new Doc({guid, ...opts})): the options re-derived, an own string `guid` wins
      const DocOpts d = doc_opts(c, c.A, s.b.off, s.b.off + s.b.n);
      if (c.err) break;
      Span g = s.a;
      if (d.has_guid) {
        uint64_t q = d.guid_val;
        const uint32_t L = cv_vu(c.A, q);
        g.off = q; g.n = L; g.fffd = 0;
        uint32_t n16 = 0;
        utf8_check(c, q, L, &n16);
        g.n16 = n16;
      }
      e_string(e, c, g);
      SinkOut so = {&e.rest};
      s_doc_opts(c, so, c.A, d, s.b.off + s.b.n);
      break;
    }
    default: seterr(c, ST_UNEXPECTED); break;
  }
}

// Item.write / GC.write / Skip.write (Item.js:625-658, GC.js:45-48, 13.5.16 ui.write)
YM_BIG void struct_write(Ctx &c, Enc &e, const SStruct &s, int64_t off) {
  if (s.kind == K_GC) { e_info(e, 0); e_len(e, s.len - off); return; }
  if (s.kind == K_SKIP) { e_info(e, 10); ovu(e.rest, s.len - off); return; }
  bool has_origin = off > 0 ? true : s.has_origin;
  int64_t oc = s.oc, ok = s.ok;
  if (off > 0) { oc = s.client; ok = s.clock + off - 1; }
  int info = (s.ref & 31) | (has_origin ? 0x80 : 0) | (s.has_right ? 0x40 : 0) | (s.has_psub ? 0x20 : 0);
  e_info(e, info);
  if (has_origin) e_left(e, oc, ok);
  if (s.has_right) e_right(e, s.rc, s.rk);
  if (!has_origin && !s.has_right) {
    if (s.parent_kind == 1) { e_parent_info(e, 1); e_string(e, c, s.pkey); }
    else if (s.parent_kind == 2) { e_parent_info(e, 0); e_left(e, s.pc, s.pk); }
    else { seterr(c, ST_UNEXPECTED); return; }
    if (s.has_psub) e_string(e, c, s.psub);
  }
  content_write(c, e, s, off);
}

// sliceStruct (13.5.16 as@38661) incl. ContentString.splice's U+FFFD rule (ContentString.js:51-66)
YM_BIG void slice_struct(Ctx &c, SStruct &s, int64_t diff) {
  if (s.kind != K_ITEM) { s.clock += diff; s.len -= diff; return; }
  s.has_origin = 1;
  s.oc = s.client;
  s.ok = s.clock + diff - 1;
  s.clock += diff;
  switch (s.ref) {
    case 1: s.cnt -= diff; s.len = s.cnt; break;
    case 2: {
      UOptCol ls;
      Span from = json_elems_from(c, s, diff, &ls);
      if (s.lsb) { s.lsnap = ls; s.lsb = from.off; }
      s.a = from;
      s.cnt = s.cnt > diff ? s.cnt - diff : 0;
      s.len = s.cnt;
      break;
    }
    case 8: {
      uint64_t p = any_skip_n(c, s.a.off, s.a.n, diff);
      s.a.n = (uint32_t)(s.a.off + s.a.n - p);
      s.a.off = p;
      s.cnt = s.cnt > diff ? s.cnt - diff : 0;
      s.len = s.cnt;
      break;
    }
    case 4: {
      Span t = s.a;
      int64_t k = diff;
      if (k > (int64_t)t.n16) k = t.n16;
      if (t.fffd && k >= 1) { t.fffd = 0; k--; t.n16--; }
      if (t.lo && k >= 1) { t.lo = 0; k--; t.n16--; }  // charCodeAt(0) is a low surrogate: no U+FFFD rule
      int split = 0;
      uint64_t b = utf8_unit_offset(c, t.off, t.n, (uint64_t)k, &split);
      if (split) {
        // left part ends with a high surrogate: right = U+FFFD + (rest after the 4-byte char)
        t.off += b + 4;
        t.n -= (uint32_t)(b + 4);
        t.fffd = 1;
        t.n16 = (uint32_t)((int64_t)t.n16 - k);
      } else {
        t.off += b;
        t.n -= (uint32_t)b;
        t.n16 = (uint32_t)((int64_t)t.n16 - k);
      }
      s.a = t;
      s.len = t.n16;
      break;
    }
    default: seterr(c, ST_METHOD); break;
  }
}


// ------------------------------------------------------------------------------------------------
// Output layout of one document (pass 1 computes it, pass 2 writes into it)
//   V2: vu(0) | col kc | col cl | col lc | col rc | col in | vu(|sb|+|sl|+vu(|sb|)) vu(|sb|) sb sl | col pi
//       | col tr | col ln | rest          (col x = vu(|x|) x;  UpdateEncoder.js:289-304)
//   V1: rest
//   rest = vu(nparts) | per part: vu(written) part-bytes | delete set      (LazyStructWriter ws@41612)
// ------------------------------------------------------------------------------------------------
enum { C_KC = 0, C_CL, C_LC, C_RC, C_IN, C_SB, C_SL, C_PI, C_TR, C_LN, C_N };
struct Layout {
  uint64_t col[C_N];
  uint64_t parts_bytes;  // sum over parts of (vu(written) + bytes)
  uint64_t nparts;
  uint64_t ds_bytes;
  uint64_t total;
  uint64_t svcount;      // sv_doc: number of (client, clock) pairs
};
YM_INL uint64_t layout_header_bytes(const Layout &L, uint32_t v2) {
  if (!v2) return 0;
  uint64_t h = 1;
  for (int i = 0; i < C_N; i++) {
    if (i == C_SB || i == C_SL) continue;
    h += vu_size(L.col[i]) + L.col[i];
  }
  uint64_t sc = vu_size(L.col[C_SB]) + L.col[C_SB] + L.col[C_SL];
  h += vu_size(sc) + sc;
  return h;
}
YM_INL void layout_finish(Layout &L, uint32_t v2) {
  L.total = layout_header_bytes(L, v2) + vu_size(L.nparts) + L.parts_bytes + L.ds_bytes;
}
// pass 2: point every stream of `e` at its final place in the document's output bytes
YM_BIG uint64_t layout_bind(const Layout &L, Enc &e, uint8_t *base) {
  uint64_t pos = 0;
  Out hdr = {base, 0};
  if (e.v2) {
    o8(hdr, 0);
    Out *cols[C_N] = {&e.kc, &e.cl, &e.lc, &e.rc, &e.in, &e.sb, &e.sl, &e.pi, &e.tr, &e.ln};
    for (int i = 0; i < C_N; i++) {
      if (i == C_SL) continue;
      if (i == C_SB) {
        uint64_t sc = vu_size(L.col[C_SB]) + L.col[C_SB] + L.col[C_SL];
        ovu(hdr, (int64_t)sc);
        ovu(hdr, (int64_t)L.col[C_SB]);
        e.sb.p = base; e.sb.n = hdr.n;
        hdr.n += L.col[C_SB];
        e.sl.p = base; e.sl.n = hdr.n;
        hdr.n += L.col[C_SL];
        continue;
      }
      ovu(hdr, (int64_t)L.col[i]);
      cols[i]->p = base;
      cols[i]->n = hdr.n;
      hdr.n += L.col[i];
    }
  }
  pos = hdr.n;
  e.rest.p = base;
  e.rest.n = pos;
  ovu(e.rest, (int64_t)L.nparts);
  return pos;
}

// ------------------------------------------------------------------------------------------------
// LazyStructWriter (13.5.16 rs/ps/gs/ws)
// ------------------------------------------------------------------------------------------------
struct PartRec { uint64_t written; uint64_t bytes; };
struct LW {
  int64_t currClient, written;
  uint64_t part_start;
  uint32_t nparts, cap, pass;
  PartRec *parts;
  uint64_t parts_bytes;
};
YM_INL void lw_flush(Ctx &c, LW &w, Enc &e) {
  if (w.written > 0) {
    uint64_t bytes = e.rest.n - w.part_start;
    if (w.pass == 1) {
      if (w.nparts < w.cap) { w.parts[w.nparts].written = (uint64_t)w.written; w.parts[w.nparts].bytes = bytes; }
      else seterr(c, ST_RETRY);
      w.parts_bytes += vu_size((uint64_t)w.written) + bytes;
    }
    w.nparts++;
    w.written = 0;
  }
}
YM_BIG void lw_write(Ctx &c, LW &w, Enc &e, const SStruct &s, int64_t off) {
  if (w.written > 0 && w.currClient != s.client) lw_flush(c, w, e);
  if (c.err) return;
  if (w.written == 0) {
    if (w.pass == 2) {  // the part header precedes the part bytes in the final layout
      if (w.nparts >= w.cap) { seterr(c, ST_RETRY); return; }
      ovu(e.rest, (int64_t)w.parts[w.nparts].written);
    }
    w.part_start = e.rest.n;
    w.currClient = s.client;
    e_client(e, s.client);
    ovu(e.rest, s.clock + off);
  }
  struct_write(c, e, s, off);
  w.written++;
}

// ------------------------------------------------------------------------------------------------
// DeleteSet: read all, group by first appearance, (merge: sort by clock + union), write
// ------------------------------------------------------------------------------------------------
struct DSE { uint32_t client; uint32_t seq; int64_t clock; int64_t len; };
struct DSG { uint32_t first; uint32_t start; uint32_t count; uint32_t pad; };

template <class T, class Less>
YM_INL void heap_sort(T *a, uint64_t n, Less less) {
  if (n < 2) return;
  auto sift = [&](uint64_t i, uint64_t m) {
    for (;;) {
      uint64_t l = 2 * i + 1, r = l + 1, mx = i;
      if (l < m && less(a[mx], a[l])) mx = l;
      if (r < m && less(a[mx], a[r])) mx = r;
      if (mx == i) return;
      T t = a[i]; a[i] = a[mx]; a[mx] = t;
      i = mx;
    }
  };
  for (uint64_t i = n / 2; i-- > 0;) sift(i, n);
  for (uint64_t m = n - 1; m > 0; m--) {
    T t = a[0]; a[0] = a[m]; a[m] = t;
    sift(0, m);
  }
}

// readDeleteSet of one decoder, appended to ds[] with increasing seq
YM_BIG void ds_gather(Ctx &c, Reader &r, DSE *ds, uint64_t cap, uint64_t &n) {
  uint32_t nc = rd_vu(c, r.rest);
  for (uint32_t i = 0; i < nc && !c.err; i++) {
    r.dsCurr = 0;
    uint32_t client = rd_vu(c, r.rest);
    uint32_t m = rd_vu(c, r.rest);
    for (uint32_t j = 0; j < m && !c.err; j++) {
      int64_t clock, len;
      if (r.v2) {
        r.dsCurr += rd_vu(c, r.rest);
        clock = r.dsCurr;
        len = (int64_t)rd_vu(c, r.rest) + 1;
        r.dsCurr += len;
      } else {
        clock = rd_vu(c, r.rest);
        len = rd_vu(c, r.rest);
      }
      if (c.err) return;
      if (n >= cap) { seterr(c, ST_RETRY); return; }
      ds[n].client = client; ds[n].seq = (uint32_t)n; ds[n].clock = clock; ds[n].len = len;
      n++;
    }
  }
}

// Writes the DS of n gathered entries: merge=1 -> mergeDeleteSets (sort by clock + union, le@10242),
// merge=2 -> the reference's mergeDeleteSets (stable sort by clock, only exactly adjacent ranges
// coalesce: DeleteSet.js:113-135), merge=0 -> readDeleteSet + writeDeleteSet only (entries regrouped by
// first client appearance).
YM_BIG void ds_emit(Ctx &c, Enc &e, DSE *ds, uint64_t n, DSG *g, int merge) {
  if (merge) heap_sort(ds, n, [](const DSE &x, const DSE &y) {
    return x.client != y.client ? x.client < y.client : x.clock != y.clock ? x.clock < y.clock : x.seq < y.seq;
  });
  else heap_sort(ds, n, [](const DSE &x, const DSE &y) { return x.client != y.client ? x.client < y.client : x.seq < y.seq; });
  uint64_t ng = 0;
  for (uint64_t i = 0; i < n;) {
    uint64_t j = i;
    uint32_t first = ds[i].seq;
    while (j < n && ds[j].client == ds[i].client) { if (ds[j].seq < first) first = ds[j].seq; j++; }
    g[ng].first = first; g[ng].start = (uint32_t)i; g[ng].count = (uint32_t)(j - i);
    ng++;
    i = j;
  }
  heap_sort(g, ng, [](const DSG &x, const DSG &y) { return x.first < y.first; });
  ovu(e.rest, (int64_t)ng);
  for (uint64_t gi = 0; gi < ng && !c.err; gi++) {
    DSE *it = ds + g[gi].start;
    uint32_t cnt = g[gi].count;
    e.dsCurr = 0;
    ovu(e.rest, it[0].client);
    if (merge) {  // in-place union (>= merges touching ranges, max of ends)
      uint32_t j = 1;
      for (uint32_t i = 1; i < cnt; i++) {
        DSE &left = it[j - 1];
        if (merge == 2 ? left.clock + left.len == it[i].clock : left.clock + left.len >= it[i].clock) {
          if (merge == 2) left.len += it[i].len;
          else {
            int64_t m = it[i].clock + it[i].len - left.clock;
            if (m > left.len) left.len = m;
          }
        } else {
          if (j < i) it[j] = it[i];
          j++;
        }
      }
      cnt = j;
    }
    ovu(e.rest, cnt);
    for (uint32_t i = 0; i < cnt; i++) {
      if (e.v2) {
        ovu(e.rest, it[i].clock - e.dsCurr);
        e.dsCurr = it[i].clock;
        if (it[i].len == 0) { seterr(c, ST_UNEXPECTED); return; }
        ovu(e.rest, it[i].len - 1);
        e.dsCurr += it[i].len;
      } else {
        ovu(e.rest, it[i].clock);
        ovu(e.rest, it[i].len);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// mergeUpdatesV2 (13.5.16 ds@39007) for one document
// ------------------------------------------------------------------------------------------------
struct DocWS {          // per-document workspace (global memory), carved by the host
  Reader *rs;           // k readers
  uint32_t *arr, *tmp;  // reader order (k each)
  PartRec *parts; uint32_t parts_cap;
  DSE *ds; DSG *dsg; uint64_t ds_cap;
  int64_t *sv;  uint32_t sv_cap;   // diff: decoded state vector (client, clock) pairs
  Span *keys; uint64_t keys_cap;   // V2 readKey caches of all readers
  uint32_t mul;                    // capacity multiplier of this attempt (grown on ST_RETRY)
};
// a V2 reader's readKey cache: (its bytes / 64 + 4) * mul entries carved from the doc's pool
YM_INL void reader_keys(Ctx &c, Reader &r, DocWS &ws, uint64_t &used) {
  if (!r.v2) return;
  const uint64_t cap = (r.rest.len / 64 + 4) * ws.mul;
  if (used + cap > ws.keys_cap) { seterr(c, ST_RETRY); return; }
  r.keys = ws.keys + used;
  r.keys_cap = (uint32_t)cap;
  used += cap;
}

// reader comparator of the 13.5.16 sort; *inconsistent is set for a GC/Item tie
YM_INL int rcmp(const Reader &a, const Reader &b, int *inconsistent) {
  const SStruct &x = a.curr, &y = b.curr;
  if (x.client == y.client) {
    int64_t d = x.clock - y.clock;
    if (d == 0) {
      if (x.kind == y.kind) return 0;
      if (x.kind != K_SKIP && y.kind != K_SKIP) *inconsistent = 1;
      return x.kind == K_SKIP ? 1 : -1;
    }
    return d < 0 ? -1 : 1;
  }
  return y.client - x.client < 0 ? -1 : 1;
}
YM_INL bool rtie_bad(const Reader &a, const Reader &b) {  // GC/Item tie (comparator inconsistent)
  return a.curr.client == b.curr.client && a.curr.clock == b.curr.clock && a.curr.kind != b.curr.kind &&
         a.curr.kind != K_SKIP && b.curr.kind != K_SKIP;
}
// V8's Array.prototype.sort (TimSort of third_party/v8/builtins/array-sort.tq in the reference's Node),
// restated operation by operation over reader indices: runs by CountAndMakeRun, extended to minrun by
// BinaryInsertionSort, a pending-run stack collapsed by MergeCollapse, merges by MergeLow / MergeHigh
// with galloping (minGallop starts at 7).  The reader comparator is inconsistent for a GC / Item tie
// (compare(a, b) = compare(b, a) = -1), so the order 13.5.16's mergeUpdates produces depends on exactly
// which pairs V8 compares; below 64 readers only the first two steps run.  tmp: n scratch slots.
struct V8Sort {
  Reader *rs;
  uint32_t *a, *t;
  uint32_t base[80], len[80];
  int nruns;
  int64_t min_gallop;
  YM_INL int cmp(uint32_t x, uint32_t y) { int inc = 0; return rcmp(rs[x], rs[y], &inc); }
};
YM_BIG int64_t v8_gallop_left(V8Sort &S, const uint32_t *arr, uint32_t key, int64_t base, int64_t length, int64_t hint) {
  int64_t last = 0, ofs = 1;
  if (S.cmp(arr[base + hint], key) < 0) {
    const int64_t maxo = length - hint;
    while (ofs < maxo) {
      if (S.cmp(arr[base + hint + ofs], key) >= 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    last += hint;
    ofs += hint;
  } else {
    const int64_t maxo = hint + 1;
    while (ofs < maxo) {
      if (S.cmp(arr[base + hint - ofs], key) < 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    const int64_t t = last;
    last = hint - ofs;
    ofs = hint - t;
  }
  last++;
  while (last < ofs) {
    const int64_t m = last + ((ofs - last) >> 1);
    if (S.cmp(arr[base + m], key) < 0) last = m + 1; else ofs = m;
  }
  return ofs;
}
YM_BIG int64_t v8_gallop_right(V8Sort &S, const uint32_t *arr, uint32_t key, int64_t base, int64_t length, int64_t hint) {
  int64_t last = 0, ofs = 1;
  if (S.cmp(key, arr[base + hint]) < 0) {
    const int64_t maxo = hint + 1;
    while (ofs < maxo) {
      if (S.cmp(key, arr[base + hint - ofs]) >= 0) break;
      last = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxo;
    }
    if (ofs > maxo) ofs = maxo;
    const int64_t t = last;
    last = hint - ofs;
    ofs = hint - t;
  } else {
    const int64_t maxo = length - hint;
    while (ofs < maxo) {
      if (S.cmp(key, arr[base + hint + ofs]) < 0) break;
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
    const int64_t m = last + ((ofs - last) >> 1);
    if (S.cmp(key, arr[base + m]) < 0) ofs = m; else last = m + 1;
  }
  return ofs;
}
YM_INL void v8_copy(uint32_t *dst, const uint32_t *src, int64_t n) {  // memmove
  if (dst < src) for (int64_t i = 0; i < n; i++) dst[i] = src[i];
  else for (int64_t i = n - 1; i >= 0; i--) dst[i] = src[i];
}
YM_BIG void v8_merge_low(V8Sort &S, int64_t baseA, int64_t lenA, int64_t baseB, int64_t lenB) {
  uint32_t *a = S.a, *t = S.t;
  v8_copy(t, a + baseA, lenA);
  int64_t dest = baseA, ct = 0, cb = baseB;
  a[dest++] = a[cb++];
  if (--lenB == 0) goto succeed;
  if (lenA == 1) goto copy_b;
  for (;;) {
    int64_t wa = 0, wb = 0;
    for (;;) {
      if (S.cmp(a[cb], t[ct]) < 0) {
        a[dest++] = a[cb++]; wb++; lenB--; wa = 0;
        if (lenB == 0) goto succeed;
        if (wb >= S.min_gallop) break;
      } else {
        a[dest++] = t[ct++]; wa++; lenA--; wb = 0;
        if (lenA == 1) goto copy_b;
        if (wa >= S.min_gallop) break;
      }
    }
    S.min_gallop++;
    bool first = true;
    while (wa >= 7 || wb >= 7 || first) {
      first = false;
      S.min_gallop = S.min_gallop - 1 > 1 ? S.min_gallop - 1 : 1;
      wa = v8_gallop_right(S, t, a[cb], ct, lenA, 0);
      if (wa > 0) {
        v8_copy(a + dest, t + ct, wa);
        dest += wa; ct += wa; lenA -= wa;
        if (lenA == 1) goto copy_b;
        if (lenA == 0) goto succeed;  // impossible for a consistent comparator
      }
      a[dest++] = a[cb++];
      if (--lenB == 0) goto succeed;
      wb = v8_gallop_left(S, a, t[ct], cb, lenB, 0);
      if (wb > 0) {
        v8_copy(a + dest, a + cb, wb);
        dest += wb; cb += wb; lenB -= wb;
        if (lenB == 0) goto succeed;
      }
      a[dest++] = t[ct++];
      if (--lenA == 1) goto copy_b;
    }
    S.min_gallop++;
  }
succeed:
  if (lenA > 0) v8_copy(a + dest, t + ct, lenA);
  return;
copy_b:
  v8_copy(a + dest, a + cb, lenB);
  a[dest + lenB] = t[ct];
}
YM_BIG void v8_merge_high(V8Sort &S, int64_t baseA, int64_t lenA, int64_t baseB, int64_t lenB) {
  uint32_t *a = S.a, *t = S.t;
  v8_copy(t, a + baseB, lenB);
  int64_t dest = baseB + lenB - 1, ct = lenB - 1, ca = baseA + lenA - 1;
  a[dest--] = a[ca--];
  if (--lenA == 0) goto succeed;
  if (lenB == 1) goto copy_a;
  for (;;) {
    int64_t wa = 0, wb = 0;
    for (;;) {
      if (S.cmp(t[ct], a[ca]) < 0) {
        a[dest--] = a[ca--]; wa++; lenA--; wb = 0;
        if (lenA == 0) goto succeed;
        if (wa >= S.min_gallop) break;
      } else {
        a[dest--] = t[ct--]; wb++; lenB--; wa = 0;
        if (lenB == 1) goto copy_a;
        if (wb >= S.min_gallop) break;
      }
    }
    S.min_gallop++;
    bool first = true;
    while (wa >= 7 || wb >= 7 || first) {
      first = false;
      S.min_gallop = S.min_gallop - 1 > 1 ? S.min_gallop - 1 : 1;
      int64_t k = v8_gallop_right(S, a, t[ct], baseA, lenA, lenA - 1);
      wa = lenA - k;
      if (wa > 0) {
        dest -= wa; ca -= wa;
        v8_copy(a + dest + 1, a + ca + 1, wa);
        lenA -= wa;
        if (lenA == 0) goto succeed;
      }
      a[dest--] = t[ct--];
      if (--lenB == 1) goto copy_a;
      k = v8_gallop_left(S, t, a[ca], 0, lenB, lenB - 1);
      wb = lenB - k;
      if (wb > 0) {
        dest -= wb; ct -= wb;
        v8_copy(a + dest + 1, t + ct + 1, wb);
        lenB -= wb;
        if (lenB == 1) goto copy_a;
        if (lenB == 0) goto succeed;  // impossible for a consistent comparator
      }
      a[dest--] = a[ca--];
      if (--lenA == 0) goto succeed;
    }
    S.min_gallop++;
  }
succeed:
  if (lenB > 0) v8_copy(a + dest - (lenB - 1), t, lenB);
  return;
copy_a:
  dest -= lenA; ca -= lenA;
  v8_copy(a + dest + 1, a + ca + 1, lenA);
  a[dest] = t[ct];
}
YM_BIG void v8_merge_at(V8Sort &S, int i) {
  int64_t baseA = S.base[i], lenA = S.len[i], baseB = S.base[i + 1], lenB = S.len[i + 1];
  S.len[i] = (uint32_t)(lenA + lenB);
  if (i == S.nruns - 3) { S.base[i + 1] = S.base[i + 2]; S.len[i + 1] = S.len[i + 2]; }
  S.nruns--;
  const int64_t k = v8_gallop_right(S, S.a, S.a[baseB], baseA, lenA, 0);
  baseA += k;
  lenA -= k;
  if (lenA == 0) return;
  lenB = v8_gallop_left(S, S.a, S.a[baseA + lenA - 1], baseB, lenB, lenB - 1);
  if (lenB == 0) return;
  if (lenA <= lenB) v8_merge_low(S, baseA, lenA, baseB, lenB);
  else v8_merge_high(S, baseA, lenA, baseB, lenB);
}
YM_INL bool v8_run_inv(const V8Sort &S, int n) { return n < 2 || S.len[n - 2] > S.len[n - 1] + S.len[n]; }
YM_BIG void v8_sort(Reader *rs, uint32_t *a, uint32_t *tmp, uint32_t n) {
  if (n < 2) return;
  V8Sort S;
  S.rs = rs; S.a = a; S.t = tmp; S.nruns = 0; S.min_gallop = 7;
  int64_t remaining = n, low = 0;
  int64_t minrun = remaining, r = 0;
  while (minrun >= 64) { r |= minrun & 1; minrun >>= 1; }
  minrun += r;
  while (remaining != 0) {
    int64_t run;  // CountAndMakeRun(low, low + remaining)
    if (remaining == 1) {
      run = 1;
    } else {
      run = 2;
      const bool desc = S.cmp(a[low + 1], a[low]) < 0;
      uint32_t prev = a[low + 1];
      for (int64_t i = low + 2; i < low + remaining; i++) {
        const int o = S.cmp(a[i], prev);
        if (desc ? o >= 0 : o < 0) break;
        prev = a[i];
        run++;
      }
      if (desc)
        for (int64_t i = low, j = low + run - 1; i < j; i++, j--) { uint32_t x = a[i]; a[i] = a[j]; a[j] = x; }
    }
    if (run < minrun) {  // BinaryInsertionSort(low, low + run, low + forced)
      const int64_t forced = minrun < remaining ? minrun : remaining;
      for (int64_t start = low + run; start < low + forced; start++) {
        const uint32_t pivot = a[start];
        int64_t left = low, right = start;
        while (left < right) {
          const int64_t mid = left + ((right - left) >> 1);
          if (S.cmp(pivot, a[mid]) < 0) right = mid; else left = mid + 1;
        }
        for (int64_t p = start; p > left; p--) a[p] = a[p - 1];
        a[left] = pivot;
      }
      run = forced;
    }
    S.base[S.nruns] = (uint32_t)low;
    S.len[S.nruns] = (uint32_t)run;
    S.nruns++;
    while (S.nruns > 1) {  // MergeCollapse
      int m = S.nruns - 2;
      if (!v8_run_inv(S, m + 1) || !v8_run_inv(S, m)) {
        if (S.len[m - 1] < S.len[m + 1]) m--;
        v8_merge_at(S, m);
      } else if (S.len[m] <= S.len[m + 1]) {
        v8_merge_at(S, m);
      } else {
        break;
      }
    }
    low += run;
    remaining -= run;
  }
  while (S.nruns > 1) {  // MergeForceCollapse
    int m = S.nruns - 2;
    if (m > 0 && S.len[m - 1] < S.len[m + 1]) m--;
    v8_merge_at(S, m);
  }
}
// stable merge sort (initial order), bottom-up: V8's result whenever the comparator is consistent
YM_BIG void stable_sort(Reader *rs, uint32_t *a, uint32_t *t, uint32_t n) {
  int inc = 0;
  for (uint32_t w = 1; w < n; w *= 2) {
    for (uint32_t lo = 0; lo < n; lo += 2 * w) {
      uint32_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      uint32_t i = lo, j = mid, k = lo;
      while (i < mid && j < hi) t[k++] = rcmp(rs[a[j]], rs[a[i]], &inc) < 0 ? a[j++] : a[i++];
      while (i < mid) t[k++] = a[i++];
      while (j < hi) t[k++] = a[j++];
    }
    for (uint32_t i = 0; i < n; i++) a[i] = t[i];
  }
}

YM_BIG void merge_doc(Ctx &c, DocWS &ws, const uint64_t *upd_off, uint32_t u0, uint32_t k, uint32_t v2, int pass,
                      Layout &L, uint8_t *out) {
  Reader *rs = ws.rs;
  uint32_t *arr = ws.arr;
  uint64_t kused = 0;
  for (uint32_t i = 0; i < k && !c.err; i++) {
    reader_open(c, rs[i], upd_off[u0 + i], upd_off[u0 + i + 1] - upd_off[u0 + i], v2);
    reader_keys(c, rs[i], ws, kused);
  }
  for (uint32_t i = 0; i < k && !c.err; i++) { rs[i].filter = 1; reader_next(c, rs[i]); }
  if (c.err) return;
  Enc e;
  enc_init(e, v2);
  if (pass == 2) layout_bind(L, e, out);
  LW w;
  __builtin_memset(&w, 0, sizeof(LW));
  w.pass = (uint32_t)pass;
  w.parts = ws.parts;
  w.cap = ws.parts_cap;
  uint32_t na = 0;
  for (uint32_t i = 0; i < k; i++) if (rs[i].has_curr) arr[na++] = i;
  // first sort: exact V8 emulation below 64 readers; otherwise a stable sort (identical whenever the
  // comparator is consistent); afterwards the array stays sorted and only the head reader moves.
  bool literal = false;
  if (na < 64) { v8_sort(rs, arr, ws.tmp, na); }
  else stable_sort(rs, arr, ws.tmp, na);
  for (uint32_t i = 1; i < na; i++)
    if (rtie_bad(rs[arr[i - 1]], rs[arr[i]])) {
      literal = true;
      if (na >= 64) {  // the stable sort is not V8's order here: sort the input order as V8 does
        na = 0;
        for (uint32_t q = 0; q < k; q++) if (rs[q].has_curr) arr[na++] = q;
        v8_sort(rs, arr, ws.tmp, na);
      }
      break;
    }
  SStruct cur;
  bool has_cur = false;
  bool first_iter = true;
  while (!c.err) {
    if (!first_iter) {
      // re-sort after the head reader (arr[0]) moved
      if (literal) {
        uint32_t m = 0;
        for (uint32_t i = 0; i < na; i++) if (rs[arr[i]].has_curr) arr[m++] = arr[i];
        na = m;
        v8_sort(rs, arr, ws.tmp, na);
      } else {
        uint32_t R = arr[0];
        if (!rs[R].has_curr) {
          for (uint32_t i = 1; i < na; i++) arr[i - 1] = arr[i];
          na--;
        } else {
          // lower bound of R's key in arr[1..na): R goes before equal keys (stable, R was first)
          uint32_t lo = 1, hi = na;
          int inc = 0;
          while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (rcmp(rs[arr[mid]], rs[R], &inc) < 0) lo = mid + 1; else hi = mid;
          }
          bool bad = (lo < na && rtie_bad(rs[R], rs[arr[lo]])) || (lo > 1 && rtie_bad(rs[R], rs[arr[lo - 1]]));
          if (bad) {
            literal = true;
            v8_sort(rs, arr, ws.tmp, na);  // every reader still has a struct here
          } else {
            for (uint32_t i = 1; i < lo; i++) arr[i - 1] = arr[i];
            arr[lo - 1] = R;
          }
        }
      }
    }
    first_iter = false;
    if (na == 0) break;
    Reader &R = rs[arr[0]];
    int64_t first_client = R.curr.client;
    if (has_cur) {
      bool iterated = false;
      bool have = true;
      while (have && R.curr.clock + R.curr.len <= cur.clock + cur.len && R.curr.client >= cur.client) {
        have = reader_next(c, R);
        iterated = true;
      }
      if (c.err) return;
      if (!have || R.curr.client != first_client || (iterated && R.curr.clock > cur.clock + cur.len)) continue;
      SStruct s = R.curr;
      if (first_client != cur.client) {
        lw_write(c, w, e, cur, 0);
        cur = s;
        reader_next(c, R);
      } else if (cur.clock + cur.len < s.clock) {
        if (cur.kind == K_SKIP) {
          cur.len = s.clock + s.len - cur.clock;
        } else {
          lw_write(c, w, e, cur, 0);
          int64_t diff = s.clock - cur.clock - cur.len;
          SStruct sk;
          __builtin_memset(&sk, 0, sizeof(SStruct));
          sk.kind = K_SKIP;
          sk.client = first_client;
          sk.clock = cur.clock + cur.len;
          sk.len = diff;
          cur = sk;
        }
      } else {
        int64_t d = cur.clock + cur.len - s.clock;
        if (d > 0) {
          if (cur.kind == K_SKIP) cur.len -= d;
          else slice_struct(c, s, d);
        }
        bool merged = cur.kind != K_ITEM && cur.kind == s.kind;  // GC/Skip.mergeWith; Items never merge
        if (merged) cur.len += s.len;
        else {
          lw_write(c, w, e, cur, 0);
          cur = s;
          reader_next(c, R);
        }
      }
    } else {
      cur = R.curr;
      has_cur = true;
      reader_next(c, R);
    }
    while (!c.err && R.has_curr && R.curr.client == first_client && R.curr.clock == cur.clock + cur.len && R.curr.kind != K_SKIP) {
      lw_write(c, w, e, cur, 0);
      cur = R.curr;
      reader_next(c, R);
    }
  }
  if (c.err) return;
  if (has_cur) lw_write(c, w, e, cur, 0);
  lw_flush(c, w, e);
  if (c.err) return;
  // delete sets of all inputs, in input order
  uint64_t nds = 0;
  for (uint32_t i = 0; i < k && !c.err; i++) ds_gather(c, rs[i], ws.ds, ws.ds_cap, nds);
  if (c.err) return;
  uint64_t ds0 = e.rest.n;
  ds_emit(c, e, ws.ds, nds, ws.dsg, 1);
  e_flush_columns(c, e);
  if (pass == 1) {
    L.col[C_KC] = e.kc.n; L.col[C_CL] = e.cl.n; L.col[C_LC] = e.lc.n; L.col[C_RC] = e.rc.n; L.col[C_IN] = e.in.n;
    L.col[C_SB] = e.sb.n; L.col[C_SL] = e.sl.n; L.col[C_PI] = e.pi.n; L.col[C_TR] = e.tr.n; L.col[C_LN] = e.ln.n;
    L.nparts = w.nparts;
    L.parts_bytes = w.parts_bytes;
    L.ds_bytes = e.rest.n - ds0;
    layout_finish(L, v2);
  }
}

// ------------------------------------------------------------------------------------------------
// diffUpdateV2 (13.5.16 us@40707) for one document (one update + one encoded state vector)
// ------------------------------------------------------------------------------------------------
YM_BIG void diff_doc(Ctx &c, DocWS &ws, uint64_t uoff, uint64_t ulen, const uint8_t *svp, uint64_t svlen, uint32_t v2,
                     int pass, Layout &L, uint8_t *out) {
  // decodeStateVector (encoding.js:536-565): later entries override earlier ones
  Ctx cs = {0, svp};
  Rd sd = {0, svlen, 0};
  uint32_t ns = rd_vu(cs, sd);
  uint32_t nsv = 0;
  for (uint32_t i = 0; i < ns && !cs.err; i++) {
    int64_t client = rd_vu(cs, sd);
    int64_t clock = rd_vu(cs, sd);
    if (cs.err) break;
    uint32_t j = 0;
    while (j < nsv && ws.sv[2 * j] != client) j++;
    if (j == nsv) {
      if (nsv >= ws.sv_cap) { seterr(c, ST_RETRY); return; }
      ws.sv[2 * j] = client;
      nsv++;
    }
    ws.sv[2 * j + 1] = clock;
  }
  if (cs.err) seterr(c, cs.err);
  if (c.err) return;
  Enc e;
  enc_init(e, v2);
  if (pass == 2) layout_bind(L, e, out);
  LW w;
  __builtin_memset(&w, 0, sizeof(LW));
  w.pass = (uint32_t)pass;
  w.parts = ws.parts;
  w.cap = ws.parts_cap;
  Reader &r = ws.rs[0];
  reader_open(c, r, uoff, ulen, v2);
  { uint64_t kused = 0; reader_keys(c, r, ws, kused); }
  if (c.err) return;
  reader_next(c, r);
  int64_t last_client = -1, last_k = 0;
  while (!c.err && r.has_curr) {
    int64_t client = r.curr.client;
    int64_t k = 0;
    if (client == last_client) k = last_k;
    else {
      for (uint32_t j = 0; j < nsv; j++) if (ws.sv[2 * j] == client) k = ws.sv[2 * j + 1];
      last_client = client;
      last_k = k;
    }
    if (r.curr.kind == K_SKIP) { reader_next(c, r); continue; }
    if (r.curr.clock + r.curr.len > k) {
      int64_t off = k - r.curr.clock;
      if (off < 0) off = 0;
      lw_write(c, w, e, r.curr, off);
      reader_next(c, r);
      while (!c.err && r.has_curr && r.curr.client == client) { lw_write(c, w, e, r.curr, 0); reader_next(c, r); }
    } else {
      while (!c.err && r.has_curr && r.curr.client == client && r.curr.clock + r.curr.len <= k) reader_next(c, r);
    }
  }
  if (c.err) return;
  lw_flush(c, w, e);
  uint64_t nds = 0;
  ds_gather(c, r, ws.ds, ws.ds_cap, nds);
  if (c.err) return;
  uint64_t ds0 = e.rest.n;
  ds_emit(c, e, ws.ds, nds, ws.dsg, 0);
  e_flush_columns(c, e);
  if (pass == 1) {
    L.col[C_KC] = e.kc.n; L.col[C_CL] = e.cl.n; L.col[C_LC] = e.lc.n; L.col[C_RC] = e.rc.n; L.col[C_IN] = e.in.n;
    L.col[C_SB] = e.sb.n; L.col[C_SL] = e.sl.n; L.col[C_PI] = e.pi.n; L.col[C_TR] = e.tr.n; L.col[C_LN] = e.ln.n;
    L.nparts = w.nparts;
    L.parts_bytes = w.parts_bytes;
    L.ds_bytes = e.rest.n - ds0;
    layout_finish(L, v2);
  }
}

// ------------------------------------------------------------------------------------------------
// convertUpdateFormat (13.5.16 ms@41803): every struct, Skips included, re-written with offset 0 by a
// LazyStructWriter of the other format; readDeleteSet + writeDeleteSet.  v2 = the input format.
// ------------------------------------------------------------------------------------------------
YM_BIG void conv_doc(Ctx &c, DocWS &ws, uint64_t uoff, uint64_t ulen, uint32_t v2, int pass, Layout &L, uint8_t *out) {
  Enc e;
  enc_init(e, !v2);
  e.xfmt = 1;
  if (pass == 2) layout_bind(L, e, out);
  LW w;
  __builtin_memset(&w, 0, sizeof(LW));
  w.pass = (uint32_t)pass;
  w.parts = ws.parts;
  w.cap = ws.parts_cap;
  Reader &r = ws.rs[0];
  reader_open(c, r, uoff, ulen, v2);
  { uint64_t kused = 0; reader_keys(c, r, ws, kused); }
  if (c.err) return;
  reader_next(c, r);
  while (!c.err && r.has_curr) {
    lw_write(c, w, e, r.curr, 0);
    reader_next(c, r);
  }
  if (c.err) return;
  lw_flush(c, w, e);
  uint64_t nds = 0;
  ds_gather(c, r, ws.ds, ws.ds_cap, nds);
  if (c.err) return;
  uint64_t ds0 = e.rest.n;
  ds_emit(c, e, ws.ds, nds, ws.dsg, 0);
  e_flush_columns(c, e);
  if (pass == 1) {
    L.col[C_KC] = e.kc.n; L.col[C_CL] = e.cl.n; L.col[C_LC] = e.lc.n; L.col[C_RC] = e.rc.n; L.col[C_IN] = e.in.n;
    L.col[C_SB] = e.sb.n; L.col[C_SL] = e.sl.n; L.col[C_PI] = e.pi.n; L.col[C_TR] = e.tr.n; L.col[C_LN] = e.ln.n;
    L.nparts = w.nparts;
    L.parts_bytes = w.parts_bytes;
    L.ds_bytes = e.rest.n - ds0;
    layout_finish(L, !v2);
  }
}

// ------------------------------------------------------------------------------------------------
// encodeStateVectorFromUpdateV2 (13.5.16 os@37724): output vu(count) | (client, clock)*
// ------------------------------------------------------------------------------------------------
YM_BIG void sv_doc(Ctx &c, DocWS &ws, uint64_t uoff, uint64_t ulen, uint32_t v2, int pass, Layout &L, uint8_t *out) {
  Reader &r = ws.rs[0];
  reader_open(c, r, uoff, ulen, v2);
  { uint64_t kused = 0; reader_keys(c, r, ws, kused); }
  if (c.err) return;
  reader_next(c, r);
  if (c.err) return;
  Out o = {pass == 2 ? out : nullptr, 0};
  if (pass == 2) ovu(o, (int64_t)L.svcount);
  uint64_t cnt = 0;
  if (r.has_curr) {
    int64_t client = r.curr.client;
    bool stop = r.curr.clock != 0;
    int64_t clock = stop ? 0 : r.curr.clock + r.curr.len;
    for (bool have = true; have && !c.err; have = reader_next(c, r)) {
      if (client != r.curr.client) {
        if (clock != 0) { cnt++; ovu(o, client); ovu(o, clock); }
        client = r.curr.client;
        clock = 0;
        stop = r.curr.clock != 0;
      }
      if (r.curr.kind == K_SKIP) stop = true;
      if (!stop) clock = r.curr.clock + r.curr.len;
    }
    if (c.err) return;
    if (clock != 0) { cnt++; ovu(o, client); ovu(o, clock); }
  }
  if (pass == 1) {
    __builtin_memset(&L, 0, sizeof(Layout));
    L.svcount = cnt;
    L.total = vu_size(cnt) + o.n;
  }
}

// ------------------------------------------------------------------------------------------------
// parseUpdateMetaV2 (13.5.16 parseUpdateMeta / parseUpdateMetaV2): a LazyStructReader that keeps Skips;
// `from` takes a client's first clock when its section starts, `to` the end of its last struct when the
// next section starts (JS Maps: a client met again keeps its position and takes the new value).
// Output: from then to, each vu(count) | (client, clock)* in Map order.  ws.sv holds (client, from, to)
// triples.
// ------------------------------------------------------------------------------------------------
YM_INL void meta_put(Ctx &c, DocWS &ws, uint32_t &n, int64_t client, int64_t v, int slot) {
  uint32_t cap = (uint32_t)((2ull * ws.sv_cap) / 3);
  int64_t *t = ws.sv;
  for (uint32_t i = n; i-- > 0;) {  // the most recent section's client is the usual hit
    if (t[3 * i] == client) { t[3 * i + slot] = v; return; }
  }
  if (n >= cap) { seterr(c, ST_RETRY); return; }
  t[3 * n] = client; t[3 * n + 1] = 0; t[3 * n + 2] = 0;
  t[3 * n + slot] = v;
  n++;
}
YM_BIG void meta_doc(Ctx &c, DocWS &ws, uint64_t uoff, uint64_t ulen, uint32_t v2, int pass, Layout &L, uint8_t *out) {
  Reader &r = ws.rs[0];
  reader_open(c, r, uoff, ulen, v2);
  { uint64_t kused = 0; reader_keys(c, r, ws, kused); }
  r.lax = 1;
  if (c.err) return;
  reader_next(c, r);
  if (c.err) return;
  uint32_t n = 0;
  if (r.has_curr) {
    int64_t client = r.curr.client, clock = r.curr.clock;
    meta_put(c, ws, n, client, clock, 1);
    for (bool have = true; have && !c.err; have = reader_next(c, r)) {
      if (client != r.curr.client) {
        meta_put(c, ws, n, client, clock, 2);
        meta_put(c, ws, n, r.curr.client, r.curr.clock, 1);
        client = r.curr.client;
      }
      clock = r.curr.clock + r.curr.len;
    }
    if (c.err) return;
    meta_put(c, ws, n, client, clock, 2);
    if (c.err) return;
  }
  Out o = {pass == 2 ? out : nullptr, 0};
  for (int slot = 1; slot <= 2; slot++) {
    ovu(o, (int64_t)n);
    for (uint32_t i = 0; i < n; i++) { ovu(o, ws.sv[3 * i]); ovu(o, ws.sv[3 * i + slot]); }
  }
  if (pass == 1) {
    __builtin_memset(&L, 0, sizeof(Layout));
    L.svcount = n;
    L.total = o.n;
  }
}

// ------------------------------------------------------------------------------------------------
// PermanentUserData's delete-set merge (PermanentUserData.js:49-54): k encoded delete sets (DSEncoderV1
// / DSEncoderV2 rest bytes, as encodeSnapshot[V2] writes them, Snapshot.js:84-101) read by
// readDeleteSet, merged by mergeDeleteSets (13.5.16 he@10482 + le@10242 union), written by
// writeDeleteSet.  Input i of the document is the byte range [upd_off[u0+i], upd_off[u0+i+1]).
// ------------------------------------------------------------------------------------------------
YM_BIG void dsmerge_doc(Ctx &c, DocWS &ws, const uint64_t *upd_off, uint32_t u0, uint32_t k, uint32_t v2, int pass,
                        Layout &L, uint8_t *out, bool ref) {
  uint64_t nds = 0;
  for (uint32_t i = 0; i < k && !c.err; i++) {
    Reader &r = ws.rs[0];
    __builtin_memset(&r, 0, sizeof(Reader));
    r.rest.start = upd_off[u0 + i];
    r.rest.len = upd_off[u0 + i + 1] - upd_off[u0 + i];
    r.v2 = v2;
    ds_gather(c, r, ws.ds, ws.ds_cap, nds);
  }
  if (c.err) return;
  Enc e;
  enc_init(e, v2);
  e.rest.p = pass == 2 ? out : nullptr;
  ds_emit(c, e, ws.ds, nds, ws.dsg, ref ? 2 : 1);
  if (c.err) return;
  if (pass == 1) {
    __builtin_memset(&L, 0, sizeof(Layout));
    L.ds_bytes = e.rest.n;
    L.total = e.rest.n;
  }
}

// ------------------------------------------------------------------------------------------------
// Snapshot codec (Snapshot.js:84-124): encodeSnapshot[V2](decodeSnapshot[V2](bytes)) -- normalisation and
// V1 <-> V2 conversion of encoded snapshots.  decode: readDeleteSet (DeleteSet.js:241-256: a client's
// entries are appended to its first appearance, a client with no entries is not added; V2 clocks are
// delta-coded per entry run, lengths stored minus one, UpdateDecoder.js DSDecoderV2) then readStateVector
// (encoding.js:536-545: Map.set, a repeated client keeps its first position and takes the last clock).
// encode: writeDeleteSet (DeleteSet.js:219-232, Map order; DSEncoderV2.writeDsLen(0) throws
// 'Unexpected case', UpdateEncoder.js:255-261) then writeStateVector (encoding.js:572-579).  V2 clock
// deltas of out-of-order entries are negative and go through lib0 writeVarUint as JS numbers (ovu).
// Workspace: the delete set's client runs in ws.ds (client, entries, byte position), the state vector's
// pairs in ws.sv.
// ------------------------------------------------------------------------------------------------
YM_INL void snap_items(Ctx &c, Out &o, uint64_t uoff, uint64_t ulen, uint64_t pos, uint32_t count, uint32_t v2in,
                       uint32_t v2out, int64_t &cur_out) {
  Rd d = {uoff, ulen, pos};
  int64_t cur_in = 0;  // DSDecoderV2.dsCurrVal, reset per client run (readDeleteSet)
  for (uint32_t q = 0; q < count && !c.err; q++) {
    int64_t clock, len;
    if (v2in) {
      cur_in += rd_vu(c, d);
      clock = cur_in;
      len = (int64_t)rd_vu(c, d) + 1;
      cur_in += len;
    } else {
      clock = rd_vu(c, d);
      len = rd_vu(c, d);
    }
    if (c.err) return;
    if (v2out) {
      ovu(o, clock - cur_out);
      cur_out = clock;
      if (len == 0) { seterr(c, ST_UNEXPECTED); return; }
      ovu(o, len - 1);
      cur_out += len;
    } else {
      ovu(o, clock);
      ovu(o, len);
    }
  }
}
YM_BIG void snap_doc(Ctx &c, DocWS &ws, uint64_t uoff, uint64_t ulen, uint32_t v2in, uint32_t v2out, int pass, Layout &L,
                     uint8_t *out) {
  Rd d = {uoff, ulen, 0};
  const uint32_t ncl = rd_vu(c, d);
  uint64_t nrun = 0;
  for (uint32_t i = 0; i < ncl && !c.err; i++) {
    const uint32_t client = rd_vu(c, d);
    const uint32_t m = rd_vu(c, d);
    if (c.err) return;
    if (m > 0) {
      if (nrun >= ws.ds_cap) { seterr(c, ST_RETRY); return; }
      DSE &e = ws.ds[nrun++];
      e.client = client;
      e.seq = m;
      e.clock = (int64_t)d.pos;
    }
    for (uint32_t q = 0; q < m && !c.err; q++) { rd_vu(c, d); rd_vu(c, d); }
  }
  if (c.err) return;
  const uint32_t nsv = rd_vu(c, d);
  uint32_t npair = 0;
  for (uint32_t i = 0; i < nsv && !c.err; i++) {
    const uint32_t client = rd_vu(c, d);
    const uint32_t clock = rd_vu(c, d);
    if (c.err) return;
    if (npair >= ws.sv_cap) { seterr(c, ST_RETRY); return; }
    ws.sv[2 * npair] = client;
    ws.sv[2 * npair + 1] = clock;
    npair++;
  }
  if (c.err) return;
  Out o = {pass == 2 ? out : nullptr, 0};
  // writeDeleteSet: clients in first-appearance order, each with the entries of all its runs
  uint64_t ndist = 0;
  for (uint64_t r = 0; r < nrun; r++) {
    bool first = true;
    for (uint64_t t = 0; t < r && first; t++) first = ws.ds[t].client != ws.ds[r].client;
    ndist += first;
  }
  ovu(o, (int64_t)ndist);
  for (uint64_t r = 0; r < nrun && !c.err; r++) {
    bool first = true;
    for (uint64_t t = 0; t < r && first; t++) first = ws.ds[t].client != ws.ds[r].client;
    if (!first) continue;
    int64_t total = 0;
    for (uint64_t t = r; t < nrun; t++) if (ws.ds[t].client == ws.ds[r].client) total += ws.ds[t].seq;
    ovu(o, ws.ds[r].client);
    ovu(o, total);
    int64_t cur_out = 0;  // DSEncoderV2.resetDsCurVal per client
    for (uint64_t t = r; t < nrun && !c.err; t++)
      if (ws.ds[t].client == ws.ds[r].client)
        snap_items(c, o, uoff, ulen, (uint64_t)ws.ds[t].clock, ws.ds[t].seq, v2in, v2out, cur_out);
  }
  if (c.err) return;
  // writeStateVector: Map order, the last clock of each client
  uint32_t nd = 0;
  for (uint32_t i = 0; i < npair; i++) {
    bool first = true;
    for (uint32_t t = 0; t < i && first; t++) first = ws.sv[2 * t] != ws.sv[2 * i];
    nd += first;
  }
  ovu(o, nd);
  for (uint32_t i = 0; i < npair; i++) {
    bool first = true;
    for (uint32_t t = 0; t < i && first; t++) first = ws.sv[2 * t] != ws.sv[2 * i];
    if (!first) continue;
    int64_t clock = ws.sv[2 * i + 1];
    for (uint32_t t = i + 1; t < npair; t++) if (ws.sv[2 * t] == ws.sv[2 * i]) clock = ws.sv[2 * t + 1];
    ovu(o, ws.sv[2 * i]);
    ovu(o, clock);
  }
  if (pass == 1) {
    __builtin_memset(&L, 0, sizeof(Layout));
    L.total = o.n;
  }
}

// ------------------------------------------------------------------------------------------------
// The general path's per-document entry (k_general in ym_general.hip; the test-only host build in
// tests/native/core_host.cpp runs the very same function on the CPU)
// ------------------------------------------------------------------------------------------------
enum : uint32_t { OP_MERGE = 0, OP_DIFF = 1, OP_SV = 2, OP_CONV = 3, OP_META = 4, OP_DSMERGE = 5, OP_SNAP = 6, OP_COMPACT = 7 };

struct GeneralWsSize {
  uint64_t rs, arr, parts, ds, dsg, sv, keys, total;
  uint32_t mul;
  uint64_t keys_cap;
  uint32_t parts_cap, sv_cap;
  uint64_t ds_cap;
};
YM_INL uint64_t al16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }
YM_INL GeneralWsSize general_ws_size(uint32_t k, uint64_t bytes, uint32_t parts_mul, uint64_t svbytes, uint32_t v2) {
  GeneralWsSize z;
  z.rs = al16((uint64_t)(k ? k : 1) * sizeof(Reader));
  z.arr = al16((uint64_t)(k + 1) * 4);
  z.parts_cap = (uint32_t)((2ull * k + 16) * parts_mul);
  z.parts = al16((uint64_t)z.parts_cap * sizeof(PartRec));
  z.ds_cap = bytes / 2 + 2;  // every delete-set entry occupies >= 2 input bytes
  z.ds = al16(z.ds_cap * sizeof(DSE));
  z.dsg = al16(z.ds_cap * sizeof(DSG));
  z.sv_cap = (uint32_t)(svbytes / 2 + 2);
  z.sv = al16((uint64_t)z.sv_cap * 16);
  z.mul = parts_mul;
  // readKey caches (V2 only): a small start, grown by the retry rounds for key-heavy documents
  z.keys_cap = v2 ? (bytes / 64 + 4ull * (k ? k : 1)) * parts_mul : 0;
  z.keys = al16(z.keys_cap * sizeof(Span));
  z.total = z.rs + 2 * z.arr + z.parts + z.ds + z.dsg + z.sv + z.keys;
  return z;
}
// the state-vector table: diff = the decoded state vector; meta = (client, from, to) triples, at most one
// client per update byte
YM_INL uint64_t general_sv_bytes(uint32_t op, uint64_t svlen, uint64_t bytes) {
  if (op == OP_DIFF) return svlen;
  if (op == OP_META) return 3 * bytes + 6;
  if (op == OP_SNAP) return bytes + 4;  // state-vector pairs: >= 2 bytes each
  return 0;
}
YM_INL void general_carve(uint8_t *p, const GeneralWsSize &z, DocWS &w) {
  w.rs = (Reader *)p; p += z.rs;
  w.arr = (uint32_t *)p; p += z.arr;
  w.tmp = (uint32_t *)p; p += z.arr;
  w.parts = (PartRec *)p; p += z.parts; w.parts_cap = z.parts_cap;
  w.ds = (DSE *)p; p += z.ds; w.ds_cap = z.ds_cap;
  w.dsg = (DSG *)p; p += z.dsg;
  w.sv = (int64_t *)p; p += z.sv; w.sv_cap = z.sv_cap;
  w.keys = (Span *)p; w.keys_cap = z.keys_cap;
  w.mul = z.mul;
}
// One document, pass 1 (sizes into L) or 2 (writes to out).  Document = updates u0 .. u0+k-1 of the
// arena (upd_off absolute); sv = its encoded state vector (diff).  Status in c.err.
// v2: 1 = V2 encoding; bit 8 (ym_ds_merge): the reference's adjacency-only delete-set coalescing;
// bit 9 (ym_snapshot): V2 output encoding
YM_BIG void general_doc(Ctx &c, DocWS &w, uint32_t op, uint32_t v2f, const uint64_t *upd_off, uint32_t u0, uint32_t k,
                        const uint8_t *sv, uint64_t svlen, int pass, Layout &L, uint8_t *out) {
  const uint32_t v2 = v2f & 1;
  if (op == OP_MERGE) {
    if (k == 1) {  // `if (updates.length === 1) return updates[0]`
      uint64_t n = upd_off[u0 + 1] - upd_off[u0];
      if (pass == 1) { __builtin_memset(&L, 0, sizeof(Layout)); L.total = n; }
      else for (uint64_t b = 0; b < n; b++) out[b] = c.A[upd_off[u0] + b];
    } else {
      merge_doc(c, w, upd_off, u0, k, v2, pass, L, out);
    }
    return;
  }
  if (op == OP_DSMERGE) { dsmerge_doc(c, w, upd_off, u0, k, v2, pass, L, out, (v2f >> 8) & 1); return; }
  if (k != 1) { c.err = ST_UNEXPECTED; return; }
  const uint64_t uoff = upd_off[u0], ulen = upd_off[u0 + 1] - upd_off[u0];
  if (op == OP_DIFF) diff_doc(c, w, uoff, ulen, sv, svlen, v2, pass, L, out);
  else if (op == OP_META) meta_doc(c, w, uoff, ulen, v2, pass, L, out);
  else if (op == OP_CONV) conv_doc(c, w, uoff, ulen, v2, pass, L, out);
  else if (op == OP_SNAP) snap_doc(c, w, uoff, ulen, v2, (v2f >> 9) & 1, pass, L, out);
  else sv_doc(c, w, uoff, ulen, v2, pass, L, out);
}

}  // namespace ym
