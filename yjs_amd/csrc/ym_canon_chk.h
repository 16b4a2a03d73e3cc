// ym_canon_chk.h -- canonical-form checks of nested payloads for the verbatim-copy paths (LDS merges, the
// streamed and chunked diff / state-vector walkers): a payload may be copied byte for byte only when
// re-encoding it the way yjs does would give the same bytes.
//   any_canon_ptr   one lib0 `any` value (ContentAny elements; V2 ContentEmbed / ContentFormat values):
//                   writeAny(readAny(bytes)) == bytes, scalars and Uint8Array / BigInt64 / nested arrays and
//                   objects (lib0 0.2.42 readAny / writeAny)
//   json_canon_ptr  one V1 JSON text (ContentEmbed / ContentFormat values, readJSON / writeJSON):
//                   JSON.stringify(JSON.parse(text)) == text, for literals, integers of up to 15 digits,
//                   strings without escapes or control characters, arrays and objects
// Both read through a generic pointer (LDS or global) and decline (return false) anything outside the
// subset they can decide: the general path then re-encodes exactly (ym_canon.h).  An object's keys must not
// start with a digit (array-index keys are re-ordered by Object.keys / JSON.stringify), must not repeat
// (the later value wins at the earlier position) and must not be `__proto__` (readAny sets the prototype).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ymk {
namespace cchk {

// Nesting depth and open-object keys: the containers' state lives in registers (every array index below is a
// select over the unrolled entries, so nothing is placed in scratch memory); deeper or wider payloads decline.
constexpr uint32_t DEPTH = 4, KEYS = 8;
template <uint32_t N>
__device__ __forceinline__ uint32_t rsel(const uint32_t (&a)[N], uint32_t i) {
  uint32_t v = a[0];
#pragma unroll
  for (uint32_t k = 1; k < N; k++) v = i == k ? a[k] : v;
  return v;
}
template <uint32_t N>
__device__ __forceinline__ void wsel(uint32_t (&a)[N], uint32_t i, uint32_t v) {
#pragma unroll
  for (uint32_t k = 0; k < N; k++) a[k] = i == k ? v : a[k];
}

__device__ __forceinline__ bool bytes_eq(const uint8_t *b, uint32_t p, uint32_t q, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (b[p + i] != b[q + i]) return false;
  return true;
}
// canonical varuint < 2^32 at p (lib0 readVarUint): value, *p advanced; false past e / non-canonical
__device__ __forceinline__ bool vu(const uint8_t *b, uint32_t &p, uint32_t e, uint32_t &v) {
  v = 0;
  for (uint32_t k = 0; k < 5; k++) {
    if (p >= e) return false;
    const uint32_t x = b[p++];
    v |= (x & 127u) << (7 * k);
    if (x < 128) return !(k > 0 && x == 0) && !(k == 4 && x > 15);
  }
  return false;
}
// strict UTF-8 of [p, p + n) (lib0 readVarString's decodeURIComponent(escape(..)))
__device__ __forceinline__ bool utf8_ok(const uint8_t *b, uint32_t p, uint32_t n) {
  const uint32_t e = p + n;
  while (p < e) {
    const uint32_t x = b[p];
    if (x < 0x80) { p++; continue; }
    uint32_t len, cp, mn;
    if ((x & 0xE0) == 0xC0) { len = 2; cp = x & 0x1F; mn = 0x80; }
    else if ((x & 0xF0) == 0xE0) { len = 3; cp = x & 0x0F; mn = 0x800; }
    else if ((x & 0xF8) == 0xF0) { len = 4; cp = x & 0x07; mn = 0x10000; }
    else return false;
    if (p + len > e) return false;
    for (uint32_t q = 1; q < len; q++) {
      const uint32_t y = b[p + q];
      if ((y & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (y & 0x3F);
    }
    if (cp < mn || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
    p += len;
  }
  return true;
}
// an object key (bytes [p, p + n)) acceptable for a verbatim copy, and not among the open object's keys
// (entries k0 .. nk - 1 of kp / kl)
__device__ __forceinline__ bool key_ok(const uint8_t *b, uint32_t p, uint32_t n, const uint32_t (&kp)[KEYS],
                                       const uint32_t (&kl)[KEYS], uint32_t k0, uint32_t nk) {
  if (n > 0 && b[p] >= '0' && b[p] <= '9') return false;
  if (n == 9 && b[p] == '_' && b[p + 1] == '_' && b[p + 2] == 'p' && b[p + 3] == 'r' &&
      b[p + 4] == 'o' && b[p + 5] == 't' && b[p + 6] == 'o' && b[p + 7] == '_' && b[p + 8] == '_')
    return false;
  bool dup = false;
#pragma unroll
  for (uint32_t k = 0; k < KEYS; k++)
    if (k >= k0 && k < nk && kl[k] == n) dup |= bytes_eq(b, kp[k], p, n);
  return !dup;
}

// One `any` value at p (< e): true and *end = its end when the bytes are what writeAny emits for it.
__device__ __forceinline__ bool any_canon_ptr(const uint8_t *b, uint32_t p, uint32_t e, uint32_t *end) {
  uint32_t rem[DEPTH] = {}, obj[DEPTH] = {}, kp[KEYS] = {}, kl[KEYS] = {};
  uint32_t depth = 0, nk = 0;
  for (;;) {
    if (depth > 0 && rsel(obj, depth - 1)) {  // an object: a key before each value
      uint32_t n;
      if (!vu(b, p, e, n) || n > e - p) return false;
      if (nk >= KEYS || !key_ok(b, p, n, kp, kl, rsel(obj, depth - 1) - 1, nk) || !utf8_ok(b, p, n)) return false;
      wsel(kp, nk, p);
      wsel(kl, nk, n);
      nk++;
      p += n;
    }
    if (p >= e) return false;
    const uint32_t tag = b[p++];
    switch (tag) {
      case 127: case 126: case 121: case 120: break;  // undefined, null, false, true
      case 125: {  // varInt: minimal, int32 range when positive (larger is written as a float)
        if (p >= e) return false;
        uint32_t x = b[p++];
        uint64_t mag = x & 63;
        const bool neg = (x & 64) != 0;
        uint32_t s = 6, nb = 1;
        while (x & 128) {
          if (p >= e || s > 34) return false;
          x = b[p++];
          mag |= (uint64_t)(x & 127) << s;
          s += 7;
          nb++;
        }
        if ((nb > 1 && x == 0) || (!neg && mag > 2147483647ull) || mag > 0xffffffffull) return false;
        break;
      }
      case 124: {  // float32: not NaN, not an integer writeAny would write as a varInt
        if (e - p < 4) return false;
        const uint32_t u = ((uint32_t)b[p] << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
        const float f = __uint_as_float(u);
        if (f != f || (truncf(f) == f && (double)f <= 2147483647.0)) return false;
        p += 4;
        break;
      }
      case 123: {  // float64: not a small integer, not float32-exact
        if (e - p < 8) return false;
        uint64_t u = 0;
        for (int k = 0; k < 8; k++) u = (u << 8) | b[p + k];
        const double x = __longlong_as_double((long long)u);
        if (x == x && ((trunc(x) == x && x <= 2147483647.0) || (double)(float)x == x)) return false;
        p += 8;
        break;
      }
      case 122:  // BigInt64: 8 bytes as they are
        if (e - p < 8) return false;
        p += 8;
        break;
      case 119: {  // string
        uint32_t n;
        if (!vu(b, p, e, n) || n > e - p || !utf8_ok(b, p, n)) return false;
        p += n;
        break;
      }
      case 116: {  // Uint8Array
        uint32_t n;
        if (!vu(b, p, e, n) || n > e - p) return false;
        p += n;
        break;
      }
      case 117: case 118: {  // array / object: count, then the values
        uint32_t n;
        if (!vu(b, p, e, n) || n > e - p || depth >= DEPTH) return false;
        if (n > 0) {
          wsel(rem, depth, n);
          wsel(obj, depth, tag == 118 ? nk + 1 : 0);
          depth++;
          continue;
        }
        break;
      }
      default: return false;
    }
    while (depth > 0) {  // a value completed: close the containers it finished
      const uint32_t r = rsel(rem, depth - 1) - 1;
      wsel(rem, depth - 1, r);
      if (r > 0) break;
      depth--;
      const uint32_t o = rsel(obj, depth);
      if (o) nk = o - 1;
    }
    if (depth == 0) { *end = p; return true; }
  }
}

// a JSON string token at p (a quote): no escapes, no control characters; *q = past its closing quote
__device__ __forceinline__ bool jstr(const uint8_t *b, uint32_t p, uint32_t e, uint32_t &q) {
  if (p >= e || b[p] != '"') return false;
  for (q = p + 1; q < e; q++) {
    const uint32_t x = b[q];
    if (x == '"') { q++; return true; }
    if (x == '\\' || x < 0x20) return false;
  }
  return false;
}
// The V1 JSON text [p, p + n) (already UTF-8-validated by the caller) in the form JSON.stringify gives.
__device__ __forceinline__ bool json_canon_ptr(const uint8_t *b, uint32_t p, uint32_t n) {
  const uint32_t e = p + n;
  uint32_t obj[DEPTH] = {}, kp[KEYS] = {}, kl[KEYS] = {};
  uint32_t depth = 0, nk = 0;
  for (;;) {
    if (depth > 0 && rsel(obj, depth - 1)) {  // key ':'
      uint32_t q;
      if (!jstr(b, p, e, q) || q >= e || b[q] != ':') return false;
      const uint32_t kn = q - p - 2;
      if (nk >= KEYS || !key_ok(b, p + 1, kn, kp, kl, rsel(obj, depth - 1) - 1, nk)) return false;
      wsel(kp, nk, p + 1);
      wsel(kl, nk, kn);
      nk++;
      p = q + 1;
    }
    if (p >= e) return false;
    const uint32_t x = b[p];
    if (x == 't') {
      if (e - p < 4 || b[p + 1] != 'r' || b[p + 2] != 'u' || b[p + 3] != 'e') return false;
      p += 4;
    } else if (x == 'f') {
      if (e - p < 5 || b[p + 1] != 'a' || b[p + 2] != 'l' || b[p + 3] != 's' || b[p + 4] != 'e') return false;
      p += 5;
    } else if (x == 'n') {
      if (e - p < 4 || b[p + 1] != 'u' || b[p + 2] != 'l' || b[p + 3] != 'l') return false;
      p += 4;
    } else if (x == '"') {
      uint32_t q;
      if (!jstr(b, p, e, q)) return false;
      p = q;
    } else if (x == '-' || (x >= '0' && x <= '9')) {  // an integer: -?(0|[1-9][0-9]{0,14}), not -0
      uint32_t q = p + (x == '-');
      if (q >= e || b[q] < '0' || b[q] > '9') return false;
      if (b[q] == '0') {
        if (x == '-') return false;
        q++;
      } else {
        const uint32_t q0 = q;
        while (q < e && b[q] >= '0' && b[q] <= '9') q++;
        if (q - q0 > 15) return false;
      }
      if (q < e && (b[q] == '.' || b[q] == 'e' || b[q] == 'E')) return false;  // fractions, exponents: general path
      p = q;
    } else if (x == '[' || x == '{') {
      if (depth >= DEPTH || e - p < 2) return false;
      if (b[p + 1] == (x == '[' ? ']' : '}')) {
        p += 2;  // an empty container
      } else {
        wsel(obj, depth, x == '{' ? nk + 1 : 0);
        depth++;
        p++;
        continue;
      }
    } else {
      return false;
    }
    for (;;) {  // after a value: ',' (next element) or the closing bracket
      if (depth == 0) return p == e;
      if (p >= e) return false;
      if (b[p] == ',') { p++; break; }
      if (b[p] != (rsel(obj, depth - 1) ? '}' : ']')) return false;
      p++;
      depth--;
      const uint32_t o = rsel(obj, depth);
      if (o) nk = o - 1;
    }
  }
}

}  // namespace cchk
}  // namespace ymk
