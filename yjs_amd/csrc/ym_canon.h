// ym_canon.h -- canonical re-encoding of payload values (general path; included by ym_core.h).
//
// yjs never copies a payload value: it decodes it to a JavaScript value and encodes that again.
//   ContentAny elements, V2 embed / format values .... readAny -> writeAny            (lib0 any, G_ANY -> T_ANY)
//   V1 embed / format texts, ContentJSON elements .... JSON.parse -> JSON.stringify   (G_JSON -> T_JSON)
//   convertUpdateFormat V1 -> V2 (embed / format) ..... JSON.parse -> writeAny         (G_JSON -> T_ANY)
//   convertUpdateFormat V2 -> V1 (embed / format) ..... readAny -> JSON.stringify      (G_ANY -> T_JSONANY)
//   ContentDoc options ................................ readAny -> new Doc({guid, ...opts}) -> re-derived opts
// (ContentAny.js:80-87, ContentJSON.js:83-90, ContentEmbed.js:80-82, ContentFormat.js:86-89,
// ContentDoc.js:116-135, UpdateEncoder.js:217-219 writeJSON / UpdateDecoder.js readJSON, 13.5.16
// convertUpdateFormat ms@41803.)  The readers copy a payload whose bytes are already what this
// re-encoding yields (the common case: yjs wrote them); a payload that is not is flagged and written
// through these routines instead, so the output is byte-identical to yjs's either way.
//
// JavaScript semantics reproduced: numbers are binary64 (ym_num.h: JSON.parse rounding, Number::toString),
// writeAny's int / float32 / float64 choice, strings are UTF-16 (surrogate pairs; a lone surrogate makes
// writeVarString throw URIError and is escaped \udxxx by JSON.stringify), object keys follow
// OrdinaryOwnPropertyKeys (array-index keys ascending, then first-insertion order, the last duplicate's
// value), readAny's `obj[key] = v` never creates an own "__proto__" key (JSON.parse does), and
// JSON.stringify drops undefined object members, writes null for undefined array elements and a
// Uint8Array as an object of index keys, and throws TypeError on a bigint.
//
// The input was validated by the reader (grammar, UTF-8, depth), so these routines only navigate it.
// Objects are walked by re-scanning their entries (no workspace): quadratic in the entry count, which
// is small for the values yjs documents carry.
#pragma once
#include "ym_num.h"

namespace ym {

enum : uint8_t { G_ANY = 0, G_JSON = 1 };
enum : uint8_t { T_ANY = 0, T_JSON = 1, T_JSONANY = 2 };

// ------------------------------------------------------------------------------------------------
// output sinks (anything with put(byte)): SinkOut (ym_core.h: an Out, counting or writing), or a UTF-8 /
// UTF-16 length counter
// ------------------------------------------------------------------------------------------------
struct SinkLen {
  uint64_t bytes, u16;
  YM_INL void put(uint32_t b) { bytes++; u16 += ((b & 0xC0) != 0x80) + (b >= 0xF0 ? 1 : 0); }
};
template <class S> YM_INL void s_vu(S &s, uint64_t v) {
  while (v > 127) { s.put(0x80 | (uint32_t)(v & 127)); v = (uint32_t)v >> 7; }
  s.put((uint32_t)v);
}
template <class S> YM_INL void s_ascii(S &s, const char *t) {
  while (*t) s.put((uint8_t)*t++);
}

// ------------------------------------------------------------------------------------------------
// source navigation (validated input)
// ------------------------------------------------------------------------------------------------
YM_INL uint32_t cv_vu(const uint8_t *A, uint64_t &p) {
  uint32_t s = 0;
  unsigned n = 0;
  for (;;) {
    const uint32_t b = A[p++];
    s |= (b & 127) << (n & 31);
    n += 7;
    if (b < 128) return s;
  }
}
// end of one lib0 `any` value
YM_INL uint64_t any_end(const uint8_t *A, uint64_t p) {
  uint32_t left[YM_ANY_DEPTH + 1];
  uint8_t obj[YM_ANY_DEPTH + 1];
  int sp = 0;
  for (;;) {
    const int tag = A[p++];
    switch (tag) {
      case 125: while (A[p] & 0x80) p++; p++; break;
      case 124: p += 4; break;
      case 123: case 122: p += 8; break;
      case 119: case 116: { const uint32_t L = cv_vu(A, p); p += L; break; }
      case 118: case 117: {
        const uint32_t n = cv_vu(A, p);
        if (n && sp <= YM_ANY_DEPTH) { left[sp] = n; obj[sp] = tag == 118; sp++; }
        break;
      }
      default: break;
    }
    for (;;) {
      if (sp == 0) return p;
      if (left[sp - 1] == 0) { sp--; continue; }
      left[sp - 1]--;
      if (obj[sp - 1]) { const uint32_t L = cv_vu(A, p); p += L; }  // the entry's key
      break;
    }
  }
}
YM_INL bool js_is_ws(uint8_t ch) { return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r'; }
YM_INL uint64_t js_ws(const uint8_t *A, uint64_t p, uint64_t end) {
  while (p < end && js_is_ws(A[p])) p++;
  return p;
}
YM_INL uint64_t js_str_end(const uint8_t *A, uint64_t p) {  // p at '"': returns the position after the closing quote
  p++;
  for (;;) {
    const uint8_t ch = A[p++];
    if (ch == '"') return p;
    if (ch == '\\') p++;
  }
}
YM_INL uint64_t js_end(const uint8_t *A, uint64_t p, uint64_t end) {  // end of one JSON value starting at p
  uint8_t ch = A[p];
  if (ch == '"') return js_str_end(A, p);
  if (ch == '{' || ch == '[') {
    int depth = 0;
    for (;;) {
      ch = A[p];
      if (ch == '"') { p = js_str_end(A, p); continue; }
      p++;
      if (ch == '{' || ch == '[') depth++;
      else if ((ch == '}' || ch == ']') && --depth == 0) return p;
    }
  }
  while (p < end) {
    ch = A[p];
    if ((ch >= '0' && ch <= '9') || ch == '-' || ch == '+' || ch == '.' || (ch >= 'a' && ch <= 'z') || ch == 'E') p++;
    else break;
  }
  return p;
}

// ------------------------------------------------------------------------------------------------
// strings as UTF-16 code-unit streams
// ------------------------------------------------------------------------------------------------
struct U16 {
  const uint8_t *A;
  uint64_t p, end;
  int32_t pend;  // the low surrogate of a 4-byte UTF-8 character, still to be returned
  uint8_t json;  // JSON string body (escapes) or raw UTF-8
};
YM_INL U16 u16_any(const uint8_t *A, uint64_t p) {  // p at a varString (length prefix)
  const uint32_t L = cv_vu(A, p);
  U16 u = {A, p, p + L, -1, 0};
  return u;
}
YM_INL U16 u16_json(const uint8_t *A, uint64_t p) {  // p at the opening quote
  const uint64_t e = js_str_end(A, p);
  U16 u = {A, p + 1, e - 1, -1, 1};
  return u;
}
YM_INL U16 u16_utf8(const uint8_t *A, uint64_t off, uint64_t n) {
  U16 u = {A, off, off + n, -1, 0};
  return u;
}
YM_INL int hexv(uint8_t h) {
  return h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10 : h - 'A' + 10;
}
YM_INL int32_t u16_next(U16 &it) {
  if (it.pend >= 0) { const int32_t v = it.pend; it.pend = -1; return v; }
  if (it.p >= it.end) return -1;
  const uint32_t b = it.A[it.p];
  if (it.json && b == '\\') {
    const uint8_t e = it.A[it.p + 1];
    it.p += 2;
    switch (e) {
      case 'b': return 8;
      case 'f': return 12;
      case 'n': return 10;
      case 'r': return 13;
      case 't': return 9;
      case 'u': {
        const int32_t v = (hexv(it.A[it.p]) << 12) | (hexv(it.A[it.p + 1]) << 8) | (hexv(it.A[it.p + 2]) << 4) |
                          hexv(it.A[it.p + 3]);
        it.p += 4;
        return v;
      }
      default: return e;  // \" \\ \/
    }
  }
  if (b < 0x80) { it.p++; return (int32_t)b; }
  if (b < 0xE0) {
    const int32_t cp = ((b & 31) << 6) | (it.A[it.p + 1] & 63);
    it.p += 2;
    return cp;
  }
  if (b < 0xF0) {
    const int32_t cp = ((b & 15) << 12) | ((it.A[it.p + 1] & 63) << 6) | (it.A[it.p + 2] & 63);
    it.p += 3;
    return cp;
  }
  int32_t cp = ((b & 7) << 18) | ((it.A[it.p + 1] & 63) << 12) | ((it.A[it.p + 2] & 63) << 6) | (it.A[it.p + 3] & 63);
  it.p += 4;
  cp -= 0x10000;
  it.pend = 0xDC00 + (cp & 0x3FF);
  return 0xD800 + (cp >> 10);
}
YM_INL bool u16_eq(U16 a, U16 b) {
  for (;;) {
    const int32_t x = u16_next(a), y = u16_next(b);
    if (x != y) return false;
    if (x < 0) return true;
  }
}
YM_INL bool u16_is(U16 a, const char *t) {
  for (;; t++) {
    const int32_t x = u16_next(a);
    if (*t == 0) return x < 0;
    if (x != (uint8_t)*t) return false;
  }
}
// canonical array index ("0" .. "4294967294", no leading zero) -> value, else -1
YM_INL int64_t u16_index(U16 a) {
  int64_t v = 0;
  int n = 0;
  for (;;) {
    const int32_t x = u16_next(a);
    if (x < 0) break;
    if (x < '0' || x > '9' || n >= 10) return -1;
    if (n == 1 && v == 0) return -1;  // leading zero
    v = v * 10 + (x - '0');
    n++;
  }
  return n > 0 && v < 4294967295ll ? v : -1;
}
// UTF-8 of the code units (writeVarString / StringEncoder: a lone surrogate throws URIError)
template <class S> YM_INL void s_utf8(Ctx &c, S &s, U16 it) {
  for (;;) {
    int32_t u = u16_next(it);
    if (u < 0) return;
    if (u >= 0xD800 && u <= 0xDFFF) {
      U16 peek = it;
      const int32_t l = u <= 0xDBFF ? u16_next(peek) : -1;
      if (l < 0xDC00 || l > 0xDFFF) { seterr(c, ST_URI); return; }
      it = peek;
      const uint32_t cp = 0x10000 + (((uint32_t)u - 0xD800) << 10) + ((uint32_t)l - 0xDC00);
      s.put(0xF0 | (cp >> 18)); s.put(0x80 | ((cp >> 12) & 63)); s.put(0x80 | ((cp >> 6) & 63)); s.put(0x80 | (cp & 63));
    } else if (u < 0x80) {
      s.put((uint32_t)u);
    } else if (u < 0x800) {
      s.put(0xC0 | (u >> 6)); s.put(0x80 | (u & 63));
    } else {
      s.put(0xE0 | (u >> 12)); s.put(0x80 | ((u >> 6) & 63)); s.put(0x80 | (u & 63));
    }
  }
}
// JSON.stringify of a string (QuoteJSONString, well-formed: lone surrogates escaped), UTF-8 output
template <class S> YM_INL void s_json_quote(S &s, U16 it) {
  const char *hx = "0123456789abcdef";
  s.put('"');
  for (;;) {
    int32_t u = u16_next(it);
    if (u < 0) break;
    switch (u) {
      case 8: s_ascii(s, "\\b"); continue;
      case 9: s_ascii(s, "\\t"); continue;
      case 10: s_ascii(s, "\\n"); continue;
      case 12: s_ascii(s, "\\f"); continue;
      case 13: s_ascii(s, "\\r"); continue;
      case '"': s_ascii(s, "\\\""); continue;
      case '\\': s_ascii(s, "\\\\"); continue;
      default: break;
    }
    bool lone = false;
    if (u >= 0xD800 && u <= 0xDBFF) {
      U16 peek = it;
      const int32_t l = u16_next(peek);
      if (l >= 0xDC00 && l <= 0xDFFF) {
        it = peek;
        const uint32_t cp = 0x10000 + (((uint32_t)u - 0xD800) << 10) + ((uint32_t)l - 0xDC00);
        s.put(0xF0 | (cp >> 18)); s.put(0x80 | ((cp >> 12) & 63)); s.put(0x80 | ((cp >> 6) & 63)); s.put(0x80 | (cp & 63));
        continue;
      }
      lone = true;
    } else if (u >= 0xDC00 && u <= 0xDFFF) {
      lone = true;
    }
    if (u < 0x20 || lone) {
      s.put('\\'); s.put('u');
      s.put(hx[(u >> 12) & 15]); s.put(hx[(u >> 8) & 15]); s.put(hx[(u >> 4) & 15]); s.put(hx[u & 15]);
    } else if (u < 0x80) {
      s.put((uint32_t)u);
    } else if (u < 0x800) {
      s.put(0xC0 | (u >> 6)); s.put(0x80 | (u & 63));
    } else {
      s.put(0xE0 | (u >> 12)); s.put(0x80 | ((u >> 6) & 63)); s.put(0x80 | (u & 63));
    }
  }
  s.put('"');
}
// writeVarString of the code units: UTF-8 byte length, then the bytes
template <class S> YM_INL void s_varstring(Ctx &c, S &s, U16 it) {
  SinkLen n = {0, 0};
  s_utf8(c, n, it);
  s_vu(s, n.bytes);
  s_utf8(c, s, it);
}

// ------------------------------------------------------------------------------------------------
// numbers
// ------------------------------------------------------------------------------------------------
// writeAny(number): integer <= 2^31-1 -> varInt (writeVarInt: first byte from the magnitude, the rest
// ToUint32-wrapped), float32 when exact, else float64 (big-endian)
template <class S> YM_INL void s_any_number(S &s, double x) {
  if (f64_is_int(x) && x <= 2147483647.0) {
    const bool neg = x < 0 || (x == 0 && f64_signbit(x));
    const double m = x < 0 ? -x : x;
    const uint32_t lo = f64_touint32(m);
    s.put(125);
    s.put((m > 63 ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (lo & 63));
    uint32_t r = lo >> 6;
    while (r > 0) { s.put((r > 127 ? 0x80u : 0u) | (r & 127)); r >>= 7; }
    return;
  }
  const float f = (float)x;
  if ((double)f == x) {  // NaN fails, +-Infinity pass
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    s.put(124); s.put(u >> 24); s.put((u >> 16) & 255); s.put((u >> 8) & 255); s.put(u & 255);
    return;
  }
  const uint64_t u = f64_bits(x);
  s.put(123);
  for (int i = 7; i >= 0; i--) s.put((uint32_t)((u >> (8 * i)) & 255));
}
template <class S> YM_INL void s_json_number(S &s, double x) {
  if (!f64_finite(x)) { s_ascii(s, "null"); return; }
  char buf[40];
  const int n = f64_to_js(x, buf);
  for (int i = 0; i < n; i++) s.put((uint8_t)buf[i]);
}
YM_INL double any_number(const uint8_t *A, uint64_t p, int tag) {  // p after the tag
  if (tag == 125) {
    uint32_t b = A[p++];
    uint32_t num = b & 63;
    const bool neg = (b & 64) != 0;
    unsigned len = 6;
    while (b & 128) {
      b = A[p++];
      num |= (b & 127) << (len & 31);
      len += 7;
    }
    return neg ? -(double)num : (double)num;
  }
  if (tag == 124) {
    const uint32_t u = ((uint32_t)A[p] << 24) | ((uint32_t)A[p + 1] << 16) | ((uint32_t)A[p + 2] << 8) | A[p + 3];
    float f;
    __builtin_memcpy(&f, &u, 4);
    return (double)f;
  }
  uint64_t u = 0;
  for (int i = 0; i < 8; i++) u = (u << 8) | A[p + i];
  return f64_from(u);
}

// ------------------------------------------------------------------------------------------------
// containers
// ------------------------------------------------------------------------------------------------
struct CvEntry { uint64_t key, val, next; };
struct CvFrame {
  uint64_t body;     // first element / entry
  uint64_t cur;      // arrays: next element; objects (phase 1): next entry
  uint32_t n;        // G_ANY: element / entry count
  uint32_t i;        // elements / entries consumed (arrays, object phase 1)
  uint32_t emitted;  // values written (separators)
  int64_t lastidx;   // objects, phase 0: last array-index key handled
  uint64_t head;     // the container's value position (its tag / opening bracket)
  uint8_t obj, phase;
  uint8_t sim;       // G_ANY object with "__proto__" keys: entry liveness from obj_sim
  uint8_t parr;      // G_ANY object whose prototype chain ends in an Array, written as writeAny's array
};
// entry at position p (the i-th of frame f); false past the last one
YM_INL bool cv_entry(const uint8_t *A, uint8_t g, uint64_t end, const CvFrame &f, uint64_t p, uint32_t i, CvEntry &e) {
  if (g == G_ANY) {
    if (i >= f.n) return false;
    e.key = p;
    uint64_t q = p;
    const uint32_t L = cv_vu(A, q);
    e.val = q + L;
    e.next = any_end(A, e.val);
    return true;
  }
  if (A[p] == '}') return false;
  e.key = p;
  uint64_t q = js_ws(A, js_str_end(A, p), end);  // ':'
  e.val = js_ws(A, q + 1, end);
  q = js_ws(A, js_end(A, e.val, end), end);
  if (A[q] == ',') q = js_ws(A, q + 1, end);
  e.next = q;
  return true;
}
YM_INL U16 cv_key(const uint8_t *A, uint8_t g, const CvEntry &e) { return g == G_ANY ? u16_any(A, e.key) : u16_json(A, e.key); }
// ------------------------------------------------------------------------------------------------
// readAny builds objects by `obj[key] = v` ([[Set]] in strict module code), so a "__proto__" key can
// replace the prototype (Object.prototype's setter; a primitive is ignored), and the prototype chain
// then decides what later assignments do and what writeAny sees:
//   * a null prototype, or a prototype object owning a "__proto__" data property: "__proto__" keys
//     become own properties;
//   * a Uint8Array in the chain: its getters (length, byteLength, byteOffset, buffer) and the
//     read-only BYTES_PER_ELEMENT make the assignment throw TypeError; a canonical numeric key is
//     created only when it is an index below the array's length (V8 of the reference's Node), else
//     ignored; writeAny reads byteLength on the object (`instanceof Uint8Array`): TypeError;
//   * an Array in the chain: writeAny takes its array branch (`instanceof Array`): length and elements
//     read through the chain.
// JSON.parse uses CreateDataProperty: every JSON key (including "__proto__") is an own property.
// The simulation re-scans entries on demand (no workspace); prototype objects nest at most PROTO_DEPTH
// levels (deeper: UNSUPPORTED).
// ------------------------------------------------------------------------------------------------
enum : int { SET_OWN = 0, SET_IGNORE = 1, SET_PROTO = 2, SET_DEEP = 4, SET_TYPEERR = 8 };  // SET_TYPEERR + key index
enum : uint8_t { PK_PLAIN = 0, PK_NULL = 1, PK_ARRAY = 2, PK_BYTES = 3 };
constexpr int PROTO_DEPTH = 4;
struct ObjSim { uint64_t proto; int err; int live; };  // proto: value position (0 = Object.prototype)

YM_INL bool key_is_any(U16 k, const char *const *names, int n) {
  for (int i = 0; i < n; i++)
    if (u16_is(k, names[i])) return true;
  return false;
}
// CanonicalNumericIndexString (ES2019 7.1.16): 1 numeric, 0 not; *idx = integer index or -1
YM_NUM_FN int key_numeric(U16 k, int64_t *idx) {
  char buf[48];
  int n = 0;
  for (;;) {
    const int32_t u = u16_next(k);
    if (u < 0) break;
    if (u > 127 || n >= 40) return 0;
    buf[n++] = (char)u;
  }
  buf[n] = 0;
  *idx = -1;
  const char *sp[4] = {"-0", "NaN", "Infinity", "-Infinity"};
  for (int i = 0; i < 4; i++) {
    int j = 0;
    while (sp[i][j] && sp[i][j] == buf[j]) j++;
    if (!sp[i][j] && !buf[j]) return 1;
  }
  // Number::toString output grammar: -?digits(.digits)?(e[+-]digits)?
  int i = 0;
  if (buf[i] == '-') i++;
  if (buf[i] < '0' || buf[i] > '9') return 0;
  for (int j = i; j < n; j++) {
    const char ch = buf[j];
    if (!((ch >= '0' && ch <= '9') || ch == '.' || ch == 'e' || ch == '+' || ch == '-')) return 0;
  }
  const double x = json_num_to_f64((const uint8_t *)buf, (uint64_t)n);
  char t[48];
  const int m = f64_to_js(x, t);
  if (m != n) return 0;
  for (int j = 0; j < n; j++)
    if (t[j] != buf[j]) return 0;
  if (f64_is_int(x) && x >= 0 && !(x == 0 && f64_signbit(x))) *idx = (int64_t)x;
  return 1;
}
template <int D> YM_NUM_FN ObjSim obj_sim(const uint8_t *A, uint64_t end, uint64_t q, uint32_t upto);
// does the (fully built) object at q own `key` as a live entry: 1, 0, or -1 (too deep)
template <int D> YM_NUM_FN int obj_owns(const uint8_t *A, uint64_t end, uint64_t q, U16 key) {
  CvFrame f;
  uint64_t p = q + 1;
  f.n = cv_vu(A, p);
  f.body = p;
  CvEntry e;
  int owns = 0;
  for (uint32_t i = 0; cv_entry(A, G_ANY, end, f, p, i, e); i++, p = e.next) {
    if (!u16_eq(cv_key(A, G_ANY, e), key)) continue;
    const ObjSim st = obj_sim<D>(A, end, q, i);
    if (st.err == ST_UNSUPPORTED) return -1;
    if (st.err) return owns;  // readAny threw at an earlier entry: reported where the value is read
    if (st.live) owns = 1;
  }
  return owns;
}
// what `obj[key] = v` does given obj's current prototype (the chain walk of OrdinarySet)
template <int D> YM_NUM_FN int set_kind(const uint8_t *A, uint64_t end, uint64_t proto, U16 key, uint8_t vtag) {
  const bool dunder = u16_is(key, "__proto__");
  const int setter = vtag == 118 || vtag == 117 || vtag == 116 || vtag == 126 ? SET_PROTO : SET_IGNORE;
  uint64_t P = proto;
  for (int hop = 0; hop <= PROTO_DEPTH; hop++) {
    if (P == 0) return dunder ? setter : SET_OWN;  // Object.prototype
    const uint8_t t = A[P];
    if (t == 126) return SET_OWN;                    // null: end of the chain
    if (t == 117) return dunder ? setter : SET_OWN;  // Array (writable data) -> Array.prototype -> Object.prototype
    if (t == 116) {
      const char *ro[5] = {"length", "byteLength", "byteOffset", "buffer", "BYTES_PER_ELEMENT"};
      for (int q = 0; q < 5; q++)
        if (key_is_any(key, ro + q, 1)) return SET_TYPEERR + q;
      int64_t idx;
      if (key_numeric(key, &idx)) {
        uint64_t qq = P + 1;
        const uint32_t L = cv_vu(A, qq);
        return idx >= 0 && idx < (int64_t)L ? SET_OWN : SET_IGNORE;
      }
      return dunder ? setter : SET_OWN;
    }
    if constexpr (D <= 0) {
      return SET_DEEP;
    } else {
      const int own = obj_owns<D - 1>(A, end, P, key);
      if (own < 0) return SET_DEEP;
      if (own) return SET_OWN;  // a writable data property on the prototype: created on the receiver
      const ObjSim ps = obj_sim<D - 1>(A, end, P, 0xFFFFFFFFu);
      if (ps.err == ST_UNSUPPORTED) return SET_DEEP;
      P = ps.proto;
    }
  }
  return SET_DEEP;
}
// readAny's assignments of the object at q (a 118 value), entries [0, upto] (upto = ~0u: all).
// .live: entry `upto` created or overwrote an own property; .err: ST_TYPE (readAny threw), ST_UNSUPPORTED
template <int D> YM_NUM_FN ObjSim obj_sim(const uint8_t *A, uint64_t end, uint64_t q, uint32_t upto) {
  ObjSim r = {0, 0, 0};
  CvFrame f;
  uint64_t p = q + 1;
  f.n = cv_vu(A, p);
  f.body = p;
  CvEntry e;
  bool own_dunder = false;
  for (uint32_t i = 0; i <= upto && cv_entry(A, G_ANY, end, f, p, i, e); i++, p = e.next) {
    const U16 k = cv_key(A, G_ANY, e);
    int live = 1;
    const bool dunder = u16_is(k, "__proto__");
    if (dunder && own_dunder) {
      live = 1;  // overwrites the own "__proto__" data property
    } else if (r.proto != 0 || dunder) {  // on the default chain every other key is a plain own property
      const int sk = set_kind<D>(A, end, r.proto, k, A[e.val]);
      if (sk == SET_DEEP) { r.err = ST_UNSUPPORTED; return r; }
      if (sk >= SET_TYPEERR) {  // an accessor without a setter / a read-only property on the chain (strict mode)
        r.err = sk == SET_TYPEERR + 4 ? st_d(ST_TYPE, D_SET_RO) : st_d(ST_TYPE, D_SET_GETTER, sk - SET_TYPEERR);
        return r;
      }
      if (sk == SET_PROTO) { r.proto = e.val; live = 0; }
      else if (sk == SET_IGNORE) live = 0;
      else if (dunder) own_dunder = true;
    }
    r.live = live;
  }
  return r;
}
template <int D> YM_NUM_FN int proto_kind(const uint8_t *A, uint64_t end, uint64_t proto) {  // -1 too deep / threw
  if (proto == 0) return PK_PLAIN;
  const uint8_t t = A[proto];
  if (t == 126) return PK_NULL;
  if (t == 117) return PK_ARRAY;
  if (t == 116) return PK_BYTES;
  if constexpr (D <= 0) {
    return -1;
  } else {
    const ObjSim ps = obj_sim<D - 1>(A, end, proto, 0xFFFFFFFFu);
    if (ps.err) return -1;
    return proto_kind<D - 1>(A, end, ps.proto);
  }
}
// does the object at q carry a "__proto__" key (only then is the simulation needed)
YM_INL bool obj_has_dunder(const uint8_t *A, uint64_t end, uint64_t q) {
  CvFrame f;
  uint64_t p = q + 1;
  f.n = cv_vu(A, p);
  f.body = p;
  CvEntry e;
  for (uint32_t i = 0; cv_entry(A, G_ANY, end, f, p, i, e); i++, p = e.next)
    if (u16_is(cv_key(A, G_ANY, e), "__proto__")) return true;
  return false;
}

// An entry is live when it creates or overwrites an own property: every entry of a JSON object, every
// readAny entry of an object without "__proto__" keys (f.sim == 0), else per obj_sim.
YM_INL bool cv_live(const uint8_t *A, uint8_t g, uint64_t end, const CvFrame &f, uint32_t i) {
  if (g != G_ANY || !f.sim) return true;
  return obj_sim<PROTO_DEPTH>(A, end, f.head, i).live != 0;
}
// the value of the last live entry whose key equals e0's (e0 = entry i0, live)
YM_INL uint64_t cv_last_value(const uint8_t *A, uint8_t g, uint64_t end, const CvFrame &f, const CvEntry &e0, uint32_t i0) {
  uint64_t v = e0.val;
  const U16 k = cv_key(A, g, e0);
  CvEntry e;
  uint64_t p = e0.next;
  for (uint32_t i = i0 + 1; cv_entry(A, g, end, f, p, i, e); i++, p = e.next)
    if (u16_eq(cv_key(A, g, e), k) && cv_live(A, g, end, f, i)) v = e.val;
  return v;
}
// is the live entry i0 the first live one with its key
YM_INL bool cv_first_occurrence(const uint8_t *A, uint8_t g, uint64_t end, const CvFrame &f, const CvEntry &e0, uint32_t i0) {
  const U16 k = cv_key(A, g, e0);
  CvEntry e;
  uint64_t p = f.body;
  for (uint32_t i = 0; i < i0 && cv_entry(A, g, end, f, p, i, e); i++, p = e.next)
    if (u16_eq(cv_key(A, g, e), k) && cv_live(A, g, end, f, i)) return false;
  return true;
}
YM_INL uint32_t cv_own_keys(const uint8_t *A, uint8_t g, uint64_t end, const CvFrame &f) {
  uint32_t n = 0;
  CvEntry e;
  uint64_t p = f.body;
  for (uint32_t i = 0; cv_entry(A, g, end, f, p, i, e); i++, p = e.next)
    if (cv_live(A, g, end, f, i) && cv_first_occurrence(A, g, end, f, e, i)) n++;
  return n;
}
YM_INL void cv_open_any_object(const uint8_t *A, uint64_t end, CvFrame &f, uint64_t q) {
  uint64_t p = q + 1;
  f.n = cv_vu(A, p);
  f.body = p;
  f.cur = p;
  f.head = q;
  f.sim = A[q] == 118 && obj_has_dunder(A, end, q);
}
// [[Get]](obj, key) along a readAny prototype chain that ends in an Array: the value position of the
// first live own `key` found, 0 = none (the array's element / length), ~0 = unsupported
YM_INL uint64_t chain_get(const uint8_t *A, uint64_t end, uint64_t q, U16 key, uint64_t *arr) {
  uint64_t P = q;
  for (int hop = 0; hop <= PROTO_DEPTH + 1; hop++) {
    const uint8_t t = A[P];
    if (t == 117) { *arr = P; return 0; }
    if (t != 118) return ~0ull;
    CvFrame f;
    cv_open_any_object(A, end, f, P);
    CvEntry e;
    uint64_t found = 0, p = f.body;
    for (uint32_t i = 0; cv_entry(A, G_ANY, end, f, p, i, e); i++, p = e.next)
      if (u16_eq(cv_key(A, G_ANY, e), key) && cv_live(A, G_ANY, end, f, i)) found = e.val;
    if (found) return found;
    const ObjSim ps = obj_sim<PROTO_DEPTH>(A, end, P, 0xFFFFFFFFu);
    if (ps.err || ps.proto == 0) return ~0ull;
    P = ps.proto;
  }
  return ~0ull;
}
// readAny's TypeError cases (a Uint8Array prototype's getters / read-only property assigned) anywhere
// inside the value at p: ST_TYPE, ST_UNSUPPORTED (too deep) or 0.  Only called for values whose
// objects carry "__proto__" keys (the canonicity scan flags them).
YM_INL int any_read_check(const uint8_t *A, uint64_t p, uint64_t end) {
  const uint64_t e = any_end(A, p);
  // every 118 tag at a value position: walk the value with the navigation of any_end
  uint32_t left[YM_ANY_DEPTH + 1];
  uint8_t obj[YM_ANY_DEPTH + 1];
  int sp = 0;
  while (p < e) {
    const uint64_t v = p;
    const int tag = A[p++];
    switch (tag) {
      case 125: while (A[p] & 0x80) p++; p++; break;
      case 124: p += 4; break;
      case 123: case 122: p += 8; break;
      case 119: case 116: { const uint32_t L = cv_vu(A, p); p += L; break; }
      case 118: case 117: {
        if (tag == 118 && obj_has_dunder(A, end, v)) {
          const ObjSim st = obj_sim<PROTO_DEPTH>(A, end, v, 0xFFFFFFFFu);
          if (st.err) return st.err;
        }
        const uint32_t n = cv_vu(A, p);
        if (n && sp <= YM_ANY_DEPTH) { left[sp] = n; obj[sp] = tag == 118; sp++; }
        break;
      }
      default: break;
    }
    for (;;) {
      if (sp == 0) return 0;
      if (left[sp - 1] == 0) { sp--; continue; }
      left[sp - 1]--;
      if (obj[sp - 1]) { const uint32_t L = cv_vu(A, p); p += L; }
      break;
    }
  }
  return 0;
}

YM_INL uint32_t cv_array_len(const uint8_t *A, uint8_t g, uint64_t end, const CvFrame &f) {
  if (g == G_ANY) return f.n;
  uint32_t n = 0;
  uint64_t p = f.body;
  while (A[p] != ']') {
    p = js_ws(A, js_end(A, p, end), end);
    if (A[p] == ',') p = js_ws(A, p + 1, end);
    n++;
  }
  return n;
}
YM_INL bool cv_undefined(const uint8_t *A, uint8_t g, uint64_t v) { return g == G_ANY && A[v] == 127; }

// Finds the next object member to write (canonical order), or returns false when the object is done.
YM_INL bool cv_next_member(const uint8_t *A, uint8_t g, uint8_t t, uint64_t end, CvFrame &f, CvEntry &out, uint64_t &val) {
  CvEntry e;
  while (f.phase == 0) {  // array-index keys, ascending
    int64_t best = -1;
    CvEntry be = {0, 0, 0};
    uint32_t bi = 0;
    uint64_t p = f.body;
    for (uint32_t i = 0; cv_entry(A, g, end, f, p, i, e); i++, p = e.next) {
      const int64_t ix = u16_index(cv_key(A, g, e));
      if (ix > f.lastidx && (best < 0 || ix < best)) { best = ix; be = e; bi = i; }
    }
    if (best < 0) { f.phase = 1; f.cur = f.body; f.i = 0; break; }
    f.lastidx = best;
    val = cv_last_value(A, g, end, f, be, bi);
    if (t == T_JSONANY && cv_undefined(A, g, val)) continue;
    out = be;
    return true;
  }
  while (cv_entry(A, g, end, f, f.cur, f.i, e)) {
    const uint32_t i = f.i;
    f.cur = e.next;
    f.i++;
    if (u16_index(cv_key(A, g, e)) >= 0 || !cv_live(A, g, end, f, i) || !cv_first_occurrence(A, g, end, f, e, i)) continue;
    val = cv_last_value(A, g, end, f, e, i);
    if (t == T_JSONANY && cv_undefined(A, g, val)) continue;
    out = e;
    return true;
  }
  return false;
}

// ------------------------------------------------------------------------------------------------
// one value: G source at p (no leading whitespace) -> T target
// ------------------------------------------------------------------------------------------------
template <class S>
YM_BIG void canon_value(Ctx &c, S &s, const uint8_t *A, uint64_t p, uint64_t end, uint8_t g, uint8_t t) {
  CvFrame st[YM_ANY_DEPTH + 2];
  int sp = 0;
  const bool json_out = t != T_ANY;
  for (;;) {
    // ---- write the value at p (scalars entirely, containers: their head, then a frame) ----
    if (g == G_ANY) {
      const int tag = A[p];
      switch (tag) {
        case 127: if (json_out) s_ascii(s, "null"); else s.put(127); break;  // array element (members are skipped)
        case 126: if (json_out) s_ascii(s, "null"); else s.put(126); break;
        case 121: if (json_out) s_ascii(s, "false"); else s.put(121); break;
        case 120: if (json_out) s_ascii(s, "true"); else s.put(120); break;
        case 125: case 124: case 123: {
          const double x = any_number(A, p + 1, tag);
          if (json_out) s_json_number(s, x); else s_any_number(s, x);
          break;
        }
        case 122:
          if (json_out) { seterr(c, st_d(ST_TYPE, D_BIGINT_JSON)); return; }  // JSON.stringify(bigint)
          for (int i = 0; i < 9; i++) s.put(A[p + i]);
          break;
        case 119: {
          const U16 u = u16_any(A, p + 1);
          if (json_out) s_json_quote(s, u); else { s.put(119); s_varstring(c, s, u); }
          break;
        }
        case 116: {
          uint64_t q = p + 1;
          const uint32_t L = cv_vu(A, q);
          if (json_out) {  // a Uint8Array is an object of index keys
            s.put('{');
            for (uint32_t i = 0; i < L; i++) {
              char buf[40];
              if (i) s.put(',');
              s.put('"');
              int n = f64_to_js((double)i, buf);
              for (int k = 0; k < n; k++) s.put((uint8_t)buf[k]);
              s.put('"'); s.put(':');
              n = f64_to_js((double)A[q + i], buf);
              for (int k = 0; k < n; k++) s.put((uint8_t)buf[k]);
            }
            s.put('}');
          } else {
            s.put(116); s_vu(s, L);
            for (uint32_t i = 0; i < L; i++) s.put(A[q + i]);
          }
          break;
        }
        default: {  // 118 object, 117 array
          if (sp > YM_ANY_DEPTH) { seterr(c, ST_UNSUPPORTED); return; }
          CvFrame &f = st[sp++];
          cv_open_any_object(A, end, f, p);
          f.i = 0; f.emitted = 0; f.lastidx = -1; f.phase = 0; f.obj = tag == 118; f.parr = 0;
          if (f.sim) {
            const ObjSim os = obj_sim<PROTO_DEPTH>(A, end, p, 0xFFFFFFFFu);
            const int kind = os.err ? -1 : proto_kind<PROTO_DEPTH>(A, end, os.proto);
            if ((os.err & 0xff) == ST_TYPE) { seterr(c, os.err); return; }
            if (kind < 0) { seterr(c, ST_UNSUPPORTED); return; }
            // writeAny: `instanceof Uint8Array` reads byteLength off a plain object (TypeError);
            // `instanceof Array` writes length and elements read through the prototype chain.
            // JSON.stringify serialises own keys whatever the prototype.
            if (kind == PK_BYTES && !json_out) { seterr(c, st_d(ST_TYPE, D_BYTELENGTH)); return; }
            if (kind == PK_ARRAY && !json_out) {
              uint64_t arr = 0;
              const uint8_t lk[6] = {'l', 'e', 'n', 'g', 't', 'h'};
              if (chain_get(A, end, p, u16_utf8(lk, 0, 6), &arr) != 0) { seterr(c, ST_UNSUPPORTED); return; }
              uint64_t q = arr + 1;
              f.n = cv_vu(A, q);
              f.obj = 0;
              f.parr = 1;
              s.put(117);
              s_vu(s, f.n);
              break;
            }
          }
          if (json_out) s.put(f.obj ? '{' : '[');
          else { s.put(tag); s_vu(s, f.obj ? cv_own_keys(A, g, end, f) : f.n); }
          break;
        }
      }
    } else {
      const uint8_t ch = A[p];
      if (ch == '"') {
        const U16 u = u16_json(A, p);
        if (json_out) s_json_quote(s, u); else { s.put(119); s_varstring(c, s, u); }
      } else if (ch == 't') {
        if (json_out) s_ascii(s, "true"); else s.put(120);
      } else if (ch == 'f') {
        if (json_out) s_ascii(s, "false"); else s.put(121);
      } else if (ch == 'n') {
        if (json_out) s_ascii(s, "null"); else s.put(126);
      } else if (ch == '{' || ch == '[') {
        if (sp > YM_ANY_DEPTH) { seterr(c, ST_UNSUPPORTED); return; }
        CvFrame &f = st[sp++];
        f.body = js_ws(A, p + 1, end); f.cur = f.body; f.n = 0; f.i = 0; f.emitted = 0; f.lastidx = -1; f.phase = 0;
        f.head = p; f.sim = 0; f.parr = 0;
        f.obj = ch == '{';
        if (json_out) s.put(ch);
        else { s.put(f.obj ? 118 : 117); s_vu(s, f.obj ? cv_own_keys(A, g, end, f) : cv_array_len(A, g, end, f)); }
      } else {
        const double x = json_num_to_f64(A + p, js_end(A, p, end) - p);
        if (json_out) s_json_number(s, x); else s_any_number(s, x);
      }
    }
    if (c.err) return;
    // ---- find the next value: the next element / member of the innermost open container ----
    for (;;) {
      if (sp == 0) return;
      CvFrame &f = st[sp - 1];
      if (f.parr) {  // writeAny's array branch over an object whose prototype chain ends in an Array
        if (f.i >= f.n) { sp--; continue; }
        char buf[40];
        const int nb = f64_to_js((double)f.i, buf);
        uint64_t arr = 0;
        const uint64_t v = chain_get(A, end, f.head, u16_utf8((const uint8_t *)buf, 0, (uint64_t)nb), &arr);
        if (v == ~0ull) { seterr(c, ST_UNSUPPORTED); return; }
        if (v) p = v;
        else {
          uint64_t q = arr + 1;
          cv_vu(A, q);
          for (uint32_t k = 0; k < f.i; k++) q = any_end(A, q);
          p = q;
        }
        f.i++;
        break;
      }
      if (!f.obj) {
        const bool more = g == G_ANY ? f.i < f.n : A[f.cur] != ']';
        if (!more) { if (json_out) s.put(']'); sp--; continue; }
        p = f.cur;
        if (g == G_ANY) f.cur = any_end(A, p);
        else { uint64_t q = js_ws(A, js_end(A, p, end), end); if (A[q] == ',') q = js_ws(A, q + 1, end); f.cur = q; }
        f.i++;
        if (json_out && f.emitted) s.put(',');
        f.emitted++;
        break;
      }
      CvEntry e;
      uint64_t v;
      if (!cv_next_member(A, g, t, end, f, e, v)) { if (json_out) s.put('}'); sp--; continue; }
      if (json_out) {
        if (f.emitted) s.put(',');
        s_json_quote(s, cv_key(A, g, e));
        s.put(':');
      } else {
        s_varstring(c, s, cv_key(A, g, e));
      }
      f.emitted++;
      p = v;
      break;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// ContentDoc options: new Doc({guid, ...readAny(opts)}) then ContentDoc's re-derived opts
// (13.5.16 ContentDoc constructor: {gc: false}? {autoLoad: true}? {meta}?; Doc defaults gc = true,
// autoLoad = false, meta = null; ContentDoc.js:116-135).  *guid_key: the entry of an own "guid" string
// key (it replaces the guid read before the options), else 0.  A non-string or undefined guid (a random
// uuid) is reported UNSUPPORTED, as the oracle does.
// ------------------------------------------------------------------------------------------------
YM_INL bool any_truthy(const uint8_t *A, uint64_t v) {
  const int tag = A[v];
  switch (tag) {
    case 127: case 126: case 121: return false;
    case 120: return true;
    case 125: case 124: case 123: { const double x = any_number(A, v + 1, tag); return !(x == 0 || x != x); }
    case 119: { uint64_t q = v + 1; return cv_vu(A, q) != 0; }
    case 122: { for (int i = 1; i <= 8; i++) if (A[v + i]) return true; return false; }
    default: return true;
  }
}
struct DocOpts { uint64_t guid_val; uint8_t has_guid, gc, autoload, has_meta; uint64_t meta; };
YM_INL DocOpts doc_opts(Ctx &c, const uint8_t *A, uint64_t p, uint64_t end) {
  DocOpts d = {0, 0, 1, 0, 0, 0};
  uint64_t guid = 0;
  if (A[p] != 118) return d;  // spreading a non-object contributes no gc / autoLoad / meta / guid
  CvFrame f;
  uint64_t q = p + 1;
  f.n = cv_vu(A, q);
  f.body = q;
  CvEntry e;
  uint64_t pos = f.body;
  for (uint32_t i = 0; cv_entry(A, G_ANY, end, f, pos, i, e); i++, pos = e.next) {
    const U16 k = cv_key(A, G_ANY, e);
    const uint64_t v = e.val;  // later entries override earlier ones (obj[key] = v)
    if (u16_is(k, "gc")) d.gc = A[v] == 127 ? 1 : any_truthy(A, v);
    else if (u16_is(k, "autoLoad")) d.autoload = A[v] == 127 ? 0 : any_truthy(A, v);
    else if (u16_is(k, "meta")) { d.has_meta = A[v] != 127 && A[v] != 126; d.meta = v; }
    else if (u16_is(k, "guid")) guid = v;
  }
  if (guid) {
    if (A[guid] != 119) { seterr(c, ST_UNSUPPORTED); return d; }
    d.has_guid = 1;
    d.guid_val = guid + 1;
  }
  return d;
}
template <class S> YM_INL void s_doc_opts(Ctx &c, S &s, const uint8_t *A, const DocOpts &d, uint64_t end) {
  s.put(118);
  s_vu(s, (uint64_t)(!d.gc) + d.autoload + d.has_meta);
  if (!d.gc) { s.put(2); s.put('g'); s.put('c'); s.put(121); }
  if (d.autoload) { s.put(8); s_ascii(s, "autoLoad"); s.put(120); }
  if (d.has_meta) { s.put(4); s_ascii(s, "meta"); canon_value(c, s, A, d.meta, end, G_ANY, T_ANY); }
}

}  // namespace ym
