// ym_lane.h -- per-lane lib0 / V1 struct parser over global memory, for the chunk-parallel walk of large
// updates (ym_pwalk.hip).  Each lane runs its own cursor (divergent across lanes, unlike the wave-uniform
// scalar walker of ym_scalar.h); the next bytes sit in a 16-byte register window (lo, hi) refilled by one
// unaligned 8-byte global load per ~8 consumed bytes, so a ~11-byte struct costs one or two loads.
//
// Same semantics and canonical-form checks as ym_scalar.h / ym_fast_common.h (lib0 0.2.42 readVarUint /
// readVarString / readAny, UpdateDecoder.js:127-243, Item.js:665-683): a struct this parser accepts is
// one the verbatim copy reproduces exactly; anything else is rejected.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ym_canon_chk.h"
#include "ym_utf8.h"

namespace ymk {
namespace ln {

// bytes [p, e) of the document at b; reads may run up to 15 bytes past e (the arena is padded)
struct LCur {
  const uint8_t *b;
  uint32_t p, e;
  bool bad;
  uint64_t lo, hi;
  uint32_t nv;
  uint32_t cap;  // longest string / ContentAny the parse accepts (bounds a speculative parse)
};
__device__ __forceinline__ uint64_t ld8(const uint8_t *b, uint32_t p) {
  uint64_t x;
  __builtin_memcpy(&x, b + p, 8);
  return x;
}
__device__ __forceinline__ uint32_t byte(const uint8_t *b, uint32_t p) { return b[p]; }
__device__ __forceinline__ void fill(LCur &c) {  // nv >= 8 afterwards
  if (c.nv >= 8) return;
  const uint64_t x = ld8(c.b, c.p + c.nv);
  if (c.nv == 0) {
    c.lo = x;
    c.hi = 0;
  } else {
    c.lo |= x << (8 * c.nv);
    c.hi = x >> (64 - 8 * c.nv);
  }
  c.nv += 8;
}
__device__ __forceinline__ LCur make(const uint8_t *b, uint32_t p, uint32_t e, uint32_t cap = 0xffffffffu) {
  LCur c = {b, p, e, false, 0, 0, 0, cap};
  fill(c);
  return c;
}
__device__ __forceinline__ void skip(LCur &c, uint32_t n) {
  if (n >= c.nv) {
    c.p += n;
    c.nv = 0;
  } else if (n > 0) {
    if (n < 8) {
      c.lo = (c.lo >> (8 * n)) | (c.hi << (64 - 8 * n));
      c.hi >>= 8 * n;
    } else {
      c.lo = c.hi >> (8 * (n - 8));
      c.hi = 0;
    }
    c.p += n;
    c.nv -= n;
  }
  fill(c);
}
__device__ __forceinline__ uint64_t peek8(const LCur &c, uint32_t o) {
  if (o == 0) return c.lo;
  if (o + 8 <= c.nv) return o < 8 ? (c.lo >> (8 * o)) | (c.hi << (64 - 8 * o)) : c.hi >> (8 * (o - 8));
  return ld8(c.b, c.p + o);
}
__device__ __forceinline__ uint32_t vu_nb(uint32_t lo, uint32_t hi) {
  const uint32_t s_lo = ~lo & 0x80808080u;
  const uint32_t s_hi = (~hi & 0x80u) | 0x8000u;
  const uint32_t t = __builtin_ctzg(s_lo, 32 + __builtin_ctz(s_hi));
  return (t >> 3) + 1;
}
__device__ __forceinline__ bool vu_bad(uint32_t lo, uint32_t hi, uint32_t nb, uint32_t p, uint32_t e) {
  const uint32_t last = nb <= 4 ? (lo >> (8 * nb - 8)) & 0xffu : hi & 0xffu;
  return (nb > 5) | (p + nb > e) | ((nb > 1) & (last == 0)) | ((nb == 5) & ((hi & 0x70u) != 0));
}
// lib0 readVarUint (u32, canonical encodings only)
__device__ __forceinline__ uint32_t rvu(LCur &c) {
  const uint32_t lo = (uint32_t)c.lo, hi = (uint32_t)(c.lo >> 32);
  const uint32_t nb = vu_nb(lo, hi);
  const uint32_t v = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u) | (hi << 28);
  const uint32_t m = (uint32_t)((1ull << (7 * (nb < 5 ? nb : 5))) - 1);
  c.bad |= vu_bad(lo, hi, nb, c.p, c.e);
  skip(c, nb < 6 ? nb : 0);
  return v & m;
}
__device__ __forceinline__ void skvu(LCur &c) { (void)rvu(c); }
__device__ __forceinline__ uint32_t rdb(LCur &c) {
  c.bad |= c.p >= c.e;
  const uint32_t v = (uint32_t)c.lo & 0xffu;
  skip(c, 1);
  return v;
}
__device__ __forceinline__ bool room(const LCur &c, uint32_t n) { return c.p <= c.e && n <= c.e - c.p; }
// strict UTF-8 (lib0: decodeURIComponent(escape(..))); the UTF-16 length
__device__ __forceinline__ uint32_t utf8_slow(const uint8_t *b, uint32_t i, uint32_t e, bool &bad) {
  return utf8::units<uint32_t>([b](uint32_t p) { return (uint32_t)ld8(b, p); }, i, e, bad);  // (ym_utf8.h: 4 bytes per step)
}
__device__ __forceinline__ uint64_t mask_bytes(uint64_t x, uint32_t n) { return n >= 8 ? x : x & ((1ull << (8 * n)) - 1); }
__device__ __forceinline__ uint32_t utf16_len(LCur &c, uint32_t n) {
  if (!room(c, n) || n > c.cap) { c.bad = true; return 0; }
  uint64_t hi = 0;
  for (uint32_t o = 0; o < n; o += 8) hi |= mask_bytes(peek8(c, o), n - o);
  uint32_t u = n;
  if (hi & 0x8080808080808080ull) u = utf8_slow(c.b, c.p, c.p + n, c.bad);
  skip(c, n);
  return u;
}
__device__ __forceinline__ uint32_t rstr(LCur &c) {
  const uint32_t n = rvu(c);
  return c.bad ? 0 : utf16_len(c, n);
}
__device__ __forceinline__ uint64_t has_byte(uint64_t x, uint64_t v) {
  const uint64_t y = x ^ (0x0101010101010101ull * v);
  return (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
}
__device__ __forceinline__ uint64_t has_ctl(uint64_t x) { return (x - 0x2020202020202020ull) & ~x & 0x8080808080808080ull; }
// JSON text as yjs writes it for formats / embeds: true | false | null | "string without escapes"
template <bool NESTED = false>
__device__ __forceinline__ void json_lit(LCur &c) {
  const uint32_t n = rvu(c);
  if (c.bad || !room(c, n) || n > c.cap) { c.bad = true; return; }
  const uint64_t w = c.lo;
  bool ok;
  if (n == 4) ok = (uint32_t)w == 0x65757274u || (uint32_t)w == 0x6c6c756eu;
  else if (n == 5) ok = (w & 0xffffffffffull) == 0x65736c6166ull;
  else ok = false;
  if (!ok && n >= 2 && (w & 0xff) == '"' && byte(c.b, c.p + n - 1) == '"') {
    uint64_t bad = 0;
    for (uint32_t o = 1; o + 1 < n; o += 8) {
      const uint64_t x = mask_bytes(peek8(c, o), n - 1 - o);
      const uint64_t pad = (n - 1 - o) >= 8 ? 0 : ~0ull << (8 * (n - 1 - o));
      const uint64_t xs = x | (pad & 0x4040404040404040ull);
      bad |= has_byte(xs, '"') | has_byte(xs, '\\') | (has_ctl(xs) & ~xs);
    }
    ok = bad == 0;
  }
  // numbers, objects, arrays: JSON.stringify(JSON.parse(text)) == text (ym_canon_chk.h)
  if (NESTED && !ok) ok = cchk::json_canon_ptr(c.b, c.p, n);
  if (!ok) { c.bad = true; return; }
  utf16_len(c, n);
}
// one scalar `any` value in the canonical form lib0 writeAny emits
__device__ __forceinline__ void any_scalar(LCur &c) {
  const uint32_t tag = rdb(c);
  switch (tag) {
    case 127: case 126: case 121: case 120: return;
    case 125: {
      uint32_t x = rdb(c);
      uint64_t mag = x & 63;
      const bool neg = x & 64;
      int s = 6, nb = 1;
      while ((x & 128) && !c.bad) {
        x = rdb(c);
        if (s > 34) { c.bad = true; return; }
        mag |= (uint64_t)(x & 127) << s;
        s += 7;
        nb++;
      }
      if ((nb > 1 && x == 0) || (!neg && mag > 2147483647ull) || mag > 0xffffffffull) c.bad = true;
      return;
    }
    case 124: {
      if (!room(c, 4)) { c.bad = true; return; }
      const float f = __uint_as_float(__builtin_bswap32((uint32_t)c.lo));
      if (f != f || (truncf(f) == f && (double)f <= 2147483647.0)) c.bad = true;
      skip(c, 4);
      return;
    }
    case 123: {
      if (!room(c, 8)) { c.bad = true; return; }
      const double x = __longlong_as_double((long long)__builtin_bswap64(c.lo));
      if (x == x && ((trunc(x) == x && x <= 2147483647.0) || (double)(float)x == x)) c.bad = true;
      skip(c, 8);
      return;
    }
    case 119: rstr(c); return;
    default: c.bad = true; return;
  }
}
// One `any` value of any shape in the form lib0 0.2.42 writeAny emits for what readAny returns, so the
// bytes round-trip: scalars as any_scalar, Uint8Array (116), BigInt64 (122), and arrays (117) / objects
// (118) nested up to AC_DEPTH levels.  An object's re-encoding follows Object.keys order, which equals the
// stored order only when no key is an array index and no key repeats, and readAny's `__proto__` key
// mutates the prototype instead of adding a key -- so keys starting with a digit, `__proto__` and
// repeated keys (compared byte-wise against the object's earlier keys, at most AC_KEYS open keys) are
// rejected (the general path re-encodes those exactly).  The containers' state is register-resident
// (cchk::rsel / wsel selects over unrolled entries: no scratch memory); deeper or wider values decline.
constexpr uint32_t AC_DEPTH = cchk::DEPTH, AC_KEYS = cchk::KEYS;
__device__ __forceinline__ bool key_eq(const uint8_t *b, uint32_t p, uint32_t q, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (b[p + i] != b[q + i]) return false;
  return true;
}
__device__ __forceinline__ void any_nested(LCur &c);
__device__ __forceinline__ void any_canon(LCur &c) {
  const uint32_t tag = (uint32_t)c.lo & 0xffu;
  if (tag == 116 || tag == 117 || tag == 118 || tag == 122) any_nested(c);
  else any_scalar(c);
}
__device__ __forceinline__ void any_nested(LCur &c) {
  uint32_t rem[AC_DEPTH] = {};   // values left in each open array / object
  uint32_t obj[AC_DEPTH] = {};   // 1 + first key slot of an open object, 0 for an array
  uint32_t kp[AC_KEYS] = {}, kl[AC_KEYS] = {};
  uint32_t depth = 0, nk = 0;
  for (;;) {
    if (c.bad) return;
    // an object expects a key before each value
    if (depth > 0 && cchk::rsel(obj, depth - 1)) {
      const uint32_t n = rvu(c);
      if (c.bad || !room(c, n) || n > c.cap) { c.bad = true; return; }
      const uint32_t p = c.p;
      const uint32_t b0 = n > 0 ? (uint32_t)c.lo & 0xffu : 0;
      c.bad |= n > 0 && b0 >= '0' && b0 <= '9';
      c.bad |= n == 9 && peek8(c, 0) == 0x5f6f746f72705f5full && (uint32_t)(peek8(c, 8) & 0xff) == '_';  // "__proto__"
      const uint32_t k0 = cchk::rsel(obj, depth - 1) - 1;
#pragma unroll
      for (uint32_t k = 0; k < AC_KEYS; k++)
        if (k >= k0 && k < nk && kl[k] == n && !c.bad) c.bad |= key_eq(c.b, kp[k], p, n);
      utf16_len(c, n);
      if (c.bad || nk >= AC_KEYS) { c.bad = true; return; }
      cchk::wsel(kp, nk, p);
      cchk::wsel(kl, nk, n);
      nk++;
    }
    const uint32_t tag = (uint32_t)c.lo & 0xffu;
    if (tag == 117 || tag == 118) {  // array / object: count, then the values
      rdb(c);
      const uint32_t n = rvu(c);
      if (c.bad || n > c.cap || depth >= AC_DEPTH) { c.bad = true; return; }
      if (n > 0) {
        cchk::wsel(rem, depth, n);
        cchk::wsel(obj, depth, tag == 118 ? nk + 1 : 0);
        depth++;
        continue;
      }
    } else if (tag == 116) {  // Uint8Array: varUint8Array
      rdb(c);
      const uint32_t n = rvu(c);
      if (c.bad || !room(c, n) || n > c.cap) { c.bad = true; return; }
      skip(c, n);
    } else if (tag == 122) {  // BigInt64: 8 bytes, read and written as they are
      rdb(c);
      if (!room(c, 8)) { c.bad = true; return; }
      skip(c, 8);
    } else {
      any_scalar(c);
    }
    // a value completed: close the containers it finished
    while (depth > 0 && !c.bad) {
      const uint32_t r = cchk::rsel(rem, depth - 1) - 1;
      cchk::wsel(rem, depth - 1, r);
      if (r > 0) break;
      depth--;
      const uint32_t o = cchk::rsel(obj, depth);
      if (o) nk = o - 1;
    }
    if (depth == 0) return;
  }
}

// Item fields and content after the info byte; false for kinds the verbatim path does not verify
// (ContentJSON, ContentDoc, bad refs) or any anomaly.  `len` = the Item's clock length.
// NESTED: nested `any` values and JSON texts through ym_canon_chk.h's out-of-line checks.  The chunk walk and
// its stitch do without (their call stack and registers would halve the walk's occupancy): a nested value
// fails there, and the document goes to the streamed walker, which checks it.
template <bool NESTED = false>
__device__ __forceinline__ bool item_body(LCur &c, uint32_t info, uint32_t &len) {
  if (info & 0x80) { skvu(c); skvu(c); }
  if (info & 0x40) { skvu(c); skvu(c); }
  if ((info & 0xC0) == 0) {
    const uint32_t pi = rvu(c);
    c.bad |= pi > 1;
    if (pi == 1) rstr(c);
    else { skvu(c); skvu(c); }
    if (info & 0x20) rstr(c);
  }
  len = 1;
  switch (info & 31) {
    case 1: len = rvu(c); break;
    case 3: { const uint32_t n = rvu(c); if (!room(c, n) || n > c.cap) c.bad = true; else skip(c, n); break; }
    case 4: len = rstr(c); break;
    case 5: json_lit<NESTED>(c); break;
    case 6: rstr(c); json_lit<NESTED>(c); break;
    case 7: {
      const uint32_t t = rvu(c);
      c.bad |= t > 6;
      if (t == 3 || t == 5) rstr(c);
      break;
    }
    case 8:
      len = rvu(c);
      c.bad |= len > c.cap;
      for (uint32_t i = 0; i < len && !c.bad; i++) {
        if (NESTED) any_canon(c);
        else any_scalar(c);
      }
      break;
    default: c.bad = true; break;
  }
  return !c.bad && len != 0;
}

// Record flags of one parsed struct (ym_pwalk.hip step records, bits 28-31 of the position word)
constexpr uint32_t F_FAIL = 1u << 28;   // no struct parses here (the walk resumes one byte later)
constexpr uint32_t F_SKIP = 1u << 29;   // a Skip (info 10)
constexpr uint32_t F_PATCH = 1u << 30;  // the writer re-encodes the info byte differently (0x20 cleared / GC := 0)
constexpr uint32_t POS_MASK = (1u << 28) - 1;

// One V1 struct at the cursor (GC / Skip / Item, readClientsStructRefs' cases): on success the cursor
// is after it (its register window still valid, so a walk carries it to the next struct), `len` is its
// clock length and `fl` its flags.  The cursor's `cap` bounds string / ContentAny lengths (a speculative
// parse of a position that may not start a struct; the stitch re-parses uncapped).
template <bool NESTED = false>
__device__ __forceinline__ bool parse_at(LCur &c, uint32_t &len, uint32_t &fl) {
  c.bad = false;
  const uint32_t info = rdb(c);
  const bool sk = info == 10, gc = !sk && (info & 31) == 0;
  bool ok;
  if (sk || gc) {
    len = rvu(c);
    ok = !c.bad;
  } else {
    ok = item_body<NESTED>(c, info, len);
  }
  ok = ok && !c.bad && c.p <= c.e;
  const uint32_t ni = sk ? info : gc ? 0 : ((info & 0xC0) ? info & ~0x20u : info);
  fl = (sk ? F_SKIP : 0) | (ni != info ? F_PATCH : 0);
  return ok;
}
template <bool NESTED = false>
__device__ __forceinline__ bool parse_struct(const uint8_t *b, uint32_t p, uint32_t e, uint32_t &next, uint32_t &len,
                                             uint32_t &fl, uint32_t cap = 0xffffffffu) {
  LCur c = make(b, p, e, cap);
  const bool ok = parse_at<NESTED>(c, len, fl);
  next = c.p;
  return ok;
}

// Branch-free short cut for the commonest structs, from one 32-byte window at p: GC / Skip, and Items with
// an origin whose content is ContentDeleted or an ASCII ContentString (C3: ~all structs) whose varuints
// end in the first 16 bytes and whose string ends inside the window.  Works on byte masks (bit 7 of each
// byte of a u64): varuint ends are the stop bytes, found by clearing the lowest set bit; overlong ends
// (a 0x00 after a continuation byte) by one SWAR mask; 5-byte varuints are left to the full parser.
// Returns true with next / len / fl exactly as parse_at would; false = not decided here (the caller runs
// parse_at, which also gives every rejection its exact meaning).
__device__ __forceinline__ uint64_t lowbytes(uint32_t n) { return n >= 8 ? ~0ull : (1ull << (8 * n)) - 1; }
__device__ __forceinline__ bool parse_fast(const uint8_t *b, uint32_t p, uint32_t e, uint32_t &next, uint32_t &len,
                                           uint32_t &fl) {
  if (p + 32 > e) return false;
  typedef uint4 __attribute__((aligned(1))) u4a;
  const uint4 A = *reinterpret_cast<const u4a *>(b + p), Bq = *reinterpret_cast<const u4a *>(b + p + 16);
  constexpr uint64_t H = 0x8080808080808080ull, L7 = 0x7f7f7f7f7f7f7f7full;
  const uint64_t w0 = ((uint64_t)A.y << 32) | A.x, w1 = ((uint64_t)A.w << 32) | A.z;
  const uint64_t w2 = ((uint64_t)Bq.y << 32) | Bq.x, w3 = ((uint64_t)Bq.w << 32) | Bq.z;
  const uint32_t info = A.x & 0xffu, ref = info & 31;
  const bool sk = info == 10, gc = !sk && ref == 0;
  const bool item = (info & 0xC0) != 0 && (ref == 1 || ref == 4);
  const uint32_t V = (sk || gc) ? 1 : 1 + 2 * ((info >> 7) & 1) + 2 * ((info >> 6) & 1);
  // stop bytes of bytes 1..15 (the info byte is not part of a varuint)
  uint64_t s0 = ~w0 & H & ~0x80ull, s1 = ~w1 & H;
  uint64_t E0 = 0, E1 = 0;  // the first V stop bytes
  uint32_t ev = 0, ep = 0, prev = 0, longest = 0;
#pragma unroll
  for (uint32_t t = 1; t <= 5; t++) {
    const uint64_t l0 = s0 & (0 - s0), l1 = s0 ? 0 : s1 & (0 - s1);
    const uint32_t et = s0 ? (uint32_t)__builtin_ctzll(s0) >> 3 : s1 ? 8 + ((uint32_t)__builtin_ctzll(s1) >> 3) : 16;
    if (t <= V) {
      E0 |= l0;
      E1 |= l1;
      longest = et - prev > longest ? et - prev : longest;
      prev = et;
    }
    if (t == V - 1) ep = et;
    if (t == V) ev = et;
    s0 ^= l0;
    s1 ^= l1;
  }
  if (!(sk || gc || item) || ev >= 16 || longest >= 5) return false;
  // overlong: a zero stop byte right after a continuation byte (the info byte does not count)
  const uint64_t z0 = ~(((w0 & L7) + L7) | w0) & H, z1 = ~(((w1 & L7) + L7) | w1) & H;
  const uint64_t c0 = ((w0 & ~0xffull) << 8) & H, c1 = ((w1 << 8) | (w0 >> 56)) & H;
  if ((E0 & z0 & c0) | (E1 & z1 & c1)) return false;
  // the last varuint's value (bytes ep+1 .. ev, at most 4)
  const uint32_t o = ep + 1;
  const uint64_t x = o == 0 ? w0 : o < 8 ? (w0 >> (8 * o)) | (w1 << (64 - 8 * o)) : w1 >> (8 * (o - 8));
  const uint32_t lo = (uint32_t)x;
  const uint32_t nb = ev - ep;
  const uint32_t v = ((lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u)) &
                     ((1u << (7 * nb)) - 1);
  uint32_t end = ev + 1;
  if (ref == 4 && item) {  // ASCII string ending inside the window
    if (v == 0 || ev + v >= 32) return false;
    const uint32_t a0 = ev + 1, a1 = a0 + v;  // string bytes [a0, a1)
    uint64_t na = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint64_t wk = k == 0 ? w0 : k == 1 ? w1 : k == 2 ? w2 : w3;
      const uint32_t lo_b = a0 > 8 * k ? a0 - 8 * k : 0, hi_b = a1 > 8 * k ? a1 - 8 * k : 0;
      na |= wk & H & lowbytes(hi_b) & ~lowbytes(lo_b);
    }
    if (na) return false;
    end += v;
  } else if (ref == 1 && item && v == 0) {
    return false;
  }
  next = p + end;
  len = v;
  const uint32_t ni = sk ? info : gc ? 0 : info & ~0x20u;
  fl = (sk ? F_SKIP : 0) | (ni != info ? F_PATCH : 0);
  return true;
}

// First position >= q (and < lim, else lim) whose byte could start a struct parse_fast accepts: a Skip
// (10), a GC (ref 0), or ContentDeleted / ContentString (ref 1 / 4) with an origin bit.  SWAR over 8
// bytes per step; a byte-wise false positive only costs an extra attempt, none is missed.
__device__ __forceinline__ uint32_t next_cand(const uint8_t *b, uint32_t q, uint32_t lim) {
  for (uint32_t it = 0; it < 8 && q < lim; it++, q += 8) {
    const uint64_t x = ld8(b, q);
    const uint64_t r = x & 0x1f1f1f1f1f1f1f1full;
    const uint64_t org = (x | (x << 1)) & 0x8080808080808080ull;  // bit 7 or bit 6 set
    const uint64_t m = has_byte(x, 10) | has_byte(r, 0) | ((has_byte(r, 1) | has_byte(r, 4)) & org);
    if (m) {
      const uint32_t c = q + (__builtin_ctzll(m) >> 3);
      return c < lim ? c : lim;
    }
  }
  return q < lim ? q : lim;
}

}  // namespace ln
}  // namespace ymk
