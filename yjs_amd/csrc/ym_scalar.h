// ym_scalar.h -- wave-uniform lib0 / V1 readers on the scalar unit, for the sequential single-update
// walkers (ym_big.hip).  A diff or state-vector walk of one large update is inherently sequential;
// run on the VALU it pays 4 cycles per wave64 instruction plus an LDS round trip per field.  Here the
// update is read with scalar loads (s_load through the constant address space: the arena is read-only
// for the kernel) and every parsed value lives in SGPRs, so the walk issues SALU instructions (1 cycle)
// with uniform branches and needs no LDS window, no refills and no barriers.
//
// Same semantics and canonical-form checks as the LDS readers in ym_fast_common.h (lib0 0.2.42
// readVarUint / readVarString / readAny, UpdateDecoder.js:127-243, Item.js:665-683).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ym_canon_chk.h"
#include "ym_utf8.h"

namespace ymk {
namespace sc {

typedef const __attribute__((address_space(4))) uint32_t cu32;

// A cursor over bytes [p, e) of a dword-aligned base (offsets in bytes from b), with the next bytes
// held in a 16-byte shift register (lo, hi): nv >= 8 bytes starting at p are always loaded, so a field
// is parsed from registers and memory is touched once per ~8 consumed bytes (a dependent scalar load
// per field would cost its full latency every time).
struct SCur {
  cu32 *b;
  uint32_t p, e;
  bool bad;
  uint64_t lo, hi;
  uint32_t nv;
};
__device__ __forceinline__ cu32 *base_of(const uint8_t *a) {
  return (cu32 *)(uintptr_t)((uintptr_t)a & ~(uintptr_t)3);
}
// 8 bytes at byte offset p (reads up to 12 bytes past p: callers stay within 16 bytes of the end of
// an allocation)
__device__ __forceinline__ uint64_t ld8(cu32 *b, uint32_t p) {
  const uint32_t w = p >> 2, sh = (p & 3) * 8;
  const uint64_t lo = ((uint64_t)b[w + 1] << 32) | b[w];
  if (sh == 0) return lo;
  return (lo >> sh) | ((uint64_t)b[w + 2] << (64 - sh));
}
__device__ __forceinline__ uint32_t byte(cu32 *b, uint32_t p) { return (b[p >> 2] >> ((p & 3) * 8)) & 0xffu; }

__device__ __forceinline__ void fill(SCur &c) {  // nv >= 8 afterwards
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
// Wave-uniform by construction, but the compiler's divergence analysis does not always prove it (the
// walk then runs on the VALU with exec-mask branches and vector loads): readfirstlane pins the cursor
// to SGPRs at loop heads.
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) { return ((uint64_t)rfl((uint32_t)(x >> 32)) << 32) | rfl((uint32_t)x); }
__device__ __forceinline__ cu32 *rflp(cu32 *b) { return (cu32 *)(uintptr_t)rfl64((uint64_t)(uintptr_t)b); }
__device__ __forceinline__ void uni(SCur &c) {
  c.b = rflp(c.b);
  c.p = rfl(c.p);
  c.e = rfl(c.e);
  c.lo = rfl64(c.lo);
  c.hi = rfl64(c.hi);
  c.nv = rfl(c.nv);
  c.bad = rfl(c.bad) != 0;
}
__device__ __forceinline__ SCur make(cu32 *b, uint32_t p, uint32_t e) {
  SCur c = {b, p, e, false, 0, 0, 0};
  fill(c);
  return c;
}
// consumes n bytes
__device__ __forceinline__ void skip(SCur &c, uint32_t n) {
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
// the 8 bytes at p + o (o < 8 reads from the register window when it holds them)
__device__ __forceinline__ uint64_t peek8(const SCur &c, uint32_t o) {
  if (o == 0) return c.lo;
  if (o + 8 <= c.nv) return o < 8 ? (c.lo >> (8 * o)) | (c.hi << (64 - 8 * o)) : c.hi >> (8 * (o - 8));
  return ld8(c.b, c.p + o);
}

__device__ __forceinline__ uint32_t vu_nb(uint32_t lo, uint32_t hi) {
  const uint32_t s_lo = ~lo & 0x80808080u;
  const uint32_t s_hi = (~hi & 0x80u) | 0x8000u;
  const uint32_t t = s_lo ? __builtin_ctz(s_lo) : 32 + __builtin_ctz(s_hi);
  return (t >> 3) + 1;
}
__device__ __forceinline__ bool vu_bad(uint32_t lo, uint32_t hi, uint32_t nb, uint32_t p, uint32_t e) {
  const uint32_t last = nb <= 4 ? (lo >> (8 * nb - 8)) & 0xffu : hi & 0xffu;
  return (nb > 5) | (p + nb > e) | ((nb > 1) & (last == 0)) | ((nb == 5) & ((hi & 0x70u) != 0));
}
__device__ __forceinline__ uint32_t rvu(SCur &c) {
  const uint64_t x = c.lo;
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if ((lo & 0x80u) == 0) {  // the common case: one byte
    c.bad |= c.p + 1 > c.e;
    skip(c, 1);
    return lo & 0x7fu;
  }
  const uint32_t nb = vu_nb(lo, hi);
  const uint32_t v = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u) | (hi << 28);
  const uint32_t m = (uint32_t)((1ull << (7 * (nb < 5 ? nb : 5))) - 1);
  c.bad |= vu_bad(lo, hi, nb, c.p, c.e);
  skip(c, nb < 6 ? nb : 0);
  return v & m;
}
__device__ __forceinline__ void skvu(SCur &c) { (void)rvu(c); }
__device__ __forceinline__ uint32_t rdb(SCur &c) {
  c.bad |= c.p >= c.e;
  const uint32_t v = (uint32_t)c.lo & 0xffu;
  skip(c, 1);
  return v;
}
__device__ __forceinline__ bool room(const SCur &c, uint32_t n) { return c.p <= c.e && n <= c.e - c.p; }
__device__ __forceinline__ uint32_t utf8_slow(cu32 *b, uint32_t i, uint32_t e, bool &bad) {
  return utf8::units<uint32_t>([b](uint32_t p) { return (uint32_t)ld8(b, p); }, i, e, bad);  // (ym_utf8.h: 4 bytes per step)
}
__device__ __forceinline__ uint64_t mask_bytes(uint64_t x, uint32_t n) { return n >= 8 ? x : x & ((1ull << (8 * n)) - 1); }
__device__ __forceinline__ uint32_t utf16_len(SCur &c, uint32_t n) {
  if (!room(c, n)) { c.bad = true; return 0; }
  uint64_t hi = 0;
  for (uint32_t o = 0; o < n; o += 8) hi |= mask_bytes(peek8(c, o), n - o);
  uint32_t u = n;
  if (hi & 0x8080808080808080ull) u = utf8_slow(c.b, c.p, c.p + n, c.bad);
  skip(c, n);
  return u;
}
__device__ __forceinline__ uint32_t rstr(SCur &c) {
  const uint32_t n = rvu(c);
  return c.bad ? 0 : utf16_len(c, n);
}
__device__ __forceinline__ uint64_t has_byte(uint64_t x, uint64_t v) {
  const uint64_t y = x ^ (0x0101010101010101ull * v);
  return (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
}
__device__ __forceinline__ uint64_t has_ctl(uint64_t x) {
  return (x - 0x2020202020202020ull) & ~x & 0x8080808080808080ull;
}
__device__ __forceinline__ void json_lit(SCur &c) {  // true | false | null | "string without escapes"
  const uint32_t n = rvu(c);
  if (c.bad || !room(c, n)) { c.bad = true; return; }
  const uint64_t w = c.lo;
  bool ok;
  if (n == 4) ok = (uint32_t)w == 0x65757274u || (uint32_t)w == 0x6c6c756eu;
  else if (n == 5) ok = (w & 0xffffffffffull) == 0x65736c6166ull;
  else ok = false;
  if (!ok && n >= 2 && (w & 0xff) == '"' && byte(c.b, c.p + n - 1) == '"') {
    uint64_t bad = 0;
    for (uint32_t o = 1; o + 1 < n; o += 8) {
      uint64_t x = mask_bytes(peek8(c, o), n - 1 - o);
      const uint64_t pad = (n - 1 - o) >= 8 ? 0 : ~0ull << (8 * (n - 1 - o));
      const uint64_t xs = x | (pad & 0x4040404040404040ull);
      bad |= has_byte(xs, '"') | has_byte(xs, '\\') | (has_ctl(xs) & ~xs);
    }
    ok = bad == 0;
  }
  // numbers, objects, arrays: JSON.stringify(JSON.parse(text)) == text (ym_canon_chk.h)
  if (!ok) ok = cchk::json_canon_ptr((const uint8_t *)(uintptr_t)c.b, c.p, n);
  if (!ok) { c.bad = true; return; }
  utf16_len(c, n);
}
__device__ __forceinline__ void any_scalar(SCur &c);
// one `any` value of any shape in the form writeAny emits (nested values: ym_canon_chk.h)
__device__ __forceinline__ void any_canon(SCur &c) {
  const uint32_t tag = c.p < c.e ? byte(c.b, c.p) : 0;
  if (tag == 116 || tag == 117 || tag == 118 || tag == 122) {
    uint32_t q = c.p;
    if (!cchk::any_canon_ptr((const uint8_t *)(uintptr_t)c.b, c.p, c.e, &q)) { c.bad = true; return; }
    skip(c, q - c.p);
  } else {
    any_scalar(c);
  }
}
__device__ __forceinline__ void any_scalar(SCur &c) {
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
      const uint32_t u = __builtin_bswap32((uint32_t)c.lo);
      const float f = __uint_as_float(u);
      if (f != f || (truncf(f) == f && (double)f <= 2147483647.0)) c.bad = true;
      skip(c, 4);
      return;
    }
    case 123: {
      if (!room(c, 8)) { c.bad = true; return; }
      const uint64_t u = __builtin_bswap64(c.lo);
      const double x = __longlong_as_double((long long)u);
      if (x == x && ((trunc(x) == x && x <= 2147483647.0) || (double)(float)x == x)) c.bad = true;
      skip(c, 8);
      return;
    }
    case 119: rstr(c); return;
    default: c.bad = true; return;
  }
}
__device__ __forceinline__ bool item_body(SCur &c, uint32_t info, uint32_t &len) {
  if (info & 0x80) { skvu(c); skvu(c); }
  if (info & 0x40) { skvu(c); skvu(c); }
  if ((info & 0xC0) == 0) {
    const uint32_t pi = rvu(c);
    if (pi > 1) return false;
    if (pi == 1) rstr(c);
    else { skvu(c); skvu(c); }
    if (info & 0x20) rstr(c);
  }
  len = 1;
  switch (info & 31) {
    case 1: len = rvu(c); break;
    case 3: { const uint32_t n = rvu(c); if (!room(c, n)) c.bad = true; else skip(c, n); break; }
    case 4: len = rstr(c); break;
    case 5: json_lit(c); break;
    case 6: rstr(c); json_lit(c); break;
    case 7: {
      const uint32_t t = rvu(c);
      if (t > 6) return false;
      if (t == 3 || t == 5) rstr(c);
      break;
    }
    case 8:
      len = rvu(c);
      for (uint32_t i = 0; i < len && !c.bad; i++) any_canon(c);
      break;
    default: return false;
  }
  return !c.bad && len != 0;
}

}  // namespace sc
}  // namespace ymk
