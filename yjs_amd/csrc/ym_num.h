// ym_num.h -- exact binary64 <-> decimal conversions for the device (general path only).
//
// yjs re-encodes numbers through JavaScript: JSON.parse (ECMA-262 StringToNumber: the decimal rounded to
// the nearest binary64, ties to even) and JSON.stringify / Number::toString (ECMA-262 7.1.12.1: the
// shortest digit string that rounds back to the value, the closest of those, ties to the even digit).
// Both are done here with exact big-integer arithmetic (no libc on the device): strtod by correcting an
// approximation against exact midpoint comparisons, toString by the Steele-White / Burger-Dybvig
// free-format digit generation.  Every routine is iterative and allocation-free (private arrays).
#pragma once
#include <stdint.h>

#ifndef YM_HD
#define YM_HD __host__ __device__
#endif
// big-integer routines stay out of line on the device: inlined into their callers they would put
// their bignum arrays into every caller's scratch frame
#ifndef YM_NUM_FN
#ifdef __HIP_DEVICE_COMPILE__
#define YM_NUM_FN YM_HD __attribute__((noinline))
#else
#define YM_NUM_FN YM_HD inline
#endif
#endif

namespace ym {

// ------------------------------------------------------------------------------------------------
// little-endian u32-limb big integers, 4096 bits (enough for 780 decimal digits scaled by 2^1075 or
// 10^1124: the worst cases of the strtod comparison)
// ------------------------------------------------------------------------------------------------
constexpr int BIG_LIMBS = 128;
struct Big {
  uint32_t n;  // used limbs (no leading zero limbs)
  uint32_t d[BIG_LIMBS];
};
YM_HD inline void big_set(Big &a, uint64_t v) {
  a.n = 0;
  while (v) { a.d[a.n++] = (uint32_t)v; v >>= 32; }
}
YM_HD inline void big_trim(Big &a) {
  while (a.n && a.d[a.n - 1] == 0) a.n--;
}
YM_HD inline void big_mul_small(Big &a, uint32_t m) {
  uint64_t carry = 0;
  for (uint32_t i = 0; i < a.n; i++) {
    uint64_t t = (uint64_t)a.d[i] * m + carry;
    a.d[i] = (uint32_t)t;
    carry = t >> 32;
  }
  if (carry && a.n < BIG_LIMBS) a.d[a.n++] = (uint32_t)carry;
}
YM_HD inline void big_add_small(Big &a, uint32_t v) {
  uint64_t carry = v;
  for (uint32_t i = 0; i < a.n && carry; i++) {
    uint64_t t = (uint64_t)a.d[i] + carry;
    a.d[i] = (uint32_t)t;
    carry = t >> 32;
  }
  if (carry && a.n < BIG_LIMBS) a.d[a.n++] = (uint32_t)carry;
}
YM_HD inline void big_mul_pow10(Big &a, int32_t k) {
  while (k >= 9) { big_mul_small(a, 1000000000u); k -= 9; }
  uint32_t p = 1;
  while (k-- > 0) p *= 10;
  if (p != 1) big_mul_small(a, p);
}
YM_HD inline void big_shl(Big &a, uint32_t bits) {
  if (a.n == 0) return;
  const uint32_t w = bits >> 5, b = bits & 31;
  uint32_t n = a.n + w + 1;
  if (n > BIG_LIMBS) n = BIG_LIMBS;
  for (int32_t i = (int32_t)n - 1; i >= 0; i--) {
    const int32_t s = i - (int32_t)w;
    uint32_t hi = s >= 0 && s < (int32_t)a.n ? a.d[s] : 0;
    uint32_t lo = s - 1 >= 0 && s - 1 < (int32_t)a.n ? a.d[s - 1] : 0;
    a.d[i] = b ? (hi << b) | (lo >> (32 - b)) : hi;
  }
  a.n = n;
  big_trim(a);
}
YM_HD inline int big_cmp(const Big &a, const Big &b) {
  if (a.n != b.n) return a.n < b.n ? -1 : 1;
  for (int32_t i = (int32_t)a.n - 1; i >= 0; i--)
    if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
  return 0;
}
YM_HD inline void big_add(Big &r, const Big &a, const Big &b) {  // r may alias a
  const uint32_t n = a.n > b.n ? a.n : b.n;
  uint64_t carry = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint64_t t = (uint64_t)(i < a.n ? a.d[i] : 0) + (i < b.n ? b.d[i] : 0) + carry;
    r.d[i] = (uint32_t)t;
    carry = t >> 32;
  }
  r.n = n;
  if (carry && r.n < BIG_LIMBS) r.d[r.n++] = (uint32_t)carry;
}
YM_HD inline void big_sub(Big &a, const Big &b) {  // a -= b, a >= b
  int64_t borrow = 0;
  for (uint32_t i = 0; i < a.n; i++) {
    int64_t t = (int64_t)a.d[i] - (i < b.n ? b.d[i] : 0) - borrow;
    borrow = t < 0;
    a.d[i] = (uint32_t)(t + (borrow << 32));
  }
  big_trim(a);
}
// cmp(a + b, c) without a temporary of the sum's size class beyond one Big
YM_HD inline int big_cmp_sum(const Big &a, const Big &b, const Big &c, Big &tmp) {
  big_add(tmp, a, b);
  return big_cmp(tmp, c);
}

// ------------------------------------------------------------------------------------------------
// binary64 helpers
// ------------------------------------------------------------------------------------------------
YM_HD inline uint64_t f64_bits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
YM_HD inline double f64_from(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }
YM_HD inline bool f64_finite(double x) { return (f64_bits(x) & 0x7FF0000000000000ull) != 0x7FF0000000000000ull; }
YM_HD inline bool f64_signbit(double x) { return (f64_bits(x) >> 63) != 0; }
YM_HD inline bool f64_is_int(double x) { return f64_finite(x) && __builtin_floor(x) == x; }
// ToUint32 of a finite integral double (ECMA-262 7.1.7: the mathematical value modulo 2^32)
YM_HD inline uint32_t f64_touint32(double x) {
  if (!f64_finite(x) || x == 0) return 0;
  const bool neg = x < 0;
  double m = neg ? -x : x;
  uint32_t r;
  if (m < 18446744073709551616.0) {
    r = (uint32_t)(uint64_t)m;
  } else {
    const uint64_t u = f64_bits(m);
    const int e = (int)((u >> 52) & 0x7FF) - 1075;  // m = f * 2^e, e >= 12
    const uint64_t f = (u & 0xFFFFFFFFFFFFFull) | 0x10000000000000ull;
    r = e >= 32 ? 0u : (uint32_t)(((f & 0xFFFFFFFFull) << e) & 0xFFFFFFFFull);
  }
  return neg ? (uint32_t)(0u - r) : r;
}

// ------------------------------------------------------------------------------------------------
// decimal -> binary64 (round to nearest, ties to even).  digits: the significant decimal digits
// (no leading zeros) of M, value = M * 10^k10; sticky = nonzero digits were dropped after them.
// ------------------------------------------------------------------------------------------------
constexpr int DEC_MAX_DIGITS = 780;  // > 767: enough to decide every binary64 rounding
YM_NUM_FN double dec_to_f64(const uint8_t *digits, int nd, int32_t k10, bool sticky) {
  if (nd == 0) return 0.0;
  const int32_t top = nd + k10;  // value in [10^(top-1), 10^top)
  if (top > 310) return __builtin_inf();
  if (top < -324) return 0.0;
  // approximation from the first 19 digits
  uint64_t m19 = 0;
  const int n19 = nd < 19 ? nd : 19;
  for (int i = 0; i < n19; i++) m19 = m19 * 10 + digits[i];
  double x = (double)m19;
  int32_t e10 = k10 + (nd - n19);
  // x * 10^e10 by exact powers of ten (each step rounds once: a few ulps off at most; the exact
  // correction below fixes them)
  const double p10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  while (e10 > 22 && f64_finite(x)) { x *= 1e22; e10 -= 22; }
  while (e10 < -22 && x != 0) { x /= 1e22; e10 += 22; }
  if (e10 > 0) x *= p10[e10 > 22 ? 22 : e10];
  else if (e10 < 0) x /= p10[-e10 > 22 ? 22 : -e10];
  if (!f64_finite(x)) x = 1.7976931348623157e308;
  if (x == 0) x = 4.9406564584124654e-324;
  // M as a big integer
  Big M;
  big_set(M, 0);
  for (int i = 0; i < nd; i++) {
    if (M.n == 0) big_set(M, digits[i]);
    else { big_mul_small(M, 10); big_add_small(M, digits[i]); }
  }
  // correction: compare M*10^k10 with the midpoints of x's neighbourhood
  for (int it = 0; it < 64; it++) {
    const uint64_t u = f64_bits(x);
    const int be = (int)((u >> 52) & 0x7FF);
    uint64_t m = u & 0xFFFFFFFFFFFFFull;
    int32_t q;
    if (be == 0) { q = -1074; } else { m |= 0x10000000000000ull; q = be - 1075; }
    // side 0: upper midpoint (2m + 1) * 2^(q-1); side 1: lower midpoint (2m - 1) * 2^(q-1), or
    // (4m - 1) * 2^(q-2) at the bottom of a binade (m = 2^52, be > 1)
    int move = 0;
    for (int side = 0; side < 2 && move == 0; side++) {
      Big L = M, R;
      uint64_t A;
      int32_t B;
      if (side == 0) { A = 2 * m + 1; B = q - 1; }
      else if (m == 0x10000000000000ull && be > 1) { A = 4 * m - 1; B = q - 2; }
      else { A = 2 * m - 1; B = q - 1; }
      big_set(R, A);
      if (k10 >= 0) big_mul_pow10(L, k10); else big_mul_pow10(R, -k10);
      if (B >= 0) big_shl(R, (uint32_t)B); else big_shl(L, (uint32_t)(-B));
      int cmp = big_cmp(L, R);
      if (cmp == 0 && sticky) cmp = 1;
      if (side == 0 && (cmp > 0 || (cmp == 0 && (m & 1)))) move = 1;       // above the upper midpoint
      if (side == 1 && (cmp < 0 || (cmp == 0 && (m & 1)))) move = -1;      // below the lower midpoint
    }
    if (move == 0) return x;
    if (move > 0) {
      if (u == 0x7FEFFFFFFFFFFFFFull) return __builtin_inf();
      x = f64_from(u + 1);
    } else {
      if (u == 1) return 0.0;
      x = f64_from(u - 1);
    }
  }
  return x;
}

// ------------------------------------------------------------------------------------------------
// binary64 -> shortest decimal digits (Number::toString's s, k, n): x finite, > 0.  Writes the digits
// (ASCII) to buf (>= 18 bytes), returns their count; *n10 = n (value = 0.d1d2..dk * 10^n).
// ------------------------------------------------------------------------------------------------
YM_NUM_FN int f64_shortest(double x, char *buf, int32_t *n10) {
  const uint64_t u = f64_bits(x);
  const int be = (int)((u >> 52) & 0x7FF);
  uint64_t f = u & 0xFFFFFFFFFFFFFull;
  int32_t e;
  if (be == 0) e = -1074; else { f |= 0x10000000000000ull; e = be - 1075; }
  const bool even = (f & 1) == 0;
  const bool unequal = f == 0x10000000000000ull && be > 1;  // lower gap is half the upper one
  Big r, s, mp, mm, t;
  if (e >= 0) {
    big_set(r, f); big_shl(r, (uint32_t)e + (unequal ? 2 : 1));
    big_set(s, unequal ? 4 : 2);
    big_set(mp, 1); big_shl(mp, (uint32_t)e + (unequal ? 1 : 0));
    big_set(mm, 1); big_shl(mm, (uint32_t)e);
  } else {
    big_set(r, f); big_shl(r, unequal ? 2 : 1);
    big_set(s, 1); big_shl(s, (uint32_t)(-e) + (unequal ? 2 : 1));
    big_set(mp, unequal ? 2 : 1);
    big_set(mm, 1);
  }
  // k estimate: ceil(log10(x)) - (0 or 1)
  int bl = 0;
  for (uint64_t g = f; g; g >>= 1) bl++;
  const int e2 = e + bl - 1;  // x in [2^e2, 2^(e2+1))
  int32_t k = (int32_t)__builtin_ceil((double)e2 * 0.30102999566398114 - 1e-10);
  if (k >= 0) big_mul_pow10(s, k);
  else { big_mul_pow10(r, -k); big_mul_pow10(mp, -k); big_mul_pow10(mm, -k); }
  {
    const int c = big_cmp_sum(r, mp, s, t);
    if (even ? c >= 0 : c > 0) { big_mul_small(s, 10); k++; }
  }
  *n10 = k;
  int nd = 0;
  for (;;) {
    big_mul_small(r, 10); big_mul_small(mp, 10); big_mul_small(mm, 10);
    big_trim(r);
    int d = 0;
    while (big_cmp(r, s) >= 0) { big_sub(r, s); d++; }
    const int cl = big_cmp(r, mm);
    const bool tc1 = even ? cl <= 0 : cl < 0;
    const int ch = big_cmp_sum(r, mp, s, t);
    const bool tc2 = even ? ch >= 0 : ch > 0;
    if (!tc1 && !tc2) {
      buf[nd++] = (char)('0' + d);
      if (nd < 20) continue;  // never reached: 17 digits always terminate
      break;
    }
    if (tc1 && tc2) {
      Big r2 = r;
      big_add(r2, r2, r);  // 2r
      const int c = big_cmp(r2, s);
      if (c > 0 || (c == 0 && (d & 1))) d++;
    } else if (tc2) {
      d++;
    }
    buf[nd++] = (char)('0' + d);
    break;
  }
  return nd;
}

// Number::toString(x) (ECMA-262 7.1.12.1) into buf (>= 32 bytes); returns the length.  NaN / Infinity
// spelled as JS does (JSON.stringify maps non-finite numbers to "null" before calling this).
YM_NUM_FN int f64_to_js(double x, char *buf) {
  int o = 0;
  if (x != x) { const char *t = "NaN"; while (*t) buf[o++] = *t++; return o; }
  if (x == 0) { buf[0] = '0'; return 1; }
  if (x < 0) { buf[o++] = '-'; x = -x; }
  if (!f64_finite(x)) { const char *t = "Infinity"; while (*t) buf[o++] = *t++; return o; }
  char dg[24];
  int32_t n;
  const int k = f64_shortest(x, dg, &n);
  if (k <= n && n <= 21) {
    for (int i = 0; i < k; i++) buf[o++] = dg[i];
    for (int i = 0; i < n - k; i++) buf[o++] = '0';
  } else if (0 < n && n <= 21) {
    for (int i = 0; i < n; i++) buf[o++] = dg[i];
    buf[o++] = '.';
    for (int i = n; i < k; i++) buf[o++] = dg[i];
  } else if (-6 < n && n <= 0) {
    buf[o++] = '0';
    buf[o++] = '.';
    for (int i = 0; i < -n; i++) buf[o++] = '0';
    for (int i = 0; i < k; i++) buf[o++] = dg[i];
  } else {
    buf[o++] = dg[0];
    if (k > 1) {
      buf[o++] = '.';
      for (int i = 1; i < k; i++) buf[o++] = dg[i];
    }
    buf[o++] = 'e';
    int32_t ex = n - 1;
    buf[o++] = ex >= 0 ? '+' : '-';
    if (ex < 0) ex = -ex;
    char eb[8];
    int ne = 0;
    do { eb[ne++] = (char)('0' + ex % 10); ex /= 10; } while (ex);
    while (ne) buf[o++] = eb[--ne];
  }
  return o;
}

// JSON number text (grammar already validated) -> binary64
YM_NUM_FN double json_num_to_f64(const uint8_t *a, uint64_t n) {
  uint64_t i = 0;
  bool neg = false;
  if (i < n && a[i] == '-') { neg = true; i++; }
  uint8_t dg[DEC_MAX_DIGITS];
  int nd = 0;
  bool sticky = false;
  int32_t k10 = 0;  // value = 0.? no: value = digits * 10^k10
  bool seen = false;  // a nonzero digit seen
  // integer part
  while (i < n && a[i] >= '0' && a[i] <= '9') {
    const uint8_t v = a[i] - '0';
    if (seen || v) {
      seen = true;
      if (nd < DEC_MAX_DIGITS) dg[nd++] = v;
      else { k10++; if (v) sticky = true; }
    }
    i++;
  }
  if (i < n && a[i] == '.') {
    i++;
    while (i < n && a[i] >= '0' && a[i] <= '9') {
      const uint8_t v = a[i] - '0';
      if (seen || v) {
        seen = true;
        if (nd < DEC_MAX_DIGITS) { dg[nd++] = v; k10--; }
        else if (v) sticky = true;
      } else {
        k10--;
      }
      i++;
    }
  }
  int64_t ex = 0;
  if (i < n && (a[i] == 'e' || a[i] == 'E')) {
    i++;
    bool eneg = false;
    if (i < n && (a[i] == '+' || a[i] == '-')) { eneg = a[i] == '-'; i++; }
    while (i < n && a[i] >= '0' && a[i] <= '9') {
      if (ex < 100000000) ex = ex * 10 + (a[i] - '0');
      i++;
    }
    if (eneg) ex = -ex;
  }
  // trailing zeros of the significand
  while (nd > 0 && dg[nd - 1] == 0) { nd--; k10++; }
  double x;
  if (nd == 0) x = 0.0;
  else {
    int64_t kk = (int64_t)k10 + ex;
    if (kk + nd > 400) x = __builtin_inf();
    else if (kk + nd < -400) x = 0.0;
    else x = dec_to_f64(dg, nd, (int32_t)kk, sticky);
  }
  return neg ? -x : x;
}

}  // namespace ym
