// Test-only host check of ym_utf8.h (the SWAR strict UTF-8 validator, 4- and 8-byte words, / UTF-16 length of the device parsers)
// against a byte-wise decoder with lib0's rules (decodeURIComponent(escape(s)): strict UTF-8).  Exhaustive over
// every 1-, 2- and 3-byte input at several alignments inside ASCII padding, random 4-byte inputs, and random
// texts of valid characters with random corruptions at every length up to 80.  Prints "ok <cases>" or the
// first mismatch and exits 1.
#define YM_HD
#include "../../yjs_amd/csrc/ym_utf8.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

static uint32_t ref_units(const uint8_t *b, uint32_t i, uint32_t e, bool &bad) {
  uint32_t u = 0;
  while (i < e) {
    const uint32_t x = b[i];
    if (x < 0x80) { u++; i++; continue; }
    uint32_t len, cp, mn;
    if ((x & 0xE0) == 0xC0) { len = 2; cp = x & 0x1F; mn = 0x80; }
    else if ((x & 0xF0) == 0xE0) { len = 3; cp = x & 0x0F; mn = 0x800; }
    else if ((x & 0xF8) == 0xF0) { len = 4; cp = x & 0x07; mn = 0x10000; }
    else { bad = true; return 0; }
    if (i + len > e) { bad = true; return 0; }
    for (uint32_t q = 1; q < len; q++) {
      const uint32_t cb = b[i + q];
      if ((cb & 0xC0) != 0x80) { bad = true; return 0; }
      cp = (cp << 6) | (cb & 0x3F);
    }
    if (cp < mn || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) { bad = true; return 0; }
    u += cp >= 0x10000 ? 2 : 1;
    i += len;
  }
  return u;
}

static uint8_t buf[256];
static long cases = 0;

static void check(uint32_t i, uint32_t e) {
  bool rb = false, sb = false;
  const uint32_t ru = ref_units(buf, i, e, rb);
  const uint32_t su = ymk::utf8::units<uint64_t>([](uint32_t p) { uint64_t x; memcpy(&x, buf + p, 8); return x; }, i, e, sb);
  bool sb4 = false;
  const uint32_t su4 = ymk::utf8::units<uint32_t>([](uint32_t p) { uint32_t x; memcpy(&x, buf + p, 4); return x; }, i, e, sb4);
  cases++;
  if (rb != sb || (!rb && ru != su) || rb != sb4 || (!rb && ru != su4)) {
    printf("mismatch at [%u, %u): ref bad %d units %u, swar8 bad %d units %u, swar4 bad %d units %u; bytes", i, e, rb, ru,
           sb, su, sb4, su4);
    for (uint32_t k = i; k < e; k++) printf(" %02x", buf[k]);
    printf("\n");
    exit(1);
  }
}

int main() {
  std::mt19937_64 rng(12345);
  // exhaustive 1 / 2 / 3-byte inputs at offsets 0..7 (3 bytes: offsets 0, 5, 6, 7), ASCII and junk around them
  for (uint32_t n = 1; n <= 3; n++) {
    const uint64_t total = 1ull << (8 * n);
    for (uint64_t v = 0; v < total; v++) {
      for (uint32_t off = 0; off < 8; off++) {
        if (n == 3 && off != 0 && off < 5) continue;
        memset(buf, 'a', sizeof buf);
        for (uint32_t k = 0; k < n; k++) buf[16 + off + k] = (uint8_t)(v >> (8 * k));
        check(16 + off, 16 + off + n);              // the bytes alone
        check(16, 16 + off + n + 3);                // inside ASCII
        buf[16 + off + n] = 0xBF;                   // a continuation right after
        check(16 + off, 16 + off + n + 1);
      }
    }
  }
  // random 4-byte inputs
  for (long t = 0; t < 20000000; t++) {
    const uint64_t v = rng();
    const uint32_t off = (uint32_t)(v >> 40) & 7;
    memset(buf, 'a', 64);
    for (uint32_t k = 0; k < 4; k++) buf[16 + off + k] = (uint8_t)(v >> (8 * k));
    check(16 + off, 20 + off);
    check(16, 24 + off);
  }
  // random texts: valid characters (ASCII, 2, 3, 4 bytes, edge code points), some corrupted
  static const uint32_t edges[] = {0x7f, 0x80, 0x7ff, 0x800, 0xd7ff, 0xe000, 0xfffd, 0xffff, 0x10000, 0x10ffff};
  for (long t = 0; t < 3000000; t++) {
    uint32_t len = 0;
    const uint32_t want = (uint32_t)(rng() % 81);
    while (len < want && len < 200) {
      const uint64_t r = rng();
      uint32_t cp;
      switch (r % 6) {
        case 0: case 1: cp = 0x20 + (uint32_t)(r >> 8) % 0x5f; break;
        case 2: cp = 0x80 + (uint32_t)(r >> 8) % 0x780; break;
        case 3: cp = 0x800 + (uint32_t)(r >> 8) % 0xf800; if (cp >= 0xd800 && cp < 0xe000) cp = 0x4e00; break;
        case 4: cp = 0x10000 + (uint32_t)(r >> 8) % 0x100000; break;
        default: cp = edges[(r >> 8) % 10];
      }
      uint8_t *o = buf + 8 + len;
      if (cp < 0x80) { o[0] = (uint8_t)cp; len += 1; }
      else if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 63); len += 2; }
      else if (cp < 0x10000) { o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 63); o[2] = 0x80 | (cp & 63); len += 3; }
      else { o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 63); o[2] = 0x80 | ((cp >> 6) & 63); o[3] = 0x80 | (cp & 63); len += 4; }
    }
    if (t % 3 == 0 && len > 0) buf[8 + rng() % len] = (uint8_t)rng();  // one corrupted byte
    const uint32_t a = (uint32_t)(rng() % (len + 1)), b = a + (uint32_t)(rng() % (len - a + 1));
    check(8, 8 + len);
    check(8 + a, 8 + b);  // any slice (may cut characters)
  }
  printf("ok %ld\n", cases);
  return 0;
}
