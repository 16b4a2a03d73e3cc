// ym_fast.hip -- LDS fast path: one 64-lane wave per document, the whole document staged in LDS.
//
// Takes mergeUpdates (V1) documents whose inputs are "simple": every update's structs increase in
// (client desc, clock asc), no two structs overlap, no GC/Skip structs, canonical encodings, payloads
// of the kinds yjs writes (strings, formats/embeds with literal JSON, scalar `any` values).  For such
// documents yjs 13.5.16's k-way merge (bundle ds@39007) reduces to: all structs sorted by
// (client desc, clock asc), a Skip before every clock gap, consecutive same-client structs grouped
// into one part (SURVEY.md App. B "Consequences for the GPU design"); the delete set is the per-client
// union of all inputs' ranges with clients in first-appearance order (DeleteSet.js:113-161, 13.5.16
// le@10242 / he@10482).  Everything else is declined (status ST_PENDING) and handled exactly by the
// general path (ym_general.hip).
//
// Per document (one wave, ~10 KB of LDS, no scratch):
//   16-B loads of the update bytes into LDS -> lanes walk updates (count pass, wave scan, emit pass)
//   -> bitonic sort of (client, clock) keys -> struct sizes + part headers by wave scans -> delete-set
//   union, one lane per client -> output staged in LDS -> 16-B stores into the doc's slot.
// Output slot of doc d: 2 * (input bytes before d) + 64 * d, 16-aligned (a bound the kernel checks),
// so the fast path needs no global atomics; the general path appends after that region.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ym_kernels.h"

namespace ymk {

template <int IN, int UPD, int REC, int DS, int OUT>
struct FastCfg {
  static constexpr int kIn = IN, kUpd = UPD, kRec = REC, kDs = DS, kOut = OUT;
};

// LDS layout (byte offsets into the dynamic LDS block), every array 16-aligned
template <class C>
struct Lay {
  static constexpr int a16(int x) { return (x + 15) & ~15; }
  static constexpr int rkey = 0;                                 // u64[REC] (client desc, clock)
  static constexpr int dkey = a16(rkey + 8 * C::kRec);           // u64[DS]  (client, clock)
  static constexpr int rlen = a16(dkey + 8 * C::kDs);            // u32[REC] struct length
  static constexpr int dlen = a16(rlen + 4 * C::kRec);           // u32[DS]  range length (by idx)
  static constexpr int dend = a16(dlen + 4 * C::kDs);            // u32[DS]  union end at interval start
  static constexpr int rpos = a16(dend + 4 * C::kDs);            // u16[REC] inclusive struct-count prefix
  static constexpr int rstart = a16(rpos + 2 * C::kRec);         // u16[REC] struct start in `in`
  static constexpr int rblen = a16(rstart + 2 * C::kRec);        // u16[REC] struct bytes incl. info
  static constexpr int ridx = a16(rblen + 2 * C::kRec);          // u16[REC] sort payload
  static constexpr int didx = a16(ridx + 2 * C::kRec);           // u16[DS]  sort payload = appearance
  static constexpr int dseq = a16(didx + 2 * C::kDs);            // u16[DS]  (update << 8 | position) by slot
  static constexpr int dflag = a16(dseq + 2 * C::kDs);           // u8[DS]   interval start flags
  static constexpr int rinfo = a16(dflag + C::kDs);              // u8[REC]
  static constexpr int uoff = a16(rinfo + C::kRec);              // u16[UPD+1]
  static constexpr int ubase = a16(uoff + 2 * (C::kUpd + 1));    // u16[UPD]
  static constexpr int dbase = a16(ubase + 2 * C::kUpd);         // u16[UPD]
  static constexpr int gstart = a16(dbase + 2 * C::kUpd);        // u16[DS+1] group start entry
  static constexpr int gmin = a16(gstart + 2 * (C::kDs + 1));    // u16[DS]  group first appearance
  static constexpr int gsz = a16(gmin + 2 * C::kDs);             // u16[DS]  group bytes
  static constexpr int gcnt = a16(gsz + 2 * C::kDs);             // u16[DS]  group interval count
  static constexpr int grank = a16(gcnt + 2 * C::kDs);           // u16[DS]  group -> rank
  static constexpr int roff = a16(grank + 2 * C::kDs);           // u16[DS]  rank -> byte offset
  static constexpr int misc = a16(roff + 2 * C::kDs);            // u32[16]
  static constexpr int in = a16(misc + 64);                      // u8[IN + 16]
  static constexpr int out = a16(in + C::kIn + 16);              // u8[OUT]
  static constexpr int total = a16(out + C::kOut);
};

extern __shared__ __attribute__((aligned(16))) uint8_t g_smem[];

template <class T>
__device__ __forceinline__ T *lds(int off) { return reinterpret_cast<T *>(g_smem + off); }

// ---- wave primitives ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

__device__ __forceinline__ uint32_t vsz(uint64_t v) {
  uint32_t n = 1;
  while (v > 127) { v >>= 7; n++; }
  return n;
}
__device__ __forceinline__ uint32_t put_vu(uint8_t *o, uint32_t p, uint64_t v) {
  while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
  o[p++] = (uint8_t)v;
  return p;
}

// ---- lean V1 walker over LDS bytes -------------------------------------------------------------
// Any anomaly (truncation, non-canonical varint, invalid UTF-8, a payload kind this path does not
// verify) sets `bad`; the general path then reproduces yjs's exact result or error.
struct Cur {
  uint32_t p, end;  // byte offsets into the dynamic LDS block
  bool bad;
};
__device__ __forceinline__ uint32_t lb(uint32_t off) { return g_smem[off]; }
__device__ __forceinline__ uint32_t rdb(Cur &c) {
  if (c.p >= c.end) { c.bad = true; return 0; }
  return g_smem[c.p++];
}
// unaligned 8-byte little-endian window at LDS offset p (two aligned dword reads + funnel shift);
// the staging buffer has >= 8 bytes of slack past every document
__device__ __forceinline__ uint64_t win8(uint32_t p) {
  const uint32_t a = p & ~3u;
  const uint32_t w0 = *reinterpret_cast<const uint32_t *>(g_smem + a);
  const uint32_t w1 = *reinterpret_cast<const uint32_t *>(g_smem + a + 4);
  const uint32_t w2 = *reinterpret_cast<const uint32_t *>(g_smem + a + 8);
  const uint32_t sh = (p & 3u) * 8u;
  const uint64_t lo = ((uint64_t)w1 << 32) | w0;
  return sh ? (lo >> sh) | ((uint64_t)w2 << (64 - sh)) : lo;
}
// lib0 readVarUint, canonical encodings only, branch-free over a 5-byte window
__device__ __forceinline__ uint32_t rvu(Cur &c) {
  const uint64_t x = win8(c.p);
  const uint64_t stop = ~x & 0x8080808080ull;
  if (stop == 0) { c.bad = true; return 0; }
  const uint32_t nb = (uint32_t)(__builtin_ctzll(stop) >> 3) + 1;
  uint64_t v = (x & 0x7full) | ((x >> 1) & (0x7full << 7)) | ((x >> 2) & (0x7full << 14)) |
               ((x >> 3) & (0x7full << 21)) | ((x >> 4) & (0x7full << 28));
  v &= (1ull << (7 * nb)) - 1;
  const uint32_t last = (uint32_t)(x >> (8 * (nb - 1))) & 0xff;
  if ((nb > 1 && last == 0) || v > 0xffffffffull || nb > c.end - c.p) c.bad = true;
  c.p += nb;
  return (uint32_t)v;
}
// strict UTF-8 (decodeURIComponent(escape(..))) over the next n bytes; returns the UTF-16 length
__device__ __forceinline__ uint32_t utf8_len16(Cur &c, uint32_t n) {
  if (n > c.end - c.p) { c.bad = true; return 0; }
  {  // ASCII fast path: 8 bytes per window
    uint64_t hi = 0;
    for (uint32_t o = 0; o < n; o += 8) {
      uint64_t x = win8(c.p + o);
      if (n - o < 8) x &= (1ull << (8 * (n - o))) - 1;
      hi |= x;
    }
    if ((hi & 0x8080808080808080ull) == 0) { c.p += n; return n; }
  }
  uint32_t i = c.p, u = 0;
  const uint32_t e = c.p + n;
  while (i < e) {
    const uint32_t b = lb(i);
    if (b < 0x80) { u++; i++; continue; }
    uint32_t len, cp, mn;
    if ((b & 0xE0) == 0xC0) { len = 2; cp = b & 0x1F; mn = 0x80; }
    else if ((b & 0xF0) == 0xE0) { len = 3; cp = b & 0x0F; mn = 0x800; }
    else if ((b & 0xF8) == 0xF0) { len = 4; cp = b & 0x07; mn = 0x10000; }
    else { c.bad = true; return 0; }
    if (i + len > e) { c.bad = true; return 0; }
    for (uint32_t q = 1; q < len; q++) {
      const uint32_t cb = lb(i + q);
      if ((cb & 0xC0) != 0x80) { c.bad = true; return 0; }
      cp = (cp << 6) | (cb & 0x3F);
    }
    if (cp < mn || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) { c.bad = true; return 0; }
    u += cp >= 0x10000 ? 2 : 1;
    i += len;
  }
  c.p = e;
  return u;
}
__device__ __forceinline__ uint32_t rstr(Cur &c) {  // varString -> UTF-16 length
  const uint32_t n = rvu(c);
  if (c.bad) return 0;
  return utf8_len16(c, n);
}
// JSON text as yjs writes it for formats / embeds: true | false | null | "string without escapes"
__device__ __forceinline__ void json_lit(Cur &c) {
  const uint32_t n = rvu(c);
  if (c.bad || n > c.end - c.p) { c.bad = true; return; }
  const uint8_t *t = g_smem + c.p;
  bool ok = false;
  if (n == 4 && t[0] == 't' && t[1] == 'r' && t[2] == 'u' && t[3] == 'e') ok = true;
  else if (n == 4 && t[0] == 'n' && t[1] == 'u' && t[2] == 'l' && t[3] == 'l') ok = true;
  else if (n == 5 && t[0] == 'f' && t[1] == 'a' && t[2] == 'l' && t[3] == 's' && t[4] == 'e') ok = true;
  else if (n >= 2 && t[0] == '"' && t[n - 1] == '"') {
    ok = true;
    for (uint32_t i = 1; i + 1 < n; i++)
      if (t[i] < 0x20 || t[i] == '"' || t[i] == '\\') ok = false;
  }
  if (!ok) { c.bad = true; return; }
  utf8_len16(c, n);
}
// one scalar `any` value in the canonical form lib0 writeAny emits (objects/arrays: general path)
__device__ __forceinline__ void any_scalar(Cur &c) {
  const uint32_t tag = rdb(c);
  switch (tag) {
    case 127: case 126: case 121: case 120: return;
    case 125: {  // varInt: minimal, and <= 2^31-1 when positive (larger is written as a float)
      uint32_t b = rdb(c);
      uint64_t mag = b & 63;
      const bool neg = b & 64;
      int s = 6, nb = 1;
      while (b & 128) {
        b = rdb(c);
        if (c.bad || s > 34) { c.bad = true; return; }
        mag |= (uint64_t)(b & 127) << s;
        s += 7;
        nb++;
      }
      if ((nb > 1 && b == 0) || (!neg && mag > 2147483647ull) || mag > 0xffffffffull) c.bad = true;
      return;
    }
    case 124: {  // float32, not an integer <= 2^31-1 (those are written as varInt), not NaN
      if (c.end - c.p < 4) { c.bad = true; return; }
      const uint32_t u = (lb(c.p) << 24) | (lb(c.p + 1) << 16) | (lb(c.p + 2) << 8) | lb(c.p + 3);
      const float f = __uint_as_float(u);
      if (f != f || (truncf(f) == f && (double)f <= 2147483647.0)) c.bad = true;
      c.p += 4;
      return;
    }
    case 123: {  // float64 that is neither a small integer nor float32-exact
      if (c.end - c.p < 8) { c.bad = true; return; }
      uint64_t u = 0;
      for (int i = 0; i < 8; i++) u = (u << 8) | lb(c.p + i);
      const double x = __longlong_as_double((long long)u);
      if (x == x && ((trunc(x) == x && x <= 2147483647.0) || (double)(float)x == x)) c.bad = true;
      c.p += 8;
      return;
    }
    case 119: rstr(c); return;
    default: c.bad = true; return;
  }
}

// Walks update u (LDS bytes [base+uoff[u], base+uoff[u+1])) and appends its structs and delete-set
// entries to the document's record arrays through LDS atomic slot counters (misc[2], misc[3]); the
// records are sorted afterwards, and a delete entry's payload (update << 8 | position) keeps yjs's
// first-appearance order.  Returns false to decline the document.
template <class C>
__device__ __attribute__((noinline)) bool walk_v1(uint32_t base, uint32_t u) {
  using L = Lay<C>;
  const uint16_t *uoff = lds<uint16_t>(L::uoff);
  uint32_t *misc = lds<uint32_t>(L::misc);
  Cur c = {(uint32_t)L::in + base + uoff[u], (uint32_t)L::in + base + uoff[u + 1], false};
  const uint32_t nclients = rvu(c);
  uint64_t prev = 0;
  bool have_prev = false;
  for (uint32_t ci = 0; ci < nclients && !c.bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = rvu(c);
    uint64_t clock = rvu(c);
    for (uint32_t si = 0; si < nstructs && !c.bad; si++) {
      const uint32_t s0 = c.p;
      const uint32_t info = rdb(c);
      if (c.bad || info == 10 || (info & 31) == 0) return false;  // Skip / GC -> general path
      if (info & 0x80) { rvu(c); rvu(c); }
      if (info & 0x40) { rvu(c); rvu(c); }
      if ((info & 0xC0) == 0) {
        const uint32_t pi = rvu(c);
        if (pi > 1) return false;  // parentInfo re-encodes as 0/1
        if (pi == 1) rstr(c);
        else { rvu(c); rvu(c); }
        if (info & 0x20) rstr(c);
      }
      uint64_t len = 1;
      switch (info & 31) {
        case 1: len = rvu(c); break;                                           // ContentDeleted
        case 3: { const uint32_t n = rvu(c); if (n > c.end - c.p) c.bad = true; else c.p += n; break; }  // Binary
        case 4: len = rstr(c); break;                                          // ContentString
        case 5: json_lit(c); break;                                            // ContentEmbed
        case 6: rstr(c); json_lit(c); break;                                   // ContentFormat
        case 7: {                                                              // ContentType
          const uint32_t t = rvu(c);
          if (t > 6) return false;
          if (t == 3 || t == 5) rstr(c);
          break;
        }
        case 8:                                                                // ContentAny
          len = rvu(c);
          for (uint64_t i = 0; i < len && !c.bad; i++) any_scalar(c);
          break;
        default: return false;  // ContentJSON, ContentDoc, invalid refs
      }
      if (c.bad || len == 0) return false;
      const uint64_t end = clock + len;
      if (end > 0xffffffffull) return false;
      const uint64_t key = ((uint64_t)(~client) << 32) | clock;
      if (have_prev && key <= prev) return false;  // each update must already be in merge order
      prev = key + len - 1;
      have_prev = true;
      const uint32_t q = atomicAdd(&misc[2], 1u);
      if (q >= (uint32_t)C::kRec) return false;
      lds<uint64_t>(L::rkey)[q] = key;
      lds<uint32_t>(L::rlen)[q] = (uint32_t)len;
      lds<uint16_t>(L::rstart)[q] = (uint16_t)(s0 - L::in);
      lds<uint16_t>(L::rblen)[q] = (uint16_t)(c.p - s0);
      lds<uint8_t>(L::rinfo)[q] = (uint8_t)info;
      lds<uint16_t>(L::ridx)[q] = (uint16_t)q;
      clock = end;
    }
  }
  if (c.bad) return false;
  const uint32_t ndc = rvu(c);  // delete set (DeleteSet.js:219-256)
  uint32_t pos = 0;
  for (uint32_t i = 0; i < ndc && !c.bad; i++) {
    const uint32_t client = rvu(c);
    const uint32_t m = rvu(c);
    for (uint32_t q = 0; q < m && !c.bad; q++, pos++) {
      const uint32_t clock = rvu(c);
      const uint32_t len = rvu(c);
      if (c.bad || pos > 255) return false;
      const uint32_t x = atomicAdd(&misc[3], 1u);
      if (x >= (uint32_t)C::kDs) return false;
      lds<uint64_t>(L::dkey)[x] = ((uint64_t)client << 32) | clock;
      lds<uint32_t>(L::dlen)[x] = len;
      lds<uint16_t>(L::didx)[x] = (uint16_t)x;
      lds<uint16_t>(L::dseq)[x] = (uint16_t)((u << 8) | pos);
    }
  }
  return !c.bad;
}

__device__ __forceinline__ void bitonic(uint64_t *key, uint16_t *idx, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t size = 2; size <= n; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (uint32_t t = lane; t < n / 2; t += 64) {
        const uint32_t i = 2 * t - (t & (stride - 1));
        const uint32_t q = i + stride;
        const bool up = (i & size) == 0;
        const uint64_t a = key[i], b = key[q];
        if ((a > b) == up) {
          key[i] = b;
          key[q] = a;
          const uint16_t x = idx[i];
          idx[i] = idx[q];
          idx[q] = x;
        }
      }
    }
  }
  __syncthreads();
}

// STOP > 0 builds a timing-only variant that ends every document after phase STOP (profiling the
// phases by ablation, cdna_hip_programming.md §7); outputs of such builds are not meaningful.
#define YM_STOP(n)                                          \
  if (STOP == (n)) {                                        \
    if (lane == 0) { j.status[d] = ym::ST_OK; j.out_len[d] = 0; } \
    __syncthreads();                                        \
    continue;                                               \
  }
template <class C, int STOP>
__global__ void __launch_bounds__(64) k_fast_merge_v1(GeneralJob j) {
  using L = Lay<C>;
  const uint32_t lane = threadIdx.x;
  uint32_t *misc = lds<uint32_t>(L::misc);
  uint8_t *in = lds<uint8_t>(L::in);
  uint8_t *out = lds<uint8_t>(L::out);
  uint64_t *rkey = lds<uint64_t>(L::rkey);
  uint64_t *dkey = lds<uint64_t>(L::dkey);
  uint32_t *rlen = lds<uint32_t>(L::rlen);
  uint32_t *dlen = lds<uint32_t>(L::dlen);
  uint32_t *dend = lds<uint32_t>(L::dend);
  uint16_t *rpos = lds<uint16_t>(L::rpos);
  uint16_t *rstart = lds<uint16_t>(L::rstart);
  uint16_t *rblen = lds<uint16_t>(L::rblen);
  uint16_t *ridx = lds<uint16_t>(L::ridx);
  uint16_t *didx = lds<uint16_t>(L::didx);
  uint16_t *dseq = lds<uint16_t>(L::dseq);
  uint8_t *dflag = lds<uint8_t>(L::dflag);
  uint8_t *rinfo = lds<uint8_t>(L::rinfo);
  uint16_t *uoff = lds<uint16_t>(L::uoff);
  uint16_t *ubase = lds<uint16_t>(L::ubase);
  uint16_t *dbase = lds<uint16_t>(L::dbase);
  uint16_t *gstart = lds<uint16_t>(L::gstart);
  uint16_t *gmin = lds<uint16_t>(L::gmin);
  uint16_t *gsz = lds<uint16_t>(L::gsz);
  uint16_t *gcnt = lds<uint16_t>(L::gcnt);
  uint16_t *grank = lds<uint16_t>(L::grank);
  uint16_t *roff = lds<uint16_t>(L::roff);
  constexpr int ROUNDS = (C::kUpd + 63) / 64;
  const uint64_t arena0 = j.upd_off[0];

  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    const uint32_t u0 = j.doc_upd[d], k = j.doc_upd[d + 1] - u0;
    const uint64_t b0 = j.upd_off[u0], bytes = j.upd_off[u0 + k] - b0;
    if (k <= 1 || k > (uint32_t)C::kUpd || bytes > (uint64_t)C::kIn) {
      if (lane == 0) j.status[d] = ST_PENDING;
      continue;
    }
    // 1. stage with 16-B loads covering [b0, b0 + bytes); `base` = b0 & 15
    const uint32_t base = (uint32_t)(b0 & 15);
    {
      const uint4 *src = reinterpret_cast<const uint4 *>(j.A + (b0 - base));
      const uint32_t nvec = (uint32_t)((base + bytes + 15) >> 4);
      for (uint32_t v = lane; v < nvec; v += 64) reinterpret_cast<uint4 *>(in)[v] = src[v];
    }
    for (uint32_t i = lane; i <= k; i += 64) uoff[i] = (uint16_t)(j.upd_off[u0 + i] - b0);
    __syncthreads();
    YM_STOP(1)
    // 2. one pass over the updates, one lane per update; records appended through LDS atomics
    if (lane == 0) { misc[2] = 0; misc[3] = 0; }
    __syncthreads();
    bool ok = true;
#pragma unroll 1
    for (uint32_t u = lane; u < k; u += 64) ok &= walk_v1<C>(base, u);
    if (__any(!ok)) {
      if (lane == 0) j.status[d] = ST_PENDING;
      __syncthreads();
      continue;
    }
    __syncthreads();
    const uint32_t nrec = misc[2], nds = misc[3];
    if (nrec == 0 || nrec > (uint32_t)C::kRec || nds > (uint32_t)C::kDs) {
      if (lane == 0) j.status[d] = ST_PENDING;
      __syncthreads();
      continue;
    }
    YM_STOP(3)
    uint32_t np2 = 64;
    while (np2 < nrec) np2 <<= 1;
    for (uint32_t i = nrec + lane; i < np2; i += 64) { rkey[i] = ~0ull; ridx[i] = 0; }
    uint32_t dp2 = 64;
    while (dp2 < nds) dp2 <<= 1;
    for (uint32_t i = nds + lane; i < dp2; i += 64) { dkey[i] = ~0ull; didx[i] = 0; }
    // 4. sorts: structs by (client desc, clock asc); delete ranges by (client, clock)
    bitonic(rkey, ridx, np2);
    if (nds > 1) bitonic(dkey, didx, dp2);
    YM_STOP(4)
    // 5. struct section; lane owns sorted records [lo, hi)
    const uint32_t per = (nrec + 63) >> 6;
    const uint32_t lo = lane * per < nrec ? lane * per : nrec;
    const uint32_t hi = lo + per < nrec ? lo + per : nrec;
    bool bad = false;
    uint32_t units = 0;
    for (uint32_t i = lo; i < hi; i++) {
      uint32_t un = 1;
      if (i > 0 && (rkey[i - 1] >> 32) == (rkey[i] >> 32)) {
        const uint64_t pend = (rkey[i - 1] & 0xffffffffull) + rlen[ridx[i - 1]];
        const uint64_t cl = rkey[i] & 0xffffffffull;
        if (pend > cl) bad = true;       // overlapping inputs: general path
        else if (pend < cl) un = 2;      // a Skip fills the gap
      }
      units += un;
    }
    if (__any(bad)) {
      if (lane == 0) j.status[d] = ST_PENDING;
      __syncthreads();
      continue;
    }
    {
      uint32_t tot_units;
      uint32_t acc = wave_excl_scan(units, &tot_units);
      for (uint32_t i = lo; i < hi; i++) {
        uint32_t un = 1;
        if (i > 0 && (rkey[i - 1] >> 32) == (rkey[i] >> 32) &&
            (rkey[i - 1] & 0xffffffffull) + rlen[ridx[i - 1]] < (rkey[i] & 0xffffffffull))
          un = 2;
        acc += un;
        rpos[i] = (uint16_t)acc;  // inclusive prefix of output structs (incl. Skips)
      }
    }
    __syncthreads();
    uint32_t bytes_l = 0, parts_l = 0;
    for (uint32_t i = lo; i < hi; i++) {
      const uint64_t key = rkey[i];
      bytes_l += rblen[ridx[i]];
      if (i == 0 || (rkey[i - 1] >> 32) != (key >> 32)) {  // part header: vu(#structs) vu(client) vu(clock)
        uint32_t e = i + 1;
        while (e < nrec && (rkey[e] >> 32) == (key >> 32)) e++;
        const uint32_t run_units = rpos[e - 1] - (i ? rpos[i - 1] : 0);
        bytes_l += vsz(run_units) + vsz(~(uint32_t)(key >> 32)) + vsz(key & 0xffffffffull);
        parts_l++;
      } else {
        const uint64_t pend = (rkey[i - 1] & 0xffffffffull) + rlen[ridx[i - 1]];
        if (pend < (key & 0xffffffffull)) bytes_l += 1 + vsz((key & 0xffffffffull) - pend);
      }
    }
    uint32_t struct_bytes, nparts;
    const uint32_t b_excl = wave_excl_scan(bytes_l, &struct_bytes);
    wave_excl_scan(parts_l, &nparts);
    const uint32_t hdr = vsz(nparts);
    YM_STOP(5)
    // 6. delete set.  Groups = clients (runs of equal client in the sorted entries).
    const uint32_t dper = (nds + 63) >> 6;
    const uint32_t dlo = lane * dper < nds ? lane * dper : nds;
    const uint32_t dhi = dlo + dper < nds ? dlo + dper : nds;
    uint32_t gs_l = 0;
    for (uint32_t i = dlo; i < dhi; i++) gs_l += (i == 0 || (dkey[i] >> 32) != (dkey[i - 1] >> 32));
    uint32_t ngroups;
    uint32_t g = wave_excl_scan(gs_l, &ngroups);
    for (uint32_t i = dlo; i < dhi; i++)
      if (i == 0 || (dkey[i] >> 32) != (dkey[i - 1] >> 32)) gstart[g++] = (uint16_t)i;
    if (lane == 0) gstart[ngroups] = (uint16_t)nds;
    __syncthreads();
    // one lane per group: in-place union (>= merges touching ranges), count, bytes, first appearance
    for (uint32_t gg = lane; gg < ngroups; gg += 64) {
      const uint32_t s = gstart[gg], e = gstart[gg + 1];
      uint32_t mn = 0xffff, cnt = 0, sz = 0, open = s;
      uint64_t cure = 0;
      for (uint32_t i = s; i < e; i++) {
        const uint32_t id = didx[i];
        if (dseq[id] < mn) mn = dseq[id];
        const uint64_t c0 = dkey[i] & 0xffffffffull;
        const uint64_t en = c0 + dlen[id];
        if (i == s || c0 > cure) {
          if (i != s) { dend[open] = (uint32_t)cure; sz += vsz(dkey[open] & 0xffffffffull) + vsz(cure - (dkey[open] & 0xffffffffull)); }
          open = i;
          cure = en;
          dflag[i] = 1;
          cnt++;
        } else {
          dflag[i] = 0;
          if (en > cure) cure = en;
        }
      }
      dend[open] = (uint32_t)cure;
      sz += vsz(dkey[open] & 0xffffffffull) + vsz(cure - (dkey[open] & 0xffffffffull));
      sz += vsz(dkey[s] >> 32) + vsz(cnt);
      gmin[gg] = (uint16_t)mn;
      gsz[gg] = (uint16_t)sz;
      gcnt[gg] = (uint16_t)cnt;
    }
    __syncthreads();
    // rank groups by first appearance; lay out their bytes in rank order
    for (uint32_t gg = lane; gg < ngroups; gg += 64) {
      uint32_t r = 0;
      const uint32_t m = gmin[gg];
      for (uint32_t h = 0; h < ngroups; h++) r += gmin[h] < m;
      grank[gg] = (uint16_t)r;
      roff[r] = gsz[gg];
    }
    __syncthreads();
    {
      const uint32_t gper = (ngroups + 63) >> 6;
      const uint32_t glo = lane * gper < ngroups ? lane * gper : ngroups;
      const uint32_t ghi = glo + gper < ngroups ? glo + gper : ngroups;
      uint32_t s = 0;
      for (uint32_t r = glo; r < ghi; r++) s += roff[r];
      uint32_t tot;
      uint32_t ex = wave_excl_scan(s, &tot);
      for (uint32_t r = glo; r < ghi; r++) { const uint32_t v = roff[r]; roff[r] = (uint16_t)ex; ex += v; }
      if (lane == 0) misc[1] = tot;
    }
    __syncthreads();
    const uint32_t ds_bytes = vsz(ngroups) + misc[1];
    const uint32_t total = hdr + struct_bytes + ds_bytes;
    // output slot: 16-aligned inside the bound 2 * in + 64 per doc
    const uint64_t slot = 2 * (b0 - arena0) + 64ull * d;
    const uint64_t slot_al = (slot + 15) & ~15ull;
    if (total > (uint32_t)C::kOut || slot_al + total > slot + 2 * bytes + 64) {
      if (lane == 0) j.status[d] = ST_PENDING;
      __syncthreads();
      continue;
    }
    if (slot_al + total > j.cap) {  // caller's arena is smaller than the fast region
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    YM_STOP(6)
    // 7. struct section into LDS staging
    if (lane == 0) put_vu(out, 0, nparts);
    {
      uint32_t p = hdr + b_excl;
      for (uint32_t i = lo; i < hi; i++) {
        const uint32_t id = ridx[i];
        const uint64_t key = rkey[i];
        const uint64_t clock = key & 0xffffffffull;
        if (i == 0 || (rkey[i - 1] >> 32) != (key >> 32)) {
          uint32_t e = i + 1;
          while (e < nrec && (rkey[e] >> 32) == (key >> 32)) e++;
          const uint32_t run_units = rpos[e - 1] - (i ? rpos[i - 1] : 0);
          p = put_vu(out, p, run_units);
          p = put_vu(out, p, ~(uint32_t)(key >> 32));
          p = put_vu(out, p, clock);
        } else {
          const uint64_t pend = (rkey[i - 1] & 0xffffffffull) + rlen[ridx[i - 1]];
          if (pend < clock) {  // Skip: info 10 + varuint length (13.5.16 ui.write)
            out[p++] = 10;
            p = put_vu(out, p, clock - pend);
          }
        }
        uint32_t info = rinfo[id];
        if (info & 0xC0) info &= ~0x20u;  // parentSub is only read / re-written without origins
        out[p++] = (uint8_t)info;
        const uint32_t s0 = rstart[id] + 1, n = rblen[id] - 1;
        for (uint32_t b = 0; b < n; b++) out[p + b] = in[s0 + b];
        p += n;
      }
    }
    // 8. delete set: vu(ngroups) | per client (first-appearance order): client, count, ranges
    {
      const uint32_t dsb = hdr + struct_bytes;
      if (lane == 0) put_vu(out, dsb, ngroups);
      const uint32_t gbase = dsb + vsz(ngroups);
      for (uint32_t gg = lane; gg < ngroups; gg += 64) {
        const uint32_t s = gstart[gg], e = gstart[gg + 1];
        uint32_t p = gbase + roff[grank[gg]];
        p = put_vu(out, p, dkey[s] >> 32);
        p = put_vu(out, p, gcnt[gg]);
        for (uint32_t q = s; q < e; q++) {
          if (!dflag[q]) continue;
          const uint32_t c0 = (uint32_t)(dkey[q] & 0xffffffffull);
          p = put_vu(out, p, c0);
          p = put_vu(out, p, dend[q] - c0);
        }
      }
    }
    __syncthreads();
    YM_STOP(8)
    // 9. 16-B stores into the doc's slot
    {
      uint8_t *dst = j.out + slot_al;
      const uint32_t nvec = total >> 4;
      for (uint32_t v = lane; v < nvec; v += 64) reinterpret_cast<uint4 *>(dst)[v] = reinterpret_cast<const uint4 *>(out)[v];
      for (uint32_t b = (nvec << 4) + lane; b < total; b += 64) dst[b] = out[b];
    }
    if (lane == 0) {
      j.out_off[d] = slot_al;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}

using SmallCfg = FastCfg<2560, 128, 128, 128, 2048>;

// the general path's bump allocator starts after the fast path's slot region
__global__ void k_fast_region(GeneralJob j, uint32_t n_upd) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *j.used = 2 * (j.upd_off[n_upd] - j.upd_off[0]) + 64ull * j.n + 64;
}

int fast_launch(uint32_t op, const GeneralJob &j, uint32_t n_upd, hipStream_t st) {
  if (op != OP_MERGE || j.v2) return 0;  // fast path: V1 merges (the C2/C4 headline configs)
  k_fast_region<<<1, 64, 0, st>>>(j, n_upd);
  const uint32_t grid = j.n < 131072 ? j.n : 131072;
  static int stop = -1;
  if (stop < 0) { const char *e = getenv("YMERGE_FAST_STOP"); stop = e ? atoi(e) : 0; }
  const size_t lds = Lay<SmallCfg>::total;
  switch (stop) {
    case 1: k_fast_merge_v1<SmallCfg, 1><<<grid, 64, lds, st>>>(j); break;
    case 2: k_fast_merge_v1<SmallCfg, 2><<<grid, 64, lds, st>>>(j); break;
    case 3: k_fast_merge_v1<SmallCfg, 3><<<grid, 64, lds, st>>>(j); break;
    case 4: k_fast_merge_v1<SmallCfg, 4><<<grid, 64, lds, st>>>(j); break;
    case 5: k_fast_merge_v1<SmallCfg, 5><<<grid, 64, lds, st>>>(j); break;
    case 6: k_fast_merge_v1<SmallCfg, 6><<<grid, 64, lds, st>>>(j); break;
    case 8: k_fast_merge_v1<SmallCfg, 8><<<grid, 64, lds, st>>>(j); break;
    default: k_fast_merge_v1<SmallCfg, 0><<<grid, 64, lds, st>>>(j); break;
  }
  return 1;
}

}  // namespace ymk
