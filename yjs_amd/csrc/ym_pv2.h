// ym_pv2.h -- definitions shared by the column-parallel V2 diff / state-vector kernels: the single-section
// path (ym_pv2.hip, BASELINE configs[2] C3) and the multi-section path (ym_pv2ms.hip, configs[4] C5).
//
// A V2 update spreads every struct over up to nine RLE columns (UpdateEncoder.js:229-408, column order
// keyClock client leftClock rightClock info string parentInfo typeRef len) plus the rest stream.  The
// kernels decode each column on its own (K1), recover every struct's column indices by block prefix sums
// (K2), and rebuild the written columns from re-encoded heads and verbatim entry runs (K3 / K4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ym_fast_common.h"
#include "ym_kernels.h"
#include "ym_lane.h"

namespace ymk {
namespace pv2 {
using namespace fastc;

constexpr uint64_t PV_MIN = 32768;  // smaller updates stay on k_big_v2
constexpr uint32_t NONE = 0xffffffffu;
// column kinds decoded by K1 / spliced by K3 (the V2 column index: col_of)
enum { K_INFO = 0, K_PI, K_SL, K_LN, K_CL, K_LC, K_RC, K_TR, K_KC, NK };
__host__ __device__ constexpr uint32_t col_of(uint32_t k) {  // V2 column order: kc cl lc rc in sl pi tr ln
  return k == K_INFO ? 4 : k == K_PI ? 6 : k == K_SL ? 5 : k == K_LN ? 8 : k == K_CL ? 1 : k == K_LC ? 2
         : k == K_RC ? 3 : k == K_TR ? 7 : 0;
}
__host__ __device__ constexpr bool k_rle(uint32_t k) { return k == K_INFO || k == K_PI; }              // RleDecoder<u8>
__host__ __device__ constexpr bool k_dif(uint32_t k) { return k == K_LC || k == K_RC || k == K_KC; }   // IntDiffOptRle
constexpr uint32_t HB = 64;      // encoded head bytes per (document, column)
constexpr uint32_t CKSTEP = 16;  // column entries per checkpoint (K3 starts its decode at the last one)

// per-document state, in HBM
struct Meta {
  uint32_t ok;                // eligible (K0) and still good
  uint32_t why;               // where a document was declined (debugging aid, ym__pv2_why)
  uint32_t ms;                // several client sections (ym_pv2ms.hip)
  uint32_t col0[9], col1[9];  // column spans (update-relative); the string column's lengths part
  uint32_t sb0, sn;           // string body [sb0, sb0 + sn)
  uint32_t n;                 // structs (multi-section: counted by the rest walk)
  uint32_t nsec;              // client sections (header)
  uint32_t r0;                // rest stream: the first section header
  uint32_t client;            // single section: the section's client (first value of the client column)
  uint32_t clock0;            // single section: the section's first clock
  uint32_t ds0;               // delete set start (rest stream)
  uint32_t nitem;             // multi-section: structs with rest payloads (Skip / Binary / Embed / Format / Any)
  // multi-section rest walk, column passes -> walk: payload list length, counted structs, token kinds present,
  // the info column's endless final entry (value, payload kind, first struct / payload / len ordinal), len entries
  uint32_t mr_npay, mr_kinds, mr_fin, mr_finpk, mr_fink, mr_finl, mr_nle, mr_ltot;
  uint64_t mr_nstr, mr_fini;
  uint64_t soff;              // scratch offset (value arrays, checkpoints, column outputs)
  uint64_t soff1;             // multi-section: section table + payload starts
  uint64_t o_tr, o_sl, o_ln, o_cl, o_ck, o_col[NK];  // scratch layout (relative to soff)
  uint32_t ocap[NK];          // multi-section: column output capacity
  uint32_t ck0[NK];           // K1 checkpoints of each column (uint4: entry position, value index, running
                              // value) every CKSTEP entries, at the scratch's checkpoint area + ck0
  uint32_t nck[NK];
  // K1: values per kind; RLE<u8> kinds: values in counted entries, and whether a final (endless) entry exists
  uint32_t nval[NK], fin[NK], finv[NK];
  // K2 (single section): the cut and the column indices around it
  uint32_t f;                 // cut struct (NONE: no struct ends past the state vector)
  uint32_t off, fclock_lo;    // Item.write offset; clock of the cut struct
  uint32_t pf[NK], pf1[NK];   // values of each kind consumed before struct f / f + 1
  uint32_t tot[NK];           // values of each kind consumed by all structs
  uint32_t body_f, body_fc, body_f1, body_end;  // string body offsets: before struct f, its content string, after it; consumed end
  uint32_t info_f, pi_f, clen_f;
  // K2 (multi-section): kept sections, keys written, item structs
  uint32_t nkept, kc_out, clock_tot;
  // K3
  uint32_t hlen[NK], vstart[NK];  // single section
  uint32_t osz[NK];               // multi-section: column output bytes
  uint8_t head[NK][HB];
};

// one client section of a multi-section update (ym_pv2ms.hip)
struct Sec {
  unsigned long long skipk;    // K2 pass 1: first Skip struct: index << 32 | clock-length prefix before it
  // rest walk (MR)
  uint32_t S, W, clock;        // first struct, structs, first clock
  uint32_t pay0, pay1;         // rest-stream payloads of its structs
  uint32_t ibase;              // item ordinal (structs with payloads) at S
  // K2 pass 1
  uint32_t C0, C1;             // clock-length prefix at S, after S
  uint32_t client, sv;         // the section's client, the state vector's clock for it
  uint32_t body0;              // string body bytes before S
  uint32_t kw0;                // structs writing a key (Format, XmlElement / XmlHook types) before S
  uint32_t pre[NK];            // values of each kind consumed before S (client: the section's client value)
  // K2 pass 2: the cut (f = NONE: nothing written)
  uint32_t f, off, fclock, info_f, pi_f, tr_f, clen_f, iord_f, kwf;
  uint32_t body_f, body_fc, body_f1;
  uint32_t pf[NK], pf1[NK];
  // K4
  uint32_t rs, ob, orr;        // output rest start (after a ContentAny offset); body / rest output offsets
};

static_assert(sizeof(Sec) % 8 == 0, "Sec holds a u64 atomic");

struct Job {
  GeneralJob j;
  Meta *meta;
  uint8_t *scr;   // per-document value arrays
  uint8_t *scr1;  // multi-section: section tables, payload starts
  uint8_t *done;
};
__device__ __forceinline__ uint8_t *a_info(const Job &J, const Meta &M) { return J.scr + M.soff; }
__device__ __forceinline__ uint8_t *a_pi(const Job &J, const Meta &M) { return J.scr + M.soff + M.n; }
__device__ __forceinline__ uint8_t *a_tr(const Job &J, const Meta &M) { return J.scr + M.soff + M.o_tr; }
__device__ __forceinline__ uint32_t *a_sl(const Job &J, const Meta &M) { return reinterpret_cast<uint32_t *>(J.scr + M.soff + M.o_sl); }
__device__ __forceinline__ uint32_t *a_ln(const Job &J, const Meta &M) { return reinterpret_cast<uint32_t *>(J.scr + M.soff + M.o_ln); }
__device__ __forceinline__ uint32_t *a_cl(const Job &J, const Meta &M) { return reinterpret_cast<uint32_t *>(J.scr + M.soff + M.o_cl); }
__device__ __forceinline__ uint4 *a_ck(const Job &J, const Meta &M, uint32_t kind) {
  return reinterpret_cast<uint4 *>(J.scr + M.soff + M.o_ck) + M.ck0[kind];
}
__device__ __forceinline__ uint8_t *a_col(const Job &J, const Meta &M, uint32_t kind) { return J.scr + M.soff + M.o_col[kind]; }
__device__ __forceinline__ Sec *a_sec(const Job &J, const Meta &M) { return reinterpret_cast<Sec *>(J.scr1 + M.soff1); }
__device__ __forceinline__ uint32_t *a_istart(const Job &J, const Meta &M) {
  return reinterpret_cast<uint32_t *>(J.scr1 + M.soff1 + (((uint64_t)M.nsec * sizeof(Sec) + 15) & ~15ull));
}
// multi-section rest walk (MR): the payload structs in struct order -- struct index, and kind | count / len
// ordinal -- and the len column's entries (first value ordinal, value); icap = rest bytes + 1 bounds both
// the payload structs and the payload starts
__host__ __device__ inline uint32_t ms_icap(uint32_t len, uint32_t r0) { return len - r0 + 1; }
__host__ __device__ inline uint64_t ms_scr1_bytes(uint32_t nsec, uint32_t len, uint32_t r0, uint32_t lncol) {
  return ((((uint64_t)nsec * sizeof(Sec) + 15) & ~15ull) + 12ull * ms_icap(len, r0) + 8ull * (lncol + 2) + 511) & ~255ull;
}
__device__ __forceinline__ uint32_t *a_pidx(const Job &J, const Meta &M, uint32_t len) { return a_istart(J, M) + ms_icap(len, M.r0); }
__device__ __forceinline__ uint32_t *a_pkl(const Job &J, const Meta &M, uint32_t len) { return a_istart(J, M) + 2ull * ms_icap(len, M.r0); }
__device__ __forceinline__ uint2 *a_lent(const Job &J, const Meta &M, uint32_t len) {  // (16-aligned: the slack of ms_scr1_bytes)
  return reinterpret_cast<uint2 *>((reinterpret_cast<uintptr_t>(a_istart(J, M) + 3ull * ms_icap(len, M.r0)) + 15) & ~(uintptr_t)15);
}
// value capacity of kind k's expanded / counted values
__host__ __device__ inline uint64_t kind_cap(uint32_t k, uint32_t n, uint32_t nsec) {
  return k == K_SL ? 3ull * n + 1 : k == K_CL ? 2ull * n + nsec + 1 : n;
}
// scratch layout of a document: info u8[n], pi u8[n], tr u8[n], sl u32[3n + 1], ln u32[n], cl u32[2n + nsec + 1]
// (multi-section only), then the K1 checkpoints (16-aligned), then the multi-section column outputs.
// Returns the bytes; fills the offsets.  `colb[k]` = input bytes of kind k's column.
__host__ __device__ inline uint64_t scr_layout(Meta &M, uint32_t n, uint32_t nsec, bool ms, const uint32_t *colb) {
  uint64_t o = 3ull * n;
  M.o_tr = 2ull * n;
  o = (o + 3) & ~3ull;
  M.o_sl = o;
  o += 4ull * (3ull * n + 1);
  M.o_ln = o;
  o += 4ull * n;
  M.o_cl = o;
  if (ms) o += 4ull * kind_cap(K_CL, n, nsec);
  o = (o + 15) & ~15ull;
  M.o_ck = o;
  uint32_t ck = 0;  // an entry is at least one byte: a column of b bytes needs b / CKSTEP + 1 checkpoints
  for (uint32_t k = 0; k < NK; k++) {
    M.ck0[k] = ck;
    ck += colb[k] / CKSTEP + 2;
  }
  o += 16ull * ck;
  for (uint32_t k = 0; k < NK; k++) {
    M.o_col[k] = o;
    M.ocap[k] = 0;
    if (ms && k != K_KC) {
      M.ocap[k] = colb[k] + 96u * nsec + 64;
      o += (M.ocap[k] + 15) & ~15ull;
    }
  }
  return o;
}

// lib0 readVarInt as k_big_v2's s_vi: canonical, <= 5 bytes, |v| < 2^31 + (sign); returns the magnitude
__device__ __forceinline__ uint32_t rvi(ln::LCur &c, bool &neg) {
  const uint32_t lo = (uint32_t)c.lo, hi = (uint32_t)(c.lo >> 32);
  const uint32_t nb = ln::vu_nb(lo, hi);
  neg = (lo & 0x40) != 0;
  uint32_t m = (lo & 0x3fu) | ((lo >> 2) & 0x1fc0u) | ((lo >> 3) & 0xfe000u) | ((lo >> 4) & 0x7f00000u) | ((hi & 0x7fu) << 27);
  const uint32_t bits = 6 + 7 * (nb - 1);
  if (nb < 5) m &= (1u << bits) - 1u;
  const uint32_t last = nb <= 4 ? (lo >> (8 * nb - 8)) & 0xffu : hi & 0xffu;
  c.bad |= (nb > 5) | (c.p + nb > c.e) | ((nb > 1) & (last == 0)) | ((nb == 5) & ((hi & 0x7fu) > 0x1fu));
  ln::skip(c, nb < 6 ? nb : 0);
  return m;
}

// ---- the column automaton (K1; the multi-section rest walk's column passes) ----------------------
constexpr uint32_t F_ID = 0xE4;  // identity on 4 states, 2 bits per state
__device__ __forceinline__ uint32_t fcompose(uint32_t a, uint32_t b) {  // b after a
  uint32_t c = 0;
#pragma unroll
  for (uint32_t st = 0; st < 4; st++) c |= ((b >> (2 * ((a >> (2 * st)) & 3))) & 3) << (2 * st);
  return c;
}
#define CDPP(x, ctl, rm) (uint32_t) __builtin_amdgcn_update_dpp((int)F_ID, (int)(x), ctl, rm, 0xf, false)
__device__ __forceinline__ uint32_t wave_incl_compose(uint32_t f) {
  f = fcompose(CDPP(f, 0x111, 0xf), f);
  f = fcompose(CDPP(f, 0x112, 0xf), f);
  f = fcompose(CDPP(f, 0x114, 0xf), f);
  f = fcompose(CDPP(f, 0x118, 0xf), f);
  f = fcompose(CDPP(f, 0x142, 0xa), f);
  f = fcompose(CDPP(f, 0x143, 0xc), f);
  return f;
}
__device__ __forceinline__ uint64_t wave_incl_add64(uint64_t x) {
#define A64(ctl, rm)                                                                                 \
  {                                                                                                  \
    const uint32_t rl = YM_DPP((uint32_t)x, ctl, rm), rh = YM_DPP((uint32_t)(x >> 32), ctl, rm);    \
    x += ((uint64_t)rh << 32) | rl;                                                                  \
  }
  A64(0x111, 0xf) A64(0x112, 0xf) A64(0x114, 0xf) A64(0x118, 0xf) A64(0x142, 0xa) A64(0x143, 0xc)
#undef A64
  return x;
}
__device__ __forceinline__ uint32_t tstep(uint32_t st, uint32_t b, bool rle, uint32_t fb) {
  const bool stop = b < 0x80;
  if (rle) return st == 0 ? 1 : (stop ? 0 : 1);
  if (st == 0) { const bool fl = (b >> fb) & 1; return stop ? (fl ? 3 : 0) : (fl ? 1 : 2); }
  if (st == 1) return stop ? 3 : 1;
  if (st == 2) return stop ? 0 : 2;
  return stop ? 0 : 3;
}

struct Ent {
  uint32_t val, cnt;
  int32_t df;
  bool fin, bad;
  uint32_t end;  // position after the entry
};
// the entry at pos: value (RLE: the byte; Opt: the varint's magnitude), count, IntDiff diff; fin = an
// RLE<u8> value byte that ends the column (no count: the final run never ends)
__device__ __forceinline__ Ent dec_entry(const uint8_t *D, uint32_t pos, uint32_t c1, uint32_t kind) {
  Ent e{0, 0, 0, false, false, c1};
  if (k_rle(kind)) {
    e.val = D[pos];
    e.bad = kind == K_PI && e.val > 1;
    if (pos + 1 >= c1) { e.fin = true; return e; }
    ln::LCur c = ln::make(D, pos + 1, c1);
    e.cnt = ln::rvu(c) + 1;
    e.bad |= c.bad || e.cnt == 0;
    e.end = c.p;
    return e;
  }
  ln::LCur c = ln::make(D, pos, c1);
  bool neg;
  const uint32_t m = rvi(c, neg);
  if (k_dif(kind)) {
    const int32_t t = neg ? -(int32_t)m : (int32_t)m;
    e.df = t >> 1;
    e.cnt = (t & 1) ? ln::rvu(c) + 2 : 1;
    e.bad = (neg && m == 0) || e.df < -(1 << 30) || e.df >= (1 << 30) || ((t & 1) && e.cnt < 2);
  } else {
    e.cnt = neg ? ln::rvu(c) + 2 : 1;
    e.bad = neg && e.cnt < 2;
  }
  e.val = m;
  e.bad |= c.bad;
  e.end = c.p;
  return e;
}

// lib0 encoders into a byte sink
struct Buf {
  uint8_t *b;
  uint32_t n, cap;
  bool over;
  bool wr = true;  // this lane stores (a wave-uniform encoder stores from lane 0 only)
  __device__ void byte(uint32_t v) { if (n < cap) { if (wr) b[n] = (uint8_t)v; } else over = true; n++; }
  __device__ void vu(uint32_t v) { while (v > 127) { byte(0x80 | (v & 127)); v >>= 7; } byte(v); }
  __device__ void vi(bool neg, uint32_t m) {
    byte((m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63));
    m >>= 6;
    while (m > 0) { byte((m > 127 ? 0x80 : 0) | (m & 127)); m >>= 7; }
  }
};
struct Enc {  // one encoder of kind `kind`: (s, count, diff, started)
  uint32_t s = 0, cnt = 0, started = 0;
  int32_t df = 0;
  bool bad = false;
  __device__ void put(Buf &B, uint32_t kind, uint32_t v) {
    if (k_rle(kind)) {  // RleEncoder<u8>
      if (started && s == v) { cnt++; return; }
      if (cnt > 0) B.vu(cnt - 1);
      B.byte(v);
      s = v; cnt = 1; started = 1;
    } else if (k_dif(kind)) {  // IntDiffOptRleEncoder
      const int64_t dd = (int64_t)v - (int64_t)s;
      if (dd < -(1ll << 30) || dd >= (1ll << 30)) { bad = true; return; }
      if (df == (int32_t)dd) { s = v; cnt++; return; }
      flush(B, kind);
      s = v; cnt = 1; df = (int32_t)dd;
    } else {  // UintOptRleEncoder
      if (s == v && cnt > 0) { cnt++; return; }
      flush(B, kind);
      s = v; cnt = 1;
    }
  }
  // closes the pending run (before verbatim entries, or at the column's end: an RLE<u8> final count is
  // not written then)
  __device__ void flush(Buf &B, uint32_t kind, bool at_end = false) {
    if (cnt == 0) return;
    if (k_rle(kind)) {
      if (!at_end) B.vu(cnt - 1);
    } else if (k_dif(kind)) {
      const int32_t x = (int32_t)((uint32_t)df << 1) | (cnt == 1 ? 0 : 1);
      B.vi(x < 0, x < 0 ? (uint32_t)(-(int64_t)x) : (uint32_t)x);
      if (cnt > 1) B.vu(cnt - 2);
    } else {
      B.vi(cnt != 1, s);
      if (cnt > 1) B.vu(cnt - 2);
    }
    cnt = 0;
  }
};

// ---- block-wide helpers (K2) ---------------------------------------------------------------------------
constexpr uint32_t KT = 256;       // threads
constexpr uint32_t PER = 4;        // structs per thread per tile
constexpr uint32_t TILE = KT * PER;
// exclusive block scan of NS u32 sums (+ totals), KT threads
template <uint32_t NS>
__device__ __forceinline__ void block_scan(uint32_t (&x)[NS], uint32_t (&tot)[NS], uint32_t *sh) {
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t incl[NS];
#pragma unroll
  for (uint32_t q = 0; q < NS; q++) incl[q] = wave_incl_add(x[q]);
  __syncthreads();
  if (lane == 63)
#pragma unroll
    for (uint32_t q = 0; q < NS; q++) sh[w * NS + q] = incl[q];
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < NS; q++) {
    uint32_t pre = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < KT / 64; k++) {
      const uint32_t s = sh[k * NS + q];
      pre += k < w ? s : 0;
      all += s;
    }
    x[q] = pre + incl[q] - x[q];
    tot[q] = all;
  }
}


// wave copy of n bytes (unaligned 16-byte loads / stores)
typedef uint4 __attribute__((aligned(1))) u4u;
__device__ __forceinline__ void wcopy(uint8_t *dst, const uint8_t *src, uint32_t n) {
  const uint32_t nv = n >> 4;
  for (uint32_t v = threadIdx.x; v < nv; v += 64) reinterpret_cast<u4u *>(dst)[v] = reinterpret_cast<const u4u *>(src)[v];
  for (uint32_t i = (nv << 4) + threadIdx.x; i < n; i += 64) dst[i] = src[i];
}


// multi-section path (ym_pv2ms.hip), launched by pv2_run
void ms_rest(const Job &J, hipStream_t st);                            // MR: the rest walk
void ms_sizes(const Job &J, uint64_t *sizes, hipStream_t st);          // phase-2 scratch sizes
void ms_run(uint32_t op, const Job &J, hipStream_t st);                // K2 .. K4 (after K1)

}  // namespace pv2
}  // namespace ymk
