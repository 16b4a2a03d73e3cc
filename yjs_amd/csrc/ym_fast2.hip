// ym_fast2.hip -- LDS fast path for batched mergeUpdatesV2: one 64-lane wave per document.
//
// The V1 fast path (ym_fast.hip) over the V2 layout (UpdateDecoder.js:245-392, UpdateEncoder.js:229-408).
// It takes the same "simple" documents (every update's structs increasing in (client desc, clock asc),
// no overlap, no GC/Skip inputs, canonical payloads) plus: ASCII string columns.  For them 13.5.16's
// mergeUpdatesV2 (ds@39007) = all structs sorted by (client desc, clock asc), Skips at clock gaps,
// parts per client run, each struct re-encoded into the nine columns; delete sets united per client,
// clients in first-appearance order.
//
// Per document (one wave, ~12.4 KB of LDS):
//   1. stage the bytes;  2. one lane per update: V2 header, per-lane lib0 RLE column decoders, struct
//   records (values, not bytes) + delete ranges into LDS;  3. rank sort;  4. layout by DPP scans;
//   5. every struct's column entries are scattered into per-column value arrays (counts scanned per
//   column), then each column is RLE-encoded wave-parallel: run starts/ends by neighbour compares,
//   run lengths by a running-max scan of start positions, run bytes by a prefix sum (UintOptRle,
//   IntDiffOptRle, Rle<u8>, StringEncoder);  6. rest stream (part headers, Skip lengths, verbatim
//   any/binary payloads) and the V2 delete set (clock deltas, len - 1).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ym_fast_common.h"
#include "ym_kernels.h"

namespace ymk {
namespace fastv2 {
using namespace fastc;

constexpr uint32_t IN = 3584, UPD = 128, E = 2, REC = 64 * E, DSN = 64 * E;

constexpr uint32_t L_IN = 0;                       // u8[IN + 16]
constexpr uint32_t L_UOFF = IN + 16;               // u16[UPD + 1]
constexpr uint32_t L_MISC = L_UOFF + 272;          // u32[16]
constexpr uint32_t R = L_MISC + 64;
// struct records (walk slots, then rank order in place)
constexpr uint32_t L_RKEY = R;                     // u64 (~client << 32 | clock)
constexpr uint32_t L_RLEN = L_RKEY + 8 * REC;      // u32
constexpr uint32_t L_RAUX = L_RLEN + 4 * REC;      // u32 info | pi << 8 | typeRef << 16
constexpr uint32_t L_RF = L_RAUX + 4 * REC;        // u32[4]: origin (or parent id) client, clock; right origin client, clock
constexpr uint32_t L_RS = L_RF + 16 * REC;         // u32[3]: strings (se_make): ykey, parentSub, content/key/name
constexpr uint32_t L_RSP = L_RS + 12 * REC;        // u32 rest span (LDS offset | n << 16)
constexpr uint32_t L_RSLOT = L_RSP + 4 * REC;      // u8
constexpr uint32_t L_RCEND = L_RSLOT + REC;
// delete ranges
constexpr uint32_t L_DKEY = L_RCEND;               // u64 (client << 32 | clock << 7 | slot)
constexpr uint32_t L_DLEN = L_DKEY + 8 * DSN;      // u32
constexpr uint32_t L_DSEQ = L_DLEN + 4 * DSN;      // u16
constexpr uint32_t L_DSLOT = L_DSEQ + 2 * DSN;     // u8
constexpr uint32_t L_PFIRST = L_DSLOT + DSN;       // u16[REC]
constexpr uint32_t L_PLAST = L_PFIRST + 2 * REC;   // u16[REC]
constexpr uint32_t L_END = L_PLAST + 2 * REC;
// output staging (merged outputs are about the input size; larger ones decline to the general path)
constexpr uint32_t L_OUT = (L_END + 15) & ~15u, OUTCAP = IN + 1024;
constexpr uint32_t LDS_BYTES = L_OUT + OUTCAP;
static_assert(8 * LDS_BYTES <= 160 * 1024, "staging keeps 2 waves per SIMD (the VGPR bound)");
// phase 5: per-column value arrays over the record region (the records are held in registers)
constexpr uint32_t V_CL = R;                       // u32[3 * REC]
constexpr uint32_t V_LC = V_CL + 12 * REC;         // u32[REC]
constexpr uint32_t V_RC = V_LC + 4 * REC;          // u32[REC]
constexpr uint32_t V_LN = V_RC + 4 * REC;          // u32[REC]
constexpr uint32_t V_ST = V_LN + 4 * REC;          // u32[3 * REC] (se_make)
constexpr uint32_t V_TR = V_ST + 12 * REC;         // u8[REC]
constexpr uint32_t V_IN = V_TR + REC;              // u8[2 * REC]
constexpr uint32_t V_PI = V_IN + 2 * REC;          // u8[REC]
constexpr uint32_t V_END = V_PI + REC;
static_assert(V_END <= L_RCEND, "column arrays fit the record region");
// phase 6 (delete set) over the record region again
constexpr uint32_t L_QCLK = R, L_QEND = L_QCLK + 4 * DSN, L_QGRP = L_QEND + 4 * DSN, L_QPRE = L_QGRP + DSN;
constexpr uint32_t L_GFIRST = L_QPRE + 272, L_GCLI = L_GFIRST + 272, L_GB2 = L_GCLI + 4 * DSN, L_GBYR = L_GB2 + 4 * DSN;
constexpr uint32_t L_GMIN = L_PFIRST;
static_assert(L_GBYR + 2 * DSN <= L_RCEND, "delete-set arrays fit the record region");

// a string of the document's string columns: its LDS offset (12 bits), UTF-8 bytes and UTF-16 units (10 bits each)
static_assert(IN + 16 <= 4096, "string offsets fit 12 bits");
__device__ __forceinline__ uint32_t se_make(uint32_t off, uint32_t bytes, uint32_t units) { return off | (bytes << 12) | (units << 22); }
__device__ __forceinline__ uint32_t se_off(uint32_t e) { return e & 0xfffu; }
__device__ __forceinline__ uint32_t se_bytes(uint32_t e) { return (e >> 12) & 0x3ffu; }
__device__ __forceinline__ uint32_t se_units(uint32_t e) { return e >> 22; }

// ---- per-lane lib0 decoders over LDS (canonical inputs only; anything else declines) -------------
// readVarInt: sign (incl. -0) + u32 magnitude, at most 5 bytes
__device__ __forceinline__ uint32_t rvi(Cur &c, bool &neg) {
  const uint64_t x = ld8(c.p);
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  neg = (lo & 0x40) != 0;
  if (__all((lo & 0x80u) == 0)) {  // every active lane: a one-byte varInt
    c.bad |= c.p >= c.e;
    c.p += 1;
    return lo & 0x3fu;
  }
  const uint32_t nb = vu_nb(lo, hi);
  uint32_t m = (lo & 0x3fu) | ((lo >> 2) & 0x1fc0u) | ((lo >> 3) & 0xfe000u) | ((lo >> 4) & 0x7f00000u) | ((hi & 0x7fu) << 27);
  const uint32_t bits = 6 + 7 * (nb - 1);
  if (nb < 5) m &= (1u << bits) - 1u;
  c.bad |= (nb > 5) | (c.p + nb > c.e) | ((nb == 5) & ((hi & 0x7fu) > 0x1fu));
  c.p += nb < 6 ? nb : 0;
  return m;
}
struct RleD { Cur c; uint32_t s, n; };              // RleDecoder<u8>
struct UoptD { Cur c; uint32_t s, n; };             // UintOptRleDecoder
struct IdifD { Cur c; uint32_t s, n; int32_t d; };  // IntDiffOptRleDecoder
__device__ __forceinline__ uint32_t rd_rle(RleD &r) {
  if (r.n == 0) {
    r.s = rdb(r.c);
    r.n = r.c.p < r.c.e ? rvu(r.c) + 1 : 0xffffffffu;  // the final run never ends
  }
  if (r.n != 0xffffffffu) r.n--;
  return r.s;
}
__device__ __forceinline__ uint32_t rd_uopt(UoptD &r) {
  if (r.n == 0) {
    bool neg;
    r.s = rvi(r.c, neg);
    r.n = neg ? rvu(r.c) + 2 : 1;
  }
  r.n--;
  return r.s;
}
__device__ __forceinline__ uint32_t rd_idif(IdifD &r) {
  if (r.n == 0) {
    bool neg;
    const uint32_t m = rvi(r.c, neg);
    const int32_t t = (int32_t)(neg ? 0u - m : m);  // ToInt32(sign * mag)
    r.d = t >> 1;
    r.n = (t & 1) ? rvu(r.c) + 2 : 1;
  }
  const int64_t v = (int64_t)r.s + r.d;
  r.c.bad |= v < 0 || v > 0xffffffffll;  // clocks: this path keeps them u32
  r.s = (uint32_t)v;
  r.n--;
  return r.s;
}

__device__ __forceinline__ void decline(const GeneralJob &j, uint32_t d) {
  j.status[d] = ST_PENDING;
  const uint32_t q = atomicAdd(j.pend_count, 1u);
  if (j.pend_list) j.pend_list[q] = d + j.doc_base;  // (ym_merge_async: declines are only counted)
}

// Walks one V2 update (lane-private decoders) and appends struct records and delete ranges.  NESTED:
// nested any values (objects, arrays) are checked canonical too (the retry pass, ym_canon_chk.h).
template <bool NESTED = false>
__device__ __forceinline__ bool walk_v2(uint32_t u) {
  const uint32_t p0 = at<uint16_t>(L_UOFF + 2 * u), p1 = at<uint16_t>(L_UOFF + 2 * u + 2);
  Cur h = {p0, p1, false};
  rvu(h);  // feature flag
  Cur col[9];
#pragma unroll
  for (uint32_t k = 0; k < 9; k++) {
    const uint32_t n = rvu(h);
    if (!room(h, n)) return false;
    col[k] = Cur{h.p, h.p + n, false};
    h.p += n;
  }
  if (h.bad) return false;
  // StringDecoder: varString(body) then the UintOptRle of UTF-16 lengths.  The body must be valid UTF-8 (the
  // decoder's replacement characters would re-encode differently); each string is then sliced by its UTF-16
  // length: bytes = units for an ASCII body, else a walk over the lead bytes (round 6; ASCII only before)
  const uint32_t sn = rvu(col[5]);
  if (col[5].bad || !room(col[5], sn)) return false;
  const uint32_t sb = col[5].p;
  bool sascii;
  uint32_t sunits = sn;
  {
    uint64_t hi = 0;
    for (uint32_t o = 0; o < sn; o += 8) hi |= mask_bytes(ld8(sb + o), sn - o);
    sascii = (hi & 0x8080808080808080ull) == 0;
    if (!sascii) {
      bool ub = false;
      sunits = utf8_slow(sb, sb + sn, ub);
      if (ub) return false;
    }
  }
  col[5].p += sn;
  IdifD kc = {col[0], 0, 0, 0};
  UoptD cl = {col[1], 0, 0};
  IdifD lc = {col[2], 0, 0, 0}, rc = {col[3], 0, 0, 0};
  RleD in = {col[4], 0, 0};
  UoptD sl = {col[5], 0, 0};
  RleD pi_ = {col[6], 0, 0};
  UoptD tr = {col[7], 0, 0}, ln = {col[8], 0, 0};
  uint32_t spos = 0, supos = 0, keys = 0;
  Cur c = h;  // rest stream
  bool bad = false;
  auto rstr = [&]() -> uint32_t {  // StringDecoder.read(): LDS offset | bytes << 12 | UTF-16 units << 22 (SE_*)
    const uint32_t n = rd_uopt(sl);
    uint32_t nb = n;
    if (!sascii) nb = utf8_span(sb + spos, sb + sn, n, bad);
    bad |= spos + nb > sn || supos + n > sunits || n > 1023 || nb > 1023;
    const uint32_t v = se_make(sb + spos, nb, n);
    spos += nb;
    supos += n;
    return v;
  };
  const uint32_t nclients = rvu(c);
  uint64_t prev = 0;
  bool have_prev = false;
  for (uint32_t ci = 0; ci < nclients && !c.bad && !bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = rd_uopt(cl);
    uint32_t clock = rvu(c);
    for (uint32_t si = 0; si < nstructs && !c.bad && !bad; si++) {
      const uint32_t info = rd_rle(in);
      // declines set `bad` (one exit edge per loop instead of one per check)
      bad |= info == 10 || (info & 31) == 0 || info > 255;  // Skip / GC inputs: general path
      uint32_t f0 = 0, f1 = 0, f2 = 0, f3 = 0, s0 = 0, s1 = 0, s2 = 0, sp = 0, pi = 0, t = 0;
      if (info & 0x80) { f0 = rd_uopt(cl); f1 = rd_idif(lc); }
      if (info & 0x40) { f2 = rd_uopt(cl); f3 = rd_idif(rc); }
      if ((info & 0xC0) == 0) {
        pi = rd_rle(pi_) == 1 ? 1 : 0;  // readParentInfo() === 1
        if (pi) s0 = rstr();
        else { f0 = rd_uopt(cl); f1 = rd_idif(lc); }
        if (info & 0x20) s1 = rstr();
      }
      uint32_t len = 1;
      switch (info & 31) {
        case 1: len = rd_uopt(ln); break;                                  // ContentDeleted
        case 3: {                                                          // ContentBinary (rest)
          const uint32_t a = c.p, n = rvu(c);
          if (!room(c, n)) bad = true;
          else c.p += n;
          sp = a | ((c.p - a) << 16);
          break;
        }
        case 4: s2 = rstr(); len = se_units(s2); break;                    // ContentString
        case 5: case 6: {                                                  // Embed / Format (+ key)
          if ((info & 31) == 6) s2 = rstr();
          const uint32_t a = c.p;
          any_canon<NESTED>(c);
          sp = a | ((c.p - a) << 16);
          break;
        }
        case 7:                                                            // ContentType
          t = rd_uopt(tr);
          bad |= t > 6;
          if (t == 3 || t == 5) {  // readKey: a cached key (keyClock < keys read) reads no string
            bad |= rd_idif(kc) < keys;
            keys++;
            s2 = rstr();
          }
          break;
        case 8: {                                                          // ContentAny
          len = rd_uopt(ln);
          const uint32_t a = c.p;
          for (uint32_t i = 0; i < len && !c.bad; i++) any_canon<NESTED>(c);
          sp = a | ((c.p - a) << 16);
          break;
        }
        default: bad = true; break;  // ContentJSON, ContentDoc, invalid refs
      }
      const uint64_t key = ((uint64_t)(~client) << 32) | clock;
      bad |= c.bad | (len == 0) | ((sp >> 16) > 0x7fff) | ((uint64_t)clock + len > 0xffffffffull) |
             (have_prev && key <= prev);  // each update must already be in merge order
      if (!bad) {
        prev = key + len - 1;
        have_prev = true;
        const uint32_t q = atomicAdd(&at<uint32_t>(L_MISC), 1u);
        bad |= q >= REC;
        if (q < REC) {
          at<uint64_t>(L_RKEY + 8 * q) = key;
          at<uint32_t>(L_RLEN + 4 * q) = len;
          at<uint32_t>(L_RAUX + 4 * q) = info | (pi << 8) | (t << 16);
          at<uint4>(L_RF + 16 * q) = make_uint4(f0, f1, f2, f3);
          at<uint32_t>(L_RS + 12 * q) = s0;
          at<uint32_t>(L_RS + 12 * q + 4) = s1;
          at<uint32_t>(L_RS + 12 * q + 8) = s2;
          at<uint32_t>(L_RSP + 4 * q) = sp;
        }
      }
      clock += len;
    }
  }
  bad |= c.bad | cl.c.bad | lc.c.bad | rc.c.bad | in.c.bad | sl.c.bad | pi_.c.bad | tr.c.bad | ln.c.bad | kc.c.bad;
  if (bad) return false;
  // V2 delete set (rest): per client, clock deltas against dsCurr and len - 1 (UpdateDecoder.js:258-267)
  const uint32_t ndc = rvu(c);
  uint32_t pos = 0;
  for (uint32_t i = 0; i < ndc && !c.bad; i++) {
    const uint32_t client = rvu(c);
    const uint32_t m = rvu(c);
    uint64_t cur = 0;
    for (uint32_t q = 0; q < m && !c.bad; q++, pos++) {
      const uint64_t clock = cur + rvu(c);
      const uint64_t len = (uint64_t)rvu(c) + 1;
      cur = clock + len;
      c.bad |= (pos > 255) | (cur > 0xffffffffull) | (clock >= (1u << 25));
      if (!c.bad) {
        const uint32_t x = atomicAdd(&at<uint32_t>(L_MISC + 4), 1u);
        c.bad |= x >= DSN;
        // slot in the low bits: distinct keys, ranks are a permutation (duplicated ranges are common)
        if (x < DSN) {
          at<uint64_t>(L_DKEY + 8 * x) = ((uint64_t)client << 32) | ((uint32_t)clock << 7) | x;
          at<uint32_t>(L_DLEN + 4 * x) = (uint32_t)len;
          at<uint16_t>(L_DSEQ + 2 * x) = (uint16_t)((u << 8) | pos);
        }
      }
    }
  }
  return !c.bad;
}

// ---- wave-parallel RLE column encoders ------------------------------------------------------------
// lib0 writeVarInt size for a magnitude (sign lives in the first byte)
__device__ __forceinline__ uint32_t vszi(uint32_t m) { return m < 64 ? 1 : 1 + vsz(m >> 6); }
template <class O>
__device__ __forceinline__ uint32_t put_vi(O o, uint32_t p, bool neg, uint32_t m) {
  ob8(o, p++, (m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63));
  m >>= 6;
  while (m > 0) { ob8(o, p++, (m > 127 ? 0x80 : 0) | (m & 127)); m >>= 7; }
  return p;
}
// inclusive running max over lanes (u32)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  uint32_t y;
  y = YM_DPP(x, 0x111, 0xf); x = y > x ? y : x;
  y = YM_DPP(x, 0x112, 0xf); x = y > x ? y : x;
  y = YM_DPP(x, 0x114, 0xf); x = y > x ? y : x;
  y = YM_DPP(x, 0x118, 0xf); x = y > x ? y : x;
  y = YM_DPP(x, 0x142, 0xa); x = y > x ? y : x;
  y = YM_DPP(x, 0x143, 0xc); x = y > x ? y : x;
  return x;
}
enum { K_UOPT = 0, K_IDIF = 1, K_RLE = 2 };
constexpr uint32_t CPL = 6;  // column elements per lane (3 * REC / 64)
// Encodes the n values get(i) (i < n <= 64 * C) with the lib0 encoder of kind K, C consecutive
// elements per lane.  Returns the byte size; writes the bytes at o[base ..] when `wr`.  Runs are found
// from neighbour compares (diffs for IntDiffOptRle), run lengths from a running max of run-start
// positions, run bytes by a prefix sum over run ends (each run end writes its run).  Values are u32;
// diffs are computed in 32 bits and `bad` is set for values >= 2^31 or diffs outside (-2^30, 2^30).
template <int K, uint32_t C, class Get, class O>
__device__ __forceinline__ uint32_t col_enc(Get get, uint32_t n, bool wr, O o, uint32_t base, bool &bad) {
  const uint32_t lane = threadIdx.x;
  const uint32_t i0 = lane * C;
  uint32_t val[C + 2];  // values (or diffs) of elements i0 - 1 .. i0 + C
  uint32_t prev = 0;
#pragma unroll
  for (uint32_t t = 0; t < C + 2; t++) {
    const int32_t i = (int32_t)i0 + (int32_t)t - 1;
    uint32_t v = 0;
    if (i >= 0 && i < (int32_t)n) {
      v = get((uint32_t)i);
      if (K == K_IDIF) {
        const uint32_t pv = t == 0 ? (i > 0 ? get((uint32_t)i - 1) : 0) : prev;
        prev = v;
        bad |= ((v | pv) >> 31) != 0;
        v -= pv;
      }
    }
    val[t] = v;
  }
  uint32_t last_sp = 0, bytes_lane = 0;
  uint32_t rb[C];
  bool st[C];
#pragma unroll
  for (uint32_t t = 0; t < C; t++) {
    const uint32_t i = i0 + t;
    st[t] = i < n && (i == 0 || val[t + 1] != val[t]);
    if (st[t]) last_sp = i;
  }
  const uint32_t carry = YM_DPP(wave_incl_max(last_sp), 0x138, 0xf);  // wave_shr:1 -> exclusive
  uint32_t sp_local = carry;
#pragma unroll
  for (uint32_t t = 0; t < C; t++) {
    const uint32_t i = i0 + t;
    rb[t] = 0;
    if (i >= n) continue;
    if (st[t]) sp_local = i;
    const bool end = i + 1 == n || val[t + 2] != val[t + 1];
    if (!end) continue;
    const uint32_t cnt = i - sp_local + 1;
    const uint32_t v = val[t + 1];
    if (K == K_UOPT) {
      rb[t] = vszi(v) + (cnt > 1 ? vsz(cnt - 2) : 0);
    } else if (K == K_IDIF) {
      const int32_t sv = (int32_t)v;
      bad |= sv <= -(1 << 30) || sv >= (1 << 30);
      const int32_t x = (int32_t)(v << 1) | (cnt > 1 ? 1 : 0);
      rb[t] = vszi(x < 0 ? 0u - (uint32_t)x : (uint32_t)x) + (cnt > 1 ? vsz(cnt - 2) : 0);
    } else {
      rb[t] = 1 + (i + 1 == n ? 0 : vsz(cnt - 1));  // Rle<u8>: the final run's count is never written
    }
    bytes_lane += rb[t];
  }
  const uint32_t incl = wave_incl_add(bytes_lane);
  const uint32_t total = lane_read(incl, 63);
  if (wr) {
    uint32_t p = base + incl - bytes_lane;
    uint32_t sp2 = carry;
#pragma unroll
    for (uint32_t t = 0; t < C; t++) {
      const uint32_t i = i0 + t;
      if (i >= n) continue;
      if (st[t]) sp2 = i;
      if (rb[t] == 0) continue;
      const uint32_t cnt = i - sp2 + 1;
      const uint32_t v = val[t + 1];
      uint32_t q = p;
      if (K == K_UOPT) {
        q = put_vi(o, q, cnt > 1, v);  // count==1 ? v : -v (-0 for v == 0)
        if (cnt > 1) q = put_vu(o, q, cnt - 2);
      } else if (K == K_IDIF) {
        const int32_t x = (int32_t)(v << 1) | (cnt > 1 ? 1 : 0);
        q = put_vi(o, q, x < 0, x < 0 ? 0u - (uint32_t)x : (uint32_t)x);
        if (cnt > 1) q = put_vu(o, q, cnt - 2);
      } else {
        ob8(o, q++, v);
        if (i + 1 != n) q = put_vu(o, q, cnt - 1);
      }
      p += rb[t];
    }
  }
  return total;
}
// n is wave-uniform: short columns (the common case) run with one or two elements per lane.
template <int K, class Get, class O>
__device__ __forceinline__ uint32_t col_encode(Get get, uint32_t n, bool wr, O o, uint32_t base, bool &bad) {
  if (n <= 64) return col_enc<K, 1>(get, n, wr, o, base, bad);
  if (n <= 128) return col_enc<K, 2>(get, n, wr, o, base, bad);
  return col_enc<K, CPL>(get, n, wr, o, base, bad);
}

#define YM2_DECLINE()                    \
  {                                      \
    if (lane == 0) decline(j, d);        \
    __syncthreads();                     \
    continue;                            \
  }

// STOP > 0: timing-only variant ending every document after phase STOP (tools/ablate_fast.py)
#define YM2_STOP(n)                                                     \
  if (STOP == (n)) {                                                    \
    if (lane == 0) { j.status[d] = ym::ST_OK; j.out_len[d] = 0; }       \
    __syncthreads();                                                    \
    continue;                                                           \
  }
// NESTED: the retry pass over the `nd` documents listed in j.list (those the first pass declined).
template <int STOP, int OCC = 1, bool NESTED = false>
__global__ void __launch_bounds__(64, OCC) k_fast_merge_v2(GeneralJob j, uint32_t nd) {
  const uint32_t lane = threadIdx.x;
  const uint64_t arena0 = j.upd_off[0];
  for (uint32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    const uint32_t d = NESTED && j.list ? j.list[di] : di;  // (NESTED without a list: every document)
    const uint32_t u0 = j.doc_upd[d], k = j.doc_upd[d + 1] - u0;
    const uint64_t b0 = j.upd_off[u0], bytes = j.upd_off[u0 + k] - b0;
    if (k <= 1 || k > UPD || bytes > IN) {
      if (lane == 0) decline(j, d);
      continue;
    }
    // ---- 1. stage
    const uint32_t base = (uint32_t)(b0 & 15);
    {  // (offsets loaded before the vectors' stores: all of the stage's loads in flight together)
      uint64_t ov[(UPD + 64) / 64];
#pragma unroll
      for (uint32_t t = 0; t < (UPD + 64) / 64; t++) ov[t] = j.upd_off[u0 + (lane + 64 * t < k ? lane + 64 * t : k)];
      stage16<(IN + 31) / 16 / 64 + 1>(L_IN, reinterpret_cast<const uint4 *>(j.A + (b0 - base)),
                                        (uint32_t)((base + bytes + 15) >> 4));
#pragma unroll
      for (uint32_t t = 0; t < (UPD + 64) / 64; t++)
        at<uint16_t>(L_UOFF + 2 * (lane + 64 * t < k ? lane + 64 * t : k)) = (uint16_t)(ov[t] - b0 + base);
    }
    if (lane < 2) at<uint32_t>(L_MISC + 4 * lane) = 0;
    __syncthreads();
    YM2_STOP(1)
    // ---- 2. walk
    bool ok = true;
#pragma unroll 1
    for (uint32_t u = lane; u < k; u += 64) ok &= walk_v2<NESTED>(u);
    if (__any(!ok)) YM2_DECLINE()
    __syncthreads();
    const uint32_t nrec = at<uint32_t>(L_MISC), nds = at<uint32_t>(L_MISC + 4);
    if (nrec == 0 || nrec > REC || nds > DSN) YM2_DECLINE()
    if (lane == 0) {
      if (nrec & 1) at<uint64_t>(L_RKEY + 8 * nrec) = ~0ull;
      if (nds & 1) at<uint64_t>(L_DKEY + 8 * nds) = ~0ull;
    }
    __syncthreads();
    YM2_STOP(2)
    // ---- 3. struct rank sort (records move to rank order; the slot array detects duplicates)
    {
      uint64_t rk[E];
      uint32_t rr[E];
#pragma unroll
      for (uint32_t s = 0; s < E; s++) rk[s] = lane + 64 * s < nrec ? at<uint64_t>(L_RKEY + 8 * (lane + 64 * s)) : ~0ull;
      rank_le(L_RKEY, nrec, rk, rr);
      uint32_t rl[E], ra[E], s0[E], s1[E], s2[E], sp[E];
      uint4 rf[E];
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t i = lane + 64 * s;
        const bool v = i < nrec;
        rl[s] = v ? at<uint32_t>(L_RLEN + 4 * i) : 0;
        ra[s] = v ? at<uint32_t>(L_RAUX + 4 * i) : 0;
        rf[s] = v ? at<uint4>(L_RF + 16 * i) : make_uint4(0, 0, 0, 0);
        s0[s] = v ? at<uint32_t>(L_RS + 12 * i) : 0;
        s1[s] = v ? at<uint32_t>(L_RS + 12 * i + 4) : 0;
        s2[s] = v ? at<uint32_t>(L_RS + 12 * i + 8) : 0;
        sp[s] = v ? at<uint32_t>(L_RSP + 4 * i) : 0;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t i = lane + 64 * s;
        if (i < nrec) {
          const uint32_t r = rr[s];
          at<uint64_t>(L_RKEY + 8 * r) = rk[s];
          at<uint32_t>(L_RLEN + 4 * r) = rl[s];
          at<uint32_t>(L_RAUX + 4 * r) = ra[s];
          at<uint4>(L_RF + 16 * r) = rf[s];
          at<uint32_t>(L_RS + 12 * r) = s0[s];
          at<uint32_t>(L_RS + 12 * r + 4) = s1[s];
          at<uint32_t>(L_RS + 12 * r + 8) = s2[s];
          at<uint32_t>(L_RSP + 4 * r) = sp[s];
          at<uint8_t>(L_RSLOT + r) = (uint8_t)i;
        }
      }
      __syncthreads();
      bool dup = false;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t i = lane + 64 * s;
        if (i < nrec) dup |= at<uint8_t>(L_RSLOT + rr[s]) != i;
      }
      if (__any(dup)) YM2_DECLINE()
    }
    YM2_STOP(3)
    // ---- 4. layout over rank order; lane owns positions r = E*lane + s
    uint64_t sk[E];
    uint32_t sl_[E], sa[E], s0[E], s1[E], s2[E], ssp[E], pstart[E], gapv[E], runu[E];
    uint4 sf[E];
    uint32_t pu[E], nparts;
    {
      bool bad = false;
      uint32_t plastf[E], units[E];
      const uint32_t r0 = E * lane;
      uint64_t kp = r0 > 0 && r0 - 1 < nrec ? at<uint64_t>(L_RKEY + 8 * (r0 - 1)) : ~0ull;
      uint32_t lp = r0 > 0 && r0 - 1 < nrec ? at<uint32_t>(L_RLEN + 4 * (r0 - 1)) : 0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t r = r0 + s;
        const bool v = r < nrec;
        sk[s] = v ? at<uint64_t>(L_RKEY + 8 * r) : ~0ull;
        sl_[s] = v ? at<uint32_t>(L_RLEN + 4 * r) : 0;
        sa[s] = v ? at<uint32_t>(L_RAUX + 4 * r) : 0;
        sf[s] = v ? at<uint4>(L_RF + 16 * r) : make_uint4(0, 0, 0, 0);
        s0[s] = v ? at<uint32_t>(L_RS + 12 * r) : 0;
        s1[s] = v ? at<uint32_t>(L_RS + 12 * r + 4) : 0;
        s2[s] = v ? at<uint32_t>(L_RS + 12 * r + 8) : 0;
        ssp[s] = v ? at<uint32_t>(L_RSP + 4 * r) : 0;
        const uint64_t kn = r + 1 < nrec ? at<uint64_t>(L_RKEY + 8 * (r + 1)) : ~0ull;
        const bool same = v && r > 0 && (kp >> 32) == (sk[s] >> 32);
        const uint64_t pend = (kp & 0xffffffffull) + lp;
        const uint64_t cl = sk[s] & 0xffffffffull;
        bad |= same && pend > cl;
        gapv[s] = same && pend < cl ? (uint32_t)(cl - pend) : 0;
        units[s] = v ? 1 + (gapv[s] != 0) : 0;
        pstart[s] = v && !same;
        plastf[s] = v && (r + 1 >= nrec || (kn >> 32) != (sk[s] >> 32));
        kp = sk[s];
        lp = sl_[s];
      }
      if (__any(bad)) YM2_DECLINE()
      uint32_t pu_lane = 0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) pu_lane += (pstart[s] << 16) | units[s];
      const uint32_t incl = wave_incl_add(pu_lane);
      nparts = lane_read(incl, 63) >> 16;
      uint32_t run = incl - pu_lane;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        pu[s] = run;
        run += (pstart[s] << 16) | units[s];
        const uint32_t pid = (run >> 16) - 1;
        if (pstart[s]) at<uint16_t>(L_PFIRST + 2 * pid) = (uint16_t)(pu[s] & 0xffff);
        if (plastf[s]) at<uint16_t>(L_PLAST + 2 * pid) = (uint16_t)(run & 0xffff);
      }
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < E; s++)
        runu[s] = pstart[s] ? at<uint16_t>(L_PLAST + 2 * (pu[s] >> 16)) - at<uint16_t>(L_PFIRST + 2 * (pu[s] >> 16)) : 0;
    }
    YM2_STOP(4)
    // ---- 5. columns.  Entry counts per struct (Item.write / LazyStructWriter routing, V2)
    uint32_t cA[E], cB[E], cC[E];  // (cl | lc << 10 | rc << 20), (in | pi << 10 | st << 20), (kc | tr << 10 | ln << 20)
#pragma unroll
    for (uint32_t s = 0; s < E; s++) {
      const bool v = E * lane + s < nrec;
      const uint32_t info = sa[s] & 0xff, pi = (sa[s] >> 8) & 0xff, t = sa[s] >> 16, ref = info & 31;
      const bool ho = info & 0x80, hr = info & 0x40, noo = (info & 0xC0) == 0;
      const bool key = ref == 6 || (ref == 7 && (t == 3 || t == 5));
      const uint32_t ncl = pstart[s] + ho + hr + (noo && !pi);
      const uint32_t nlc = ho || (noo && !pi);
      const uint32_t nin = 1 + (gapv[s] != 0);
      const uint32_t nst = (noo && pi) + (noo && (info & 0x20)) + (ref == 4 || key);
      cA[s] = v ? ncl | (nlc << 10) | ((uint32_t)hr << 20) : 0;
      cB[s] = v ? nin | ((uint32_t)noo << 10) | (nst << 20) : 0;
      cC[s] = v ? (uint32_t)key | ((uint32_t)(ref == 7) << 10) | ((uint32_t)(ref == 1 || ref == 8) << 20) : 0;
    }
    uint32_t oA[E], oB[E], oC[E], nA, nB, nC;
    {
      uint32_t ta = cA[0] + cA[1], tb = cB[0] + cB[1], tc = cC[0] + cC[1];
      const uint32_t ia = wave_incl_add(ta), ib = wave_incl_add(tb), ic = wave_incl_add(tc);
      nA = lane_read(ia, 63); nB = lane_read(ib, 63); nC = lane_read(ic, 63);
      oA[0] = ia - ta; oB[0] = ib - tb; oC[0] = ic - tc;
      oA[1] = oA[0] + cA[0]; oB[1] = oB[0] + cB[0]; oC[1] = oC[0] + cC[0];
    }
    __syncthreads();  // the record arrays are dead (everything is in registers): the value arrays reuse R
#pragma unroll
    for (uint32_t s = 0; s < E; s++) {
      if (E * lane + s >= nrec) break;
      const uint32_t info = sa[s] & 0xff, pi = (sa[s] >> 8) & 0xff, t = sa[s] >> 16, ref = info & 31;
      const bool ho = info & 0x80, hr = info & 0x40, noo = (info & 0xC0) == 0;
      uint32_t icl = oA[s] & 0x3ff, ilc = (oA[s] >> 10) & 0x3ff, irc = oA[s] >> 20;
      uint32_t iin = oB[s] & 0x3ff, ipi = (oB[s] >> 10) & 0x3ff, ist = oB[s] >> 20;
      uint32_t ikc = oC[s] & 0x3ff, itr = (oC[s] >> 10) & 0x3ff, iln = oC[s] >> 20;
      if (pstart[s]) at<uint32_t>(V_CL + 4 * icl++) = ~(uint32_t)(sk[s] >> 32);  // writeClient at a part start
      if (gapv[s]) at<uint8_t>(V_IN + iin++) = 10;                               // Skip
      at<uint8_t>(V_IN + iin) = (uint8_t)(ho || hr ? info & ~0x20u : info);       // 0x20 only without origins
      if (ho) { at<uint32_t>(V_CL + 4 * icl++) = sf[s].x; at<uint32_t>(V_LC + 4 * ilc) = sf[s].y; }
      if (hr) { at<uint32_t>(V_CL + 4 * icl++) = sf[s].z; at<uint32_t>(V_RC + 4 * irc) = sf[s].w; }
      if (noo) {
        at<uint8_t>(V_PI + ipi) = (uint8_t)pi;
        if (pi) at<uint32_t>(V_ST + 4 * ist++) = s0[s];
        else { at<uint32_t>(V_CL + 4 * icl++) = sf[s].x; at<uint32_t>(V_LC + 4 * ilc) = sf[s].y; }
        if (info & 0x20) at<uint32_t>(V_ST + 4 * ist++) = s1[s];
      }
      if (ref == 4 || ref == 6 || (ref == 7 && (t == 3 || t == 5))) at<uint32_t>(V_ST + 4 * ist) = s2[s];
      if (ref == 6 || (ref == 7 && (t == 3 || t == 5))) (void)ikc;  // keyClock values are the entry index
      if (ref == 7) at<uint8_t>(V_TR + itr) = (uint8_t)t;
      if (ref == 1 || ref == 8) at<uint32_t>(V_LN + 4 * iln) = sl_[s];
    }
    __syncthreads();
    const uint32_t ncl = nA & 0x3ff, nlc = (nA >> 10) & 0x3ff, nrc = nA >> 20;
    const uint32_t nin = nB & 0x3ff, npi = (nB >> 10) & 0x3ff, nst = nB >> 20;
    const uint32_t nkc = nC & 0x3ff, ntr = (nC >> 10) & 0x3ff, nln = nC >> 20;
    auto g_cl = [](uint32_t i) { return at<uint32_t>(V_CL + 4 * i); };
    auto g_lc = [](uint32_t i) { return at<uint32_t>(V_LC + 4 * i); };
    auto g_rc = [](uint32_t i) { return at<uint32_t>(V_RC + 4 * i); };
    auto g_ln = [](uint32_t i) { return at<uint32_t>(V_LN + 4 * i); };
    auto g_tr = [](uint32_t i) { return (uint32_t)at<uint8_t>(V_TR + i); };
    auto g_in = [](uint32_t i) { return (uint32_t)at<uint8_t>(V_IN + i); };
    auto g_pi = [](uint32_t i) { return (uint32_t)at<uint8_t>(V_PI + i); };
    auto g_kc = [](uint32_t i) { return i; };
    auto g_sl = [](uint32_t i) { return se_units(at<uint32_t>(V_ST + 4 * i)); };
    // string body bytes and per-entry offsets
    uint32_t sbody, sboff[CPL];
    {
      uint32_t t = 0;
#pragma unroll
      for (uint32_t q = 0; q < CPL; q++) {
        const uint32_t i = lane * CPL + q;
        sboff[q] = t;
        t += i < nst ? se_bytes(at<uint32_t>(V_ST + 4 * i)) : 0;
      }
      const uint32_t incl = wave_incl_add(t);
      sbody = lane_read(incl, 63);
#pragma unroll
      for (uint32_t q = 0; q < CPL; q++) sboff[q] += incl - t;
    }
    bool cbad = false;
    const Slot none = make_slot(j.out, 0);
    uint32_t csz[9];
    csz[0] = col_encode<K_IDIF>(g_kc, nkc, false, none, 0, cbad);
    csz[1] = col_encode<K_UOPT>(g_cl, ncl, false, none, 0, cbad);
    csz[2] = col_encode<K_IDIF>(g_lc, nlc, false, none, 0, cbad);
    csz[3] = col_encode<K_IDIF>(g_rc, nrc, false, none, 0, cbad);
    csz[4] = col_encode<K_RLE>(g_in, nin, false, none, 0, cbad);
    const uint32_t slsz = col_encode<K_UOPT>(g_sl, nst, false, none, 0, cbad);
    csz[5] = vsz(sbody) + sbody + slsz;
    csz[6] = col_encode<K_RLE>(g_pi, npi, false, none, 0, cbad);
    csz[7] = col_encode<K_UOPT>(g_tr, ntr, false, none, 0, cbad);
    csz[8] = col_encode<K_UOPT>(g_ln, nln, false, none, 0, cbad);
    if (__any(cbad)) YM2_DECLINE()
    YM2_STOP(5)
    uint32_t colbytes = 1;
#pragma unroll
    for (uint32_t c = 0; c < 9; c++) colbytes += vsz(csz[c]) + csz[c];
    // rest part bytes per struct: part header (written, first clock), Skip length, payload span
    uint32_t rb[E], rest_lane = 0;
#pragma unroll
    for (uint32_t s = 0; s < E; s++) {
      rb[s] = 0;
      if (E * lane + s >= nrec) continue;
      if (pstart[s]) rb[s] += vsz(runu[s]) + vsz((uint32_t)sk[s]);
      if (gapv[s]) rb[s] += vsz(gapv[s]);
      rb[s] += ssp[s] >> 16;
      rest_lane += rb[s];
    }
    uint32_t rest_bytes, roff0;
    {
      const uint32_t incl = wave_incl_add(rest_lane);
      rest_bytes = lane_read(incl, 63);
      roff0 = incl - rest_lane;
    }
    const uint32_t rest_base = colbytes + vsz(nparts);
    // output slot (as the V1 fast path): 16-aligned inside 2 * in + 64 per doc
    const uint64_t slot = 2 * (b0 - arena0) + 64ull * (d + j.doc_base);
    const uint64_t slot_al = (slot + 15) & ~15ull;
    const uint64_t slot_end = slot + 2 * bytes + 64 < j.cap ? slot + 2 * bytes + 64 : j.cap;
    if (slot_al + rest_base + rest_bytes > slot_end) {
      if (slot_al + rest_base + rest_bytes > slot + 2 * bytes + 64) YM2_DECLINE()
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    if (rest_base + rest_bytes > OUTCAP) YM2_DECLINE()
    const LSlot dst{L_OUT};
    // ---- write the columns: vu(0) | 9 x (vu(size) | bytes)
    {
      uint32_t p = 0;
      if (lane == 0) ob8(dst, 0, 0);
      p = 1;
      uint32_t cb[9];
#pragma unroll
      for (uint32_t c = 0; c < 9; c++) {
        if (lane == 0) put_vu(dst, p, csz[c]);
        p += vsz(csz[c]);
        cb[c] = p;
        p += csz[c];
      }
      col_encode<K_IDIF>(g_kc, nkc, true, dst, cb[0], cbad);
      col_encode<K_UOPT>(g_cl, ncl, true, dst, cb[1], cbad);
      col_encode<K_IDIF>(g_lc, nlc, true, dst, cb[2], cbad);
      col_encode<K_IDIF>(g_rc, nrc, true, dst, cb[3], cbad);
      col_encode<K_RLE>(g_in, nin, true, dst, cb[4], cbad);
      if (lane == 0) put_vu(dst, cb[5], sbody);
      const uint32_t sbase = cb[5] + vsz(sbody);
#pragma unroll
      for (uint32_t q = 0; q < CPL; q++) {  // string bodies: copied from the update's string column
        const uint32_t i = lane * CPL + q;
        if (i >= nst) break;
        const uint32_t e = at<uint32_t>(V_ST + 4 * i), a = se_off(e), n = se_bytes(e);
        lds_copy(dst.b + sbase + sboff[q], a, n);
      }
      col_encode<K_UOPT>(g_sl, nst, true, dst, sbase + sbody, cbad);
      col_encode<K_RLE>(g_pi, npi, true, dst, cb[6], cbad);
      col_encode<K_UOPT>(g_tr, ntr, true, dst, cb[7], cbad);
      col_encode<K_UOPT>(g_ln, nln, true, dst, cb[8], cbad);
    }
    YM2_STOP(6)
    // ---- rest: vu(#parts) | per struct: part header, Skip length, payload
    if (lane == 0) put_vu(dst, colbytes, nparts);
    {
      uint32_t p = rest_base + roff0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        if (E * lane + s >= nrec) break;
        uint32_t q = p;
        if (pstart[s]) { q = put_vu(dst, q, runu[s]); q = put_vu(dst, q, (uint32_t)sk[s]); }
        if (gapv[s]) q = put_vu(dst, q, gapv[s]);
        const uint32_t a = ssp[s] & 0xffff, n = ssp[s] >> 16;
        lds_copy(dst.b + q, a, n);
        p += rb[s];
      }
    }
    const uint32_t dsb = rest_base + rest_bytes;
    YM2_STOP(7)
    // ---- 6. delete set (as ym_fast.hip step 5, V2 encoding: clock - previous end, len - 1)
    {
      uint64_t dk[E];
      uint32_t dl[E], dq[E], dr[E];
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t i = lane + 64 * s;
        const bool v = i < nds;
        dk[s] = v ? at<uint64_t>(L_DKEY + 8 * i) : ~0ull;
        dl[s] = v ? at<uint32_t>(L_DLEN + 4 * i) : 0;
        dq[s] = v ? at<uint16_t>(L_DSEQ + 2 * i) : 0;
      }
      rank_le(L_DKEY, nds, dk, dr);  // distinct keys: a permutation
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        if (lane + 64 * s < nds) {
          const uint32_t r = dr[s];
          at<uint64_t>(L_DKEY + 8 * r) = dk[s];
          at<uint32_t>(L_DLEN + 4 * r) = dl[s];
          at<uint16_t>(L_DSEQ + 2 * r) = (uint16_t)dq[s];
        }
      }
      __syncthreads();
    }
    uint32_t ngroups, nranges;
    bool dbad = false;
    {
      uint32_t ecl[E], ecli[E], segst[E], segid[E], eseq[E];
      uint64_t eend[E];
      uint32_t seg_lane = 0;
      const uint32_t r0 = E * lane;
      uint32_t cprev = r0 > 0 && r0 - 1 < nds ? (uint32_t)(at<uint64_t>(L_DKEY + 8 * (r0 - 1)) >> 32) : 0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t r = r0 + s;
        const bool v = r < nds;
        const uint64_t kk = v ? at<uint64_t>(L_DKEY + 8 * r) : 0;
        ecl[s] = (uint32_t)kk >> 7;
        ecli[s] = (uint32_t)(kk >> 32);
        eend[s] = v ? (uint64_t)ecl[s] + at<uint32_t>(L_DLEN + 4 * r) : 0;
        eseq[s] = v ? at<uint16_t>(L_DSEQ + 2 * r) : 0xffff;
        segst[s] = v && (r == 0 || cprev != ecli[s]);
        seg_lane += segst[s];
        cprev = ecli[s];
      }
      {
        const uint32_t incl = wave_incl_add(seg_lane);
        ngroups = lane_read(incl, 63);
        uint32_t run = incl - seg_lane;
#pragma unroll
        for (uint32_t s = 0; s < E; s++) { run += segst[s]; segid[s] = run - 1; }
      }
      uint64_t m = 0, rmax[E];
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint64_t x = r0 + s < nds ? ((uint64_t)segid[s] << 33) | eend[s] : 0;
        m = x > m ? x : m;
        rmax[s] = m;
      }
      const uint64_t incl = wave_incl_max64(m);
      uint64_t ex = ((uint64_t)from_prev_lane((uint32_t)(incl >> 32)) << 32) | from_prev_lane((uint32_t)incl);
      uint32_t newr[E], nr_lane = 0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint64_t before = ex;
        rmax[s] = rmax[s] > ex ? rmax[s] : ex;
        ex = rmax[s];
        newr[s] = r0 + s < nds && (segst[s] || ecl[s] > (before & 0x1ffffffffull));
        nr_lane += newr[s];
      }
      const uint32_t incl_r = wave_incl_add(nr_lane);
      nranges = lane_read(incl_r, 63);
      uint32_t run = incl_r - nr_lane;
      const uint32_t next_first = from_next_lane(newr[0]);
      __syncthreads();  // the rank-ordered delete ranges are in registers: phase arrays reuse R
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t r = r0 + s;
        if (r >= nds) break;
        run += newr[s];
        const uint32_t rid = run - 1;
        if (newr[s]) {
          at<uint32_t>(L_QCLK + 4 * rid) = ecl[s];
          at<uint8_t>(L_QGRP + rid) = (uint8_t)segid[s];
        }
        const bool nxt_new = s + 1 < E ? newr[s + 1] != 0 : next_first != 0;
        if (r + 1 >= nds || nxt_new) {
          const uint64_t en = rmax[s] & 0x1ffffffffull;
          dbad |= en > 0xffffffffull;
          at<uint32_t>(L_QEND + 4 * rid) = (uint32_t)en;
        }
        if (segst[s]) {
          at<uint16_t>(L_GFIRST + 2 * segid[s]) = (uint16_t)rid;
          at<uint32_t>(L_GCLI + 4 * segid[s]) = ecli[s];
          at<uint32_t>(L_GMIN + 4 * segid[s]) = 0xffffffffu;
        }
      }
      if (lane == 0) at<uint16_t>(L_GFIRST + 2 * ngroups) = (uint16_t)nranges;
      if (__any(dbad)) YM2_DECLINE()
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < E; s++)
        if (r0 + s < nds) atomicMin(&at<uint32_t>(L_GMIN + 4 * segid[s]), eseq[s]);
    }
    __syncthreads();
    // merged ranges q: V2 bytes = vu(clock - end of the previous range of the client) + vu(len - 1)
    {
      uint32_t qb[E], t = 0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t q = E * lane + s;
        qb[s] = 0;
        if (q < nranges) {
          const uint32_t c0 = at<uint32_t>(L_QCLK + 4 * q), e0 = at<uint32_t>(L_QEND + 4 * q);
          const uint32_t g = at<uint8_t>(L_QGRP + q);
          const uint32_t pe = q > at<uint16_t>(L_GFIRST + 2 * g) ? at<uint32_t>(L_QEND + 4 * (q - 1)) : 0;
          qb[s] = vsz(c0 - pe) + vsz(e0 - c0 - 1);
        }
        t += qb[s];
      }
      const uint32_t incl = wave_incl_add(t);
      uint32_t run = incl - t;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t q = E * lane + s;
        if (q < nranges) at<uint16_t>(L_QPRE + 2 * q) = (uint16_t)run;
        run += qb[s];
      }
      if (lane == 63) at<uint16_t>(L_QPRE + 2 * nranges) = (uint16_t)incl;
    }
    __syncthreads();
    uint32_t grk[E], gbytes[E];
#pragma unroll
    for (uint32_t s = 0; s < E; s++) {
      const uint32_t g = lane + 64 * s;
      const bool v = g < ngroups;
      const uint32_t f0 = v ? at<uint16_t>(L_GFIRST + 2 * g) : 0, f1 = v ? at<uint16_t>(L_GFIRST + 2 * g + 2) : 0;
      gbytes[s] = v ? vsz(at<uint32_t>(L_GCLI + 4 * g)) + vsz(f1 - f0) + at<uint16_t>(L_QPRE + 2 * f1) - at<uint16_t>(L_QPRE + 2 * f0) : 0;
      const uint32_t mine = v ? at<uint32_t>(L_GMIN + 4 * g) : 0;
      uint32_t rk_ = 0;
      for (uint32_t h = 0; h < ngroups; h++) rk_ += at<uint32_t>(L_GMIN + 4 * h) < mine;
      grk[s] = rk_;
    }
#pragma unroll
    for (uint32_t s = 0; s < E; s++)
      if (lane + 64 * s < ngroups) at<uint16_t>(L_GBYR + 2 * grk[s]) = (uint16_t)gbytes[s];
    __syncthreads();
    const uint32_t ds_hdr = vsz(ngroups);
    uint32_t ds_groups_bytes;
    {
      uint32_t v[E], t = 0;
#pragma unroll
      for (uint32_t s = 0; s < E; s++) { const uint32_t r = E * lane + s; v[s] = r < ngroups ? at<uint16_t>(L_GBYR + 2 * r) : 0; t += v[s]; }
      const uint32_t incl = wave_incl_add(t);
      ds_groups_bytes = lane_read(incl, 63);
      uint32_t run = incl - t;
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < E; s++) {
        const uint32_t r = E * lane + s;
        if (r < ngroups) at<uint16_t>(L_GBYR + 2 * r) = (uint16_t)run;
        run += v[s];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t s = 0; s < E; s++) {
      const uint32_t g = lane + 64 * s;
      if (g < ngroups) {
        const uint32_t f0 = at<uint16_t>(L_GFIRST + 2 * g), f1 = at<uint16_t>(L_GFIRST + 2 * g + 2);
        const uint32_t off = dsb + ds_hdr + at<uint16_t>(L_GBYR + 2 * grk[s]);
        at<uint32_t>(L_GMIN + 4 * g) = off;
        at<uint32_t>(L_GB2 + 4 * g) = off + vsz(at<uint32_t>(L_GCLI + 4 * g)) + vsz(f1 - f0) - at<uint16_t>(L_QPRE + 2 * f0);
      }
    }
    __syncthreads();
    const uint32_t total = dsb + ds_hdr + ds_groups_bytes;
    if (slot_al + total > slot_end) {
      if (slot_al + total > slot + 2 * bytes + 64) YM2_DECLINE()
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    if (total > OUTCAP) YM2_DECLINE()
    if (lane == 0) put_vu(dst, dsb, ngroups);
#pragma unroll
    for (uint32_t s = 0; s < E; s++) {
      const uint32_t g = lane + 64 * s;
      if (g < ngroups)
        put_vu(dst, put_vu(dst, at<uint32_t>(L_GMIN + 4 * g), at<uint32_t>(L_GCLI + 4 * g)),
               at<uint16_t>(L_GFIRST + 2 * g + 2) - at<uint16_t>(L_GFIRST + 2 * g));
      const uint32_t q = E * lane + s;
      if (q < nranges) {
        const uint32_t c0 = at<uint32_t>(L_QCLK + 4 * q), e0 = at<uint32_t>(L_QEND + 4 * q);
        const uint32_t g2 = at<uint8_t>(L_QGRP + q);
        const uint32_t pe = q > at<uint16_t>(L_GFIRST + 2 * g2) ? at<uint32_t>(L_QEND + 4 * (q - 1)) : 0;
        const uint32_t off = at<uint32_t>(L_GB2 + 4 * g2) + at<uint16_t>(L_QPRE + 2 * q);
        put_vu(dst, put_vu(dst, off, c0 - pe), e0 - c0 - 1);
      }
    }
    __syncthreads();
    copy_out(j.out + slot_al, L_OUT, total, slot_end - slot_al);
    if (lane == 0) {
      j.out_off[d] = slot_al;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}

// ---- parseUpdateMetaV2 / encodeStateVectorFromUpdateV2 over small updates: one update per LANE -------------
// 13.5.16 parseUpdateMetaV2 / encodeStateVectorFromUpdateV2 (LazyStructReader over UpdateDecoderV2; the delete
// set is not read): per client section with structs its client, its first clock and the end of its last
// struct; meta writes (client, first)* then (client, end)*, the state vector (client, end) for the sections
// that start at clock 0 (os@37724: a section from a later clock counts nothing; no Skip reaches here).  A block
// takes ND consecutive single-update documents: the wave stages their (contiguous) bytes into one LDS window
// of WIN bytes with 16-byte loads, then lane l walks document l with the per-lane column decoders of the merge
// walk (walk_v2: the same acceptance -- canonical columns, ASCII string bodies, no Skip / GC, no ContentJSON /
// Doc, keys never read from the cache) and k_big_v2's rules (clients strictly descending); the wave sizes the
// outputs by a prefix sum and bump-allocates them with one atomic.  A lane that declines, or a document outside
// the window, leaves the document to k_big_v2 (done[d] stays 0) or, without a done array, to the general path.
template <uint32_t ND, uint32_t WIN, uint32_t NSEC>
struct Sv2Lay {
  static constexpr uint32_t TAB = WIN + 48;                // u32[ND][NSEC][3]: client, first, end
  static constexpr uint32_t BYTES = TAB + ND * NSEC * 12;
};
// the lane's update at LDS [p0, p1): its sections into the table at `tab` (<= nsec_max); the count, or -1 to
// decline
__device__ __forceinline__ int meta_walk_v2(uint32_t p0, uint32_t p1, uint32_t tab, uint32_t nsec_max) {
  Cur h = {p0, p1, false};
  rvu(h);  // feature flag
  Cur col[9];
#pragma unroll
  for (uint32_t k = 0; k < 9; k++) {
    const uint32_t n = rvu(h);
    if (!room(h, n)) return -1;
    col[k] = Cur{h.p, h.p + n, false};
    h.p += n;
  }
  if (h.bad) return -1;
  const uint32_t sn = rvu(col[5]);
  if (col[5].bad || !room(col[5], sn)) return -1;
  const uint32_t sb = col[5].p;
  uint32_t sunits = sn;  // the body's UTF-16 units: only lengths matter here (strings are not sliced or copied)
  {
    uint64_t hi = 0;
    for (uint32_t o = 0; o < sn; o += 8) hi |= mask_bytes(ld8(sb + o), sn - o);
    if (hi & 0x8080808080808080ull) {  // (valid UTF-8 only: the decoder's replacements would change lengths)
      bool ub = false;
      sunits = utf8_slow(sb, sb + sn, ub);
      if (ub) return -1;
    }
  }
  col[5].p += sn;
  IdifD kc = {col[0], 0, 0, 0};
  UoptD cl = {col[1], 0, 0};
  IdifD lc = {col[2], 0, 0, 0}, rc = {col[3], 0, 0, 0};
  RleD in = {col[4], 0, 0};
  UoptD sl = {col[5], 0, 0};
  RleD pi_ = {col[6], 0, 0};
  UoptD tr = {col[7], 0, 0}, ln = {col[8], 0, 0};
  uint32_t spos = 0, keys = 0;
  Cur c = h;  // rest stream
  bool bad = false;
  auto rstr = [&]() -> uint32_t {  // StringDecoder.read(): its UTF-16 length (str.slice within the body's units)
    const uint32_t n = rd_uopt(sl);
    bad |= spos + n > sunits;
    spos += n;
    return n;
  };
  const uint32_t nclients = rvu(c);
  uint32_t prev_client = 0, nsec = 0;
  for (uint32_t ci = 0; ci < nclients && !c.bad && !bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = rd_uopt(cl);
    uint64_t clock = rvu(c);
    bad |= ci > 0 && client >= prev_client;  // a repeated or ascending client: k_big_v2 declines (Map order)
    prev_client = client;
    const uint32_t first = (uint32_t)clock;
    for (uint32_t si = 0; si < nstructs && !c.bad && !bad; si++) {
      const uint32_t info = rd_rle(in);
      bad |= info == 10 || (info & 31) == 0 || info > 255;  // Skip / GC: the streamed walker
      if (info & 0x80) { rd_uopt(cl); rd_idif(lc); }
      if (info & 0x40) { rd_uopt(cl); rd_idif(rc); }
      if ((info & 0xC0) == 0) {
        if (rd_rle(pi_) == 1) rstr();
        else { rd_uopt(cl); rd_idif(lc); }
        if (info & 0x20) rstr();
      }
      uint32_t len = 1;
      switch (info & 31) {
        case 1: len = rd_uopt(ln); break;  // ContentDeleted
        case 3: {                          // ContentBinary (rest)
          const uint32_t n = rvu(c);
          if (!room(c, n)) bad = true;
          else c.p += n;
          break;
        }
        case 4: len = rstr(); break;  // ContentString
        case 5: case 6:               // Embed / Format (+ key)
          if ((info & 31) == 6) rstr();
          any_canon<false>(c);
          break;
        case 7: {  // ContentType
          const uint32_t t = rd_uopt(tr);
          bad |= t > 6;
          if (t == 3 || t == 5) {
            bad |= rd_idif(kc) < keys;
            keys++;
            rstr();
          }
          break;
        }
        case 8:  // ContentAny
          len = rd_uopt(ln);
          for (uint32_t i = 0; i < len && !c.bad; i++) any_canon<false>(c);
          break;
        default: bad = true; break;  // ContentJSON, ContentDoc, invalid refs
      }
      bad |= c.bad | (len == 0) | ((uint64_t)clock + len > 0xffffffffull);
      clock += len;
    }
    if (nstructs > 0 && !bad) {
      bad |= nsec >= nsec_max;
      if (!bad) {
        at<uint32_t>(tab + 12 * nsec) = client;
        at<uint32_t>(tab + 12 * nsec + 4) = first;
        at<uint32_t>(tab + 12 * nsec + 8) = (uint32_t)clock;
        nsec++;
      }
    }
  }
  bad |= c.bad | cl.c.bad | lc.c.bad | rc.c.bad | in.c.bad | sl.c.bad | pi_.c.bad | tr.c.bad | ln.c.bad | kc.c.bad;
  return bad ? -1 : (int)nsec;
}
template <int OP, uint32_t ND, uint32_t WIN, uint32_t NSEC>
__global__ void __launch_bounds__(64) k_small_v2(GeneralJob j, uint8_t *done, uint64_t pv_min) {
  using L = Sv2Lay<ND, WIN, NSEC>;
  const uint32_t lane = threadIdx.x;
  const uint32_t d0 = blockIdx.x * ND, d = d0 + lane;
  if (d0 >= j.n) return;
  const uint32_t dn = j.n - d0 < ND ? j.n - d0 : ND;
  // the window: the bytes of document d0 onwards (the ND documents' updates are contiguous in a packed batch)
  const uint64_t w0 = j.upd_off[j.doc_upd[d0]] & ~15ull;
  const uint64_t wend = j.upd_off[j.doc_upd[d0 + dn]];
  const uint32_t wbytes = (uint32_t)((wend - w0 < WIN ? wend - w0 : WIN) + 15) & ~15u;
  if (wbytes) stage16<(WIN + 15) / 16 / 64 + 1>(0, reinterpret_cast<const uint4 *>(j.A + w0), wbytes / 16);
  __syncthreads();
  int ns = -1;
  const uint32_t tab = L::TAB + 12 * NSEC * (lane < ND ? lane : 0);
  if (lane < dn) {
    const uint32_t u0 = j.doc_upd[d];
    if (j.doc_upd[d + 1] - u0 == 1 && !(done && done[d])) {
      const uint64_t a = j.upd_off[u0], b = j.upd_off[u0 + 1];
      // (from pv_min on, a document is the column path's: the two sets stay disjoint)
      if (a >= w0 && b <= w0 + wbytes && b > a && b - a < pv_min) ns = meta_walk_v2((uint32_t)(a - w0), (uint32_t)(b - w0), tab, NSEC);
    }
  }
  // meta: vu(n) | (client, first)* | vu(n) | (client, end)*;  sv: vu(m) | (client, end)* over the m sections
  // that start at 0
  uint32_t sz = 0, m = 0;
  if (ns >= 0) {
    for (int k = 0; k < ns; k++) {
      const uint32_t cl = at<uint32_t>(tab + 12 * k), f = at<uint32_t>(tab + 12 * k + 4), e = at<uint32_t>(tab + 12 * k + 8);
      if (OP == OP_META) sz += 2 * vsz(cl) + vsz(f) + vsz(e);
      else if (f == 0) { sz += vsz(cl) + vsz(e); m++; }
    }
    sz += OP == OP_META ? 2 * vsz((uint32_t)ns) : vsz(m);
  }
  const uint32_t incl = wave_incl_add(sz), total = lane_read(incl, 63);
  uint64_t base = 0;
  if (lane == 0 && total) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
  base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
  if (ns >= 0) {
    const uint64_t off = base + incl - sz;
    if (off + sz > j.cap) {
      j.status[d] = ym::ST_CAPACITY;
      j.out_len[d] = 0;
    } else {
      const Slot o = make_slot(j.out + off, sz);
      if (OP == OP_META) {
        uint32_t p = put_vu(o, 0, (uint32_t)ns);
        for (int k = 0; k < ns; k++) p = put_vu(o, put_vu(o, p, at<uint32_t>(tab + 12 * k)), at<uint32_t>(tab + 12 * k + 4));
        p = put_vu(o, p, (uint32_t)ns);
        for (int k = 0; k < ns; k++) p = put_vu(o, put_vu(o, p, at<uint32_t>(tab + 12 * k)), at<uint32_t>(tab + 12 * k + 8));
      } else {
        uint32_t p = put_vu(o, 0, m);
        for (int k = 0; k < ns; k++)
          if (at<uint32_t>(tab + 12 * k + 4) == 0) p = put_vu(o, put_vu(o, p, at<uint32_t>(tab + 12 * k)), at<uint32_t>(tab + 12 * k + 8));
      }
      j.out_off[d] = off;
      j.out_len[d] = sz;
      j.status[d] = ym::ST_OK;
    }
    if (done) done[d] = 1;
  } else if (lane < dn && !done) {
    decline(j, d);  // no streamed walker after this kernel: the general path
  }
}

// ---- diffUpdateV2 over small updates: one update per LANE --------------------------------------------------
// 13.5.16 diffUpdateV2 (us@40707): the structs of each client section from the first one ending past the state
// vector's clock on (that one sliced by `off`), re-encoded with the lib0 column encoders -- Item.write(encoder,
// off) as k_big_v2's v2_write -- into per-lane output streams in LDS, then vu(0) | 9 x varUint8Array(column) |
// vu(#parts) | parts (vu(written) | first clock | payloads) | delete set (copied: a canonical V2 delete set
// round-trips byte for byte).  A block takes ND consecutive single-update documents and their state vectors:
// both windows are staged into LDS with 16-byte loads, each lane decodes its state vector into a table, sizes
// its eleven output streams from its input columns (a wave prefix sum carves them out of one LDS pool), walks
// its update with the per-lane column decoders of the merge walk and writes the streams; the wave sizes the
// outputs by a prefix sum, bump-allocates them with one atomic and each lane copies its document out.  Anything
// outside this path's acceptance (Skip / GC / JSON / Doc inputs, cached keys, non-ASCII strings, clients not
// strictly descending, a stream or table overflow, documents outside the windows) leaves done[d] = 0: k_big_v2.
template <uint32_t ND, uint32_t WIN, uint32_t POOL>
struct Df2Lay {
  // (several documents per wave: at most 32 client sections / state-vector entries each -- a wider document,
  // C4's 64 clients, declines at its header and takes k_big_v2's single generation, which is faster for it)
  static constexpr uint32_t SVW = ND == 1 ? 1024 : 128 * ND, NSV = ND == 1 ? 128 : 32, NPART = NSV;
  static constexpr uint32_t SV = WIN + 48;               // u8[SVW + 16]: the state vectors
  static constexpr uint32_t SVT = SV + SVW + 16;         // u32[ND][NSV][2]: client, clock (then the ds clients)
  static constexpr uint32_t PT = SVT + ND * NSV * 8;     // u32[ND][NPART][4]: rest start, rest end, written
  static constexpr uint32_t OUT = PT + ND * NPART * 16;  // u8[POOL]: the lanes' output streams
  static constexpr uint32_t BYTES = OUT + POOL + 16;
};
namespace df2 {
struct OS { uint32_t a, n, cap; };  // an output stream in LDS: start, bytes written (may pass cap), capacity
__device__ __forceinline__ void ob(OS &s, uint32_t v) {
  if (s.n < s.cap) at<uint8_t>(s.a + s.n) = (uint8_t)v;
  s.n++;
}
__device__ __forceinline__ void ovu(OS &s, uint32_t v) {
  while (v > 127) { ob(s, 0x80 | (v & 127)); v >>= 7; }
  ob(s, v);
}
__device__ __forceinline__ void ovi(OS &s, bool neg, uint32_t m) {  // lib0 writeVarInt (sign in the first byte)
  ob(s, (m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63));
  m >>= 6;
  while (m > 0) { ob(s, (m > 127 ? 0x80 : 0) | (m & 127)); m >>= 7; }
}
__device__ __forceinline__ void ospan(OS &s, uint32_t a, uint32_t n) {  // LDS bytes [a, a + n)
  if (s.n + n <= s.cap) lds_copy(s.a + s.n, a, n);
  s.n += n;
}
// LDS bytes [src, src + n) to dst <= src (ascending 8-byte chunks: safe when the regions overlap)
__device__ __forceinline__ void lds_move_down(uint32_t dst, uint32_t src, uint32_t n) {
  if (dst == src) return;
  lds_copy(dst, src, n);
}
struct UE { uint32_t s, n; };             // UintOptRleEncoder
struct IE { uint32_t s, n; int32_t d; };  // IntDiffOptRleEncoder
struct RE { uint32_t s, n; };             // RleEncoder<u8> (n == 0: nothing written yet)
__device__ __forceinline__ void ue_flush(OS &o, const UE &e) {
  if (e.n > 0) {
    ovi(o, e.n != 1, e.s);  // count == 1 ? s : -s (-0 for 0)
    if (e.n > 1) ovu(o, e.n - 2);
  }
}
__device__ __forceinline__ void ue_w(OS &o, UE &e, uint32_t v) {
  if (e.s == v) { e.n++; return; }
  ue_flush(o, e);
  e.s = v;
  e.n = 1;
}
__device__ __forceinline__ void ie_flush(OS &o, const IE &e) {
  if (e.n > 0) {
    const int32_t x = (int32_t)((uint32_t)e.d << 1) | (e.n == 1 ? 0 : 1);
    ovi(o, x < 0, x < 0 ? (uint32_t)(-(int64_t)x) : (uint32_t)x);
    if (e.n > 1) ovu(o, e.n - 2);
  }
}
__device__ __forceinline__ void ie_w(OS &o, IE &e, uint32_t v, bool &bad) {
  const int64_t d = (int64_t)v - (int64_t)e.s;
  bad |= d < -(1ll << 30) || d >= (1ll << 30);  // JS `diff << 1` wraps beyond
  if (e.d == (int32_t)d) { e.s = v; e.n++; return; }
  ie_flush(o, e);
  e.s = v;
  e.n = 1;
  e.d = (int32_t)d;
}
__device__ __forceinline__ void re_w(OS &o, RE &e, uint32_t v) {
  if (e.n > 0 && e.s == v) { e.n++; return; }
  if (e.n > 0) ovu(o, e.n - 1);
  ob(o, v);
  e.s = v;
  e.n = 1;
}
// output streams: the nine columns (the string column as body + lengths) and the rest stream of the parts
enum { S_KC = 0, S_CL, S_LC, S_RC, S_IN, S_SB, S_SL, S_PI, S_TR, S_LN, S_RE, NS };

// Column cursors with their next 8 bytes already in registers: the refill load is issued as soon as a value
// is consumed and waited for only at the column's next read (usually a struct later), so a struct's chain of
// column reads does not wait on one LDS round trip per field.
struct PC { uint32_t p, e; bool bad; uint64_t w; };
__device__ __forceinline__ PC pc_make(const Cur &c) { return PC{c.p, c.e, c.bad, ld8(c.p)}; }
__device__ __forceinline__ void pc_adv(PC &c, uint32_t nb) { c.p += nb; c.w = ld8(c.p); }
__device__ __forceinline__ uint32_t pc_vu(PC &c) {  // rvu
  const uint32_t lo = (uint32_t)c.w, hi = (uint32_t)(c.w >> 32);
  if (__all((lo & 0x80u) == 0)) {
    c.bad |= c.p >= c.e;
    pc_adv(c, 1);
    return lo & 0x7fu;
  }
  const uint32_t nb = vu_nb(lo, hi);
  const uint32_t v = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u) | (hi << 28);
  const uint32_t m = (uint32_t)((1ull << (7 * (nb < 5 ? nb : 5))) - 1);
  c.bad |= vu_bad(lo, hi, nb, c.p, c.e);
  pc_adv(c, nb < 6 ? nb : 0);
  return v & m;
}
__device__ __forceinline__ uint32_t pc_vi(PC &c, bool &neg) {  // rvi
  const uint32_t lo = (uint32_t)c.w, hi = (uint32_t)(c.w >> 32);
  neg = (lo & 0x40) != 0;
  if (__all((lo & 0x80u) == 0)) {
    c.bad |= c.p >= c.e;
    pc_adv(c, 1);
    return lo & 0x3fu;
  }
  const uint32_t nb = vu_nb(lo, hi);
  uint32_t m = (lo & 0x3fu) | ((lo >> 2) & 0x1fc0u) | ((lo >> 3) & 0xfe000u) | ((lo >> 4) & 0x7f00000u) | ((hi & 0x7fu) << 27);
  const uint32_t bits = 6 + 7 * (nb - 1);
  if (nb < 5) m &= (1u << bits) - 1u;
  c.bad |= (nb > 5) | (c.p + nb > c.e) | ((nb == 5) & ((hi & 0x7fu) > 0x1fu));
  pc_adv(c, nb < 6 ? nb : 0);
  return m;
}
__device__ __forceinline__ uint32_t pc_b(PC &c) {  // rdb
  c.bad |= c.p >= c.e;
  const uint32_t v = (uint32_t)c.w & 0xffu;
  pc_adv(c, 1);
  return v;
}
struct PRle { PC c; uint32_t s, n; };
struct PUopt { PC c; uint32_t s, n; };
struct PIdif { PC c; uint32_t s, n; int32_t d; };
__device__ __forceinline__ uint32_t pd_rle(PRle &r) {  // rd_rle
  if (r.n == 0) {
    r.s = pc_b(r.c);
    r.n = r.c.p < r.c.e ? pc_vu(r.c) + 1 : 0xffffffffu;  // the final run never ends
  }
  if (r.n != 0xffffffffu) r.n--;
  return r.s;
}
__device__ __forceinline__ uint32_t pd_uopt(PUopt &r) {  // rd_uopt
  if (r.n == 0) {
    bool neg;
    r.s = pc_vi(r.c, neg);
    r.n = neg ? pc_vu(r.c) + 2 : 1;
  }
  r.n--;
  return r.s;
}
__device__ __forceinline__ uint32_t pd_idif(PIdif &r) {  // rd_idif
  if (r.n == 0) {
    bool neg;
    const uint32_t m = pc_vi(r.c, neg);
    const int32_t t = (int32_t)(neg ? 0u - m : m);
    r.d = t >> 1;
    r.n = (t & 1) ? pc_vu(r.c) + 2 : 1;
  }
  const int64_t v = (int64_t)r.s + r.d;
  r.c.bad |= v < 0 || v > 0xffffffffll;
  r.s = (uint32_t)v;
  r.n--;
  return r.s;
}
}  // namespace df2

template <uint32_t ND, uint32_t WIN, uint32_t POOL, int OCC>
__global__ void __launch_bounds__(64, OCC) k_diff_small_v2(GeneralJob j, uint8_t *done, uint64_t pv_min, uint32_t retry) {
  using namespace df2;
  using L = Df2Lay<ND, WIN, POOL>;
  const uint32_t lane = threadIdx.x;
  const uint32_t d0 = blockIdx.x * ND, d = d0 + lane;
  if (d0 >= j.n) return;
  if (retry && ND == 1 && done[d0] != 2 && done[d0] != 5) return;  // (retry launches: most blocks have nothing to do)
  const uint32_t dn = j.n - d0 < ND ? j.n - d0 : ND;
  // the windows: the ND updates and their state vectors (each contiguous in a packed batch)
  const uint64_t w0 = j.upd_off[j.doc_upd[d0]] & ~15ull, wend = j.upd_off[j.doc_upd[d0 + dn]];
  const uint32_t wbytes = (uint32_t)((wend - w0 < WIN ? wend - w0 : WIN) + 15) & ~15u;
  const uint64_t v0 = j.sv_off[d0] & ~15ull, vend = j.sv_off[d0 + dn];
  const uint32_t vbytes = (uint32_t)((vend - v0 < L::SVW ? vend - v0 : L::SVW) + 15) & ~15u;
  if (wbytes) stage16<(WIN + 15) / 16 / 64 + 1>(0, reinterpret_cast<const uint4 *>(j.A + w0), wbytes / 16);
  if (vbytes) stage16<(L::SVW + 15) / 16 / 64 + 1>(L::SV, reinterpret_cast<const uint4 *>(j.sv + v0), vbytes / 16);
  __syncthreads();
  bool ok = false, sel = false;
  uint32_t p0 = 0, p1 = 0, s0 = 0, s1 = 0;
  if (lane < dn) {
    const uint32_t u0 = j.doc_upd[d];
    // retry: only the documents a previous launch left outside its windows or its shared output pool (done 2
    // or 5; one document per wave)
    sel = retry ? done[d] == 2 || done[d] == 5 : !done[d];
    if (j.doc_upd[d + 1] - u0 == 1 && sel) {
      const uint64_t a = j.upd_off[u0], b = j.upd_off[u0 + 1], sa = j.sv_off[d], sb = j.sv_off[d + 1];
      ok = a >= w0 && b <= w0 + wbytes && b > a && b - a < pv_min && sa >= v0 && sb <= v0 + vbytes && sb >= sa;
      p0 = (uint32_t)(a - w0); p1 = (uint32_t)(b - w0);
      s0 = L::SV + (uint32_t)(sa - v0); s1 = L::SV + (uint32_t)(sb - v0);
    }
  }
  // decline reasons (done[d], read by ym__pv2_done): 2 not in the windows / several updates, 3 state vector,
  // 4 header, 5 output pool, 6 walk, 7 delete set, 8 stream overflow, 9 in-place assembly
  uint32_t why = ok || !sel ? 0 : 2;  // (a document this launch does not select keeps its done value)
  const uint32_t svt = L::SVT + 8 * L::NSV * (lane < ND ? lane : 0);
  const uint32_t pt = L::PT + 16 * L::NPART * (lane < ND ? lane : 0);
  // decodeStateVector into the lane's table (a later entry for a client wins: the lookup scans backwards)
  uint32_t nsv = 0;
  if (ok) {
    Cur c = {s0, s1, false};
    const uint32_t n = rvu(c);
    ok = !c.bad && n <= L::NSV;
    for (uint32_t i = 0; ok && i < n; i++) {
      const uint32_t cl = rvu(c), ck = rvu(c);
      at<uint2>(svt + 8 * i) = make_uint2(cl, ck);
    }
    ok &= !c.bad;
    nsv = n;
    if (!ok && !why) why = 3;
  }
  // header: the nine column spans, the ASCII string body, the rest stream's client count
  Cur col[9], c = {0, 0, false};
  uint32_t sn = 0, sb = 0, sunits = 0, nclients = 0, need = 0;
  bool sascii = true;
  uint32_t in_sz[NS];
  if (ok) {
    Cur h = {p0, p1, false};
    rvu(h);  // feature flag
#pragma unroll
    for (uint32_t k = 0; k < 9; k++) {
      const uint32_t n = rvu(h);
      ok &= room(h, n);
      col[k] = Cur{h.p, h.p + n, false};
      h.p += ok ? n : 0;
    }
    ok &= !h.bad;
    sn = rvu(col[5]);
    ok &= !col[5].bad && room(col[5], sn);
    sb = col[5].p;
    if (ok) {
      uint64_t hi = 0;
      for (uint32_t o = 0; o < sn; o += 8) hi |= mask_bytes(ld8(sb + o), sn - o);
      sascii = (hi & 0x8080808080808080ull) == 0;
      if (!sascii) {  // valid UTF-8 only (round 6; ASCII only before): strings are sliced by UTF-16 units
        bool ub = false;
        sunits = utf8_slow(sb, sb + sn, ub);
        ok &= !ub;
      } else {
        sunits = sn;
      }
      col[5].p += sn;
    }
    c = h;  // rest stream
    nclients = rvu(c);
    ok &= !c.bad && nclients <= L::NPART;
    in_sz[S_KC] = col[0].e - col[0].p; in_sz[S_CL] = col[1].e - col[1].p; in_sz[S_LC] = col[2].e - col[2].p;
    in_sz[S_RC] = col[3].e - col[3].p; in_sz[S_IN] = col[4].e - col[4].p; in_sz[S_SB] = sn;
    in_sz[S_SL] = col[5].e - col[5].p; in_sz[S_PI] = col[6].e - col[6].p; in_sz[S_TR] = col[7].e - col[7].p;
    in_sz[S_LN] = col[8].e - col[8].p; in_sz[S_RE] = p1 - c.p;
    // room per stream: what the written structs can add over their input bytes -- run splits at every part
    // (one per client section at most), the cut struct's new origin (client + left clock) and sliced length,
    // the part headers in the rest stream; the string body only shrinks.  A stream that still overflows
    // declines the document (k_big_v2).
    const uint32_t nc = nclients;
    const uint32_t room[NS] = {8, 8 + 16 * nc, 8 + 16 * nc, 8 + 8 * nc, 8 + 4 * nc, 0, 8 + 4 * nc, 8 + 2 * nc, 8, 8 + 8 * nc, 8 + 8 * nc};
#pragma unroll
    for (uint32_t k = 0; k < NS; k++) {
      in_sz[k] += (k == S_SB || k == S_KC || k == S_TR || k == S_PI || k == S_LN ? 0 : in_sz[k] >> 3) + room[k];
      need += in_sz[k];
    }
    need = (need + 16 + 15) & ~15u;  // (16 bytes ahead of the streams: the output is assembled in place)
    if (!ok && !why) why = 4;
  }
  // the lanes' output streams out of the pool
  const uint32_t incl = wave_incl_add(ok ? need : 0);
  ok &= incl <= POOL;
  if (!ok && !why) why = 5;
  OS os[NS];
  {
    uint32_t a = L::OUT + incl - (ok ? need : 0) + 16;
#pragma unroll
    for (uint32_t k = 0; k < NS; k++) { os[k] = OS{a, 0, ok ? in_sz[k] : 0}; a += ok ? in_sz[k] : 0; }
  }
  PIdif kc = {pc_make(col[0]), 0, 0, 0};
  PUopt cl = {pc_make(col[1]), 0, 0};
  PIdif lc = {pc_make(col[2]), 0, 0, 0}, rc = {pc_make(col[3]), 0, 0, 0};
  PRle in = {pc_make(col[4]), 0, 0};
  PUopt sl = {pc_make(col[5]), 0, 0};
  PRle pi_ = {pc_make(col[6]), 0, 0};
  PUopt tr = {pc_make(col[7]), 0, 0}, ln = {pc_make(col[8]), 0, 0};
  UE e_cl = {0, 0}, e_sl = {0, 0}, e_tr = {0, 0}, e_ln = {0, 0};
  IE e_kc = {0, 0, 0}, e_lc = {0, 0, 0}, e_rc = {0, 0, 0};
  RE e_in = {0, 0}, e_pi = {0, 0};
  uint32_t spos = 0, supos = 0, keys = 0, kclock = 0, nparts = 0, prev_client = 0;
  bool bad = !ok, uri = false;
  // a string: its body offset a and n = bytes | UTF-16 units << 16
  auto rstr = [&](uint32_t &a, uint32_t &n) {  // StringDecoder.read(): str.slice(spos, spos + units)
    const uint32_t u = pd_uopt(sl);
    const uint32_t nb = sascii ? u : utf8_span(sb + spos, sb + sn, u, bad);
    bad |= spos + nb > sn || supos + u > sunits || u > 0xffff;
    a = sb + spos;
    n = nb | (u << 16);
    spos += nb;
    supos += u;
  };
  auto wstr = [&](uint32_t a, uint32_t n) {  // StringEncoder.write
    ospan(os[S_SB], a, n & 0xffff);
    ue_w(os[S_SL], e_sl, n >> 16);
  };
  auto wkey = [&]() {  // writeKey: keyClock++ (never cached, E9)
    ie_w(os[S_KC], e_kc, kclock, bad);
    kclock++;
  };
  for (uint32_t ci = 0; ci < nclients && !bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = pd_uopt(cl);
    uint32_t clock = rvu(c);
    bad |= ci > 0 && client >= prev_client;  // a repeated or ascending client: k_big_v2
    prev_client = client;
    uint32_t k = 0;  // state.get(client) || 0
    for (uint32_t i = nsv; i-- > 0;) {
      const uint2 e = at<uint2>(svt + 8 * i);
      if (e.x == client) { k = e.y; break; }
    }
    bool copying = false;
    uint32_t written = 0, prest0 = 0;
    for (uint32_t si = 0; si < nstructs && !bad; si++) {
      const uint32_t info = pd_rle(in);
      bad |= info == 10 || (info & 31) == 0 || info > 255;  // Skip / GC inputs: k_big_v2
      // the struct (LazyStructReader): what Item.write needs to re-encode it
      uint32_t oc = 0, ok_ = 0, rcl = 0, rk = 0, pi = 0, ya = 0, yn = 0, pc = 0, pk = 0, pa = 0, pn = 0;
      uint32_t ca = 0, cn = 0, ka = 0, kn = 0, t = 0, r0 = 0, r1 = 0, len = 1;
      if (info & 0x80) { oc = pd_uopt(cl); ok_ = pd_idif(lc); }
      if (info & 0x40) { rcl = pd_uopt(cl); rk = pd_idif(rc); }
      if ((info & 0xC0) == 0) {
        pi = pd_rle(pi_) == 1 ? 1 : 0;
        if (pi) rstr(ya, yn);
        else { pc = pd_uopt(cl); pk = pd_idif(lc); }
        if (info & 0x20) rstr(pa, pn);
      }
      switch (info & 31) {
        case 1: len = pd_uopt(ln); break;  // ContentDeleted
        case 3: {                          // ContentBinary: rest varUint8Array
          r0 = c.p;
          const uint32_t n = rvu(c);
          if (!room(c, n)) bad = true;
          else c.p += n;
          r1 = c.p;
          break;
        }
        case 4: rstr(ca, cn); len = cn >> 16; break;  // ContentString
        case 5: case 6:                         // Embed / Format: rest any (Format reads its key as a string)
          if ((info & 31) == 6) rstr(ka, kn);
          r0 = c.p;
          any_canon<true>(c);
          r1 = c.p;
          break;
        case 7:  // ContentType
          t = pd_uopt(tr);
          bad |= t > 6;
          if (t == 3 || t == 5) {  // readKey: a cached key (keyClock < keys read) reads no string
            bad |= pd_idif(kc) < keys;
            keys++;
            rstr(ka, kn);
          }
          break;
        case 8:  // ContentAny: len column + rest values
          len = pd_uopt(ln);
          r0 = c.p;
          for (uint32_t i = 0; i < len && !c.bad; i++) any_canon<true>(c);
          r1 = c.p;
          break;
        default: bad = true; break;  // ContentJSON, ContentDoc, invalid refs
      }
      bad |= c.bad | (len == 0) | ((uint64_t)clock + len > 0xffffffffull);
      if (bad) break;
      uint32_t off = 0;
      bool wr = copying;
      if (!copying && clock + len > k) {  // the cut (us@40707): LazyStructWriter starts a part
        copying = true;
        wr = true;
        written = 0;
        off = k > clock ? k - clock : 0;
        ue_w(os[S_CL], e_cl, client);
        prest0 = os[S_RE].n;
        ovu(os[S_RE], clock + off);
      }
      if (wr) {  // Item.write(encoder, off) (k_big_v2 v2_write)
        written++;
        const uint32_t ref = info & 31;
        const bool noorig = (info & 0xC0) == 0;
        bad |= off > 0 && ref != 1 && ref != 4 && ref != 8;
        const bool has_o = off > 0 || (info & 0x80);
        re_w(os[S_IN], e_in, ref | (has_o ? 0x80 : 0) | (info & 0x40) | (noorig ? (info & 0x20) : 0));
        if (off > 0) { ue_w(os[S_CL], e_cl, client); ie_w(os[S_LC], e_lc, clock + off - 1, bad); }
        else if (info & 0x80) { ue_w(os[S_CL], e_cl, oc); ie_w(os[S_LC], e_lc, ok_, bad); }
        if (info & 0x40) { ue_w(os[S_CL], e_cl, rcl); ie_w(os[S_RC], e_rc, rk, bad); }
        if (!has_o && !(info & 0x40)) {
          re_w(os[S_PI], e_pi, pi);
          if (pi) wstr(ya, yn);
          else { ue_w(os[S_CL], e_cl, pc); ie_w(os[S_LC], e_lc, pk, bad); }
          if (info & 0x20) wstr(pa, pn);
        }
        switch (ref) {
          case 1: ue_w(os[S_LN], e_ln, len - off); break;
          case 3: case 5: ospan(os[S_RE], r0, r1 - r0); break;
          case 4: {  // str.slice(off): a cut inside a surrogate pair leaves a lone low surrogate, which the
                     // column's writeVarString rejects (URIError, toUint8Array: after everything is read)
            bool split = false;
            const uint32_t ob = sascii ? off : utf8_span(ca, ca + (cn & 0xffff), off, split);
            uri |= split;
            if (!split) wstr(ca + ob, ((cn & 0xffff) - ob) | (((cn >> 16) - off) << 16));
            break;
          }
          case 6: wkey(); wstr(ka, kn); ospan(os[S_RE], r0, r1 - r0); break;
          case 7:
            ue_w(os[S_TR], e_tr, t);
            if (t == 3 || t == 5) { wkey(); wstr(ka, kn); }
            break;
          case 8: {
            ue_w(os[S_LN], e_ln, len - off);
            Cur v = {r0, r1, false};  // ContentAny.splice: drop `off` values
            for (uint32_t i = 0; i < off; i++) any_canon<true>(v);
            bad |= v.bad;
            ospan(os[S_RE], v.p, r1 - v.p);
            break;
          }
        }
      }
      clock += len;
    }
    if (copying && !bad) {
      bad |= nparts >= L::NPART;
      if (!bad) at<uint4>(pt + 16 * nparts) = make_uint4(prest0, os[S_RE].n, written, 0);
      nparts++;
    }
  }
  bad |= c.bad | cl.c.bad | lc.c.bad | rc.c.bad | in.c.bad | sl.c.bad | pi_.c.bad | tr.c.bad | ln.c.bad | kc.c.bad;
  if (bad && !why) why = 6;
  // the delete set (rest stream): validated, then copied (readDeleteSet / writeDeleteSet round-trip it)
  const uint32_t ds0 = c.p;
  if (!bad) {
    const uint32_t ndc = rvu(c);
    bad |= ndc > L::NSV;
    for (uint32_t i = 0; i < ndc && !bad && !c.bad; i++) {
      const uint32_t client = rvu(c), m = rvu(c);
      bad |= m == 0;  // readDeleteSet drops a client without ranges: the bytes would change
      for (uint32_t q = 0; q < i; q++) bad |= at<uint32_t>(svt + 4 * q) == client;  // a repeated client merges
      at<uint32_t>(svt + 4 * i) = client;
      for (uint32_t q = 0; q < m && !c.bad; q++) { rvu(c); rvu(c); }
    }
    bad |= c.bad;
    if (bad && !why) why = 7;
  }
  const uint32_t ds1 = c.p;
  // lib0 toUint8Array: Uint / IntDiff runs flushed, the Rle<u8> final counts omitted
  ie_flush(os[S_KC], e_kc);
  ue_flush(os[S_CL], e_cl);
  ie_flush(os[S_LC], e_lc);
  ie_flush(os[S_RC], e_rc);
  ue_flush(os[S_SL], e_sl);
  ue_flush(os[S_TR], e_tr);
  ue_flush(os[S_LN], e_ln);
#pragma unroll
  for (uint32_t k = 0; k < NS; k++) bad |= os[k].n > os[k].cap;
  if (bad && !why) why = 8;
  // the output: vu(0) | 9 x (vu(n) column) | vu(#parts) parts | delete set
  uint32_t coln[9];
  coln[0] = os[S_KC].n; coln[1] = os[S_CL].n; coln[2] = os[S_LC].n; coln[3] = os[S_RC].n; coln[4] = os[S_IN].n;
  coln[5] = vsz(os[S_SB].n) + os[S_SB].n + os[S_SL].n; coln[6] = os[S_PI].n; coln[7] = os[S_TR].n; coln[8] = os[S_LN].n;
  uint32_t total = 0;
  if (!bad) {
    total = 1 + vsz(nparts) + (ds1 - ds0);
#pragma unroll
    for (uint32_t q = 0; q < 9; q++) total += vsz(coln[q]) + coln[q];
    for (uint32_t q = 0; q < nparts; q++) {
      const uint4 e = at<uint4>(pt + 16 * q);
      total += vsz(e.z) + e.y - e.x;
    }
  }
  // assemble the output in place: each piece moves down to the end of what precedes it (the 16 bytes
  // ahead of the streams and every stream's slack hold the varuint headers); the delete set comes from the
  // input window
  const uint32_t area = os[S_KC].a - 16;
  if (!bad) {
    bad |= total + 16 > os[S_RE].a + os[S_RE].cap - area;  // (cannot happen: the slack covers the headers)
  }
  if (!bad) {
    uint32_t p = area;
    auto put = [&](uint32_t v) { while (v > 127) { at<uint8_t>(p++) = (uint8_t)(0x80 | (v & 127)); v >>= 7; } at<uint8_t>(p++) = (uint8_t)v; };
    // a piece moves only downwards; a header that reached into a piece not yet moved declines the document
    // (k_big_v2 reads the input from HBM, so the half-assembled area is simply dropped)
    auto mv = [&](uint32_t src, uint32_t n) {
      bad |= p > src;
      if (!bad) lds_move_down(p, src, n);
      p += n;
    };
    put(0);
#pragma unroll
    for (uint32_t q = 0; q < 9; q++) {
      put(coln[q]);
      if (q == 5) {
        put(os[S_SB].n);
        mv(os[S_SB].a, os[S_SB].n);
        mv(os[S_SL].a, os[S_SL].n);
      } else {
        const uint32_t k = q == 0 ? S_KC : q == 1 ? S_CL : q == 2 ? S_LC : q == 3 ? S_RC : q == 4 ? S_IN : q == 6 ? S_PI : q == 7 ? S_TR : S_LN;
        mv(os[k].a, os[k].n);
      }
    }
    put(nparts);
    for (uint32_t q = 0; q < nparts; q++) {
      const uint4 e = at<uint4>(pt + 16 * q);
      put(e.z);
      mv(os[S_RE].a + e.x, e.y - e.x);
    }
    if (!bad) lds_copy(p, ds0, ds1 - ds0);
    if (bad && !why) why = 9;
  }
  // a valid document whose result is yjs's URIError (a string cut inside a surrogate pair): no output
  const bool uerr = !bad && uri;
  if (uerr) bad = true;
  // sizes: one bump allocation per wave; every output starts 16-byte aligned (the cooperative copy's stores)
  const uint32_t total16 = bad ? 0 : (total + 15) & ~15u;
  const uint32_t oincl = wave_incl_add(total16), otot = lane_read(oincl, 63);
  uint64_t base = 0;
  if (lane == 0 && otot) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)otot + 15);
  base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
  base = (base + 15) & ~15ull;
  const uint64_t off = base + oincl - total16;
  const bool fits = off + total16 <= j.cap;
  if (bad && lane < dn && why) done[d] = (uint8_t)why;
  if (uerr) {
    done[d] = 1;
    j.status[d] = ym::ST_URI;
    j.out_len[d] = 0;
    j.out_off[d] = 0;
  }
  if (!bad) {
    done[d] = 1;
    if (fits) {
      j.out_off[d] = off;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    } else {
      j.status[d] = ym::ST_CAPACITY;
      j.out_len[d] = 0;
    }
  }
  // the wave copies each completed output out of LDS with 16-byte accesses
  for (uint32_t q = 0; q < dn; q++) {
    const uint32_t n = lane_read(bad || !fits ? 0 : total16, q);
    if (n == 0) continue;
    const uint32_t src = lane_read(area, q);
    const uint64_t dst = ((uint64_t)lane_read((uint32_t)(off >> 32), q) << 32) | lane_read((uint32_t)off, q);
    for (uint32_t k = lane; k < n / 16; k += 64)
      *reinterpret_cast<uint4 *>(j.out + dst + 16 * k) = at<uint4>(src + 16 * k);
  }
}

}  // namespace fastv2

// parseUpdateMetaV2 / encodeStateVectorFromUpdateV2 over small single updates, one per lane (k_small_v2);
// done: the streamed walker's done array (nullptr: the kernel is the call's only specialised pass, its
// declines go to the general path).  Meta: 64 updates of an update log per wave (4 KB window); state
// vectors: 4 merged documents per wave (~1 KB each: an 8 KB window, 32 sections each).
// pv_min: the column path's smallest update in this call (its documents are not taken here); ~0: no column path
int small_v2_launch(uint32_t op, const GeneralJob &j, uint8_t *done, hipStream_t st, uint32_t diff_min, uint64_t pv_min) {
  static const bool off = getenv("YMERGE_NO_SMALL_V2") != nullptr;
  if (off || !j.v2 || j.n == 0) return 0;
  using namespace fastv2;
  if (op == OP_META) {
    k_small_v2<OP_META, 64, 4096, 8><<<(j.n + 63) / 64, 64, Sv2Lay<64, 4096, 8>::BYTES, st>>>(j, done, pv_min);
  } else if (op == OP_SV) {
    // 4 documents per wave with an 8 KB window: one generation of short waves (C2, 10 k documents: 0.41 ms at
    // 16 per wave, 0.42 at 8, 0.31 at 4 and 0.32 at 2)
    k_small_v2<OP_SV, 4, 8192, 32><<<(j.n + 3) / 4, 64, Sv2Lay<4, 8192, 32>::BYTES, st>>>(j, done, pv_min);
  } else if (op == OP_DIFF && done && j.sv) {
    // documents per wave so that the batch is one generation of waves (2 per SIMD: 2,048 on the chip; a
    // second generation doubles the call: C2, 10 k documents, 4 per wave 0.93 ms against 5 per wave 0.56),
    // each wave with a 7.5 KB window and 7.5 KB of output streams (its documents share both)
    // Batches that fit one generation of k_big_v2's one-document waves (<= 4,096 documents here) stay on it:
    // per document the lane walk is faster only for narrow documents (C2R 4 k: 0.87 against 1.25 ms), and
    // slower for wide rich ones (C4R 4 k, 64 clients with object values: 2.7 against 1.9 ms), which a batch
    // does not announce (YMERGE_DF2_MIN lowers the threshold: tests)
    if (getenv("YMERGE_NO_DF2")) return 0;
    if (const char *e = getenv("YMERGE_DF2_MIN")) diff_min = (uint32_t)strtoul(e, nullptr, 10);
    if (j.n <= diff_min) return 0;
    const uint32_t nd = j.n <= 2048 ? 1 : j.n <= 4096 ? 2 : j.n <= 6144 ? 3 : j.n <= 8192 ? 4 : 5;
#define DF2(N) \
  if (nd == N) k_diff_small_v2<N, 7680, 7680, 1><<<(j.n + N - 1) / N, 64, Df2Lay<N, 7680, 7680>::BYTES, st>>>(j, done, pv_min, 0);
    DF2(1) DF2(2) DF2(3) DF2(4) DF2(5)
#undef DF2
    // documents larger than their share of a shared window or output pool (done 2 / 5: e.g. merged C2U documents,
    // five to a 7.5 KB window) once more one per wave before k_big_v2, whose walker takes ASCII string columns only
    if (nd > 1) k_diff_small_v2<1, 7680, 7680, 1><<<j.n, 64, Df2Lay<1, 7680, 7680>::BYTES, st>>>(j, done, pv_min, 1);
  } else {
    return 0;
  }
  return 1;
}

int fast2_launch(uint32_t op, const GeneralJob &j, uint32_t n_upd, hipStream_t st) {
  if (op != OP_MERGE || !j.v2) return 0;
  (void)n_upd;
  const uint32_t grid = j.n < 131072 ? j.n : 131072;
  static int stop = -1, occ = -1;
  if (stop < 0) { const char *e = getenv("YMERGE_FAST_STOP"); stop = e ? atoi(e) : 0; }
  if (occ < 0) { const char *e = getenv("YMERGE_FAST2_OCC"); occ = e ? atoi(e) : 3; }  // min waves / SIMD (3: 168 VGPRs, no spills)
  if (stop == 0 && occ >= 2) {
    if (occ == 2) fastv2::k_fast_merge_v2<0, 2><<<grid, 64, fastv2::LDS_BYTES, st>>>(j, j.n);
    else if (occ == 3) fastv2::k_fast_merge_v2<0, 3><<<grid, 64, fastv2::LDS_BYTES, st>>>(j, j.n);
    else fastv2::k_fast_merge_v2<0, 4><<<grid, 64, fastv2::LDS_BYTES, st>>>(j, j.n);
    return 1;
  }
  switch (stop) {
#define YM2_L(S) case S: fastv2::k_fast_merge_v2<S><<<grid, 64, fastv2::LDS_BYTES, st>>>(j, j.n); break;
    YM2_L(1) YM2_L(2) YM2_L(3) YM2_L(4) YM2_L(5) YM2_L(6) YM2_L(7)
    default: fastv2::k_fast_merge_v2<0><<<grid, 64, fastv2::LDS_BYTES, st>>>(j, j.n); break;
#undef YM2_L
  }
  return 1;
}

// The V2 retry pass with nested payload checks (see fast_nested_launch, ym_fast.hip).
int fast2_nested_launch(const GeneralJob &j, uint32_t n, hipStream_t st) {
  if (j.op != OP_MERGE || !j.v2 || n == 0) return 0;
  static int off = -1;
  if (off < 0) { const char *e = getenv("YMERGE_FAST_NESTED"); off = e && atoi(e) == 0 ? 1 : 0; }
  if (off) return 0;
  fastv2::k_fast_merge_v2<0, 3, true><<<n < 131072 ? n : 131072, 64, fastv2::LDS_BYTES, st>>>(j, n);
  return 1;
}

}  // namespace ymk
