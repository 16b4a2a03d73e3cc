// ym_big2.hip -- V2 diffUpdateV2 / encodeStateVectorFromUpdateV2 over single updates of any size.
//
// The V1 walker of ym_big.hip, generalised to the V2 layout (UpdateDecoder.js:245-392,
// UpdateEncoder.js:229-408): ten input streams -- the rest stream and the keyClock / client /
// leftClock / rightClock / info / string-length / parentInfo / typeRef / len columns -- each read
// through its own LDS window, with the lib0 RLE decoders (RleDecoder, UintOptRleDecoder,
// IntDiffOptRleDecoder) run by the whole wave in lockstep.  The string column's UTF-8 body is
// validated up front by all lanes (StringDecoder decodes the whole column in its constructor) and is
// never walked: this path takes ASCII string columns, where a UTF-16 slice is a byte slice.
//
// diffUpdateV2 (13.5.16 us@40707) re-encodes every column of the written structs with the lib0
// encoders (UintOptRleEncoder, IntDiffOptRleEncoder, RleEncoder, StringEncoder) into per-stream
// scratch in the output arena, then assembles vu(0) | 9 x varUint8Array(column) | rest, where rest =
// vu(#parts) | parts (vu(written) | first clock | payloads) | delete set (copied: the V2 delete set
// round-trips byte for byte when canonical).  Everything else follows ym_big.hip.
#include <hip/hip_runtime.h>

#include "ym_fast_common.h"
#include "ym_kernels.h"
#include "ym_cmap.h"
#include "ym_pv2.h"

namespace ymk {
namespace big2 {
using namespace fastc;

// input streams
enum { I_REST = 0, I_KC, I_CL, I_LC, I_RC, I_IN, I_SL, I_PI, I_TR, I_LN, NIN };
// output streams (scratch): the nine columns (string split in body + lengths) and the part bytes
enum { O_KC = 0, O_CL, O_LC, O_RC, O_IN, O_SB, O_SL, O_PI, O_TR, O_LN, O_REST, NOUT };
constexpr uint32_t WREST = 4096, MREST = 1024;  // rest window / margin (any payloads live here)
constexpr uint32_t WCOL = 256, MCOL = 24;       // column windows / margin (one varint or byte)
constexpr uint32_t NSEC = BS_NSEC, NSV = BS_NSV;  // parts / state-vector entries (per-block HBM scratch)

constexpr uint32_t L_WREST = 0;
constexpr uint32_t L_WCOL = WREST + 16;                      // (NIN-1) x (WCOL + 16)
constexpr uint32_t LDS_BYTES = L_WCOL + (NIN - 1) * (WCOL + 16);

// The walk is wave-uniform: every lane computes the same stream cursors, decoder and encoder states,
// so they live in registers (Doc::st_*), identical in all 64 lanes -- no LDS round trip and no barrier
// per field.  Only the stream windows (LDS) and the output bytes (stored by lane 0) are shared.
enum { M_BAD = 0, M_KEYS, M_KCLOCK, M_SPOS };
#define ist(s, f) D.st_in[s][f]    // input streams: pos, end, wdelta, wlim
#define dec(s, f) D.st_dec[s][f]   // RLE decoders: s, count, diff
#define ost(s, f) D.st_out[s][f]   // output streams (scratch): base, cur, cap
#define enc(s, f) D.st_enc[s][f]   // RLE encoders: s, count, diff, started
#define misc(f) D.st_misc[f]
#define set_bad() (D.st_misc[M_BAD] = 1)
#define is_bad() (D.st_misc[M_BAD] != 0)

// per-block HBM scratch (ym_kernels.h BS_*): parts (rest start, rest end, written), state vector,
// delete-set clients
struct Scr {
  uint32_t *part, *svt, *dsc, *map;
};
__device__ __forceinline__ Scr scratch(const GeneralJob &j) {
  uint8_t *b = j.bscratch + (uint64_t)blockIdx.x * BS_BYTES;
  return Scr{(uint32_t *)(b + BS_SEC), (uint32_t *)(b + BS_SVT), (uint32_t *)(b + BS_DSC), (uint32_t *)(b + BS_MAP)};
}
__device__ __forceinline__ uint32_t sv_lookup(const uint32_t *svt, uint32_t nsv, uint32_t client) {
  int best = -1;  // decodeStateVector: a later entry for the same client wins
  for (uint32_t i0 = 0; i0 < nsv; i0 += 64) {
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t m = __ballot(i < nsv && svt[2 * i] == client);
    if (m) best = (int)(i0 + 63 - __builtin_clzll(m));
  }
  return best >= 0 ? svt[2 * best + 1] : 0;
}

struct Doc {
  const uint8_t *A;  // arena
  uint64_t b0;       // update start (absolute)
  uint32_t len;      // update bytes
  uint8_t *O;        // output arena
  uint32_t st_in[NIN][4], st_dec[NIN][4], st_out[NOUT][4], st_enc[NOUT][4], st_misc[4];
};

__device__ __forceinline__ uint32_t win_lds(uint32_t s) { return s == I_REST ? L_WREST : L_WCOL + (s - 1) * (WCOL + 16); }
// (re)loads stream s's window at its cursor; every lane takes part (the walk is wave-uniform)
__device__ __forceinline__ void s_load(Doc &D, uint32_t s) {
  const uint32_t W = s == I_REST ? WREST : WCOL;
  const uint32_t pos = ist(s, 0), end = ist(s, 1);
  __syncthreads();
  const uint64_t wa = (D.b0 + pos) & ~15ull;
  const uint64_t eabs = D.b0 + end;
  // (a cursor that overran its stream end after a malformed varuint loads nothing)
  const uint32_t n = (uint32_t)(wa >= eabs ? 0 : wa + W < eabs ? W : eabs - wa);
  const uint4 *src = reinterpret_cast<const uint4 *>(D.A + wa);
  const uint32_t base = win_lds(s);
  for (uint32_t v = threadIdx.x; v < (n + 15) >> 4; v += 64) at<uint4>(base + 16 * v) = src[v];
  __syncthreads();
  ist(s, 2) = (uint32_t)(base - (wa - D.b0));  // LDS address = pos + wdelta
  ist(s, 3) = (uint32_t)(wa - D.b0) + n;       // loaded through (update-relative)
}
// cursor of stream s as an LDS Cur with at least `need` bytes loaded (or the stream's end)
__device__ __forceinline__ Cur s_cur(Doc &D, uint32_t s, uint32_t need) {
  uint32_t pos = ist(s, 0), end = ist(s, 1), lim = ist(s, 3);
  if (pos + need > lim && lim < end) {
    s_load(D, s);
    lim = ist(s, 3);
  }
  const uint32_t wd = ist(s, 2);
  Cur c = {pos + wd, (end < lim ? end : lim) + wd, false};
  return c;
}
__device__ __forceinline__ void s_commit(Doc &D, uint32_t s, const Cur &c) {
  ist(s, 0) = c.p - ist(s, 2);
  if (c.bad) set_bad();
}
__device__ __forceinline__ uint32_t s_vu(Doc &D, uint32_t s) {
  Cur c = s_cur(D, s, MCOL);
  const uint32_t v = rvu(c);
  s_commit(D, s, c);
  return v;
}
__device__ __forceinline__ uint32_t s_u8(Doc &D, uint32_t s) {
  Cur c = s_cur(D, s, MCOL);
  const uint32_t v = rdb(c);
  s_commit(D, s, c);
  return v;
}
// lib0 readVarInt (canonical, <= 5 bytes): sign flag incl. -0, u32 magnitude
__device__ __forceinline__ uint32_t s_vi(Doc &D, uint32_t s, bool &neg) {
  Cur c = s_cur(D, s, MCOL);
  const uint64_t x = ld8(c.p);
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const uint32_t nb = vu_nb(lo, hi);
  neg = (lo & 0x40) != 0;
  uint32_t m = (lo & 0x3fu) | ((lo >> 2) & 0x1fc0u) | ((lo >> 3) & 0xfe000u) | ((lo >> 4) & 0x7f00000u) | ((hi & 0x7fu) << 27);
  const uint32_t bits = 6 + 7 * (nb - 1);
  if (nb < 5) m &= (1u << bits) - 1u;
  const uint32_t last = nb <= 4 ? (lo >> (8 * nb - 8)) & 0xffu : hi & 0xffu;
  c.bad |= (nb > 5) | (c.p + nb > c.e) | ((nb > 1) & (last == 0)) | ((nb == 5) & ((hi & 0x7fu) > 0x1fu));
  c.p += nb < 6 ? nb : 0;
  s_commit(D, s, c);
  return m;
}
__device__ __forceinline__ bool s_has(Doc &D, uint32_t s) { return ist(s, 0) < ist(s, 1); }

// lib0 decoders (state in L_DEC): RleDecoder<u8>, UintOptRleDecoder, IntDiffOptRleDecoder
__device__ __forceinline__ uint32_t rle_read(Doc &D, uint32_t s) {
  uint32_t v = dec(s, 0), n = dec(s, 1);
  if (n == 0) {
    v = s_u8(D, s);
    n = s_has(D, s) ? s_vu(D, s) + 1 : 0xffffffffu;  // the final run never ends
  }
  dec(s, 0) = v; dec(s, 1) = n == 0xffffffffu ? n : n - 1;
  return v;
}
__device__ __forceinline__ uint32_t uopt_read(Doc &D, uint32_t s) {
  uint32_t v = dec(s, 0), n = dec(s, 1);
  if (n == 0) {
    bool neg;
    v = s_vi(D, s, neg);
    n = neg ? s_vu(D, s) + 2 : 1;
  }
  dec(s, 0) = v; dec(s, 1) = n - 1;
  return v;
}
// IntDiffOptRleDecoder: diff = ToInt32(sign * mag) >> 1, count from its low bit; values must stay in
// [0, 2^32) for this path (clocks)
__device__ __forceinline__ uint32_t idiff_read(Doc &D, uint32_t s) {
  int64_t v = (int64_t)dec(s, 0);
  uint32_t n = dec(s, 1);
  int32_t df = (int32_t)dec(s, 2);
  if (n == 0) {
    bool neg;
    const uint32_t m = s_vi(D, s, neg);
    const int32_t t = neg ? -(int32_t)m : (int32_t)m;
    df = t >> 1;
    n = (t & 1) ? s_vu(D, s) + 2 : 1;
  }
  v += df;
  if (v < 0 || v > 0xffffffffll) set_bad();
  dec(s, 0) = (uint32_t)v; dec(s, 1) = n - 1; dec(s, 2) = (uint32_t)df;
  return (uint32_t)v;
}

// ---- output streams (scratch in the output arena) -----------------------------------------------
__device__ __forceinline__ void o_byte(Doc &D, uint32_t s, uint32_t v) {
  const uint32_t cur = ost(s, 1);
  if (cur >= ost(s, 2)) { set_bad(); return; }
  if (threadIdx.x == 0) D.O[(uint64_t)ost(s, 0) + cur] = (uint8_t)v;
  ost(s, 1) = cur + 1;
}
__device__ __forceinline__ void o_vu(Doc &D, uint32_t s, uint32_t v) {
  while (v > 127) { o_byte(D, s, 0x80 | (v & 127)); v >>= 7; }
  o_byte(D, s, v);
}
__device__ __forceinline__ void o_vi(Doc &D, uint32_t s, bool neg, uint32_t m) {  // lib0 writeVarInt
  o_byte(D, s, (m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63));
  m >>= 6;
  while (m > 0) { o_byte(D, s, (m > 127 ? 0x80 : 0) | (m & 127)); m >>= 7; }
}
// copies update bytes [a, b) to the end of output stream s (all lanes)
__device__ __forceinline__ void o_span(Doc &D, uint32_t s, uint32_t a, uint32_t b) {
  const uint32_t cur = ost(s, 1);
  if (b < a || (uint64_t)cur + (b - a) > ost(s, 2)) { set_bad(); return; }
  uint8_t *dst = D.O + ost(s, 0) + cur;
  const uint8_t *src = D.A + D.b0 + a;
  for (uint32_t i = threadIdx.x; i < b - a; i += 64) dst[i] = src[i];
  ost(s, 1) = cur + (b - a);
}
// lib0 encoders (state in L_ENC: s, count, diff, started)
__device__ __forceinline__ void uopt_flush(Doc &D, uint32_t s) {
  const uint32_t v = enc(s, 0), n = enc(s, 1);
  if (n > 0) {
    o_vi(D, s, n != 1, v);  // count==1 ? v : -v  (-0 for v==0)
    if (n > 1) o_vu(D, s, n - 2);
  }
}
__device__ __forceinline__ void uopt_w(Doc &D, uint32_t s, uint32_t v) {
  if (enc(s, 0) == v) {
    enc(s, 1) += 1;
    return;
  }
  uopt_flush(D, s);
  enc(s, 0) = v; enc(s, 1) = 1;
}
__device__ __forceinline__ void idiff_flush(Doc &D, uint32_t s) {
  const int32_t df = (int32_t)enc(s, 2);
  const uint32_t n = enc(s, 1);
  if (n > 0) {
    const int32_t x = (int32_t)((uint32_t)df << 1) | (n == 1 ? 0 : 1);
    o_vi(D, s, x < 0, x < 0 ? (uint32_t)(-(int64_t)x) : (uint32_t)x);
    if (n > 1) o_vu(D, s, n - 2);
  }
}
__device__ __forceinline__ void idiff_w(Doc &D, uint32_t s, uint32_t v) {
  const int64_t d = (int64_t)v - (int64_t)enc(s, 0);
  if (d < -(1ll << 30) || d >= (1ll << 30)) { set_bad(); return; }  // JS `diff << 1` wraps beyond
  if ((int32_t)enc(s, 2) == (int32_t)d) {
    enc(s, 0) = v; enc(s, 1) += 1;
    return;
  }
  idiff_flush(D, s);
  enc(s, 0) = v; enc(s, 1) = 1; enc(s, 2) = (uint32_t)(int32_t)d;
}
__device__ __forceinline__ void rle_w(Doc &D, uint32_t s, uint32_t v) {
  if (enc(s, 3) && enc(s, 0) == v) {
    enc(s, 1) += 1;
    return;
  }
  if (enc(s, 1) > 0) o_vu(D, s, enc(s, 1) - 1);
  o_byte(D, s, v);
  enc(s, 0) = v; enc(s, 1) = 1; enc(s, 3) = 1;
}
__device__ __forceinline__ void str_w(Doc &D, uint32_t sb0, uint32_t a, uint32_t n) {  // ASCII string
  o_span(D, O_SB, sb0 + a, sb0 + a + n);
  uopt_w(D, O_SL, n);
}

// one V2 struct, decoded (13.5.16 LazyStructReader over UpdateDecoderV2); the record keeps what
// Item.write / GC.write / Skip.write need to re-encode it (string slices are ASCII byte ranges of the
// string body, payloads are rest-stream spans)
struct Rec {
  uint32_t info, len, oc, ok, rc, rk, pi, ya, yn, pa, pn, pc, pk, ca, cn, ka, kn, t, r0, r1;
};
__device__ __forceinline__ void rstr(Doc &D, uint32_t sn, uint32_t &a, uint32_t &n) {
  const uint32_t pos = misc(M_SPOS);  // StringDecoder.read: the next slice (bytes == UTF-16 units)
  n = uopt_read(D, I_SL);
  a = pos;
  if ((uint64_t)pos + n > sn) set_bad();  // a slice past the end would shorten the string
  misc(M_SPOS) = pos + n;
}
__device__ __forceinline__ bool v2_read(Doc &D, uint32_t info, uint32_t sn, Rec &r) {
  r = Rec{};
  r.info = info;
  if (info == 10) { r.len = s_vu(D, I_REST); return !is_bad(); }           // Skip: len in rest
  if ((info & 31) == 0) { r.len = uopt_read(D, I_LN); return !is_bad(); }  // GC: len column
  if (info & 0x80) { r.oc = uopt_read(D, I_CL); r.ok = idiff_read(D, I_LC); }
  if (info & 0x40) { r.rc = uopt_read(D, I_CL); r.rk = idiff_read(D, I_RC); }
  if ((info & 0xC0) == 0) {
    r.pi = rle_read(D, I_PI);
    if (r.pi == 1) rstr(D, sn, r.ya, r.yn);
    else { r.pc = uopt_read(D, I_CL); r.pk = idiff_read(D, I_LC); }
    if (info & 0x20) rstr(D, sn, r.pa, r.pn);
  }
  r.len = 1;
  switch (info & 31) {
    case 1: r.len = uopt_read(D, I_LN); break;                          // ContentDeleted
    case 3: {                                                           // ContentBinary: rest varUint8Array
      Cur c = s_cur(D, I_REST, MREST);
      r.r0 = c.p - ist(I_REST, 2);
      const uint32_t n = rvu(c);
      if (!room(c, n)) c.bad = true; else c.p += n;
      s_commit(D, I_REST, c);
      r.r1 = ist(I_REST, 0);
      break;
    }
    case 4: rstr(D, sn, r.ca, r.cn); r.len = r.cn; break;                // ContentString
    case 5: case 6: {                                                   // Embed / Format: rest any
      if ((info & 31) == 6) rstr(D, sn, r.ka, r.kn);
      Cur c = s_cur(D, I_REST, MREST);
      r.r0 = c.p - ist(I_REST, 2);
      any_canon<true>(c);
      s_commit(D, I_REST, c);
      r.r1 = ist(I_REST, 0);
      break;
    }
    case 7:                                                             // ContentType
      r.t = uopt_read(D, I_TR);
      if (r.t > 6) { set_bad(); return false; }
      if (r.t == 3 || r.t == 5) {  // readKey: a cached key (keyClock < keys read) consumes no string
        const uint32_t kcv = idiff_read(D, I_KC);
        if (kcv < misc(M_KEYS)) { set_bad(); return false; }
        misc(M_KEYS) += 1;
        rstr(D, sn, r.ka, r.kn);
      }
      break;
    case 8: {                                                           // ContentAny: len col + rest
      r.len = uopt_read(D, I_LN);
      Cur c = s_cur(D, I_REST, MREST);
      r.r0 = c.p - ist(I_REST, 2);
      for (uint32_t i = 0; i < r.len && !c.bad; i++) any_canon<true>(c);
      s_commit(D, I_REST, c);
      r.r1 = ist(I_REST, 0);
      break;
    }
    default: set_bad(); return false;  // ContentJSON, ContentDoc, invalid refs
  }
  if (r.len == 0) set_bad();
  return !is_bad();
}
__device__ __forceinline__ void next_key(Doc &D) {  // writeKey: keyClock++ (never cached, E9)
  const uint32_t kc = misc(M_KCLOCK);
  idiff_w(D, O_KC, kc);
  misc(M_KCLOCK) = kc + 1;
}
// Item.write / GC.write / Skip.write (encoder, off) into the output streams, V2 routing
__device__ __forceinline__ void v2_write(Doc &D, const Rec &r, uint32_t off, uint32_t client, uint32_t clock, uint32_t sb0) {
  const uint32_t info = r.info;
  if (info == 10) { rle_w(D, O_IN, 10); o_vu(D, O_REST, r.len - off); return; }
  if ((info & 31) == 0) { rle_w(D, O_IN, 0); uopt_w(D, O_LN, r.len - off); return; }
  const uint32_t ref = info & 31;
  const bool noorig = (info & 0xC0) == 0;
  if (off > 0 && ref != 1 && ref != 4 && ref != 8) { set_bad(); return; }
  const bool has_o = off > 0 || (info & 0x80);
  // parentSub is read (and its bit kept) only without origins (E9)
  const uint32_t ni = (ref | (has_o ? 0x80 : 0) | (info & 0x40) | (noorig ? (info & 0x20) : 0));
  rle_w(D, O_IN, ni);
  if (off > 0) { uopt_w(D, O_CL, client); idiff_w(D, O_LC, clock + off - 1); }
  else if (info & 0x80) { uopt_w(D, O_CL, r.oc); idiff_w(D, O_LC, r.ok); }
  if (info & 0x40) { uopt_w(D, O_CL, r.rc); idiff_w(D, O_RC, r.rk); }
  if (!has_o && !(info & 0x40)) {
    rle_w(D, O_PI, r.pi == 1 ? 1 : 0);
    if (r.pi == 1) str_w(D, sb0, r.ya, r.yn);
    else { uopt_w(D, O_CL, r.pc); idiff_w(D, O_LC, r.pk); }
    if (info & 0x20) str_w(D, sb0, r.pa, r.pn);
  }
  switch (ref) {
    case 1: uopt_w(D, O_LN, r.len - off); break;
    case 3: case 5: o_span(D, O_REST, r.r0, r.r1); break;
    case 4: str_w(D, sb0, r.ca + off, r.cn - off); break;
    case 6: next_key(D); str_w(D, sb0, r.ka, r.kn); o_span(D, O_REST, r.r0, r.r1); break;
    case 7:
      uopt_w(D, O_TR, r.t);
      if (r.t == 3 || r.t == 5) { next_key(D); str_w(D, sb0, r.ka, r.kn); }
      break;
    case 8: {
      uopt_w(D, O_LN, r.len - off);
      uint32_t a = r.r0;
      if (off > 0) {  // ContentAny.splice: drop `off` values (still in the rest window: nothing was read since)
        const uint32_t wd = ist(I_REST, 2);
        if (r.r0 + wd < L_WREST || r.r1 + wd > L_WREST + WREST) { set_bad(); return; }
        Cur c = {r.r0 + wd, r.r1 + wd, false};
        for (uint32_t i = 0; i < off; i++) any_canon<true>(c);
        if (c.bad) { set_bad(); return; }
        a = c.p - wd;
      }
      o_span(D, O_REST, a, r.r1);
      break;
    }
  }
}

#define YB2_DECLINE()                                       \
  {                                                         \
    if (threadIdx.x == 0) {                                 \
      j.status[d] = ST_PENDING;                             \
      const uint32_t q_ = atomicAdd(j.pend_count, 1u);      \
      if (j.pend_list) j.pend_list[q_] = d;                 \
    }                                                       \
    __syncthreads();                                        \
    continue;                                               \
  }

template <int OP>
__global__ void __launch_bounds__(64) k_big_v2(GeneralJob j) {
  const uint32_t lane = threadIdx.x;
  const Scr X = scratch(j);
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    if (j.pw_done && j.pw_done[d] == 1) continue;  // completed by the column-parallel path
    const uint32_t u0 = j.doc_upd[d];
    if (j.doc_upd[d + 1] - u0 != 1) YB2_DECLINE()
    Doc D;
    D.A = j.A;
    D.O = j.out;
    D.b0 = j.upd_off[u0];
    const uint64_t len64 = j.upd_off[u0 + 1] - D.b0;
    if (len64 == 0 || len64 > 0xfffffff0ull) YB2_DECLINE()
    D.len = (uint32_t)len64;
#pragma unroll
    for (uint32_t a = 0; a < NIN; a++)
#pragma unroll
      for (uint32_t b = 0; b < 4; b++) { D.st_in[a][b] = 0; D.st_dec[a][b] = 0; }
#pragma unroll
    for (uint32_t a = 0; a < NOUT; a++)
#pragma unroll
      for (uint32_t b = 0; b < 4; b++) { D.st_out[a][b] = 0; D.st_enc[a][b] = 0; }
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) D.st_misc[b] = 0;
    // ---- state vector (diff)
    uint32_t nsv = 0;
    if (OP == OP_DIFF) {
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      if (s1 - s0 > WREST - 32) YB2_DECLINE()
      const uint64_t a = s0 & ~15ull;
      const uint4 *src = reinterpret_cast<const uint4 *>(j.sv + a);
      for (uint32_t v = lane; v < (uint32_t)((s1 - a + 15) >> 4); v += 64) at<uint4>(L_WREST + 16 * v) = src[v];
      __syncthreads();
      Cur c = {(uint32_t)(s0 - a), (uint32_t)(s1 - a), false};
      const uint32_t n = rvu(c);
      for (uint32_t i = 0; i < n && !c.bad; i++) {
        const uint32_t cl = rvu(c), ck = rvu(c);
        if (nsv >= NSV) { c.bad = true; break; }
        if (lane == 0) { X.svt[2 * nsv] = cl; X.svt[2 * nsv + 1] = ck; }
        nsv++;
      }
      __threadfence_block();
      __syncthreads();
      if (c.bad) YB2_DECLINE()
      if (nsv > 64) cmap::build_sv(X.map, X.svt, nsv);
    }
    // ---- header: feature flag, nine columns (UpdateDecoderV2 constructor, UpdateDecoder.js:274-293)
    ist(I_REST, 0) = 0;
    ist(I_REST, 1) = D.len;
    s_load(D, I_REST);
    uint32_t sb0 = 0, sn = 0;
    {
      s_vu(D, I_REST);  // feature flag (unused)
      const uint32_t map[9] = {I_KC, I_CL, I_LC, I_RC, I_IN, I_SL, I_PI, I_TR, I_LN};
#pragma unroll
      for (uint32_t k = 0; k < 9; k++) {  // readVarUint8Array x 9: column spans
        const uint32_t n = s_vu(D, I_REST);
        const uint32_t c0 = ist(I_REST, 0);
        if ((uint64_t)c0 + n > D.len) set_bad();
        ist(map[k], 0) = c0;
        ist(map[k], 1) = c0 + n;
        ist(I_REST, 0) = c0 + n;
      }
      if (is_bad()) YB2_DECLINE()
      // the string column = varString(body) | UintOptRle(lengths)
      s_load(D, I_SL);
      sn = s_vu(D, I_SL);
      sb0 = ist(I_SL, 0);
      if ((uint64_t)sb0 + sn > ist(I_SL, 1)) set_bad();
      ist(I_SL, 0) = sb0 + sn;
#pragma unroll
      for (uint32_t k = 0; k < 9; k++) s_load(D, map[k]);
    }
    if (is_bad()) YB2_DECLINE()
    // the string body must be ASCII (then a UTF-16 slice is a byte slice and the body is valid UTF-8)
    {
      bool nonascii = false;
      const uint8_t *p = D.A + D.b0 + sb0;
      for (uint32_t i = lane; i < sn; i += 64) nonascii |= p[i] >= 0x80;
      if (__any(nonascii)) YB2_DECLINE()
    }
    // ---- output scratch (diff): one region per stream, sized by its input stream plus slack
    const uint32_t nclients = s_vu(D, I_REST);
    if (is_bad() || nclients > NSEC) YB2_DECLINE()
    uint64_t scratch = 0;
    if (OP == OP_DIFF) {
      const uint32_t slack = 64 + 32 * nclients;
      const uint32_t in_sz[NOUT] = {ist(I_KC, 1) - ist(I_KC, 0), ist(I_CL, 1) - ist(I_CL, 0), ist(I_LC, 1) - ist(I_LC, 0),
                                    ist(I_RC, 1) - ist(I_RC, 0), ist(I_IN, 1) - ist(I_IN, 0), sn,
                                    ist(I_SL, 1) - ist(I_SL, 0), ist(I_PI, 1) - ist(I_PI, 0), ist(I_TR, 1) - ist(I_TR, 0),
                                    ist(I_LN, 1) - ist(I_LN, 0), D.len};
      uint32_t tot = 0;
#pragma unroll
      for (uint32_t k = 0; k < NOUT; k++) tot += in_sz[k] + slack;
      if (lane == 0) scratch = atomicAdd((unsigned long long *)j.used, (unsigned long long)tot);
      scratch = ((uint64_t)lane_read((uint32_t)(scratch >> 32), 0) << 32) | lane_read((uint32_t)scratch, 0);
      if (scratch + tot > j.cap) {
        if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
        __syncthreads();
        continue;
      }
      {
        uint32_t o = 0;
#pragma unroll
        for (uint32_t k = 0; k < NOUT; k++) { ost(k, 0) = o; ost(k, 1) = 0; ost(k, 2) = in_sz[k] + slack; o += in_sz[k] + slack; }
      }
      D.O = j.out + scratch;
    }
    // ---- the walk (13.5.16 LazyStructReader over V2; diff = us@40707, sv = os@37724)
    uint32_t nparts = 0;
    uint32_t sv_client = 0, sv_clock = 0, sv_n = 0;
    bool sv_stop = false, sv_any = false;
    uint32_t prev_client = 0;
    for (uint32_t ci = 0; ci < nclients && !is_bad(); ci++) {
      const uint32_t nstructs = s_vu(D, I_REST);
      const uint32_t client = uopt_read(D, I_CL);
      uint64_t clock = s_vu(D, I_REST);
      if (ci > 0 && client == prev_client) { set_bad(); break; }
      // meta (parseUpdateMeta): clients strictly descending (as yjs writes them), so none repeats
      if (OP == OP_META && ci > 0 && client > prev_client) { set_bad(); break; }
      prev_client = client;
      const uint32_t first_clock = (uint32_t)clock;
      const uint32_t k = OP != OP_DIFF ? 0 : nsv > 64 ? cmap::sv_get(X.map, X.svt, client) : sv_lookup(X.svt, nsv, client);
      if (OP == OP_SV && nstructs > 0 && sv_any && client != sv_client) {
        if (sv_clock != 0) {
          if (sv_n >= NSV) { set_bad(); break; }
          if (lane == 0) { X.svt[2 * sv_n] = sv_client; X.svt[2 * sv_n + 1] = sv_clock; }
          sv_n++;
        }
        sv_client = client; sv_clock = 0; sv_stop = clock != 0;
      }
      bool copying = false;
      uint32_t written = 0, prest0 = 0;
      for (uint32_t si = 0; si < nstructs && !is_bad(); si++) {
        const uint32_t info = rle_read(D, I_IN);
        Rec r;
        if (!v2_read(D, info, sn, r)) break;
        const uint32_t len = r.len;
        if ((uint64_t)clock + len > 0xffffffffull) { set_bad(); break; }
        if (OP == OP_SV) {
          if (!sv_any) { sv_any = true; sv_client = client; sv_stop = clock != 0; sv_clock = sv_stop ? 0 : (uint32_t)(clock + len); }
          if (info == 10) sv_stop = true;
          if (!sv_stop) sv_clock = (uint32_t)(clock + len);
        } else if (OP == OP_META) {
          // parseUpdateMeta only measures the section: nothing is cut or written
        } else if (copying) {
          written++;
          v2_write(D, r, 0, client, (uint32_t)clock, sb0);
        } else if (info != 10 && clock + len > k) {  // the cut (us@40707)
          copying = true;
          written = 1;
          const uint32_t off = k > clock ? (uint32_t)(k - clock) : 0;
          uopt_w(D, O_CL, client);  // LazyStructWriter: writeClient + first clock at a part's start
          prest0 = ost(O_REST, 1);
          o_vu(D, O_REST, (uint32_t)(clock + off));
          v2_write(D, r, off, client, (uint32_t)clock, sb0);
        }
        clock += len;
      }
      if (OP == OP_META && nstructs > 0 && !is_bad()) {  // from = first clock, to = end of the last struct
        if (sv_n >= NSV) { set_bad(); break; }
        if (lane == 0) { X.svt[2 * sv_n] = client; X.svt[2 * sv_n + 1] = first_clock; X.part[sv_n] = (uint32_t)clock; }
        sv_n++;
      }
      if (OP == OP_DIFF && copying) {
        if (nparts >= NSEC) { set_bad(); break; }
        if (lane == 0) {
          X.part[4 * nparts] = prest0;
          X.part[4 * nparts + 1] = ost(O_REST, 1);
          X.part[4 * nparts + 2] = written;
        }
        nparts++;
        __syncthreads();
      }
    }
    if (is_bad()) YB2_DECLINE()
    if (OP == OP_META) {  // from then to, each vu(n) | (client, clock)*
      __threadfence_block();
      __syncthreads();
      uint32_t tl = 0;
      for (uint32_t i = lane; i < sv_n; i += 64) tl += 2 * vsz(X.svt[2 * i]) + vsz(X.svt[2 * i + 1]) + vsz(X.part[i]);
      const uint32_t total = 2 * vsz(sv_n) + lane_read(wave_incl_add(tl), 63);
      uint64_t base = 0;
      if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
      base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
      if (base + total > j.cap) {
        if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
        __syncthreads();
        continue;
      }
      if (lane == 0) {
        uint8_t *o = j.out + base;
        uint32_t p = 0;
        auto put = [&](uint32_t v) { while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[p++] = (uint8_t)v; };
        put(sv_n);
        for (uint32_t i = 0; i < sv_n; i++) { put(X.svt[2 * i]); put(X.svt[2 * i + 1]); }
        put(sv_n);
        for (uint32_t i = 0; i < sv_n; i++) { put(X.svt[2 * i]); put(X.part[i]); }
        j.out_off[d] = base;
        j.out_len[d] = total;
        j.status[d] = ym::ST_OK;
      }
      __syncthreads();
      continue;
    }
    if (OP == OP_SV) {
      if (sv_any && sv_clock != 0) {
        if (sv_n >= NSV) YB2_DECLINE()
        if (lane == 0) { X.svt[2 * sv_n] = sv_client; X.svt[2 * sv_n + 1] = sv_clock; }
        sv_n++;
      }
      __threadfence_block();
      __syncthreads();
      uint32_t tl = 0;
      for (uint32_t i = lane; i < sv_n; i += 64) tl += vsz(X.svt[2 * i]) + vsz(X.svt[2 * i + 1]);
      const uint32_t total = vsz(sv_n) + lane_read(wave_incl_add(tl), 63);
      uint64_t base = 0;
      if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
      base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
      if (base + total > j.cap) {
        if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
        __syncthreads();
        continue;
      }
      if (lane == 0) {
        uint8_t *o = j.out + base;
        uint32_t p = 0;
        auto put = [&](uint32_t v) { while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[p++] = (uint8_t)v; };
        put(sv_n);
        for (uint32_t i = 0; i < sv_n; i++) { put(X.svt[2 * i]); put(X.svt[2 * i + 1]); }
        j.out_off[d] = base;
        j.out_len[d] = total;
        j.status[d] = ym::ST_OK;
      }
      __syncthreads();
      continue;
    }
    // ---- delete set (rest stream): validated, then copied (the V2 round trip is byte-identical)
    uint32_t ds0, ds1;
    {
      Cur c = s_cur(D, I_REST, MREST);
      ds0 = c.p - ist(I_REST, 2);
      const uint32_t ndc = rvu(c);
      s_commit(D, I_REST, c);
      const bool big = ndc > 64 && ndc <= BS_NDSC;
      if (big) cmap::clear(X.map);
      for (uint32_t i = 0; i < ndc && !is_bad(); i++) {
        c = s_cur(D, I_REST, MREST);
        const uint32_t client = rvu(c);
        const uint32_t m = rvu(c);
        s_commit(D, I_REST, c);
        if (m == 0 || i >= BS_NDSC) { set_bad(); break; }
        bool hit = false;  // readDeleteSet merges a repeated client: the bytes would change
        if (big) hit = cmap::seen_insert(X.map, client);
        else for (uint32_t h0 = 0; h0 < i; h0 += 64) hit |= __any(h0 + lane < i && X.dsc[h0 + lane] == client);
        if (hit) set_bad();
        __syncthreads();
        if (lane == 0) X.dsc[i] = client;
        __threadfence_block();
        for (uint32_t q = 0; q < m && !is_bad(); q++) {
          c = s_cur(D, I_REST, MREST);
          rvu(c);
          rvu(c);
          s_commit(D, I_REST, c);
        }
      }
      ds1 = ist(I_REST, 0);
    }
    // flush the RLE encoders (lib0 toUint8Array: Uint/IntDiff runs flushed, Rle<u8> final count omitted)
    idiff_flush(D, O_KC);
    uopt_flush(D, O_CL);
    idiff_flush(D, O_LC);
    idiff_flush(D, O_RC);
    uopt_flush(D, O_SL);
    uopt_flush(D, O_TR);
    uopt_flush(D, O_LN);
    if (is_bad()) YB2_DECLINE()
    __syncthreads();
    // ---- final layout: vu(0) | 9 x (vu(n) column) | vu(#parts) parts | delete set
    uint32_t coln[9];
    const uint32_t order[9] = {O_KC, O_CL, O_LC, O_RC, O_IN, O_SB, O_PI, O_TR, O_LN};
#pragma unroll
    for (uint32_t k = 0; k < 9; k++) coln[k] = ost(order[k], 1);
    const uint32_t sbn = ost(O_SB, 1), sln = ost(O_SL, 1);
    coln[5] = vsz(sbn) + sbn + sln;
    uint32_t total = 1;
#pragma unroll
    for (uint32_t k = 0; k < 9; k++) total += vsz(coln[k]) + coln[k];
    total += vsz(nparts);
    __threadfence_block();
    __syncthreads();
    {
      uint32_t tl = 0;
      for (uint32_t pI = lane; pI < nparts; pI += 64) tl += vsz(X.part[4 * pI + 2]) + X.part[4 * pI + 1] - X.part[4 * pI];
      total += lane_read(wave_incl_add(tl), 63);
    }
    total += ds1 - ds0;
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
    if (base + total > j.cap) {
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    // the scratch bytes were stored by lane 0 / the wave: make them visible to every lane's loads
    // (agent-scope fence: waits for the stores and invalidates the CU's vector L1)
    __threadfence();
    __syncthreads();
    uint8_t *const o = j.out + base;
    const uint8_t *const sc = j.out + scratch;
    auto put = [&](uint32_t p, uint32_t v) -> uint32_t {
      const uint32_t n = vsz(v);
      if (lane == 0) { uint32_t t = p; while (v > 127) { o[t++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[t] = (uint8_t)v; }
      return p + n;
    };
    auto copy = [&](uint32_t p, const uint8_t *src, uint32_t n) -> uint32_t {
      for (uint32_t i = lane; i < n; i += 64) o[p + i] = src[i];
      return p + n;
    };
    uint32_t p = put(0, 0);
#pragma unroll
    for (uint32_t k = 0; k < 9; k++) {
      p = put(p, coln[k]);
      if (k == 5) {
        p = put(p, sbn);
        p = copy(p, sc + ost(O_SB, 0), sbn);
        p = copy(p, sc + ost(O_SL, 0), sln);
      } else {
        p = copy(p, sc + ost(order[k], 0), coln[k]);
      }
    }
    p = put(p, nparts);
    for (uint32_t pI = 0; pI < nparts; pI++) {
      const uint32_t r0 = X.part[4 * pI], r1 = X.part[4 * pI + 1];
      p = put(p, X.part[4 * pI + 2]);
      p = copy(p, sc + ost(O_REST, 0) + r0, r1 - r0);
    }
    p = copy(p, D.A + D.b0 + ds0, ds1 - ds0);
    if (lane == 0) {
      j.out_off[d] = base;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}

}  // namespace big2

__global__ void k_big_init(GeneralJob j);  // ym_big.hip
int small_v2_launch(uint32_t op, const GeneralJob &j, uint8_t *done, hipStream_t st, uint32_t diff_min,
                    uint64_t pv_min);  // ym_fast2.hip
// batches of at most this many documents keep the V2 diff on k_big_v2 (one generation of one-document waves,
// faster for wide rich documents than the lane walk: C4R 4 k 1.9 against 2.7 ms); the sync and async paths
// share it (YMERGE_DF2_MIN overrides it, tests)
constexpr uint32_t DF2_MIN_DOCS = 4096;
int big2_launch(uint32_t op, const GeneralJob &j0, hipStream_t st, PwBufs &pwb) {
  if (!j0.v2 || (op != OP_SV && op != OP_DIFF && op != OP_META)) return 0;
  // many small updates (an update log): one update per lane (k_meta_v2), what it declines to the general path
  if (op == OP_META && j0.n > 8 * BS_GRID) return small_v2_launch(op, j0, nullptr, st, 0, ~0ull);
  k_big_init<<<1, 64, 0, st>>>(j0);
  GeneralJob j = j0;
  // large single-section updates: the column-parallel path first (ym_pv2.hip); small ones one per lane
  // (parseUpdateMeta); k_big_v2 takes the rest
  if (int r = pv2_prepare(op, j0, st, pwb, &j.pw_done); r < 0) return r;
  uint64_t pv_min = pv2::PV_MIN;  // (as pv2_prepare: the column path's documents are not the small kernels')
  if (const char *e = getenv("YMERGE_PW_MIN")) pv_min = strtoull(e, nullptr, 10);
  if (j.pw_done) small_v2_launch(op, j, const_cast<uint8_t *>(j.pw_done), st, DF2_MIN_DOCS, pv_min);
  if (int r = pv2_finish(j0, st, pwb); r < 0) return r;  // (waits for the prep's totals: the kernels above run)
  const uint32_t grid = j.n < BS_GRID ? j.n : BS_GRID;
  if (op == OP_DIFF) big2::k_big_v2<OP_DIFF><<<grid, 64, big2::LDS_BYTES, st>>>(j);
  else if (op == OP_META) big2::k_big_v2<OP_META><<<grid, 64, big2::LDS_BYTES, st>>>(j);
  else big2::k_big_v2<OP_SV><<<grid, 64, big2::LDS_BYTES, st>>>(j);
  return 1;
}

// The asynchronous form (ym_diff_async / ym_sv_async): no column-parallel pass (it sizes its records on the
// host); small state vectors one per lane, k_big_v2 the rest over at most grid_max blocks.  done: n zeroed bytes.
int big2_async_launch(uint32_t op, const GeneralJob &j0, uint8_t *done, uint32_t grid_max, hipStream_t st) {
  if (!j0.v2 || (op != OP_DIFF && op != OP_SV)) return 0;
  GeneralJob j = j0;
  j.pw_done = done;
  small_v2_launch(op, j, done, st, DF2_MIN_DOCS, ~0ull);
  const uint32_t grid = j.n < grid_max ? j.n : grid_max;
  if (op == OP_DIFF) big2::k_big_v2<OP_DIFF><<<grid, 64, big2::LDS_BYTES, st>>>(j);
  else big2::k_big_v2<OP_SV><<<grid, 64, big2::LDS_BYTES, st>>>(j);
  return 1;
}

}  // namespace ymk
