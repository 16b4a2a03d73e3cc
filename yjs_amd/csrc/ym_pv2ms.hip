// ym_pv2ms.hip -- column-parallel diffUpdateV2 / encodeStateVectorFromUpdateV2 / parseUpdateMetaV2 over
// large V2 updates with several client sections (BASELINE configs[4] C5: ~1,000 sections per document,
// XmlElement / XmlText types, formatted text, attributes).
//
// The single-section path (ym_pv2.hip) reads the one section's header from the rest stream and cuts one
// run of every column.  Here the rest stream interleaves every section's header (vu(#structs), vu(first
// clock)) with the payloads of its structs (Skip lengths, ContentAny / ContentFormat / ContentEmbed values,
// ContentBinary buffers; UpdateDecoder.js:274-293, 13.5.16 LazyStructReader), and a diff keeps a suffix
// of every section (13.5.16 diffUpdateV2 us@40707; reference writeClientsStructs encoding.js:94-116 cuts
// each client at the state vector), so every column is rebuilt from ~1,000 kept value ranges.
//
//  MR  k_ms_rest    one block per document: the rest walk -- section headers, and the payload start of every
//                   struct that has one: the info / len columns are tokenised block-parallel into the list of
//                   payload structs, then one thread follows the rest stream's tokens through per-window
//                   token-length tables.  Counts the structs, so the value arrays can be sized.
//  K1  k_v2_decw    (ym_pv2.hip) every column decoded wave-parallel, as for one section.
//  K2  k_ms_struct  one 256-thread block per document, two passes of block prefix sums over the structs:
//                   pass 1 gives each section's column indices, clock and body offsets, its client (the
//                   client column's value at the section start) and, for a state vector / meta, the answer;
//                   pass 2 finds each section's cut against sv[client] (an LDS hash map of the state vector).
//  K3  k_ms_col     one wave per (document, column): lanes locate each kept section's value range in the
//                   input column (K1 checkpoints) and describe it as runs -- the cut struct's re-encoded
//                   values (Item.write with offset), the range's first two entries, its clipped last entry --
//                   and a verbatim byte span for the entries between; then one wave-uniform lib0 encoder
//                   folds the runs of all sections in order, so runs that continue across a section boundary
//                   merge exactly as the encoder would merge them, and the spans are copied.
//  K4  k_ms_out     one wave per document: the delete set validated, string body pieces and rest pieces
//                   (vu(written) vu(first clock) payloads) per kept section, the keyClock column (writeKey
//                   numbers keys 0, 1, 2, ...: its IntDiff encoding has a closed form), the assembly.
//
// Exactly the documents k_big_v2 (ym_big2.hip) would take are taken, with identical bytes, except that
// ContentAny / Embed / Format values may be nested objects and arrays here; anything else (JSON / Doc
// content, non-ASCII string bodies, repeated or ascending clients, a Skip right before a cut, non-canonical
// columns) is declined to k_big_v2 and from there to the general path.
#include <hip/hip_runtime.h>

#include "ym_pv2.h"
#include "ym_cmap.h"
#include "ym_wave_ds.h"

namespace ymk {
namespace pv2 {

// debugging aid (ym__ms_prof), the rest walk (ticks of the 100 MHz s_memrealtime, summed over documents):
// [0] column passes A + B, [1] phase C, [2] C's serial walk, [3] windows, [4] tokens from the tables,
// [5] tokens parsed by the walker itself, [6] section headers, [7] C's table computation
__device__ unsigned long long ms_prof[16];
#ifdef YM_PW_TICKS
#define MSP(i, v) do { if (threadIdx.x == 0) atomicAdd(&ms_prof[i], (unsigned long long)(v)); } while (0)
#define MSC(x) x
#else  // (the walk's counters and timers cost it scalar registers: diagnostics builds only)
#define MSP(i, v) do { } while (0)
#define MSC(x) do { } while (0)
#endif

// ---- MR: the rest walk ---------------------------------------------------------------------------------
// ---- MR: the rest walk, block-parallel where it can be ---------------------------------------------------
// A walk of the rest stream alone is sequential (each section header's position depends on every payload
// before it), but most of what a struct-by-struct walk does is not: round 3's one-wave walk spent its steps
// on the info column (C5: ~55 k run entries per document, 0.6 us each).  Here one 256-thread block per
// document:
//  A  tokenises the info column 4 KB per block step (the RLE<u8> automaton of K1, composed across the
//     block) and writes the PAYLOAD LIST: every struct that has rest tokens (Skip: a varuint, Binary: a
//     varUint8Array, Embed / Format: one `any`, Any: `len` of them), in struct order, with its struct
//     index and kind (Any: its ordinal among the len column's consumers: GC, Deleted, Any);
//  B  tokenises the len column (UintOptRle) into its entries (first value ordinal, value) and resolves
//     every Any's value count by a binary search;
//  C  walks the rest stream with one thread, 4 KB window by window: the whole block first computes, for
//     every byte offset of the window, the length of the token a varuint / varUint8Array / scalar `any`
//     would have there (0: not decidable from the window, or invalid -- the walker then parses that token
//     itself), so each step of the chain is a table lookup: a section header (two varuints, parsed), then
//     the tokens of the payload structs up to the section's end (payload list, staged into LDS per window).
// Outputs: the section table (first struct, structs, clock, payload span, payload
// ordinal), every payload struct's rest position, the struct and payload counts, the delete set's start.
constexpr uint32_t MR_T = 256, MR_W = 4096, MR_MARG = 256, MR_PC = 1024;
// a store to global memory through an address-space-1 pointer: the walker's stores through generic pointers
// (flat stores) counted against the LDS counter too, so each next table read waited for the previous
// store's round trip to HBM (~0.9 us per token)
template <class T>
__device__ __forceinline__ void gst(T *p, T v) { *(__attribute__((address_space(1))) T *)p = v; }
// per-thread 16-byte slice transition of the RLE<u8> / UintOptRle automaton (K1's tstep), packed 2 bits per state
__device__ __forceinline__ uint32_t mr_slice_f(const uint8_t (&b)[16], uint32_t q, uint32_t c1, bool rle, uint32_t fb) {
  uint32_t s0 = 0, s1 = 1, s2 = 2, s3 = 3;
#pragma unroll
  for (uint32_t k = 0; k < 16; k++)
    if (q + k < c1) { s0 = tstep(s0, b[k], rle, fb); s1 = tstep(s1, b[k], rle, fb); s2 = tstep(s2, b[k], rle, fb); s3 = tstep(s3, b[k], rle, fb); }
  return s0 | (s1 << 2) | (s2 << 4) | (s3 << 6);
}
// block-wide: the transition before this thread's slice (composed over lower threads) and the block's total
__device__ __forceinline__ uint32_t mr_block_compose(uint32_t f, uint32_t *sh, uint32_t &total) {
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t incl = wave_incl_compose(f);
  const uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp((int)F_ID, (int)incl, 0x138, 0xf, 0xf, false);
  __syncthreads();
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  uint32_t pre = F_ID;
  for (uint32_t k = 0; k < w; k++) pre = fcompose(pre, sh[k]);
  total = F_ID;
  for (uint32_t k = 0; k < MR_T / 64; k++) total = fcompose(total, sh[k]);
  return fcompose(pre, excl);
}
// block-wide exclusive sums of a u64 and three u32 values (+ the block's totals)
__device__ __forceinline__ void mr_block_scan(uint64_t &a, uint32_t &b, uint32_t &c, uint32_t &e, uint64_t *sh64, uint32_t *sh,
                                              uint64_t &ta, uint32_t &tb, uint32_t &tc, uint32_t &te) {
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t ia = wave_incl_add64(a);
  const uint32_t ib = wave_incl_add(b), ic = wave_incl_add(c), ie = wave_incl_add(e);
  __syncthreads();
  if (lane == 63) { sh64[w] = ia; sh[3 * w] = ib; sh[3 * w + 1] = ic; sh[3 * w + 2] = ie; }
  __syncthreads();
  uint64_t pa = 0;
  uint32_t pb = 0, pc = 0, pe = 0;
  ta = 0; tb = 0; tc = 0; te = 0;
  for (uint32_t k = 0; k < MR_T / 64; k++) {
    if (k < w) { pa += sh64[k]; pb += sh[3 * k]; pc += sh[3 * k + 1]; pe += sh[3 * k + 2]; }
    ta += sh64[k]; tb += sh[3 * k]; tc += sh[3 * k + 1]; te += sh[3 * k + 2];
  }
  a = pa + ia - a; b = pb + ib - b; c = pc + ic - c; e = pe + ie - e;
}
// payload kinds (the low 3 bits of a payload-list entry)
enum : uint32_t { PK_NONE = 0, PK_SKIP = 1, PK_BIN = 2, PK_ONE = 3, PK_ANY = 4 };
// an info byte's rest payload kind and whether it consumes a len value; false: a kind this path declines
__device__ __forceinline__ bool mr_kind(uint32_t v, uint32_t &pk, bool &lenc) {
  pk = PK_NONE;
  lenc = false;
  if (v == 10) { pk = PK_SKIP; return true; }
  const uint32_t ref = v & 31;
  switch (ref) {
    case 0: lenc = true; return v == 0;  // GC (GC.write writes info 0)
    case 1: lenc = true; return true;    // ContentDeleted
    case 3: pk = PK_BIN; return true;
    case 5: case 6: pk = PK_ONE; return true;
    case 8: pk = PK_ANY; lenc = true; return true;
    case 4: case 7: return true;         // String / Type: columns only
    default: return false;               // JSON, Doc, invalid refs
  }
}
// the token of kind k at o of the window buffer (bytes [0, lim)): its length, 0 when not decidable here
// (strings / binaries longer than MR_CAP: 0, the walker's own parse -- an uncapped parse at a garbage offset can
// run to the window's end, and the tables would cost O(window x window))
constexpr uint32_t MR_CAP = 128;
__device__ __forceinline__ uint32_t mr_tok_len(const uint8_t *w, uint32_t o, uint32_t lim, uint32_t k) {
  ln::LCur c = ln::make(w, o, lim, MR_CAP);
  if (k == PK_SKIP) {
    const uint32_t v = ln::rvu(c);
    return c.bad || v == 0 ? 0 : c.p - o;
  }
  if (k == PK_BIN) {
    const uint32_t n = ln::rvu(c);
    if (c.bad || n > MR_CAP || !ln::room(c, n)) return 0;
    return c.p + n - o;
  }
  const uint32_t tag = (uint32_t)c.lo & 0xffu;
  if (tag == 116 || tag == 117 || tag == 118 || tag == 122) return 0;  // nested: the walker's own parse
  ln::any_scalar(c);
  return c.bad ? 0 : c.p - o;
}
// lib0 readVarUint (canonical, u32) at o of the LDS window w (bytes [0, lim)), advancing o
template <uint32_t N>
__device__ __forceinline__ uint32_t mr_vu(const uint8_t (&w)[N], uint32_t &o, uint32_t lim, bool &bad) {
  uint32_t v = 0, nb = 0, x = 0x80;
  while ((x & 0x80) && nb < 5) {
    x = o + nb < lim ? w[o + nb] : 0x80;
    v |= (x & 0x7f) << (7 * nb);
    nb++;
  }
  bad |= (x & 0x80) || (nb > 1 && x == 0) || (nb == 5 && (x & 0x70) != 0);
  o += nb;
  return v;
}
// the token of kind k at p, parsed from the document (the walker's slow path); NONE: invalid
__device__ __noinline__ uint32_t mr_tok_slow(const uint8_t *D, uint32_t p, uint32_t len, uint32_t k) {
  ln::LCur c = ln::make(D, p, len);
  if (k == PK_SKIP) c.bad |= ln::rvu(c) == 0;
  else if (k == PK_BIN) { const uint32_t nb = ln::rvu(c); if (c.bad || !ln::room(c, nb)) c.bad = true; else ln::skip(c, nb); }
  else ln::any_canon(c);
  return c.bad ? NONE : c.p;
}
// the len column's value at ordinal o (entries: first ordinal, value); NONE past its end
__device__ __forceinline__ uint32_t mr_len_at(const uint2 *le, uint32_t nle, uint32_t ltot, uint32_t o) {
  if (o >= ltot || nle == 0) return NONE;
  uint32_t lo = 0, hi = nle;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (le[mid].x <= o) lo = mid; else hi = mid;
  }
  return le[lo].y;
}

__global__ void __launch_bounds__(MR_T) k_ms_rest(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  Meta &M = J.meta[d];
  if (__builtin_amdgcn_readfirstlane((int)M.ok) == 0 || __builtin_amdgcn_readfirstlane((int)M.ms) == 0) return;
  __shared__ uint32_t shf[MR_T / 64], shs[3 * (MR_T / 64)];
  __shared__ uint64_t sh64[MR_T / 64];
  __shared__ uint32_t s_bad;
  const uint32_t u0 = j.doc_upd[d];
  const uint64_t ub = j.upd_off[u0];
  const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
  const uint8_t *D = j.A + ub;
  Sec *S = a_sec(J, M);
  uint32_t *ist = a_istart(J, M), *pidx = a_pidx(J, M, len), *pkl = a_pkl(J, M, len);
  uint2 *lent = a_lent(J, M, len);
  const uint32_t icap = ms_icap(len, M.r0);
  if (t == 0) s_bad = 0;
  const uint64_t tm0 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  // ---- A: info column -> payload list
  uint64_t nstr = 0;        // structs of the counted entries
  uint32_t npay = 0, nlc = 0, fin = 0, finv = 0, fin_k = 0, fin_l = 0;
  uint64_t fin_i = 0;
  {
    const uint32_t c0 = M.col0[4], c1 = M.col1[4];
    uint32_t st = 0;
    for (uint32_t x = c0; x < c1; x += 16 * MR_T) {
      const uint32_t q = x + 16 * t;
      uint8_t b[16];
      { const uint4 v4 = wds::load16m(D, q, c1); __builtin_memcpy(b, &v4, 16); }
      uint32_t tot;
      const uint32_t ex = mr_block_compose(mr_slice_f(b, q, c1, true, 0), shf, tot);
      uint32_t sl = (ex >> (2 * st)) & 3, starts = 0;
#pragma unroll
      for (uint32_t k = 0; k < 16; k++)
        if (q + k < c1) { if (sl == 0) starts |= 1u << k; sl = tstep(sl, b[k], true, 0); }
      uint64_t ns = 0;
      uint32_t np = 0, nl = 0, nf = 0, fv = 0;
      bool bad = false;
      for (uint32_t m = starts; m; m &= m - 1) {
        const Ent e = dec_entry(D, q + __builtin_ctz(m), c1, K_INFO);
        uint32_t pk;
        bool lc;
        bad |= e.bad || !mr_kind(e.val, pk, lc) || e.cnt > (1u << 26);
        if (e.fin) { nf = 1; fv = e.val; continue; }
        ns += e.cnt;
        np += pk != PK_NONE ? e.cnt : 0;
        nl += lc ? e.cnt : 0;
      }
      uint64_t a = ns;
      uint32_t bb = np, cc = nl, ee = nf, tb, tc, te;
      uint64_t tta;
      mr_block_scan(a, bb, cc, ee, sh64, shs, tta, tb, tc, te);
      // emission: the thread's entries' payload structs
      uint64_t si = nstr + a;
      uint32_t pi = npay + bb, li = nlc + cc;
      bad |= nstr + tta > (1ull << 26) || npay + tb > icap;
      if (!bad)
        for (uint32_t m = starts; m; m &= m - 1) {
          const Ent e = dec_entry(D, q + __builtin_ctz(m), c1, K_INFO);
          uint32_t pk;
          bool lc;
          mr_kind(e.val, pk, lc);
          if (e.fin) {  // the endless final run: its structs start after every counted one
            fin_i = nstr + tta; fin_k = npay + tb; fin_l = nlc + tc;
            continue;
          }
          if (pk != PK_NONE)
            for (uint32_t r = 0; r < e.cnt; r++) {
              pidx[pi + r] = (uint32_t)(si + r);
              pkl[pi + r] = pk == PK_ANY ? ((li + r) << 3) | PK_ANY : pk;
            }
          si += e.cnt;
          pi += pk != PK_NONE ? e.cnt : 0;
          li += lc ? e.cnt : 0;
        }
      if (bad) s_bad = 1;
      if (nf) { fin = 1; finv = fv; }
      // (the final entry is the column's last byte: one thread of the last step has it)
      st = (tot >> (2 * st)) & 3;
      nstr += tta; npay += tb; nlc += tc;
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane((int)s_bad)) break;
    }
  }
  // the final entry's values to every thread
  __shared__ uint32_t s_fin2[5];
  __shared__ uint64_t s_fini2;
  if (t == 0) { s_fin2[0] = 0; }
  __syncthreads();
  if (fin) { s_fin2[0] = 1; s_fin2[1] = finv; s_fin2[2] = fin_k; s_fin2[3] = fin_l; s_fini2 = fin_i; }
  __syncthreads();
  fin = s_fin2[0];
  if (fin) { finv = s_fin2[1]; fin_k = s_fin2[2]; fin_l = s_fin2[3]; fin_i = s_fini2; }
  uint32_t fin_pk = PK_NONE;
  {
    bool lc;
    if (fin) mr_kind(finv, fin_pk, lc);
  }
  // ---- B: len column entries; the Any structs' value counts
  uint32_t nle = 0, ltot = 0;
  if (!__builtin_amdgcn_readfirstlane((int)s_bad)) {
    const uint32_t c0 = M.col0[8], c1 = M.col1[8];
    uint32_t st = 0;
    uint64_t lsum = 0;
    for (uint32_t x = c0; x < c1; x += 16 * MR_T) {
      const uint32_t q = x + 16 * t;
      uint8_t b[16];
      { const uint4 v4 = wds::load16m(D, q, c1); __builtin_memcpy(b, &v4, 16); }
      uint32_t tot;
      const uint32_t ex = mr_block_compose(mr_slice_f(b, q, c1, false, 6), shf, tot);
      uint32_t sl = (ex >> (2 * st)) & 3, starts = 0;
#pragma unroll
      for (uint32_t k = 0; k < 16; k++)
        if (q + k < c1) { if (sl == 0) starts |= 1u << k; sl = tstep(sl, b[k], false, 6); }
      uint64_t nv = 0;
      uint32_t ne = 0;
      bool bad = false;
      for (uint32_t m = starts; m; m &= m - 1) {
        const Ent e = dec_entry(D, q + __builtin_ctz(m), c1, K_LN);
        bad |= e.bad;
        nv += e.cnt;
        ne++;
      }
      uint64_t a = nv;
      uint32_t bb = ne, cc = 0, ee = 0, tb, tc, te;
      uint64_t tta;
      mr_block_scan(a, bb, cc, ee, sh64, shs, tta, tb, tc, te);
      bad |= lsum + tta > 0xffffffffull;
      if (!bad) {
        uint64_t o = lsum + a;
        uint32_t ei = nle + bb;
        for (uint32_t m = starts; m; m &= m - 1) {
          const Ent e = dec_entry(D, q + __builtin_ctz(m), c1, K_LN);
          lent[ei++] = make_uint2((uint32_t)o, e.val);
          o += e.cnt;
        }
      }
      if (bad) s_bad = 1;
      st = (tot >> (2 * st)) & 3;
      lsum += tta;
      nle += tb;
      __syncthreads();
      if (__builtin_amdgcn_readfirstlane((int)s_bad)) break;
    }
    ltot = (uint32_t)lsum;
  }
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane((int)s_bad)) {  // Any: the count of values (the len value at its ordinal)
    bool bad = false;
    for (uint32_t k = t; k < npay; k += MR_T) {
      const uint32_t kl = pkl[k];
      if ((kl & 7) != PK_ANY) continue;
      const uint32_t v = mr_len_at(lent, nle, ltot, kl >> 3);
      bad |= v == NONE || v == 0 || v >= (1u << 28);
      pkl[k] = (v << 3) | PK_ANY;
    }
    if (bad) s_bad = 1;
  }
  __syncthreads();
  // which token kinds the document has (tables are computed for those only): Skip / Binary / any
  __shared__ uint32_t s_kinds;
  if (t == 0) s_kinds = fin ? 1u << fin_pk : 0;
  __syncthreads();
  {
    uint32_t m = 0;
    for (uint32_t k = t; k < npay; k += MR_T) m |= 1u << (pkl[k] & 7);
    if (m) atomicOr(&s_kinds, m);
  }
  __syncthreads();
  if (t == 0) {
    if (s_bad) { M.ok = 0; M.why = 50; }
    M.mr_npay = npay; M.mr_kinds = s_kinds; M.mr_fin = fin; M.mr_finpk = fin_pk; M.mr_fink = fin_k; M.mr_finl = fin_l;
    M.mr_nle = nle; M.mr_ltot = ltot; M.mr_nstr = nstr; M.mr_fini = fin_i;
  }
  MSP(0, __builtin_amdgcn_s_memrealtime() - tm0);
}

// ---- MR, the walk: one wave per document, in lockstep -----------------------------------------------------
// Every lane computes the same values (LDS reads made uniform by readfirstlane), so the chain's state stays in
// scalar registers and its branches are uniform; the wave computes each window's token-length tables
// (64 offsets per lane), then follows the chain: a section header (two varuints), then the tokens of the
// payload structs up to the section's end, each one table lookup.
__global__ void __launch_bounds__(64) k_ms_walk(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  Meta &M = J.meta[d];
  auto U = [](uint32_t x) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
  if (U(M.ok) == 0 || U(M.ms) == 0) return;
  __shared__ __attribute__((aligned(16))) uint8_t win[MR_W + MR_MARG + 16];
  __shared__ uint16_t tV[MR_W], tB[MR_W], tA[MR_W];
  __shared__ uint2 spay[MR_PC + 1]; // the window's payload structs (index, kind | token count << 3; one token: the kind)
  __shared__ uint32_t sist[MR_PC];  // their first tokens' offsets (flushed to ist at the window's end)
  __shared__ uint32_t sdum[64];     // (the fast loop's other lanes' stores)
  const uint32_t u0 = j.doc_upd[d];
  const uint64_t ub = j.upd_off[u0];
  const uint32_t len = U((uint32_t)(j.upd_off[u0 + 1] - ub));
  const uint8_t *D = j.A + ub;
  Sec *S = a_sec(J, M);
  uint32_t *ist = a_istart(J, M), *pidx = a_pidx(J, M, len), *pkl = a_pkl(J, M, len);
  const uint2 *lent = a_lent(J, M, len);
  const uint32_t icap = ms_icap(len, U(M.r0));
  const uint32_t npay = U(M.mr_npay), kinds = U(M.mr_kinds), fin = U(M.mr_fin), fin_pk = U(M.mr_finpk);
  const uint32_t fin_k = U(M.mr_fink), fin_l = U(M.mr_finl), nle = U(M.mr_nle), ltot = U(M.mr_ltot);
  const uint64_t nstr = M.mr_nstr, fin_i = M.mr_fini;
  const uint32_t nsec = U(M.nsec);
  const bool need_v = kinds & (1u << PK_SKIP), need_b = kinds & (1u << PK_BIN);
  const uint64_t tm0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t_walk = 0, t_tab = 0;
  uint32_t n_win = 0, n_tok = 0, n_slow = 0, n_hdr = 0, n_fin = 0, n_ghdr = 0, n_lc = 0;
  // the len column's cursor for the endless final run: entry lc_e - 1 holds ordinals [lc_lo, lc_hi), value lc_v
  uint32_t lc_e = 0, lc_lo = 1, lc_hi = 0, lc_v = NONE;
  // the chain's state (uniform)
  uint32_t p = U(M.r0), s = 0, k = 0, i = 0, send = 0, insec = 0, rt = 0, kind = 0;
  bool bad = false, done = false;
  uint32_t tab_wb = NONE;
  uint32_t tab_wn = 0;
  while (!bad && !done) {
    // the window: the current one while p is inside its tables, else one starting at p
    const uint32_t k0 = k, wb = tab_wb != NONE && p >= tab_wb && p < tab_wb + tab_wn ? tab_wb : p & ~15u;
    const uint32_t wl = wb + MR_W + MR_MARG < len ? wb + MR_W + MR_MARG : len;  // window bytes [wb, wl)
    const uint32_t lim = wl - wb, wn = lim < MR_W ? lim : MR_W;
    const bool fresh = wb != tab_wb;
    const uint64_t tt0 = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (fresh)
      for (uint32_t q = 16 * t; q < lim; q += 16 * 64) {
        const uint4 v = wds::load16m(D, wb + q, len);
        uint8_t tb16[16];
        __builtin_memcpy(tb16, &v, 16);
        __builtin_memcpy(win + q, tb16, 16);
      }
    for (uint32_t q = t; q < MR_PC; q += 64)
      if (k0 + q < npay) {
        const uint32_t kl = pkl[k0 + q];
        spay[q] = make_uint2(pidx[k0 + q], kl == ((1u << 3) | PK_ANY) ? (uint32_t)PK_ONE : kl);  // (Any of one value: one token)
      }
    __syncthreads();
    if (fresh) {
      for (uint32_t o = t; o < wn; o += 64) {
        const uint32_t la = mr_tok_len(win, o, lim, PK_ONE);
        tA[o] = (uint16_t)(la < 65536 ? la : 0);
        if (need_v) { const uint32_t lv = mr_tok_len(win, o, lim, PK_SKIP); tV[o] = (uint16_t)(lv < 65536 ? lv : 0); }
        if (need_b) { const uint32_t lb = mr_tok_len(win, o, lim, PK_BIN); tB[o] = (uint16_t)(lb < 65536 ? lb : 0); }
      }
      tab_wb = wb;
      tab_wn = wn;
    }
    __syncthreads();
    const uint64_t tt1 = __builtin_amdgcn_s_memrealtime();
    MSC(t_tab += tt1 - tt0);
    MSC(n_win++);
    const uint32_t wend = wb + wn;  // tokens starting before here use the tables
    // the staged entries the fast loop may take (below the payload list's end and the first-token capacity)
    const uint32_t kfast = min(min(npay, k0 + MR_PC), icap);
    for (;;) {
      if (rt > 0) {  // inside a payload struct: its tokens
        const uint16_t *tab = kind == PK_SKIP ? tV : kind == PK_BIN ? tB : tA;
        const uint32_t rt0 = rt;
        while (rt > 0 && p < wend) {
          const uint32_t L = U(tab[p - wb]);
          if (L == 0) break;
          p += L;
          rt--;
        }
        MSC(n_tok += rt0 - rt);
        (void)rt0;
        if (rt == 0) continue;
        if (p >= wend) { bad = wend >= len; break; }  // (next window; past the document's end: truncated)
        const uint32_t e = U(mr_tok_slow(D, p, len, kind == PK_ANY ? PK_ONE : kind));  // (a token the table lacks)
        if (e == NONE) { bad = true; break; }
        MSC(n_slow++);
        MSC(n_tok++);
        p = e;
        rt--;
        continue;
      }
      if (!insec) {  // a section header: vu(#structs) vu(first clock)
        if (s == nsec) { done = true; break; }
        if (p >= wend) { bad = wend >= len; break; }
        MSC(n_hdr++);
        uint32_t W, clock, pe;
        bool hb = false;
        if (p + 16 <= wl) {
          uint32_t o = p - wb;
          W = U(mr_vu(win, o, lim, hb));
          clock = U(mr_vu(win, o, lim, hb));
          pe = wb + U(o);
        } else {
          MSC(n_ghdr++);
          ln::LCur c = ln::make(D, p, len);
          W = U(ln::rvu(c));
          clock = U(ln::rvu(c));
          pe = U(c.p);
          hb = c.bad;
        }
        if (U(hb ? 1u : 0u) != 0 || W == 0 || W > (1u << 26)) { bad = true; break; }
        if (t == 0) {
          gst(&S[s].S, i);
          gst(&S[s].W, W);
          gst(&S[s].clock, clock);
          gst(&S[s].pay0, pe);
          gst(&S[s].ibase, k);
        }
        p = pe;
        send = i + W;
        if (send > (1u << 26)) { bad = true; break; }
        insec = 1;
        continue;
      }
      // fast loop: consecutive one-token payload structs of one kind inside the window and the staged list --
      // one table read per struct, the next entry's read issued before it (the general steps below take
      // everything else: section ends, Any runs, tokens the tables lack, window and list ends)
      if (k < kfast && p < wend) {
        uint2 e = spay[k - k0];
        const uint32_t code = U(e.y);
        if (U(e.x) < send && code != PK_NONE && code < PK_ANY) {
          const uint16_t *tab = code == PK_SKIP ? tV : code == PK_BIN ? tB : tA;
          for (;;) {
            // both LDS reads in flight together (the barrier keeps the compiler from sinking the entry's read
            // below the table read's wait); lane 0 records the first-token offset, the other lanes write a
            // slot of their own (no exec-mask branch, no bank conflict)
            const uint2 en = spay[k + 1 - k0];
            const uint32_t tv = tab[p - wb];
            asm volatile("" ::: "memory");
            const uint32_t L = U(tv);
            if (L == 0) break;
            *(t == 0 ? &sist[k - k0] : &sdum[t]) = p;
            p += L;
            k++;
            if (k >= kfast || p >= wend || U(en.x) >= send || U(en.y) != code) break;
          }
        }
      }
      // the next payload struct, if it belongs to this section
      uint32_t nidx, nkl;
      if (k - k0 >= MR_PC) break;  // the staged payload list (or the offsets' buffer) is used up: next window
      if (k < npay) {
        const uint2 e = spay[k - k0];
        nidx = U(e.x);
        nkl = U(e.y);
      } else if (fin && fin_pk != PK_NONE) {  // the endless final run
        const uint64_t x = fin_i + (k - fin_k);
        nidx = x < 0xffffffffull ? (uint32_t)x : NONE;
        nkl = fin_pk;
        MSC(n_fin++);
        if (fin_pk == PK_ANY) {  // (consecutive ordinals: the cursor moves to the next entry, else a search)
          const uint32_t o = fin_l + (k - fin_k);
          if (o < lc_lo || o >= lc_hi) {
            MSC(n_lc++);
            lc_v = NONE; lc_lo = 1; lc_hi = 0;
            if (o < ltot && nle != 0) {
              uint32_t e = lc_e;
              if (!(e < nle && U(lent[e].x) <= o && (e + 1 == nle || U(lent[e + 1].x) > o))) {
                uint32_t lo = 0, hi = nle;
                while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (U(lent[mid].x) <= o) lo = mid; else hi = mid; }
                e = lo;
              }
              lc_lo = U(lent[e].x); lc_v = U(lent[e].y); lc_hi = e + 1 < nle ? U(lent[e + 1].x) : ltot; lc_e = e + 1;
            }
          }
          const uint32_t v = lc_v;
          if (v == NONE || v == 0 || v >= (1u << 28)) { if (nidx < send) { bad = true; break; } }
          nkl = (v << 3) | PK_ANY;
        }
      } else {
        nidx = NONE;
        nkl = 0;
      }
      if (nidx >= send) {  // the section is complete
        if (t == 0) gst(&S[s].pay1, p);
        i = send;
        s++;
        insec = 0;
        continue;
      }
      if (k >= icap) { bad = true; break; }
      if (t == 0) sist[k - k0] = p;
      k++;
      kind = nkl & 7;
      rt = kind == PK_ANY ? nkl >> 3 : 1;
    }
    MSC(t_walk += __builtin_amdgcn_s_memrealtime() - tt1);
    __syncthreads();
    for (uint32_t q = t; q < k - k0; q += 64) ist[k0 + q] = sist[q];
  }
  if (done && !fin && (uint64_t)i > nstr) bad = true;  // the info column has fewer structs than the sections
  if (t == 0) {
    if (bad) { M.ok = 0; M.why = 50; }
    else { M.n = i; M.nitem = k; M.ds0 = p; }
  }
  MSP(1, __builtin_amdgcn_s_memrealtime() - tm0); MSP(2, t_walk); MSP(3, n_win);
  MSP(4, n_tok); MSP(5, n_slow); MSP(6, n_hdr); MSP(7, t_tab); MSP(8, n_fin); MSP(9, n_ghdr); MSP(10, n_lc);
}

__global__ void k_ms_sizes_k(Job J, uint64_t *sizes) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= J.j.n) return;
  Meta &M = J.meta[d];
  if (!M.ok || !M.ms) return;
  uint32_t colb[NK];
  for (uint32_t k = 0; k < NK; k++) colb[k] = M.col1[col_of(k)] - M.col0[col_of(k)];
  sizes[d] = (scr_layout(M, M.n, M.nsec, true, colb) + 255) & ~255ull;
}

// ---- K2: struct passes ----------------------------------------------------------------------------------
constexpr uint32_t SVMAX = 2048, SVSLOTS = 4096;  // state-vector entries / LDS hash slots
__device__ __forceinline__ uint32_t sv_hash(uint32_t c) { return (c * 0x9E3779B1u) >> 20; }
constexpr uint32_t MSEC = 4096;  // sections a document may have on this path (their starts sit in LDS)
// the section holding struct i (sections are contiguous, non-empty, in struct order; starts in LDS)
__device__ __forceinline__ uint32_t sec_of(const uint32_t *secS, uint32_t nsec, uint32_t i) {
  uint32_t lo = 0, hi = nsec;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (secS[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t put_vu_g(uint8_t *o, uint32_t p, uint32_t v) {
  while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
  o[p++] = (uint8_t)v;
  return p;
}

// per-struct values of the scans: the nine kinds, payload-struct ordinal, key writers
enum { X_IT = NK, X_KW, NX };

template <int OP>
__global__ void __launch_bounds__(KT) k_ms_struct(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  Meta &M = J.meta[d];
  if (!M.ok || !M.ms) return;
  __shared__ uint32_t sh[4 * 16];
  __shared__ uint32_t s_bad;
  __shared__ uint32_t mkey[OP == OP_DIFF ? SVSLOTS : 1], mval[OP == OP_DIFF ? SVSLOTS : 1];
  __shared__ uint32_t svclk[OP == OP_DIFF ? SVMAX : 1];
  __shared__ uint32_t secS[MSEC + 1];  // each section's first struct (sec_of)
  const uint32_t u0 = j.doc_upd[d];
  const uint64_t ub = j.upd_off[u0];
  const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
  const uint8_t *D = j.A + ub;
  const uint32_t n = M.n, nsec = M.nsec;
  Sec *S = a_sec(J, M);
  const uint32_t *ist = a_istart(J, M);
  const uint8_t *info_a = a_info(J, M), *pi_a = a_pi(J, M), *tr_a = a_tr(J, M);
  const uint32_t *sl_a = a_sl(J, M), *ln_a = a_ln(J, M), *cl_a = a_cl(J, M);
#define MS_DECLINE(code)                       \
  {                                            \
    if (t == 0) { M.ok = 0; M.why = (code); }  \
    return;                                    \
  }
  // the string body must be ASCII (a UTF-16 slice is then a byte slice; k_big_v2's condition)
  {
    bool na = false;
    for (uint32_t i = 16 * t; i < M.sn; i += 16 * KT) {
      const uint32_t m = M.sn - i < 16 ? M.sn - i : 16;
      for (uint32_t q = 0; q < m; q++) na |= D[M.sb0 + i + q] >= 0x80;
    }
    if (__syncthreads_or(na)) MS_DECLINE(21)
  }
  if (M.nval[K_CL] == 0 || nsec > MSEC) MS_DECLINE(22)
  for (uint32_t s = t; s < nsec; s += KT) {
    S[s].skipk = ~0ull;
    S[s].f = NONE;
    secS[s] = S[s].S;
  }
  if (t == 0) secS[nsec] = NONE;
  // decodeStateVector (encoding.js:536-545): a later entry for a client wins
  if (OP == OP_DIFF) {
    for (uint32_t q = t; q < SVSLOTS; q += KT) mval[q] = 0;
    __syncthreads();
    if (t == 0) {
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      ln::LCur c = ln::make(j.sv + s0, 0, (uint32_t)(s1 - s0));
      const uint32_t ns = s1 - s0 > (1u << 20) ? NONE : ln::rvu(c);
      bool bad = ns == NONE || ns > SVMAX;
      for (uint32_t q = 0; q < ns && !bad; q++) {
        const uint32_t cl = ln::rvu(c), ck = ln::rvu(c);
        bad |= c.bad;
        svclk[q] = ck;
        uint32_t h = sv_hash(cl);
        while (mval[h] != 0 && mkey[h] != cl) h = (h + 1) & (SVSLOTS - 1);
        mkey[h] = cl;
        mval[h] = q + 1;
      }
      s_bad = bad || c.bad;
    }
    __syncthreads();
    if (s_bad) MS_DECLINE(20)
  }
  __syncthreads();
  // running sums carried across tiles: NX kinds, body bytes; clock prefix in 64 bits
  uint32_t base[NX + 1];
  uint64_t clock = 0;
  for (uint32_t pass = 1; pass <= (OP == OP_DIFF ? 2u : 1u); pass++) {
#pragma unroll
    for (uint32_t q = 0; q <= NX; q++) base[q] = 0;
    clock = 0;
    for (uint32_t t0 = 0; t0 < n; t0 += TILE) {
      const uint32_t i0 = t0 + t * PER;
      uint32_t s = sec_of(secS, nsec, i0 < n ? i0 : n - 1);
      uint32_t vv[PER], pv[PER], tv[PER], sec[PER];
      bool st[PER];
      uint32_t cons[PER][NX];
      bool bad = false;
      uint32_t xp[2] = {0, 0}, pi0 = 0, tr0 = 0;
#pragma unroll
      for (uint32_t e = 0; e < PER; e++) {
        const uint32_t i = i0 + e;
        const bool valid = i < n;
        while (valid && secS[s + 1] <= i) s++;
        sec[e] = s;
        st[e] = valid && secS[s] == i;
        const uint32_t v = valid ? info_a[i] : 0;
        vv[e] = v;
        const uint32_t ref = v & 31;
        const bool sk = valid && v == 10, gc = valid && ref == 0, item = valid && !sk && !gc;
        bad |= gc && v != 0;
        bad |= item && (ref == 2 || ref == 9 || ref >= 10);
        bad |= item && (v & 0xC0) && (v & 0x20);  // parentSub bit next to an origin: re-encoded without it
        cons[e][K_PI] = item && !(v & 0xC0);
        cons[e][K_TR] = item && ref == 7;
        xp[0] += cons[e][K_PI];
        xp[1] += cons[e][K_TR];
      }
      // parentInfo / typeRef indices first (the other kinds depend on their values)
      {
        uint32_t tp[2];
        block_scan<2>(xp, tp, sh);
        uint32_t pidx = base[K_PI] + xp[0], tidx = base[K_TR] + xp[1];
#pragma unroll
        for (uint32_t e = 0; e < PER; e++) {
          pv[e] = 0;
          tv[e] = 0;
          if (cons[e][K_PI]) {
            pv[e] = pidx < M.nval[K_PI] ? pi_a[pidx] : M.finv[K_PI];
            bad |= pidx >= M.nval[K_PI] && !M.fin[K_PI];
            pidx++;
          }
          if (cons[e][K_TR]) {
            bad |= tidx >= M.nval[K_TR];
            tv[e] = tidx < M.nval[K_TR] ? tr_a[tidx] : 0;
            tidx++;
          }
        }
        pi0 = base[K_PI] + xp[0];
        tr0 = base[K_TR] + xp[1];
        base[K_PI] += tp[0];
        base[K_TR] += tp[1];
      }
      uint32_t xs[NX], tot[NX];
#pragma unroll
      for (uint32_t q = 0; q < NX; q++) xs[q] = 0;
#pragma unroll
      for (uint32_t e = 0; e < PER; e++) {
        const uint32_t v = vv[e], ref = v & 31;
        const bool valid = i0 + e < n;
        const bool sk = valid && v == 10, gc = valid && ref == 0, item = valid && !sk && !gc;
        const bool o = item && (v & 0x80), r = item && (v & 0x40), no = item && !(v & 0xC0);
        const bool key = item && ref == 7 && (tv[e] == 3 || tv[e] == 5);
        cons[e][K_INFO] = valid;
        cons[e][K_CL] = st[e] + o + r + (no && pv[e] != 1);
        cons[e][K_LC] = o + (no && pv[e] != 1);
        cons[e][K_RC] = r;
        cons[e][K_SL] = (no && pv[e] == 1) + (no && (v & 0x20)) + (item && ref == 4) + (item && ref == 6) + key;
        cons[e][K_LN] = gc + (item && (ref == 1 || ref == 8));
        cons[e][K_KC] = key;
        cons[e][X_IT] = sk + (item && (ref == 3 || ref == 5 || ref == 6 || ref == 8));
        cons[e][X_KW] = (item && ref == 6) + key;
#pragma unroll
        for (uint32_t q = 0; q < NX; q++)
          if (q != K_PI && q != K_TR) xs[q] += cons[e][q];
      }
      block_scan<NX>(xs, tot, sh);  // (PI / TR entries are zero here: their prefixes come from above)
      // string lengths -> body bytes; clock lengths
      uint32_t sli = base[K_SL] + xs[K_SL], lni = base[K_LN] + xs[K_LN], iti = base[X_IT] + xs[X_IT];
      uint32_t clen[PER], bodyb[PER];
      uint32_t xb[2] = {0, 0};
#pragma unroll
      for (uint32_t e = 0; e < PER; e++) {
        const uint32_t v = vv[e], ref = v & 31;
        const bool valid = i0 + e < n;
        const bool sk = valid && v == 10, gc = valid && ref == 0, item = valid && !sk && !gc;
        uint32_t bl = 0;
        for (uint32_t q = 0; q < cons[e][K_SL]; q++) bl += sli + q < M.nval[K_SL] ? sl_a[sli + q] : 0;
        bad |= sli + cons[e][K_SL] > M.nval[K_SL];
        uint32_t cl = 0;
        if (sk) {  // Skip: vu(length) in the rest stream
          bad |= iti >= M.nitem;
          if (iti < M.nitem) {
            ln::LCur c = ln::make(D, ist[iti], len);
            cl = ln::rvu(c);
          }
        } else if (gc || (item && (ref == 1 || ref == 8))) {
          bad |= lni >= M.nval[K_LN];
          cl = lni < M.nval[K_LN] ? ln_a[lni] : 0;
        } else if (item && ref == 4) {
          cl = sli + cons[e][K_SL] - 1 < M.nval[K_SL] ? sl_a[sli + cons[e][K_SL] - 1] : 0;  // the content string: last
        } else if (item) {
          cl = 1;
        }
        bad |= valid && (cl == 0 || cl >= (1u << 20));  // (lengths keep the block's clock sums in u32)
        clen[e] = cl;
        bodyb[e] = bl;
        xb[0] += bl;
        xb[1] += cl;
        sli += cons[e][K_SL];
        lni += cons[e][K_LN];
        iti += cons[e][X_IT];
      }
      uint32_t tb[2];
      block_scan<2>(xb, tb, sh);
      // per struct: the prefixes before it
      uint32_t pre[NX];
#pragma unroll
      for (uint32_t q = 0; q < NX; q++) pre[q] = base[q] + xs[q];
      pre[K_PI] = pi0;
      pre[K_TR] = tr0;
      uint32_t bo = base[NX] + xb[0];
      uint64_t ck = clock + xb[1];
#pragma unroll
      for (uint32_t e = 0; e < PER; e++) {
        const uint32_t i = i0 + e;
        const bool valid = i < n;
        const uint32_t v = vv[e], ref = v & 31;
        const bool sk = valid && v == 10;
        const uint32_t s2 = sec[e];
        if (pass == 1 && valid) {
          if (st[e]) {
            Sec &X = S[s2];
            X.C0 = (uint32_t)ck;
            X.C1 = (uint32_t)(ck + clen[e]);
            X.body0 = bo;
#pragma unroll
            for (uint32_t q = 0; q < NK; q++) X.pre[q] = pre[q];
            X.kw0 = pre[X_KW];
            bad |= pre[X_IT] != X.ibase;  // the rest walk and the columns agree on the payload structs
          }
          if (sk) atomicMin(&S[s2].skipk, ((unsigned long long)i << 32) | (uint32_t)ck);
        }
        if (pass == 2 && valid && !sk) {
          const Sec &X = S[s2];
          const uint64_t startc = (uint64_t)X.clock + ((uint32_t)ck - X.C0), end = startc + clen[e];
          const uint64_t svs = X.sv;
          const bool before_ok = st[e] || startc <= svs;
          // a Skip right before a struct that ends past the state vector: the cut may lie before it
          bad |= !st[e] && startc > svs && end > svs && info_a[i - 1] == 10;
          if (end > svs && before_ok) {  // the cut (us@40707): the first non-Skip struct ending past sv
            Sec &Y = S[s2];
            Y.f = i;
            Y.fclock = (uint32_t)startc;
            Y.off = svs > startc ? (uint32_t)(svs - startc) : 0;
            Y.info_f = v;
            Y.pi_f = pv[e];
            Y.tr_f = tv[e];
            Y.clen_f = clen[e];
            Y.iord_f = pre[X_IT];
            Y.kwf = pre[X_KW];
            Y.body_f = bo;
            Y.body_f1 = bo + bodyb[e];
            Y.body_fc = ref == 4 ? bo + bodyb[e] - clen[e] : bo + bodyb[e];
#pragma unroll
            for (uint32_t q = 0; q < NK; q++) {
              Y.pf[q] = pre[q] + (q == K_CL && st[e] ? 1 : 0);
              Y.pf1[q] = pre[q] + cons[e][q];
            }
          }
        }
#pragma unroll
        for (uint32_t q = 0; q < NX; q++) pre[q] += cons[e][q];
        bo += bodyb[e];
        ck += clen[e];
      }
      bad |= clock + tb[1] > 0xffffffffull;
      if (__syncthreads_or(bad)) MS_DECLINE(23)
#pragma unroll
      for (uint32_t q = 0; q < NX; q++)
        if (q != K_PI && q != K_TR) base[q] += tot[q];
      base[NX] += tb[0];
      clock += tb[1];
      __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    if (pass == 1) {
      // every column consumed exactly (as the re-encoding writes it); strings inside the body
      bool bad = false;
      uint32_t code = 24;
      if (t == 0) {
#pragma unroll
        for (uint32_t q = 0; q < NK; q++) {
          // (keyClock: only XmlElement / XmlHook types read it, while every writeKey -- formats too -- wrote
          // one: the column is read as far as needed, and rewritten from 0)
          const bool b = q == K_KC ? base[q] > M.nval[q]
                         : k_rle(q) ? (M.fin[q] ? base[q] < M.nval[q] + 1 : base[q] != M.nval[q]) : base[q] != M.nval[q];
          if (b && !bad) code = 100 + q;
          bad |= b;
          M.tot[q] = base[q];
        }
        if (!bad && base[X_IT] != M.nitem) { bad = true; code = 110; }
        if (!bad && base[NX] > M.sn) { bad = true; code = 111; }
        M.body_end = base[NX];
        M.clock_tot = (uint32_t)clock;
      }
      // each section's client: descending (as yjs writes them), so no client repeats; its sv clock
      for (uint32_t s = t; s < nsec && !bad; s += KT) {
        const uint32_t ci = S[s].pre[K_CL];
        if (ci >= M.nval[K_CL]) { bad = true; code = 25; break; }
        const uint32_t client = cl_a[ci];
        S[s].client = client;
        const uint32_t cn = s + 1 < nsec ? S[s + 1].C0 : (uint32_t)clock;
        if ((uint64_t)S[s].clock + (cn - S[s].C0) > 0xffffffffull) { bad = true; code = 26; }  // clocks stay u32
        if (s > 0 && (S[s - 1].pre[K_CL] >= M.nval[K_CL] || cl_a[S[s - 1].pre[K_CL]] <= client)) { bad = true; code = 27; }
        uint32_t svc = 0;
        if (OP == OP_DIFF) {
          uint32_t h = sv_hash(client);
          while (mval[h] != 0) {
            if (mkey[h] == client) { svc = svclk[mval[h] - 1]; break; }
            h = (h + 1) & (SVSLOTS - 1);
          }
        }
        S[s].sv = svc;
      }
      if (__syncthreads_or(bad)) {
        if (bad) M.why = code;  // (a racy but harmless debugging aid)
        if (t == 0) M.ok = 0;
        return;
      }
      __threadfence_block();
      __syncthreads();
    }
  }
  if (OP == OP_DIFF) {
    if (t == 0) {
      uint32_t nk = 0, kc = 0;
      for (uint32_t s = 0; s < nsec; s++) {
        if (S[s].f == NONE) continue;
        nk++;
        kc += (s + 1 < nsec ? S[s + 1].kw0 : base[X_KW]) - S[s].kwf;
      }
      M.nkept = nk;
      M.kc_out = kc;
    }
    return;
  }
  // encodeStateVectorFromUpdateV2 (os@37724) / parseUpdateMetaV2: one entry per section, written by one thread
  if (t != 0) return;
  const uint32_t ctot = M.clock_tot;
  auto sec_end = [&](uint32_t s) -> uint32_t {  // the section's end clock
    const uint32_t cn = s + 1 < nsec ? S[s + 1].C0 : ctot;
    return S[s].clock + (cn - S[s].C0);
  };
  auto sv_val = [&](uint32_t s) -> uint32_t {  // what the state vector records for the section's client
    const Sec &X = S[s];
    if (X.clock != 0) return 0;  // stopCounting: the client must start at 0
    if (X.skipk == ~0ull) return sec_end(s);
    const uint32_t si = (uint32_t)(X.skipk >> 32), sc = (uint32_t)X.skipk;
    if (si == X.S) return s == 0 ? X.clock + (X.C1 - X.C0) : 0;  // (the update's first struct is counted)
    return X.clock + (sc - X.C0);
  };
  uint32_t total = 0, cnt = 0;
  if (OP == OP_SV) {
    for (uint32_t s = 0; s < nsec; s++) {
      const uint32_t v = sv_val(s);
      if (v) { cnt++; total += vsz(S[s].client) + vsz(v); }
    }
    total += vsz(cnt);
  } else {
    for (uint32_t s = 0; s < nsec; s++) total += 2 * vsz(S[s].client) + vsz(S[s].clock) + vsz(sec_end(s));
    total += 2 * vsz(nsec);
  }
  const uint64_t b = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
  J.done[d] = 1;
  atomicAdd((unsigned long long *)j.pw_count, 1ull);
  if (b + total > j.cap) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; return; }
  uint8_t *o = j.out + b;
  uint32_t p = 0;
  if (OP == OP_SV) {
    p = put_vu_g(o, p, cnt);
    for (uint32_t s = 0; s < nsec; s++) {
      const uint32_t v = sv_val(s);
      if (v) { p = put_vu_g(o, p, S[s].client); p = put_vu_g(o, p, v); }
    }
  } else {
    p = put_vu_g(o, p, nsec);
    for (uint32_t s = 0; s < nsec; s++) { p = put_vu_g(o, p, S[s].client); p = put_vu_g(o, p, S[s].clock); }
    p = put_vu_g(o, p, nsec);
    for (uint32_t s = 0; s < nsec; s++) { p = put_vu_g(o, p, S[s].client); p = put_vu_g(o, p, sec_end(s)); }
  }
  j.out_off[d] = b;
  j.out_len[d] = total;
  j.status[d] = ym::ST_OK;
#undef MS_DECLINE
}

// ---- K3: columns ----------------------------------------------------------------------------------------
// an input entry with its value index and (IntDiff) running value before it
struct EW {
  uint32_t pos, end, idx, cnt, val;
  int32_t df;
  int64_t vr;
  bool ok;
};
__device__ __forceinline__ EW ew_at(const uint8_t *D, uint32_t kind, uint32_t c1, uint32_t tot, uint32_t pos, uint32_t idx, int64_t vr) {
  EW w{pos, c1, idx, 0, 0, 0, vr, false};
  if (pos >= c1 || idx >= tot) return w;
  const Ent e = dec_entry(D, pos, c1, kind);
  if (e.bad) return w;
  w.cnt = e.fin ? tot - idx : e.cnt;
  w.val = e.val;
  w.df = e.df;
  w.end = e.end;
  w.ok = w.cnt > 0 && w.end > pos;
  return w;
}
__device__ __forceinline__ EW ew_next(const uint8_t *D, uint32_t kind, uint32_t c1, uint32_t tot, const EW &w) {
  return ew_at(D, kind, c1, tot, w.end, w.idx + w.cnt, w.vr + (int64_t)w.df * w.cnt);
}
__device__ __forceinline__ uint32_t ew_value(uint32_t kind, const EW &w, uint32_t x) {
  return k_dif(kind) ? (uint32_t)(w.vr + (int64_t)w.df * (x - w.idx + 1)) : w.val;
}
// the entry holding value x: K1's last checkpoint at or before it, then at most CKSTEP entries
__device__ __forceinline__ EW locate(const Job &J, const Meta &M, const uint8_t *D, uint32_t kind, uint32_t c0, uint32_t c1,
                                     uint32_t tot, uint32_t x) {
  const uint4 *ck = a_ck(J, M, kind);
  uint32_t lo = 0, hi = M.nck[kind];
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ck[mid].y <= x) lo = mid; else hi = mid;
  }
  uint32_t pos = c0, idx = 0;
  int64_t vr = 0;
  if (M.nck[kind] > 0) {
    const uint4 c4 = ck[lo];
    pos = c4.x;
    idx = c4.y;
    vr = c4.z;
  }
  EW w{pos, c1, idx, 0, 0, 0, vr, false};
  if (pos < c0 || pos > c1 || idx > x) return w;
  w = ew_at(D, kind, c1, tot, pos, idx, vr);
  for (uint32_t g = 0; g <= 2 * CKSTEP && w.ok && x >= w.idx + w.cnt; g++) w = ew_next(D, kind, c1, tot, w);
  if (w.ok && (x < w.idx || x >= w.idx + w.cnt)) w.ok = false;
  return w;
}
struct Run {
  uint32_t v;
  int32_t d;
  uint32_t c;
};
__device__ __forceinline__ Run clip(uint32_t kind, const EW &w, uint32_t lo, uint32_t hi) {
  const uint32_t a = lo > w.idx ? lo : w.idx, b = hi < w.idx + w.cnt ? hi : w.idx + w.cnt;
  return Run{ew_value(kind, w, a), k_dif(kind) ? w.df : 0, b > a ? b - a : 0};
}
// a run of c values (v, v + d, ...) into the wave-uniform encoder
__device__ __forceinline__ void feed(Enc &E, Buf &B, uint32_t kind, const Run &r) {
  if (r.c == 0) return;
  E.put(B, kind, r.v);
  if (r.c == 1) return;
  if (k_dif(kind)) {
    const uint32_t last = (uint32_t)((int64_t)r.v + (int64_t)r.d * (r.c - 1));
    if (E.df == r.d && E.cnt > 0) {
      E.cnt += r.c - 1;
    } else {
      E.flush(B, kind);
      E.cnt = r.c - 1;
      E.df = r.d;
    }
    E.s = last;
  } else {
    E.cnt += r.c - 1;
  }
}
// Item.write(encoder, off) / GC.write of the cut struct into column `kind` (v2_write of ym_big2.hip),
// preceded on the client column by the LazyStructWriter's writeClient; fv = the struct's own input values
// of the column, in reading order
__device__ __forceinline__ uint32_t head_vals(uint32_t kind, const Sec &X, const uint32_t *fv, uint32_t nf, uint32_t *hv, bool &bad) {
  const uint32_t info = X.info_f, off = X.off, ref = info & 31;
  const bool gc = ref == 0, item = !gc;
  const bool o = item && (info & 0x80), r = item && (info & 0x40), no = item && !(info & 0xC0);
  const bool has_o = item && (off > 0 || o);
  const bool pinfo = item && !has_o && !r;  // parent info written (implies no origins and off == 0)
  const bool pp = no && X.pi_f != 1, py = no && X.pi_f == 1;
  const bool key = item && ref == 7 && (X.tr_f == 3 || X.tr_f == 5);
  uint32_t nh = 0, fi = 0;
  switch (kind) {
    case K_INFO:
      fi++;
      hv[nh++] = gc ? 0 : (ref | (has_o ? 0x80 : 0) | (info & 0x40) | (no ? (info & 0x20) : 0));
      break;
    case K_CL: {
      const uint32_t oc = o ? fv[fi++] : 0, rc = r ? fv[fi++] : 0, pc = pp ? fv[fi++] : 0;
      hv[nh++] = X.client;
      if (item && off > 0) hv[nh++] = X.client;
      else if (o) hv[nh++] = oc;
      if (r) hv[nh++] = rc;
      if (pinfo && pp) hv[nh++] = pc;
      break;
    }
    case K_LC: {
      const uint32_t ok = o ? fv[fi++] : 0, pk = pp ? fv[fi++] : 0;
      if (item && off > 0) hv[nh++] = X.fclock + off - 1;
      else if (o) hv[nh++] = ok;
      if (pinfo && pp) hv[nh++] = pk;
      break;
    }
    case K_RC:
      if (r) hv[nh++] = fv[fi++];
      break;
    case K_PI:
      if (no) fi++;
      if (pinfo) hv[nh++] = X.pi_f == 1 ? 1 : 0;
      break;
    case K_SL: {
      const uint32_t yk = py ? fv[fi++] : 0, ps = no && (info & 0x20) ? fv[fi++] : 0;
      const bool hc = item && (ref == 4 || ref == 6 || key);
      const uint32_t cs = hc ? fv[fi++] : 0;
      if (pinfo && py) hv[nh++] = yk;
      if (pinfo && (info & 0x20)) hv[nh++] = ps;
      if (item && ref == 4) hv[nh++] = cs - off;
      else if (hc) hv[nh++] = cs;
      break;
    }
    case K_LN:
      if (gc || ref == 1 || ref == 8) { fi++; hv[nh++] = X.clen_f - off; }
      break;
    case K_TR:
      if (item && ref == 7) { fi++; hv[nh++] = X.tr_f; }
      break;
  }
  bad |= fi != nf;
  return nh;
}

constexpr uint32_t NKC = K_KC;  // spliced kinds (the keyClock column is regenerated)
constexpr uint32_t RMAX = 8;    // runs before a span: <= 5 head values + the range's first two entries
__global__ void __launch_bounds__(64) k_ms_col(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x, kind = blockIdx.y, lane = threadIdx.x;
  Meta &M = J.meta[d];
  if (!M.ok || !M.ms) return;
  __shared__ Run sr[64][RMAX + 1];  // [RMAX]: the tail run after the span
  __shared__ uint32_t snr[64], sm0[64], sm1[64], ssm[64], skept[64];
  const uint8_t *D = j.A + j.upd_off[j.doc_upd[d]];
  const uint32_t c0 = M.col0[col_of(kind)], c1 = M.col1[col_of(kind)];
  const uint32_t tot = M.tot[kind], nsec = M.nsec;
  const Sec *S = a_sec(J, M);
  Buf B{a_col(J, M, kind), 0, M.ocap[kind], false};
  B.wr = lane == 0;
  Enc E;
  bool bad = false;
  for (uint32_t s0 = 0; s0 < nsec && !bad && !B.over; s0 += 64) {
    const uint32_t s = s0 + lane;
    // phase A (lane per section): the section's runs and span
    uint32_t nr = 0, m0 = 0, m1 = 0, sm = 0, kept = 0;
    Run tail{0, 0, 0};
    bool lbad = false;
    if (s < nsec && S[s].f != NONE) {
      const Sec &X = S[s];
      kept = 1;
      const uint32_t pf = X.pf[kind], pf1 = X.pf1[kind];
      const uint32_t pe = s + 1 < nsec ? S[s + 1].pre[kind] : tot;
      uint32_t fv[4] = {0, 0, 0, 0};
      const uint32_t nf = pf1 - pf;
      lbad |= pf1 < pf || nf > 4 || pe < pf1 || pe > tot;
      EW w{};
      w.ok = false;
      if (!lbad && nf > 0) {
        w = locate(J, M, D, kind, c0, c1, tot, pf);
        for (uint32_t q = 0; q < nf && w.ok; q++) {
          while (w.ok && pf + q >= w.idx + w.cnt) w = ew_next(D, kind, c1, tot, w);
          fv[q] = ew_value(kind, w, pf + q);
        }
        lbad |= !w.ok;
      }
      uint32_t hv[6];
      const uint32_t nh = lbad ? 0 : head_vals(kind, X, fv, nf, hv, lbad);
      for (uint32_t h = 0; h < nh; h++) sr[lane][nr++] = Run{hv[h], 0, 1};
      if (!lbad && pf1 < pe) {
        EW e1 = (w.ok && pf1 >= w.idx && pf1 < w.idx + w.cnt) ? w
                : (w.ok && pf1 == w.idx + w.cnt) ? ew_next(D, kind, c1, tot, w)
                                                 : locate(J, M, D, kind, c0, c1, tot, pf1);
        lbad |= !e1.ok;
        if (!lbad) {
          sr[lane][nr++] = clip(kind, e1, pf1, pe);
          if (e1.idx + e1.cnt < pe) {
            const EW e2 = ew_next(D, kind, c1, tot, e1);
            lbad |= !e2.ok;
            if (!lbad) {
              sr[lane][nr++] = clip(kind, e2, pf1, pe);
              if (e2.idx + e2.cnt < pe) {
                const EW em = locate(J, M, D, kind, c0, c1, tot, pe - 1);
                lbad |= !em.ok || em.idx < e2.idx + e2.cnt || em.pos < e2.end;
                if (!lbad) {
                  m0 = e2.end;
                  m1 = em.pos;  // the full entries strictly between: verbatim
                  sm = (uint32_t)em.vr;
                  tail = clip(kind, em, pf1, pe);
                }
              }
            }
          }
        }
      }
    }
    snr[lane] = nr;
    sm0[lane] = m0;
    sm1[lane] = m1;
    ssm[lane] = sm;
    skept[lane] = kept;
    sr[lane][RMAX] = tail;
    bad |= __any(lbad);
    __syncthreads();
    // phase B (wave-uniform): the encoder over the sections in order
    const uint32_t nl = nsec - s0 < 64 ? nsec - s0 : 64;
    for (uint32_t l = 0; l < nl && !bad; l++) {
      if (!skept[l]) continue;
      const uint32_t k = snr[l];
      for (uint32_t r = 0; r < k; r++) feed(E, B, kind, sr[l][r]);
      if (sr[l][RMAX].c > 0) {
        const uint32_t a = sm0[l], b = sm1[l];
        if (b > a) {  // the span: the pending run closes, the entries are copied, the tail starts a new run
          E.flush(B, kind);
          if ((uint64_t)B.n + (b - a) > B.cap) { B.over = true; break; }
          wcopy(B.b + B.n, D + a, b - a);
          B.n += b - a;
          E.s = ssm[l];
          E.cnt = 0;
          E.started = 0;
        }
        feed(E, B, kind, sr[l][RMAX]);
      }
    }
    __syncthreads();
  }
  E.flush(B, kind, true);
  if (lane == 0) {
    M.osz[kind] = B.n;
    if (bad || B.over || E.bad) { M.ok = 0; M.why = 60 + kind; }
  }
}

// ---- K4: output -----------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_ms_out(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t lane = threadIdx.x;
  __shared__ wds::DsLds dsl;
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    Meta &M = J.meta[d];
    if (!M.ok || !M.ms) continue;
    const uint32_t u0 = j.doc_upd[d];
    const uint64_t ub = j.upd_off[u0];
    const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
    const uint8_t *D = j.A + ub;
    Sec *S = a_sec(J, M);
    const uint32_t *ist = a_istart(J, M);
    const uint32_t nsec = M.nsec;
    // delete set: readDeleteSet's reads, canonical, no repeated or empty client (then copied); through the
    // LDS token tables, or client by client when those cannot decide
    uint32_t x = wds::ds_validate_lds(D, M.ds0, len, dsl);
    bool bad = x == NONE;
    uint32_t ndc = 0;
    if (x == wds::DS_BIG) {
      x = M.ds0;
      ln::LCur c = ln::make(D, x, len);
      ndc = ln::rvu(c);
      x = c.p;
      bad = c.bad || ndc > 4096;
    }
    uint32_t *dsc = reinterpret_cast<uint32_t *>(j.bscratch + (uint64_t)blockIdx.x * BS_BYTES + BS_DSC);
    uint32_t *map = reinterpret_cast<uint32_t *>(j.bscratch + (uint64_t)blockIdx.x * BS_BYTES + BS_MAP);
    const bool big = !bad && ndc > 64 && ndc <= BS_NDSC;
    if (big) cmap::clear(map);
    for (uint32_t i = 0; i < ndc && !bad; i++) {
      ln::LCur h = ln::make(D, x, len);
      const uint32_t client = ln::rvu(h);
      const uint32_t m = ln::rvu(h);
      x = h.p;
      if (h.bad || m == 0 || i >= BS_NDSC) { bad = true; break; }
      bool hit = false;
      if (big) hit = cmap::seen_insert(map, client);
      else for (uint32_t h0 = 0; h0 < i; h0 += 64) hit |= __any(h0 + lane < i && dsc[h0 + lane] == client);
      if (hit) { bad = true; break; }
      __syncthreads();
      if (lane == 0) dsc[i] = client;
      __threadfence_block();
      __syncthreads();
      x = wds::skip_varuints(D, x, len, 2ull * m);
      if (x == NONE) bad = true;
    }
    if (bad) { if (lane == 0) { M.ok = 0; M.why = 70; } __syncthreads(); continue; }
    const uint32_t ds1 = x;
    // kept sections: string body piece, rest piece (after the cut struct's skipped ContentAny values)
    uint32_t sbn = 0, rsz = 0, nk = 0;
    for (uint32_t s0 = 0; s0 < nsec && !bad; s0 += 64) {
      const uint32_t s = s0 + lane;
      uint32_t bb = 0, rb = 0;
      bool kept = false, lbad = false;
      if (s < nsec && S[s].f != NONE) {
        const Sec &X = S[s];
        kept = true;
        const uint32_t ref = X.info_f & 31;
        const uint32_t hs0 = X.off == 0 ? X.body_f : ref == 4 ? X.body_fc + X.off : X.body_f1;
        const uint32_t be = s + 1 < nsec ? S[s + 1].body0 : M.body_end;
        lbad |= hs0 > be || be > M.sn || X.body_f > X.body_fc || X.body_fc > X.body_f1;
        const uint32_t ie = s + 1 < nsec ? S[s + 1].ibase : M.nitem;
        uint32_t rs = X.iord_f < ie ? ist[X.iord_f] : X.pay1;
        if (ref == 8 && X.off > 0) {  // ContentAny.splice: the first `off` values are not written
          ln::LCur c = ln::make(D, rs, X.pay1);
          for (uint32_t a = 0; a < X.off && !c.bad; a++) ln::any_canon(c);
          lbad |= c.bad;
          rs = c.p;
        }
        lbad |= rs < X.pay0 || rs > X.pay1 || X.f < X.S || X.f - X.S >= X.W;
        const uint32_t wr = X.W - (X.f - X.S), cw = X.fclock + X.off;
        bb = lbad ? 0 : be - hs0;
        rb = lbad ? 0 : vsz(wr) + vsz(cw) + (X.pay1 - rs);
        S[s].rs = rs;
      }
      const uint32_t ib = wave_incl_add(bb), ir = wave_incl_add(rb);
      if (kept) {
        S[s].ob = sbn + ib - bb;
        S[s].orr = rsz + ir - rb;
      }
      sbn += lane_read(ib, 63);
      rsz += lane_read(ir, 63);
      nk += (uint32_t)__builtin_popcountll(__ballot(kept));
      bad |= __any(lbad);
    }
    bad |= nk != M.nkept;
    __threadfence_block();  // the lanes' per-section offsets, read by the whole wave below
    __syncthreads();
    if (bad) { if (lane == 0) { M.ok = 0; M.why = 71; } __syncthreads(); continue; }
    // column sizes: keyClock 0, 1, 2, ... = IntDiff runs (diff 0 x1)(diff 1 x K-1): 00 | 00 02 | 00 03 vu(K-3)
    const uint32_t K = M.kc_out;
    uint32_t cl[9];
    cl[0] = K == 0 ? 0 : K == 1 ? 1 : K == 2 ? 2 : 2 + vsz(K - 3);
    for (uint32_t k = 0; k < NKC; k++)
      if (k != K_SL) cl[col_of(k)] = M.osz[k];
    cl[5] = vsz(sbn) + sbn + M.osz[K_SL];
    uint32_t total = 1;
    for (uint32_t c = 0; c < 9; c++) total += vsz(cl[c]) + cl[c];
    total += vsz(nk) + rsz + (ds1 - M.ds0);
    uint64_t b = 0;
    if (lane == 0) b = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    b = ((uint64_t)lane_read((uint32_t)(b >> 32), 0) << 32) | lane_read((uint32_t)b, 0);
    if (lane == 0) { J.done[d] = 1; atomicAdd((unsigned long long *)j.pw_count, 1ull); }
    if (b + total > j.cap) {
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    uint8_t *o = j.out + b;
    auto put = [&](uint32_t p, uint32_t v) -> uint32_t {
      if (lane == 0) put_vu_g(o, p, v);
      return p + vsz(v);
    };
    uint32_t p = put(0, 0);
    for (uint32_t c = 0; c < 9; c++) {
      p = put(p, cl[c]);
      if (c == 0) {
        if (lane == 0 && K >= 1) o[p] = 0;
        if (lane == 0 && K == 2) o[p + 1] = 2;
        if (K >= 3) { if (lane == 0) o[p + 1] = 3; put(p + 2, K - 3); }
        p += cl[0];
        continue;
      }
      if (c == 5) {  // varString(body) | lengths
        p = put(p, sbn);
        for (uint32_t s0 = 0; s0 < nsec; s0 += 64) {  // each lane loads one section's piece, the wave copies them
          const uint32_t s = s0 + lane;
          uint32_t src = 0, dst = 0, n = 0;
          if (s < nsec && S[s].f != NONE) {
            const Sec &X = S[s];
            const uint32_t ref = X.info_f & 31;
            const uint32_t hs0 = X.off == 0 ? X.body_f : ref == 4 ? X.body_fc + X.off : X.body_f1;
            const uint32_t be = s + 1 < nsec ? S[s + 1].body0 : M.body_end;
            src = M.sb0 + hs0;
            dst = X.ob;
            n = be - hs0;
          }
          for (uint64_t m = __ballot(n > 0); m; m &= m - 1) {
            const int l = __builtin_ctzll(m);
            wcopy(o + p + lane_read(dst, l), D + lane_read(src, l), lane_read(n, l));
          }
        }
        p += sbn;
        wcopy(o + p, a_col(J, M, K_SL), M.osz[K_SL]);
        p += M.osz[K_SL];
        continue;
      }
      uint32_t k = 0;
      for (uint32_t q = 0; q < NKC; q++) if (col_of(q) == c) k = q;
      wcopy(o + p, a_col(J, M, k), cl[c]);
      p += cl[c];
    }
    p = put(p, nk);
    for (uint32_t s0 = 0; s0 < nsec; s0 += 64) {  // each lane writes its section's header, the wave copies the payloads
      const uint32_t s = s0 + lane;
      uint32_t src = 0, dst = 0, n = 0;
      bool kept = false;
      if (s < nsec && S[s].f != NONE) {
        const Sec &X = S[s];
        kept = true;
        uint32_t q = put_vu_g(o, p + X.orr, X.W - (X.f - X.S));
        q = put_vu_g(o, q, X.fclock + X.off);
        src = X.rs;
        dst = q;
        n = X.pay1 - X.rs;
      }
      (void)kept;
      for (uint64_t m = __ballot(n > 0); m; m &= m - 1) {
        const int l = __builtin_ctzll(m);
        wcopy(o + lane_read(dst, l), D + lane_read(src, l), lane_read(n, l));
      }
    }
    p += rsz;
    wcopy(o + p, D + M.ds0, ds1 - M.ds0);
    if (lane == 0) {
      j.out_off[d] = b;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}

// ---- host launchers (pv2_run, ym_pv2.hip) -------------------------------------------------------------------
void ms_rest(const Job &J, hipStream_t st) {
  k_ms_rest<<<J.j.n, MR_T, 0, st>>>(J);
  k_ms_walk<<<J.j.n, 64, 0, st>>>(J);
}
void ms_sizes(const Job &J, uint64_t *sizes, hipStream_t st) { k_ms_sizes_k<<<(J.j.n + 255) / 256, 256, 0, st>>>(J, sizes); }
void ms_run(uint32_t op, const Job &J, hipStream_t st) {
  const uint32_t n = J.j.n;
  if (op == OP_DIFF) {
    k_ms_struct<OP_DIFF><<<n, KT, 0, st>>>(J);
    k_ms_col<<<dim3(n, NKC), 64, 0, st>>>(J);
    k_ms_out<<<n < BS_GRID ? n : BS_GRID, 64, 0, st>>>(J);
  } else if (op == OP_SV) {
    k_ms_struct<OP_SV><<<n, KT, 0, st>>>(J);
  } else {
    k_ms_struct<OP_META><<<n, KT, 0, st>>>(J);
  }
}

}  // namespace pv2
}  // namespace ymk

extern "C" int ym__ms_prof(unsigned long long *host, int reset) {
  int r = (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ymk::pv2::ms_prof), 128);
  if (reset) { unsigned long long z[16] = {}; hipMemcpyToSymbol(HIP_SYMBOL(ymk::pv2::ms_prof), z, 128); }
  return r;
}
