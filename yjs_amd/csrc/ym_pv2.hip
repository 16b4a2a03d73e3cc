// ym_pv2.hip -- column-parallel diffUpdateV2 / encodeStateVectorFromUpdateV2 over large single-section
// V2 updates (BASELINE configs[2] C3 in V2: one client, ~70 k String / Deleted Items per 0.47 MB update).
//
// The V2 encoding spreads every struct over up to nine RLE columns (UpdateEncoder.js:229-408); the
// sequential walker (ym_big2.hip) advances all of them struct by struct.  Here each column is an
// independent stream:
//
//  K0 k_v2_prep   one thread per document: the header (column spans, the section header), eligibility
//                 (one update, one client section), the scratch size.
//  K1 k_v2_decw   one wave per (document, column): the lib0 RLE decoders (RleDecoder<u8>,
//                 UintOptRleDecoder, IntDiffOptRleDecoder) parallelised by an automaton tokeniser whose
//                 per-lane transition functions a wave prefix scan composes; every entry checked to be in
//                 the form lib0's encoder writes (canonical varints, runs maximal, no -0 diff, diffs < 2^30,
//                 parentInfo in {0, 1}, an RLE<u8> column ending without a count); info / parentInfo /
//                 string lengths / len values expanded into per-value arrays, the others only counted;
//                 a checkpoint (entry position, value index, running value) every CKSTEP entries.
//  K2 k_v2_struct one 256-thread block per document: per struct the values it consumes from every
//                 column (from its info byte and parentInfo), block prefix sums over the structs give each
//                 struct's column indices, its clock length and clock; the diff cut is the first struct
//                 ending past sv[client]; every column must be consumed exactly (as the re-encoding would
//                 write it).  encodeStateVectorFromUpdateV2 is answered here.
//  K3 k_v2_splice one lane per (document, column): the cut struct's values, re-encoded (Item.write with
//                 offset) with the rest of the column entry they share, by the lib0 encoders; the column's
//                 following entries are then byte-identical to what the encoder would write (the input is
//                 canonical), so they are copied.
//  K4 k_v2_out    one wave per document: the delete set validated (readDeleteSet), the output assembled:
//                 vu(0) | 9 x varUint8Array(column) | vu(#parts) | vu(written) vu(first clock) | delete set.
//
// Exactly the documents ym_big2.hip's k_big_v2 accepts among these are taken, with identical bytes;
// everything else (several clients, Skip / Any / Type / Format / Embed / Binary content, non-ASCII string
// columns, non-canonical columns) is left to k_big_v2 (and from there to the general path).
#include <hip/hip_runtime.h>
#include "ym_scan.h"

#include "ym_pv2.h"
#include "ym_cmap.h"
#include "ym_wave_ds.h"

namespace ymk {
namespace pv2 {
using namespace fastc;

// ---- K0: header ---------------------------------------------------------------------------------------
// sizes[d]: the document's value-array scratch (single section; multi-section documents get theirs after
// the rest walk counted their structs, ms_sizes); sizes1[d]: the multi-section tables.
__global__ void k_v2_prep(Job J, uint64_t pv_min, uint64_t *sizes, uint64_t *sizes1) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d > j.n) return;
  if (d == j.n) { sizes[d] = 0; sizes1[d] = 0; return; }
  Meta &M = J.meta[d];
  M.ok = 0;
  M.why = 1;
  M.ms = 0;
  J.done[d] = 0;
  sizes[d] = 0;
  sizes1[d] = 0;
  const uint32_t u0 = j.doc_upd[d];
  if (j.doc_upd[d + 1] - u0 != 1) return;
  const uint64_t ub = j.upd_off[u0], len64 = j.upd_off[u0 + 1] - ub;
  if (len64 < pv_min || len64 == 0 || len64 >= (1ull << 28)) return;
  const uint32_t len = (uint32_t)len64;
  const uint8_t *D = j.A + ub;
  ln::LCur c = ln::make(D, 0, len);
  ln::rvu(c);  // feature flag
  for (uint32_t k = 0; k < 9; k++) {
    const uint32_t n = ln::rvu(c);
    M.col0[k] = c.p;
    if (c.bad || (uint64_t)c.p + n > len) return;
    M.col1[k] = c.p + n;
    c = ln::make(D, c.p + n, len);
  }
  const uint32_t nclients = ln::rvu(c);
  if (c.bad || nclients == 0 || nclients > (1u << 16)) return;
  M.nsec = nclients;
  M.r0 = c.p;
  // string column = varString(body) | UintOptRle(lengths)
  ln::LCur s = ln::make(D, M.col0[5], M.col1[5]);
  const uint32_t sn = ln::rvu(s);
  if (s.bad || (uint64_t)s.p + sn > M.col1[5]) return;
  M.sb0 = s.p;
  M.sn = sn;
  M.col0[5] = s.p + sn;  // lengths part
  if (nclients > 1) {  // several client sections: ym_pv2ms.hip (tables sized by the rest stream's bytes)
    M.ms = 1;
    M.n = 0;
    M.ok = 1;
    M.why = 0;
    sizes1[d] = ms_scr1_bytes(nclients, len, M.r0, M.col1[8] - M.col0[8]);  // (Sec holds a u64 atomic)
    return;
  }
  // typeRef / keyClock unused by the kinds the single-section path takes
  if (M.col1[0] != M.col0[0] || M.col1[7] != M.col0[7]) return;
  const uint32_t nstructs = ln::rvu(c);
  const uint32_t clock = ln::rvu(c);
  if (c.bad || nstructs == 0 || nstructs > (1u << 26)) return;
  M.ds0 = c.p;
  M.n = nstructs;
  M.clock0 = clock;
  M.ok = 1;
  M.why = 0;
  uint32_t colb[NK];
  for (uint32_t k = 0; k < NK; k++) colb[k] = M.col1[col_of(k)] - M.col0[col_of(k)];
  sizes[d] = (scr_layout(M, nstructs, 1, false, colb) + 255) & ~255ull;
}

__global__ void k_v2_meta_off(Job J, const uint64_t *offs, uint32_t which) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= J.j.n) return;
  if (which) J.meta[d].soff1 = offs[d];
  else J.meta[d].soff = offs[d];
}

// ---- K1, wave-parallel: one wave per (document, column) ---------------------------------------------
// A column is tokenised 1 KB per wave step (16 bytes per lane) by a finite automaton whose per-lane
// transition functions are composed by a wave prefix scan, so every lane knows the state at its first
// byte without a sequential pass.  RleDecoder<u8>: 0 = at a value byte, 1 = in a count varuint.
// UintOptRle / IntDiffOptRle: 0 = at a value varint, 1 / 2 = inside one that has / has not a count
// (the flag: the sign bit, bit 6 of the first byte, resp. bit 0 of the magnitude), 3 = in a count.
// Entries start where the state is 0; each lane decodes the entries starting in its bytes, and wave
// scans give their entry / value indices and (IntDiff) running values.  Checks: canonical
// varints, maximal runs, no -0 diff, diffs < 2^30, values in [0, 2^32), parentInfo in {0, 1},
// an RLE<u8> column ending without a count.
__global__ void __launch_bounds__(64) k_v2_decw(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x, kind = blockIdx.y, lane = threadIdx.x;
  Meta &M = J.meta[d];
  if (!M.ok) return;
  const uint8_t *D = j.A + j.upd_off[j.doc_upd[d]];
  const uint32_t c0 = M.col0[col_of(kind)], c1 = M.col1[col_of(kind)];
  const uint32_t n = M.n;
  const bool rle = k_rle(kind), dif = k_dif(kind);
  const uint32_t fb = dif ? 0 : 6;
  const uint64_t cap = kind_cap(kind, n, M.nsec);
  // expanded per-value arrays: info / parentInfo / typeRef (u8), string lengths / len (u32), and for
  // multi-section documents the client column (each section's client)
  uint8_t *o8 = kind == K_INFO ? a_info(J, M) : kind == K_PI ? a_pi(J, M) : kind == K_TR ? a_tr(J, M) : nullptr;
  uint32_t *o32 = kind == K_SL ? a_sl(J, M) : kind == K_LN ? a_ln(J, M) : kind == K_CL && M.ms ? a_cl(J, M) : nullptr;
  uint4 *ck = a_ck(J, M, kind);
  const uint32_t ckcap = (c1 - c0) / CKSTEP + 2;
  uint32_t st = 0, ne = 0, fin = 0, finv = 0;  // carried across steps (wave-uniform)
  uint64_t nv = 0;
  int64_t vrun = 0;      // IntDiff: value before the next entry
  uint32_t last = 0;     // the previous entry's value (Opt / RLE) or diff (IntDiff) ...
  bool have_last = false;  // ... if any
  bool bad = false;
  for (uint32_t x = c0; x < c1 && !bad; x += 1024) {
    const uint32_t q = x + 16 * lane;
    uint8_t b[16];
    {
      const uint4 v4 = wds::load16m(D, q, c1);
      __builtin_memcpy(b, &v4, 16);
    }
    uint32_t s0 = 0, s1 = 1, s2 = 2, s3 = 3;  // the lane's transition function (bytes past the column: identity)
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
      if (q + k < c1) { s0 = tstep(s0, b[k], rle, fb); s1 = tstep(s1, b[k], rle, fb); s2 = tstep(s2, b[k], rle, fb); s3 = tstep(s3, b[k], rle, fb); }
    }
    const uint32_t f = s0 | (s1 << 2) | (s2 << 4) | (s3 << 6);
    const uint32_t incl = wave_incl_compose(f);
    const uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp((int)F_ID, (int)incl, 0x138, 0xf, 0xf, false);
    uint32_t sl = (excl >> (2 * st)) & 3;  // state at the lane's first byte
    uint32_t starts = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
      if (q + k < c1) {
        if (sl == 0) starts |= 1u << k;
        sl = tstep(sl, b[k], rle, fb);
      }
    }
    // pass 1: the lane's entries: counts, first / last key, diff sum, checks
    uint32_t lne = 0, lfirst = 0, llast = 0, lfinv = 0;
    uint64_t lnv = 0;
    int64_t lsum = 0;
    bool lbad = false, lfin = false;
    for (uint32_t m = starts; m; m &= m - 1) {
      const Ent e = dec_entry(D, q + __builtin_ctz(m), c1, kind);
      const uint32_t key = dif ? (uint32_t)e.df : e.val;
      lbad |= e.bad || (lne > 0 && key == llast) || e.cnt > cap || (kind == K_TR && e.val > 6);
      if (e.fin) { lfin = true; lfinv = e.val; }
      if (lne == 0) lfirst = key;
      llast = key;
      lne++;
      lnv += e.cnt;
      lsum += (int64_t)e.df * e.cnt;
    }
    // the entry before the lane's first: the nearest lower lane with entries, else the last step's
    const uint64_t has = __ballot(lne > 0);
    const uint64_t below = has & ((1ull << lane) - 1);
    const int src = below ? 63 - __builtin_clzll(below) : (int)lane;
    const uint32_t pk = (uint32_t)__shfl((int)llast, src);
    lbad |= lne > 0 && (below ? pk == lfirst : (have_last && last == lfirst));
    const uint32_t ne_incl = wave_incl_add(lne);
    const uint64_t nv_incl = wave_incl_add64(lnv);
    const uint64_t sum_incl = wave_incl_add64((uint64_t)lsum);
    uint32_t ei = ne + ne_incl - lne;
    uint64_t vbase = nv + nv_incl - lnv;
    int64_t vr = vrun + (int64_t)(sum_incl - (uint64_t)lsum);
    lbad |= vbase + lnv > cap || (lne > 0 && (ei + lne - 1) / CKSTEP >= ckcap);
    // pass 2: checkpoints, IntDiff ranges, expansions
    if (!__any(lbad)) {
      for (uint32_t m = starts; m; m &= m - 1) {
        const uint32_t pos = q + __builtin_ctz(m);
        const Ent e = dec_entry(D, pos, c1, kind);
        if ((ei & (CKSTEP - 1)) == 0) ck[ei / CKSTEP] = make_uint4(pos, (uint32_t)vbase, (uint32_t)vr, 0);
        if (kind == K_CL && ei == 0) M.client = e.val;  // the section header's client
        if (dif) {
          const int64_t vfirst = vr + e.df, vlast = vr + (int64_t)e.df * e.cnt;
          lbad |= vfirst < 0 || vfirst > 0xffffffffll || vlast < 0 || vlast > 0xffffffffll;
          // keyClock: readKey reads a new key string only when keyClock >= the keys read so far (value i
          // >= i for every i; linear inside an entry, so its two ends decide)
          if (kind == K_KC) lbad |= vfirst < (int64_t)vbase || vlast < (int64_t)(vbase + e.cnt - 1);
          vr = vlast;
        }
        if (vbase + e.cnt <= cap) {
          if (o8) for (uint32_t i = 0; i < e.cnt; i++) o8[vbase + i] = (uint8_t)e.val;
          if (o32) for (uint32_t i = 0; i < e.cnt; i++) o32[vbase + i] = e.val;
        }
        vbase += e.cnt;
        ei++;
      }
    }
    bad |= __any(lbad);
    const uint64_t fm = __ballot(lfin);
    if (fm) {  // the final RLE entry ends the column
      fin = 1;
      finv = (uint32_t)__shfl((int)lfinv, 63 - __builtin_clzll(fm));
    }
    st = (lane_read(incl, 63) >> (2 * st)) & 3;
    ne += lane_read(ne_incl, 63);
    nv += lane_read64(nv_incl, 63);
    vrun += (int64_t)lane_read64(sum_incl, 63);
    if (has) {
      last = (uint32_t)__shfl((int)llast, 63 - __builtin_clzll(has));
      have_last = true;
    }
  }
  if (!bad && kind == K_INFO) {  // the endless final run fills the structs left
    if (!fin && nv != n) bad = true;
    if (fin && nv <= n)
      for (uint64_t i = nv + lane; i < n; i += 64) o8[i] = (uint8_t)finv;
    else if (fin) bad = true;
  }
  if (lane == 0) {
    if (bad) { M.ok = 0; M.why = 10 + kind; }
    M.nval[kind] = (uint32_t)nv;
    M.nck[kind] = (ne + CKSTEP - 1) / CKSTEP;
    M.fin[kind] = fin;
    M.finv[kind] = finv;
  }
}

// ---- K2: struct pass ------------------------------------------------------------------------------------
constexpr uint32_t NK1 = K_TR;     // single section: the seven kinds a GC / Deleted / String struct uses
template <int OP>
__global__ void __launch_bounds__(KT) k_v2_struct(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  Meta &M = J.meta[d];
  if (!M.ok || M.ms) return;
  __shared__ uint32_t sh[4 * 16];
  __shared__ uint32_t s_bad, s_cut;
  __shared__ uint64_t s_clock;
  const uint8_t *D = j.A + j.upd_off[j.doc_upd[d]];
  const uint32_t n = M.n;
  // the state vector's clock for the client (decodeStateVector: a later entry wins)
  uint32_t k = 0;
  if (OP == OP_DIFF) {
    if (t == 0) {
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      ln::LCur c = ln::make(j.sv + s0, 0, (uint32_t)(s1 - s0));
      const uint32_t ns = s1 - s0 > (1u << 20) ? NONE : ln::rvu(c);
      bool bad = ns == NONE;
      for (uint32_t i = 0; i < ns && !bad; i++) {
        const uint32_t cl = ln::rvu(c), ck = ln::rvu(c);
        bad |= c.bad;
        if (!bad && cl == M.client) k = ck;
      }
      s_bad = bad || c.bad;
      s_cut = k;
    }
    __syncthreads();
    if (s_bad) { if (t == 0) { M.ok = 0; M.why = 20; } return; }
    k = s_cut;
  }
  // the body must be ASCII (a UTF-16 slice is then a byte slice; k_big_v2's condition)
  {
    bool na = false;
    for (uint32_t i = 16 * t; i < M.sn; i += 16 * KT) {
      uint8_t b[16];
      const uint32_t m = M.sn - i < 16 ? M.sn - i : 16;
      for (uint32_t q = 0; q < m; q++) b[q] = D[M.sb0 + i + q];
      for (uint32_t q = 0; q < m; q++) na |= b[q] >= 0x80;
    }
    if (__syncthreads_or(na)) { if (t == 0) { M.ok = 0; M.why = 21; } return; }
  }
  // the section client: the client column's first value (uopt_read)
  if (M.nval[K_CL] == 0) { if (t == 0) { M.ok = 0; M.why = 22; } return; }
  const uint8_t *info_a = a_info(J, M), *pi_a = a_pi(J, M);
  const uint32_t *sl_a = a_sl(J, M), *ln_a = a_ln(J, M);
  // running column indices (carried across tiles): [K_INFO .. K_RC] + string body bytes
  uint32_t base[NK1 + 1];
#pragma unroll
  for (uint32_t q = 0; q <= NK1; q++) base[q] = 0;
  base[K_CL] = 1;  // the section header's client
  uint64_t clock = M.clock0;
  uint32_t cut = NONE;
  if (t == 0) s_bad = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += TILE) {
    // per struct: values consumed of each kind (no Skip / Any / Type ...: only GC, Deleted, String)
    uint32_t cons[PER][NK1], info[PER], pi[PER];
    uint32_t x[NK1 + 2];  // per-thread sums: kinds, body bytes, clock
#pragma unroll
    for (uint32_t q = 0; q < NK1 + 2; q++) x[q] = 0;
    bool bad = false;
#pragma unroll
    for (uint32_t e = 0; e < PER; e++) {
      const uint32_t i = t0 + t * PER + e;
      const uint32_t v = i < n ? info_a[i] : 0;
      info[e] = v;
      const uint32_t ref = v & 31;
      const bool valid = i < n;
      const bool gc = valid && ref == 0 && v != 10;
      const bool item = valid && !gc;
      bad |= valid && (v == 10 || (item && ref != 1 && ref != 4));
      // written back as GC.write / Item.write would (13.5.16 lazy reader: parentSub only without
      // origins): a GC info byte with flags, or a parentSub bit next to an origin, would change
      bad |= gc && v != 0;
      bad |= item && (v & 0xC0) && (v & 0x20);
      const bool o = item && (v & 0x80), r = item && (v & 0x40), no = item && !(v & 0xC0);
      cons[e][K_INFO] = valid;
      cons[e][K_PI] = no;
      cons[e][K_RC] = r;
      cons[e][K_LN] = gc || (item && ref == 1);
      pi[e] = 0;  // parentInfo value: looked up after the scan (needs the index)
      cons[e][K_CL] = o + r;
      cons[e][K_LC] = o;
      cons[e][K_SL] = (item && ref == 4) + (no && (v & 0x20));
#pragma unroll
      for (uint32_t q = 0; q < NK1; q++) x[q] += cons[e][q];
    }
    // parentInfo index first (the others depend on its values)
    {
      uint32_t xp[1] = {x[K_PI]}, tp[1];
      block_scan<1>(xp, tp, sh);
      uint32_t pidx = base[K_PI] + xp[0];
#pragma unroll
      for (uint32_t e = 0; e < PER; e++) {
        if (cons[e][K_PI]) {
          const uint32_t pv = pidx < M.nval[K_PI] ? pi_a[pidx] : M.finv[K_PI];
          bad |= pidx >= M.nval[K_PI] && !M.fin[K_PI];
          pi[e] = pv;
          // readParentInfo: 1 -> a ykey string, else a parent ID (client, clock)
          cons[e][K_SL] += pv == 1;
          cons[e][K_CL] += pv != 1;
          cons[e][K_LC] += pv != 1;
          x[K_SL] += pv == 1;
          x[K_CL] += pv != 1;
          x[K_LC] += pv != 1;
          pidx++;
        }
      }
      base[K_PI] += tp[0];
    }
    // indices of every kind
    uint32_t tot[NK1];
    uint32_t xs[NK1];
#pragma unroll
    for (uint32_t q = 0; q < NK1; q++) xs[q] = x[q];
    block_scan<NK1>(xs, tot, sh);
    // string lengths -> body bytes, clock lengths
    uint32_t sli = base[K_SL] + xs[K_SL], lni = base[K_LN] + xs[K_LN];
    uint32_t clen[PER], bodyb[PER];
    x[NK1] = 0;
    x[NK1 + 1] = 0;
#pragma unroll
    for (uint32_t e = 0; e < PER; e++) {
      uint32_t bl = 0;
      for (uint32_t s = 0; s < cons[e][K_SL]; s++) bl += sli + s < M.nval[K_SL] ? sl_a[sli + s] : 0;
      const uint32_t ref = info[e] & 31;
      uint32_t cl = 0;
      if (cons[e][K_INFO]) {
        if (cons[e][K_LN]) cl = lni < M.nval[K_LN] ? ln_a[lni] : 0;
        else cl = sli + cons[e][K_SL] - 1 < M.nval[K_SL] ? sl_a[sli + cons[e][K_SL] - 1] : 0;  // ContentString: last
        bad |= (ref == 1 || ref == 4) && info[e] != 0 && cl == 0;  // Item length 0
        bad |= cl >= (1u << 20);  // keeps the block's clock sums in u32
      }
      clen[e] = cl;
      bodyb[e] = bl;
      x[NK1] += bl;
      x[NK1 + 1] += cl;
      sli += cons[e][K_SL];
      lni += cons[e][K_LN];
    }
    uint32_t xb[2] = {x[NK1], x[NK1 + 1]}, tb[2];
    block_scan<2>(xb, tb, sh);
    // the cut: first struct (non-Skip) whose end passes sv[client]
    uint64_t ck = clock + xb[1];
    uint32_t mycut = NONE;
#pragma unroll
    for (uint32_t e = 0; e < PER; e++) {
      const uint32_t i = t0 + t * PER + e;
      if (i < n && OP == OP_DIFF && mycut == NONE && cut == NONE && ck + clen[e] > k) mycut = e;
      if (mycut == NONE) ck += clen[e];
    }
    if (t == 0) s_cut = NONE;
    __syncthreads();
    if (mycut != NONE) atomicMin(&s_cut, t0 + t * PER + mycut);
    bad |= clock + tb[1] > 0xffffffffull;
    if (__syncthreads_or(bad)) { if (t == 0) { M.ok = 0; M.why = 23; } return; }
    const uint32_t tc = s_cut;
    if (tc != NONE && cut == NONE && mycut != NONE && tc == t0 + t * PER + mycut) {  // the thread holding the cut records it
      const uint32_t e = mycut;
      uint32_t pre[NK1], pre1[NK1];
#pragma unroll
      for (uint32_t q = 0; q < NK1; q++) {
        pre[q] = base[q] + xs[q];
        for (uint32_t e2 = 0; e2 < e; e2++) pre[q] += cons[e2][q];
        pre1[q] = pre[q] + cons[e][q];
        M.pf[q] = pre[q];
        M.pf1[q] = pre1[q];
      }
      uint32_t bo = base[NK1] + xb[0];
      for (uint32_t e2 = 0; e2 < e; e2++) bo += bodyb[e2];
      M.body_f = bo;
      M.body_f1 = bo + bodyb[e];
      M.body_fc = (info[e] & 31) == 4 && info[e] != 0 ? bo + bodyb[e] - clen[e] : bo + bodyb[e];
      uint64_t cf = clock + xb[1];
      for (uint32_t e2 = 0; e2 < e; e2++) cf += clen[e2];
      M.f = tc;
      M.off = k > cf ? (uint32_t)(k - cf) : 0;
      M.fclock_lo = (uint32_t)cf;
      M.info_f = info[e];
      M.pi_f = pi[e];
      M.clen_f = clen[e];
    }
    if (tc != NONE) cut = tc;
#pragma unroll
    for (uint32_t q = 0; q < NK1; q++) base[q] += tot[q];
    base[NK1] += tb[0];
    clock += tb[1];
    __syncthreads();
  }
  if (t != 0) return;
  // every column consumed exactly as the re-encoding writes it; strings inside the body
  bool bad = false;
#pragma unroll
  for (uint32_t q = 0; q < NK1; q++) {
    if (q == K_INFO || q == K_PI) bad |= M.fin[q] ? base[q] < M.nval[q] + 1 : base[q] != M.nval[q];
    else bad |= base[q] != M.nval[q];
    M.tot[q] = base[q];
  }
  bad |= base[NK1] > M.sn;
  M.body_end = base[NK1];
  if (bad) { M.ok = 0; M.why = 24; return; }
  if (cut == NONE) M.f = NONE;
  if (OP == OP_SV) {
    // encodeStateVectorFromUpdateV2: one section, no Skip -> (client, end) unless the section does not
    // start at clock 0 (then nothing is known) or ends at 0
    const uint32_t end = M.clock0 == 0 ? (uint32_t)clock : 0;
    const uint32_t total = end ? 1 + vsz(M.client) + vsz(end) : 1;
    const uint64_t b = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    J.done[d] = 1;
    atomicAdd((unsigned long long *)j.pw_count, 1ull);
    if (b + total > j.cap) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; return; }
    uint8_t *o = j.out + b;
    if (end) { o[0] = 1; uint32_t p = 1; for (uint32_t v : {M.client, end}) { while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[p++] = (uint8_t)v; } }
    else o[0] = 0;
    j.out_off[d] = b;
    j.out_len[d] = total;
    j.status[d] = ym::ST_OK;
  }
  if (OP == OP_META) {
    // parseUpdateMetaV2 of one section with structs: from = {client: first clock}, to = {client: end}
    const uint32_t end = (uint32_t)clock;
    const uint32_t total = 2 + 2 * vsz(M.client) + vsz(M.clock0) + vsz(end);
    const uint64_t b = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    J.done[d] = 1;
    atomicAdd((unsigned long long *)j.pw_count, 1ull);
    if (b + total > j.cap) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; return; }
    uint8_t *o = j.out + b;
    uint32_t p = 0;
    for (uint32_t v : {1u, M.client, M.clock0, 1u, M.client, end}) { while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[p++] = (uint8_t)v; }
    j.out_off[d] = b;
    j.out_len[d] = total;
    j.status[d] = ym::ST_OK;
  }
}

// ---- K3: splice heads ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_v2_splice(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t d = blockIdx.x * 64 + threadIdx.x, kind = blockIdx.y;
  if (d >= j.n) return;
  Meta &M = J.meta[d];
  if (!M.ok || M.ms || M.f == NONE) return;
  const uint8_t *D = j.A + j.upd_off[j.doc_upd[d]];
  const uint32_t c0 = M.col0[col_of(kind)], c1 = M.col1[col_of(kind)];
  const uint32_t q0 = M.pf[kind], q1 = M.pf1[kind], tot = M.tot[kind];
  // walk the column's entries up to the one holding value q1; collect the cut struct's values [q0, q1)
  uint32_t fv[4] = {0, 0, 0, 0};
  uint32_t idx = 0, p = c0, vstart = c1;
  uint32_t rem_v = 0, rem_n = 0;  // the entry holding q1: its value (first value at q1 for diffs) and values from q1 on
  int32_t rem_df = 0;
  bool have_rem = false;
  int64_t v = 0;  // IntDiff running value
  {  // resume at K1's last checkpoint at or before value q0 (binary search)
    const uint4 *ck = a_ck(J, M, kind);
    uint32_t lo = 0, hi = M.nck[kind];
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ck[mid].y <= q0) lo = mid; else hi = mid;
    }
    if (M.nck[kind] > 0) {
      const uint4 c4 = ck[lo];
      p = c4.x;
      idx = c4.y;
      v = c4.z;
    }
  }
  bool gbad = p < c0 || p > c1;  // guards: a resume point or entry outside the column declines
  while (idx < tot && !gbad) {
    if (p >= c1) { gbad = true; break; }
    uint32_t ev, cnt, entry_end;
    int32_t df = 0;
    if (kind == K_INFO || kind == K_PI) {
      ev = D[p];
      if (p + 1 >= c1) { cnt = tot - idx; entry_end = c1; }
      else { ln::LCur c = ln::make(D, p + 1, c1); cnt = ln::rvu(c) + 1; entry_end = c.p; }
    } else {
      ln::LCur c = ln::make(D, p, c1);
      bool neg;
      const uint32_t m = rvi(c, neg);
      if (kind == K_LC || kind == K_RC) {
        const int32_t tt = neg ? -(int32_t)m : (int32_t)m;
        df = tt >> 1;
        cnt = (tt & 1) ? ln::rvu(c) + 2 : 1;
      } else {
        cnt = neg ? ln::rvu(c) + 2 : 1;
      }
      ev = m;
      entry_end = c.p;
    }
    if (cnt == 0 || entry_end <= p || entry_end > c1) { gbad = true; break; }
    // values idx .. idx + cnt - 1 of this entry
    for (uint32_t q = q0; q < q1; q++)
      if (q >= idx && q < idx + cnt) {
        const uint32_t val = (kind == K_LC || kind == K_RC) ? (uint32_t)(v + (int64_t)df * (q - idx + 1)) : ev;
        fv[q - q0] = val;
      }
    if (q1 < idx + cnt && q1 >= idx) {
      have_rem = true;
      rem_n = idx + cnt - q1;
      rem_df = df;
      rem_v = (kind == K_LC || kind == K_RC) ? (uint32_t)(v + (int64_t)df * (q1 - idx + 1)) : ev;
      vstart = entry_end;
      if (kind == K_LC || kind == K_RC) v += (int64_t)df * cnt;
      idx += cnt;
      break;
    }
    if (kind == K_LC || kind == K_RC) v += (int64_t)df * cnt;
    idx += cnt;
    p = entry_end;
  }
  // Item.write(encoder, off) of the cut struct (v2_write), preceded for the client column by the
  // LazyStructWriter's writeClient
  const uint32_t info = M.info_f, off = M.off, ref = info & 31;
  const bool gc = ref == 0 && info != 10;
  const bool o = !gc && (info & 0x80), r = !gc && (info & 0x40), no = !gc && !(info & 0xC0);
  const bool has_o = !gc && (off > 0 || o);
  uint32_t hv[6], nh = 0;
  uint32_t fi = 0;  // next of the cut struct's own values
  if (kind == K_INFO) {
    hv[nh++] = gc ? 0 : (ref | (has_o ? 0x80 : 0) | (info & 0x40) | (no && off == 0 ? (info & 0x20) : 0));
  } else if (kind == K_CL) {
    hv[nh++] = M.client;
    if (o) { hv[nh++] = off > 0 ? M.client : fv[fi]; fi++; }
    else if (off > 0 && !gc) hv[nh++] = M.client;
    if (r) hv[nh++] = fv[fi++];
    if (no && M.pi_f != 1) { if (off == 0 && !r) hv[nh++] = fv[fi]; fi++; }
  } else if (kind == K_LC) {
    if (o) { hv[nh++] = off > 0 ? M.fclock_lo + off - 1 : fv[fi]; fi++; }
    else if (off > 0 && !gc) hv[nh++] = M.fclock_lo + off - 1;
    if (no && M.pi_f != 1) { if (off == 0 && !r) hv[nh++] = fv[fi]; fi++; }
  } else if (kind == K_RC) {
    if (r) hv[nh++] = fv[fi++];
  } else if (kind == K_PI) {
    if (no && off == 0 && !r) hv[nh++] = M.pi_f == 1 ? 1 : 0;
  } else if (kind == K_LN) {
    if (gc || ref == 1) hv[nh++] = M.clen_f - off;
  } else {  // K_SL: ykey / parentSub (written only with the parent info) and the content slice
    if (no && M.pi_f == 1) { if (off == 0 && !r) hv[nh++] = fv[fi]; fi++; }
    if (no && (info & 0x20)) { if (off == 0 && !r) hv[nh++] = fv[fi]; fi++; }
    if (ref == 4 && !gc) hv[nh++] = fv[fi] - off;
  }
  if (gbad) { M.ok = 0; M.why = 37; return; }
  uint8_t *hb = M.head[kind];
  Buf B{hb, 0, HB, false};
  Enc E;
  for (uint32_t i = 0; i < nh; i++) E.put(B, kind, hv[i]);
  bool bad = E.bad;
  if (have_rem) {
    // the rest of the entry holding q1: one run in the input; the encoder sees its first value (and for
    // diffs the second, which fixes the run's diff), every further value only extends the run
    const bool dif = kind == K_LC || kind == K_RC;
    E.put(B, kind, rem_v);
    if (rem_n >= 2) {
      if (dif) {
        E.put(B, kind, (uint32_t)((int64_t)rem_v + rem_df));
        E.cnt += rem_n - 2;
        E.s = (uint32_t)((int64_t)rem_v + (int64_t)rem_df * (rem_n - 1));
      } else {
        E.cnt += rem_n - 1;
      }
    }
    bad |= E.bad;
    // The next input entry starts a new run (the input is canonical) -- but the re-encoded head can leave
    // a pending run it continues (a diff equal to the entry's, or the same value): the encoder would merge
    // them, so that entry is re-encoded too (at most twice: after a whole entry the next one differs).
    for (int guard = 0; guard < 2 && vstart < c1 && !bad; guard++) {
      ln::LCur c = ln::make(D, vstart, c1);
      uint32_t nv, ncnt, nend;
      int32_t ndf = 0;
      if (kind == K_INFO || kind == K_PI) {
        nv = D[vstart];
        if (vstart + 1 >= c1) { ncnt = tot - idx; nend = c1; }
        else { ln::LCur cc = ln::make(D, vstart + 1, c1); ncnt = ln::rvu(cc) + 1; nend = cc.p; }
      } else {
        bool neg;
        const uint32_t m = rvi(c, neg);
        nv = m;
        if (kind == K_LC || kind == K_RC) {
          const int32_t tt = neg ? -(int32_t)m : (int32_t)m;
          ndf = tt >> 1;
          ncnt = (tt & 1) ? ln::rvu(c) + 2 : 1;
        } else {
          ncnt = neg ? ln::rvu(c) + 2 : 1;
        }
        nend = c.p;
      }
      const bool merge = E.cnt > 0 && ((kind == K_LC || kind == K_RC) ? E.df == ndf : E.s == nv);
      if (!merge) break;
      E.cnt += ncnt;  // the same run, ncnt values longer
      if (kind == K_LC || kind == K_RC) E.s = (uint32_t)((int64_t)E.s + (int64_t)ndf * ncnt);
      idx += ncnt;
      vstart = nend;
    }
    E.flush(B, kind, vstart >= c1);
  } else {
    E.flush(B, kind, true);
    vstart = c1;
  }
  if (bad || B.over) { M.ok = 0; M.why = 30 + kind; return; }
  M.hlen[kind] = B.n;
  M.vstart[kind] = vstart;
}

// ---- K4: output -----------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_v2_out(Job J) {
  const GeneralJob &j = J.j;
  const uint32_t lane = threadIdx.x;
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    Meta &M = J.meta[d];
    if (!M.ok || M.ms) continue;
    const uint32_t u0 = j.doc_upd[d];
    const uint64_t ub = j.upd_off[u0];
    const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
    const uint8_t *D = j.A + ub;
    // delete set: readDeleteSet's reads, canonical, no repeated or empty client (then copied)
    uint32_t x = M.ds0;
    bool bad = false;
    uint32_t ndc;
    {
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
    if (bad) { if (lane == 0) M.why = 40; __syncthreads(); continue; }
    const uint32_t ds1 = x;
    // sizes
    const bool part = M.f != NONE;
    uint32_t cl[9];
    for (uint32_t c = 0; c < 9; c++) cl[c] = 0;
    uint32_t sbn = 0, sln = 0;
    if (part) {  // spans the splice and the cut produced must lie inside their columns (else: decline)
      bool span_bad = M.body_f > M.body_fc || M.body_fc > M.body_f1 || M.body_f1 > M.body_end || M.body_end > M.sn;
      span_bad |= M.off != 0 && (M.info_f & 31) == 4 && M.body_fc + M.off > M.body_f1;
      for (uint32_t kk = 0; kk < NK1; kk++)
        span_bad |= M.hlen[kk] > HB || M.vstart[kk] < M.col0[col_of(kk)] || M.vstart[kk] > M.col1[col_of(kk)];
      if (span_bad) { if (lane == 0) M.why = 41; __syncthreads(); continue; }
      for (uint32_t kk = 0; kk < NK1; kk++) {
        const uint32_t c = col_of(kk);
        const uint32_t b = M.hlen[kk] + (M.col1[c] - M.vstart[kk]);
        if (kk == K_SL) sln = b;
        else cl[c] = b;
      }
      // the cut struct's strings: all of them without an offset, else only the content's tail (an offset
      // gives the Item an origin: ykey / parentSub are not written)
      const uint32_t hs0 = M.off == 0 ? M.body_f : (M.info_f & 31) == 4 ? M.body_fc + M.off : M.body_f1;
      sbn = (M.body_f1 - hs0) + (M.body_end - M.body_f1);
    }
    cl[5] = vsz(sbn) + sbn + sln;  // the string column always holds varString(body), even an empty one
    uint32_t total = 1;
    for (uint32_t c = 0; c < 9; c++) total += vsz(cl[c]) + cl[c];
    const uint32_t written = part ? M.n - M.f : 0;
    const uint32_t fclock = part ? M.fclock_lo + M.off : 0;
    total += vsz(part ? 1 : 0) + (part ? vsz(written) + vsz(fclock) : 0) + (ds1 - M.ds0);
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
      const uint32_t nb = vsz(v);
      if (lane == 0) { uint32_t q = p; while (v > 127) { o[q++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[q] = (uint8_t)v; }
      return p + nb;
    };
    uint32_t p = put(0, 0);
    for (uint32_t c = 0; c < 9; c++) {
      p = put(p, cl[c]);
      if (c == 5) p = put(p, sbn);  // string column: varString(body) | lengths
      if (!part || cl[c] == 0) continue;
      int kk = -1;
      for (uint32_t q = 0; q < NK1; q++) if (col_of(q) == c) kk = (int)q;
      if (c == 5) {
        const uint32_t hs0 = M.off == 0 ? M.body_f : (M.info_f & 31) == 4 ? M.body_fc + M.off : M.body_f1;
        wcopy(o + p, D + M.sb0 + hs0, M.body_f1 - hs0);
        p += M.body_f1 - hs0;
        wcopy(o + p, D + M.sb0 + M.body_f1, M.body_end - M.body_f1);
        p += M.body_end - M.body_f1;
      }
      if (kk < 0) continue;
      if (lane == 0) for (uint32_t q = 0; q < M.hlen[kk]; q++) o[p + q] = M.head[kk][q];
      p += M.hlen[kk];
      wcopy(o + p, D + M.vstart[kk], M.col1[c] - M.vstart[kk]);
      p += M.col1[c] - M.vstart[kk];
    }
    p = put(p, part ? 1 : 0);
    if (part) { p = put(p, written); p = put(p, fclock); }
    wcopy(o + p, D + M.ds0, ds1 - M.ds0);
    if (lane == 0) {
      j.out_off[d] = b;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}

}  // namespace pv2

namespace {
int pv_ensure(PwBufs &B, int k, size_t n) {
  if (n <= B.cap[k]) return 0;
  if (B.p[k]) hipFree(B.p[k]);
  B.p[k] = nullptr;
  B.cap[k] = 0;
  const size_t want = n + n / 8 + 4096;
  if (hipMalloc(&B.p[k], want) != hipSuccess) return -1;
  B.cap[k] = want;
  return 0;
}
}  // namespace

// Column-parallel V2 diff / sv / meta over the large documents of a call (single section: this file;
// several sections: ym_pv2ms.hip); marks the documents it completes in *done_out (k_big_v2 skips them).
// 1 = launched, 0 = not applicable, < 0 = error.
static pv2::Meta *pv2_last_meta = nullptr;
static const uint8_t *pv2_last_done = nullptr;
namespace pv2 {
// the scanned totals (scratch bytes of the single- and multi-section documents) straight into the coherent
// pinned host words pv2_finish reads (a copy op would hold the stream ~25 us)
__global__ void k_v2_totals(const uint64_t *t0, const uint64_t *t1, uint64_t *host) {
  if (threadIdx.x == 0) { host[0] = *t0; host[1] = *t1; }
}
}  // namespace pv2
// Step 1: the per-document prep and the scans of its scratch sizes; every document is marked not done
// (*done_out) and the totals start towards the host.  The small documents' kernels are enqueued next (their
// work hides that round trip; the column path only takes documents of >= PV_MIN bytes, beyond their windows).
int pv2_prepare(uint32_t op, const GeneralJob &j, hipStream_t st, PwBufs &B, const uint8_t **done_out) {
  using namespace pv2;
  *done_out = nullptr;
  B.pending = false;
  if (!j.v2 || (op != OP_DIFF && op != OP_SV && op != OP_META) || j.n == 0 || !j.pw_count || getenv("YMERGE_NO_PW")) return 0;
  uint64_t pv_min = PV_MIN;
  if (const char *e = getenv("YMERGE_PW_MIN")) pv_min = strtoull(e, nullptr, 10);
  if (!B.pinned_dev) {
    if (B.pinned) hipHostFree(B.pinned);
    B.pinned = nullptr;
    if (hipHostMalloc((void **)&B.pinned, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -2;
    if (hipHostGetDevicePointer((void **)&B.pinned_dev, B.pinned, 0) != hipSuccess) return -2;
  }
  if (!B.ev && hipEventCreateWithFlags(&B.ev, hipEventDisableTiming) != hipSuccess) return -2;
  const uint32_t n1 = j.n + 1;
  if (pv_ensure(B, 0, sizeof(Meta) * (uint64_t)j.n + 32ull * n1 + j.n + 64)) return -2;
  Job J;
  J.j = j;
  J.meta = (Meta *)B.p[0];
  uint64_t *sizes = (uint64_t *)(J.meta + j.n), *offs = sizes + n1, *sizes1 = offs + n1, *offs1 = sizes1 + n1;
  J.done = (uint8_t *)(offs1 + n1);
  pv2_last_meta = J.meta;
  pv2_last_done = J.done;
  k_v2_prep<<<(n1 + 255) / 256, 256, 0, st>>>(J, pv_min, sizes, sizes1);
  size_t tmp = 0;
  scan_excl<uint64_t>(nullptr, tmp, sizes, offs, n1, st);
  if (pv_ensure(B, 1, tmp + 16)) return -2;
  if (scan_excl<uint64_t>(B.p[1], tmp, sizes, offs, n1, st)) return -3;
  if (scan_excl<uint64_t>(B.p[1], tmp, sizes1, offs1, n1, st)) return -3;
  k_v2_totals<<<1, 64, 0, st>>>(offs + j.n, offs1 + j.n, (uint64_t *)B.pinned_dev);
  if (hipEventRecord(B.ev, st) != hipSuccess) return -3;
  *done_out = J.done;
  B.pending = true;
  B.op = op;
  return 1;
}
// Step 2: waits for the totals, then the column path over the large documents (documents it completes get
// done[d] = 1; what it leaves stays 0 for k_big_v2).
int pv2_finish(const GeneralJob &j, hipStream_t st, PwBufs &B) {
  using namespace pv2;
  if (!B.pending) return 0;
  B.pending = false;
  const uint32_t op = B.op, n1 = j.n + 1;
  Job J;
  J.j = j;
  J.meta = (Meta *)B.p[0];
  uint64_t *sizes = (uint64_t *)(J.meta + j.n), *offs = sizes + n1, *sizes1 = offs + n1, *offs1 = sizes1 + n1;
  J.done = (uint8_t *)(offs1 + n1);
  J.scr = nullptr;
  J.scr1 = nullptr;
  size_t tmp = 0;
  scan_excl<uint64_t>(nullptr, tmp, sizes, offs, n1, st);
  if (hipEventSynchronize(B.ev) != hipSuccess) return -3;  // (the small documents' kernels run meanwhile)
  uint64_t total, total1;
  __builtin_memcpy(&total, B.pinned, 8);
  __builtin_memcpy(&total1, B.pinned + 2, 8);
  bool ms = total1 > 0;
  if (ms && pv_ensure(B, 3, total1 + 256)) return 1;  // no room: k_big_v2 takes the large documents
  if (ms) {  // multi-section documents: the rest walk counts their structs, then their value arrays are sized
    J.scr1 = (uint8_t *)B.p[3];
    k_v2_meta_off<<<(j.n + 255) / 256, 256, 0, st>>>(J, offs1, 1);
    ms_rest(J, st);
    ms_sizes(J, sizes, st);
    if (scan_excl<uint64_t>(B.p[1], tmp, sizes, offs, n1, st)) return -3;
    k_v2_totals<<<1, 64, 0, st>>>(offs + j.n, offs1 + j.n, (uint64_t *)B.pinned_dev);
    if (hipStreamSynchronize(st) != hipSuccess) return -3;
    __builtin_memcpy(&total, B.pinned, 8);
  }
  if (total == 0) return 1;
  if (pv_ensure(B, 2, total + 256)) return 1;  // no room: k_big_v2 takes them (done stays 0)
  J.scr = (uint8_t *)B.p[2];
  k_v2_meta_off<<<(j.n + 255) / 256, 256, 0, st>>>(J, offs, 0);
  const dim3 g1((j.n + 63) / 64, NK1);
  k_v2_decw<<<dim3(j.n, ms ? NK : NK1), 64, 0, st>>>(J);
  if (op == OP_DIFF) {
    k_v2_struct<OP_DIFF><<<j.n, KT, 0, st>>>(J);
    k_v2_splice<<<g1, 64, 0, st>>>(J);
    const uint32_t grid = j.n < BS_GRID ? j.n : BS_GRID;
    k_v2_out<<<grid, 64, 0, st>>>(J);
  } else if (op == OP_SV) {
    k_v2_struct<OP_SV><<<j.n, KT, 0, st>>>(J);
  } else {
    k_v2_struct<OP_META><<<j.n, KT, 0, st>>>(J);
  }
  if (ms) ms_run(op, J, st);
  return 1;
}

}  // namespace ymk

// debugging aid (not part of include/ymerge.h): per document of the last V2 column-path call on this
// device, 0 = taken, 1 = not eligible, else the stage that declined it (K1: 10 + column, K2: 20-24,
// K3: 30 + column, K4: 40 delete set / 41 spans)
// ... and its done array (1 = completed by a specialised kernel, >= 2 = the small-document kernel's decline
// reason, k_diff_small_v2)
extern "C" int ym__pv2_done(uint8_t *host, uint32_t n) {
  return ymk::pv2_last_done ? (int)hipMemcpy(host, ymk::pv2_last_done, n, hipMemcpyDeviceToHost) : -1;
}
extern "C" int ym__pv2_why(uint32_t *host, uint32_t n) {
  using namespace ymk;
  if (!pv2_last_meta) return -1;
  for (uint32_t d = 0; d < n; d++)
    if (hipMemcpy(host + d, reinterpret_cast<uint8_t *>(pv2_last_meta + d) + offsetof(pv2::Meta, why), 4,
                  hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return 0;
}
