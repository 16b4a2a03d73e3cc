// ym_large.hip -- batched mergeUpdates / mergeUpdatesV2 for documents too large for the LDS fast
// paths (BASELINE configs[4] C5: ~16 k updates, ~50 k structs, 1,024 clients per document).
//
// Same contract as ym_fast.hip / ym_fast2.hip: documents whose updates are "simple" (every update's
// structs increase in (client desc, clock asc), no GC / Skip inputs, canonical payloads, no two runs
// of a client overlapping) merge to all structs sorted by (client desc, clock asc), a Skip at every
// clock gap, one part per client, the delete set = per-client interval union with clients in first-
// appearance order (yjs 13.5.16 ds@39007 / he@10482 / le@10242).  Anything else is
// declined and run by the exact general path.  Records live in HBM; the pipeline is device-wide:
//
//   1. walk (count, then emit): one lane per update, 64 consecutive updates of a document staged
//      into an LDS window per wave; struct records, client runs (the structs of one client inside one
//      update: contiguous clocks) and delete ranges go to SoA arrays at offsets from exclusive scans
//      of the per-update counts (ym_scan.h: the listed documents' updates only, counted on the device).
//   2. segmented radix sorts (ym_segsort.hip, one workgroup per document): runs by
//      (~client << 32 | clock), delete ranges by (client << 32 | clock); the ranges' values are their
//      emission index = first-appearance order.
//   3. one 1024-thread workgroup per document, tile loops with carried block scans:
//      A  runs in key order: overlap check, Skips at gaps, parts, struct / unit bases;
//      B  expand runs to the output struct order;  C  per-struct output sizes (V1 rows) or V2 column
//      entries (values scattered into per-column HBM arrays) and rest bytes;  D  V2 column sizes by
//      tiled RLE encoders (run starts by neighbour compares, lengths by a carried running max of
//      start positions);  E  delete set: carried segmented running-max scan = union, groups ranked by
//      their first appearance;  F  placement in the document's output slot;  G/H  writes.
#include <hip/hip_runtime.h>
#include <string.h>

#include "ym_scan.h"

#include "ym_fast_common.h"
#include "ym_kernels.h"

namespace ymk {
namespace lm {
using namespace fastc;

constexpr uint32_t WIN = 8192;                 // staged bytes per 64-update chunk
constexpr uint32_t L_IN = 0;                   // u8[WIN + 16]
constexpr uint32_t L_UOFF = WIN + 16;          // u32[65]
constexpr uint32_t WALK_LDS = L_UOFF + 4 * 72;
constexpr uint32_t BT = 512, NW = BT / 64;     // document workgroup
constexpr uint32_t GMAX = 4096;                // delete-set groups (clients) ranked in LDS
// per-document info passed between k_lm_doc1 -> k_lm_col -> k_lm_doc2 -> k_lm_col<write>
enum { DI_NPARTS = 0, DI_NCOL = 1, DI_SBODY = 10, DI_SECT, DI_NGROUPS, DI_NRANGES, DI_DSBYTES, DI_CSZ = 16,
       DI_CBASE = 25, DI_SLOT = 34 /* u64 */, DI_N = 40 };

struct LMJob {
  const uint8_t *A;
  const uint64_t *upd_off;
  const uint32_t *doc_upd;
  uint32_t v2, nb, stride;    // big documents; stride of the per-update count arrays (>= nbu + 1)
  const uint32_t *bdoc;       // [nb] document ids
  uint32_t *bu_off;           // [nb + 1] first big-update index of each document
  uint32_t *ch_off;           // [nb + 1] first chunk of each document
  uint32_t *bad;              // [nb] declined (general path)
  uint32_t *u_cnt, *u_off;    // [3][stride]: structs, runs, delete ranges per big update
  // struct records
  uint64_t *rkey;             // ~client << 32 | clock
  uint32_t *rlen, *raux;      // len; info | parentInfo << 8 | typeRef << 16
  uint64_t *rsrc;             // V1: arena offset of the info byte; V2: rest payload span
  uint32_t *rbn;              // V1: struct bytes incl. info; V2: rest payload bytes
  uint4 *rf;                  // V2: origin / parent id (client, clock), right origin (client, clock)
  uint64_t *rs;               // V2: 3 strings (arena offset << 24 | bytes): ykey, parentSub, content/key
  // client runs
  uint64_t *runkey, *srunkey;
  uint32_t *runidx, *srunidx, *runfirst, *runcnt, *runend;
  // delete ranges
  uint64_t *dkey, *sdkey;
  uint32_t *dlen, *didx, *sdidx;
  // per-document scratch of phase 3 (indexed by the document's record / run / range bases)
  uint32_t *a_sbase, *a_gap, *a_pid, *p_uf, *p_ul;               // runs / parts
  uint32_t *ord, *o_gap, *o_pw, *o_off;                          // output struct order
  uint32_t *q_clk, *q_end, *q_grp, *q_pre, *g_first, *g_cli, *g_min, *g_woff, *g_rb;  // delete set
  uint32_t *c_cl, *c_lc, *c_rc, *c_ln, *c_sbo;                   // V2 column values
  uint8_t *c_in, *c_pi, *c_tr;
  uint64_t *c_st;
  uint32_t *dinfo;            // [nb][DI_N] per-document sizes between the phase kernels
  // outputs
  int32_t *status;
  uint8_t *out;
  uint64_t cap;
  uint64_t *out_off, *out_len;
};

// ---- prep: per-document update / chunk counts --------------------------------------------------
__global__ void k_lm_prep(LMJob J, const uint32_t *list, uint32_t *kcnt, uint32_t *ccnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > J.nb) return;
  if (i == J.nb) { kcnt[i] = 0; ccnt[i] = 0; return; }
  const uint32_t d = list[i];
  const uint32_t k = J.doc_upd[d + 1] - J.doc_upd[d];
  const uint64_t bytes = J.upd_off[J.doc_upd[d + 1]] - J.upd_off[J.doc_upd[d]];
  const bool ok = k > 1 && bytes < (1ull << 30);
  J.bad[i] = !ok;
  kcnt[i] = ok ? k : 0;
  ccnt[i] = ok ? (k + 63) / 64 : 0;
}

// the per-update count arrays zeroed over the listed documents' updates (tot[0] + 1 entries each)
__global__ void k_lm_zero(LMJob J, const uint32_t *tot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > tot[0] || i >= J.stride) return;
  J.u_cnt[i] = 0;
  J.u_cnt[J.stride + i] = 0;
  J.u_cnt[2 * J.stride + i] = 0;
}
// the record totals (structs, runs, delete ranges) and the chunk total into the coherent pinned host words
__global__ void k_lm_totals(LMJob J, const uint32_t *tot, uint32_t *host) {
  if (threadIdx.x == 0) {
    const uint32_t nu = tot[0];
    host[0] = J.u_off[nu];
    host[1] = J.u_off[J.stride + nu];
    host[2] = J.u_off[2 * J.stride + nu];
    host[3] = tot[1];
  }
}

// ---- 1. walkers (one lane per update; LDS bytes at [p0, p1), arena offset of LDS byte 0 = gb) ------
struct Emit {
  uint32_t rq, runq, dq;  // first record / run / range slot of this update
};

template <bool EMIT>
__device__ bool walk_v1(const LMJob &J, uint32_t p0, uint32_t p1, uint64_t gb, const Emit &E, uint32_t (&cnt)[3]) {
  Cur c = {p0, p1, false};
  const uint32_t nclients = rvu(c);
  uint64_t prev = 0;
  bool have_prev = false;
  for (uint32_t ci = 0; ci < nclients && !c.bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = rvu(c);
    uint32_t clock = rvu(c);
    if (c.bad || nstructs == 0) return false;
    const uint32_t first = cnt[0], clock0 = clock;
    for (uint32_t si = 0; si < nstructs && !c.bad; si++) {
      const uint32_t s0 = c.p;
      const uint32_t info = rdb(c);
      if (info == 10 || (info & 31) == 0) return false;  // Skip / GC inputs: general path
      uint32_t len;
      if (!item_body<true>(c, info, len)) return false;
      if ((uint64_t)clock + len > 0xffffffffull) return false;
      const uint64_t key = ((uint64_t)(~client) << 32) | clock;
      if (have_prev && key <= prev) return false;  // each update must already be in merge order
      prev = key + len - 1;
      have_prev = true;
      if (EMIT) {
        const uint32_t q = E.rq + cnt[0];
        J.rkey[q] = key;
        J.rlen[q] = len;
        J.raux[q] = info;
        J.rsrc[q] = gb + s0;
        J.rbn[q] = c.p - s0;
      }
      cnt[0]++;
      clock += len;
    }
    if (EMIT) {
      const uint32_t r = E.runq + cnt[1];
      J.runkey[r] = ((uint64_t)(~client) << 32) | clock0;
      J.runidx[r] = r;
      J.runfirst[r] = E.rq + first;
      J.runcnt[r] = cnt[0] - first;
      J.runend[r] = clock;
    }
    cnt[1]++;
  }
  if (c.bad) return false;
  // delete set (DeleteSet.js:241-256)
  const uint32_t ndc = rvu(c);
  for (uint32_t i = 0; i < ndc && !c.bad; i++) {
    const uint32_t client = rvu(c);
    const uint32_t m = rvu(c);
    for (uint32_t q = 0; q < m && !c.bad; q++) {
      const uint32_t clock = rvu(c);
      const uint32_t len = rvu(c);
      if (c.bad) return false;
      if (EMIT) {
        const uint32_t x = E.dq + cnt[2];
        J.dkey[x] = ((uint64_t)client << 32) | clock;
        J.dlen[x] = len;
        J.didx[x] = x;
      }
      cnt[2]++;
    }
  }
  return !c.bad;
}

// V2 (UpdateDecoder.js:245-392): per-lane lib0 column decoders as in ym_fast2.hip
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
struct RleD { Cur c; uint32_t s, n; };
struct UoptD { Cur c; uint32_t s, n; };
struct IdifD { Cur c; uint32_t s, n; int32_t d; };
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
    const int32_t t = (int32_t)(neg ? 0u - m : m);
    r.d = t >> 1;
    r.n = (t & 1) ? rvu(r.c) + 2 : 1;
  }
  const int64_t v = (int64_t)r.s + r.d;
  r.c.bad |= v < 0 || v > 0xffffffffll;
  r.s = (uint32_t)v;
  r.n--;
  return r.s;
}

template <bool EMIT>
__device__ bool walk_v2(const LMJob &J, uint32_t p0, uint32_t p1, uint64_t gb, const Emit &E, uint32_t (&cnt)[3]) {
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
  const uint32_t sn = rvu(col[5]);  // StringDecoder: varString body (ASCII only) + UintOptRle lengths
  if (col[5].bad || !room(col[5], sn)) return false;
  const uint32_t sb = col[5].p;
  {
    uint64_t hi = 0;
    for (uint32_t o = 0; o < sn; o += 8) hi |= mask_bytes(ld8(sb + o), sn - o);
    if (hi & 0x8080808080808080ull) return false;
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
  auto rstr = [&]() -> uint64_t {  // StringDecoder.read(): arena offset << 24 | bytes
    const uint32_t n = rd_uopt(sl);
    bad |= spos + n > sn;
    const uint64_t v = ((gb + sb + spos) << 24) | n;
    spos += n;
    return v;
  };
  const uint32_t nclients = rvu(c);
  uint64_t prev = 0;
  bool have_prev = false;
  for (uint32_t ci = 0; ci < nclients && !c.bad && !bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = rd_uopt(cl);
    uint32_t clock = rvu(c);
    if (c.bad || nstructs == 0) return false;
    const uint32_t first = cnt[0], clock0 = clock;
    for (uint32_t si = 0; si < nstructs && !c.bad && !bad; si++) {
      const uint32_t info = rd_rle(in);
      if (info == 10 || (info & 31) == 0 || info > 255) return false;
      uint32_t f0 = 0, f1 = 0, f2 = 0, f3 = 0, pi = 0, t = 0;
      uint64_t s0 = 0, s1 = 0, s2 = 0, sp = 0;
      uint32_t spn = 0;
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
        case 1: len = rd_uopt(ln); break;                                   // ContentDeleted
        case 3: {                                                           // ContentBinary (rest)
          const uint32_t a = c.p, n = rvu(c);
          if (!room(c, n)) return false;
          c.p += n;
          sp = gb + a;
          spn = c.p - a;
          break;
        }
        case 4: s2 = rstr(); len = (uint32_t)(s2 & 0xffffff); break;        // ContentString (ASCII)
        case 5: case 6: {                                                   // Embed / Format (+ key)
          if ((info & 31) == 6) s2 = rstr();
          const uint32_t a = c.p;
          any_canon<true>(c);
          sp = gb + a;
          spn = c.p - a;
          break;
        }
        case 7:                                                             // ContentType
          t = rd_uopt(tr);
          if (t > 6) return false;
          if (t == 3 || t == 5) {  // readKey: a cached key (keyClock < keys read) reads no string
            if (rd_idif(kc) < keys) return false;
            keys++;
            s2 = rstr();
          }
          break;
        case 8: {                                                           // ContentAny
          len = rd_uopt(ln);
          const uint32_t a = c.p;
          for (uint32_t q = 0; q < len && !c.bad; q++) any_canon<true>(c);
          sp = gb + a;
          spn = c.p - a;
          break;
        }
        default: return false;  // ContentJSON, ContentDoc, invalid refs
      }
      if (c.bad || bad || len == 0) return false;
      if ((uint64_t)clock + len > 0xffffffffull) return false;
      const uint64_t key = ((uint64_t)(~client) << 32) | clock;
      if (have_prev && key <= prev) return false;
      prev = key + len - 1;
      have_prev = true;
      if (EMIT) {
        const uint32_t q = E.rq + cnt[0];
        J.rkey[q] = key;
        J.rlen[q] = len;
        J.raux[q] = info | (pi << 8) | (t << 16);
        J.rsrc[q] = sp;
        J.rbn[q] = spn;
        J.rf[q] = make_uint4(f0, f1, f2, f3);
        J.rs[3 * (uint64_t)q] = s0;
        J.rs[3 * (uint64_t)q + 1] = s1;
        J.rs[3 * (uint64_t)q + 2] = s2;
      }
      cnt[0]++;
      clock += len;
    }
    if (EMIT && !c.bad && !bad) {
      const uint32_t r = E.runq + cnt[1];
      J.runkey[r] = ((uint64_t)(~client) << 32) | clock0;
      J.runidx[r] = r;
      J.runfirst[r] = E.rq + first;
      J.runcnt[r] = cnt[0] - first;
      J.runend[r] = clock;
    }
    cnt[1]++;
  }
  bad |= c.bad | cl.c.bad | lc.c.bad | rc.c.bad | in.c.bad | sl.c.bad | pi_.c.bad | tr.c.bad | ln.c.bad | kc.c.bad;
  if (bad) return false;
  // V2 delete set (rest): per client, clock deltas against the previous end, len - 1 (UpdateDecoder.js:258-267)
  const uint32_t ndc = rvu(c);
  for (uint32_t i = 0; i < ndc && !c.bad; i++) {
    const uint32_t client = rvu(c);
    const uint32_t m = rvu(c);
    uint64_t cur = 0;
    for (uint32_t q = 0; q < m && !c.bad; q++) {
      const uint64_t clock = cur + rvu(c);
      const uint64_t len = (uint64_t)rvu(c) + 1;
      cur = clock + len;
      if (c.bad || cur > 0xffffffffull) return false;
      if (EMIT) {
        const uint32_t x = E.dq + cnt[2];
        J.dkey[x] = ((uint64_t)client << 32) | clock;
        J.dlen[x] = (uint32_t)len;
        J.didx[x] = x;
      }
      cnt[2]++;
    }
  }
  return !c.bad;
}

template <bool EMIT, bool V2>
__global__ void __launch_bounds__(64) k_lm_walk(LMJob J, const uint32_t *tot) {
  const uint32_t lane = threadIdx.x;
  const uint32_t nch = tot[1];
  for (uint32_t c = blockIdx.x; c < nch; c += gridDim.x) {
    uint32_t lo = 0, hi = J.nb;  // the document of chunk c: last i with ch_off[i] <= c
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (J.ch_off[mid] <= c) lo = mid; else hi = mid;
    }
    const uint32_t i = lo;
    if (EMIT && J.bad[i]) continue;
    const uint32_t d = J.bdoc[i];
    const uint32_t lc = c - J.ch_off[i];
    const uint32_t k = J.doc_upd[d + 1] - J.doc_upd[d];
    const uint32_t ug = J.doc_upd[d] + 64 * lc;
    const uint32_t n = k - 64 * lc < 64 ? k - 64 * lc : 64;
    const uint64_t b0 = J.upd_off[ug], bytes = J.upd_off[ug + n] - b0;
    const uint32_t bu = J.bu_off[i] + 64 * lc + lane;
    if (bytes > WIN) {  // a chunk of oversized updates: general path (counts stay zero)
      if (!EMIT && lane == 0) J.bad[i] = 1;
      continue;
    }
    const uint32_t base = (uint32_t)(b0 & 15);
    {
      const uint4 *src = reinterpret_cast<const uint4 *>(J.A + (b0 - base));
      const uint32_t nvec = (uint32_t)((base + bytes + 15) >> 4);
      for (uint32_t v = lane; v < nvec; v += 64) at<uint4>(L_IN + 16 * v) = src[v];
    }
    for (uint32_t l = lane; l <= n; l += 64) at<uint32_t>(L_UOFF + 4 * l) = (uint32_t)(J.upd_off[ug + l] - b0) + base;
    __syncthreads();
    if (lane < n) {
      uint32_t cnt[3] = {0, 0, 0};
      Emit E = {0, 0, 0};
      if (EMIT) E = Emit{J.u_off[bu], J.u_off[J.stride + bu], J.u_off[2 * J.stride + bu]};
      const uint32_t p0 = at<uint32_t>(L_UOFF + 4 * lane), p1 = at<uint32_t>(L_UOFF + 4 * lane + 4);
      const uint64_t gb = b0 - base;
      const bool ok = V2 ? walk_v2<EMIT>(J, p0, p1, gb, E, cnt) : walk_v1<EMIT>(J, p0, p1, gb, E, cnt);
      if (!EMIT) {
        if (!ok) J.bad[i] = 1;
        J.u_cnt[bu] = cnt[0];
        J.u_cnt[J.stride + bu] = cnt[1];
        J.u_cnt[2 * J.stride + bu] = cnt[2];
      }
    }
    __syncthreads();
  }
}

// segments of the sorts: per document [first, end) of its runs / delete ranges (empty when declined)
__global__ void k_lm_segs(LMJob J, uint32_t *seg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= J.nb) return;
  const uint32_t a = J.bu_off[i], b = J.bu_off[i + 1];
  const bool ok = !J.bad[i];
  for (uint32_t t = 0; t < 2; t++) {
    const uint32_t *o = J.u_off + (t + 1) * J.stride;
    seg[(2 * t) * J.nb + i] = o[a];
    seg[(2 * t + 1) * J.nb + i] = ok ? o[b] : o[a];
  }
}

// ---- 3. block primitives (1024 threads, carried across tiles) ------------------------------------
struct Shm {
  uint32_t s[11 * NW];
  unsigned long long m[NW];
  uint32_t gmin[GMAX];
  uint32_t flag;
};

// exclusive block scan of N values per thread in place; tot = block totals (uniform)
template <int N>
__device__ __forceinline__ void bscan(Shm &S, uint32_t (&x)[N], uint32_t (&tot)[N]) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc[N];
#pragma unroll
  for (int k = 0; k < N; k++) inc[k] = wave_incl_add(x[k]);
  if (lane == 63) {
#pragma unroll
    for (int k = 0; k < N; k++) S.s[k * NW + w] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++) {
    uint32_t pre = 0, t = 0;
#pragma unroll
    for (uint32_t v = 0; v < NW; v++) {
      const uint32_t s = S.s[k * NW + v];
      pre += v < w ? s : 0;
      t += s;
    }
    x[k] = pre + inc[k] - x[k];
    tot[k] = t;
  }
  __syncthreads();
}
// inclusive block running max (u64) with a carried prefix; tot = block max (uniform); excl = the
// running max before this thread's element
__device__ __forceinline__ uint64_t bmax(Shm &S, uint64_t x, uint64_t carry, uint64_t &tot, uint64_t *excl = nullptr) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_max64(x);
  if (lane == 63) S.m[w] = inc;
  __syncthreads();
  uint64_t pre = carry, t = carry;
#pragma unroll
  for (uint32_t v = 0; v < NW; v++) {
    const uint64_t s = S.m[v];
    if (v < w) pre = s > pre ? s : pre;
    t = s > t ? s : t;
  }
  tot = t;
  if (excl) {
    const uint64_t wex = ((uint64_t)from_prev_lane((uint32_t)(inc >> 32)) << 32) | from_prev_lane((uint32_t)inc);
    *excl = wex > pre ? wex : pre;  // lane 0 receives 0 from the shift
  }
  __syncthreads();
  return inc > pre ? inc : pre;
}
__device__ __forceinline__ bool bor(Shm &S, bool b) {
  if (threadIdx.x == 0) S.flag = 0;
  __syncthreads();
  if (b) S.flag = 1;
  __syncthreads();
  const bool r = S.flag != 0;
  __syncthreads();
  return r;
}

__device__ __forceinline__ uint32_t gvsz(uint64_t v) {
  uint32_t n = 1;
  while (v > 127) { v >>= 7; n++; }
  return n;
}
__device__ __forceinline__ uint32_t gput_vu(uint8_t *o, uint32_t p, uint64_t v) {
  while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
  o[p++] = (uint8_t)v;
  return p;
}
__device__ __forceinline__ uint32_t vszi(uint32_t m) { return m < 64 ? 1 : 1 + gvsz(m >> 6); }
__device__ __forceinline__ uint32_t gput_vi(uint8_t *o, uint32_t p, bool neg, uint32_t m) {
  o[p++] = (uint8_t)((m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63));
  m >>= 6;
  while (m > 0) { o[p++] = (uint8_t)((m > 127 ? 0x80 : 0) | (m & 127)); m >>= 7; }
  return p;
}
// One thread's copy of a struct's bytes (unaligned on both sides).  All loads of a piece are issued
// before its stores, 16 / 8 / 4 / 1 bytes wide: a byte loop waited for every load (a C5 document's
// ~16 k structs of ~30 bytes made k_lm_doc2 a chain of byte round trips).
typedef uint4 __attribute__((aligned(1))) lm_u4u;
typedef uint64_t __attribute__((aligned(1))) lm_u8u;
typedef uint32_t __attribute__((aligned(1))) lm_u32u;
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t n) {
  uint32_t b = 0;
  for (; b + 64 <= n; b += 64) {
    const uint4 v0 = *reinterpret_cast<const lm_u4u *>(src + b), v1 = *reinterpret_cast<const lm_u4u *>(src + b + 16);
    const uint4 v2 = *reinterpret_cast<const lm_u4u *>(src + b + 32), v3 = *reinterpret_cast<const lm_u4u *>(src + b + 48);
    *reinterpret_cast<lm_u4u *>(dst + b) = v0;
    *reinterpret_cast<lm_u4u *>(dst + b + 16) = v1;
    *reinterpret_cast<lm_u4u *>(dst + b + 32) = v2;
    *reinterpret_cast<lm_u4u *>(dst + b + 48) = v3;
  }
  // the rest (< 64 bytes): up to three 16-byte pieces, then 8, 4 and single bytes, loads first
  const uint32_t k = (n - b) >> 4;
  uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0, v2 = v0;
  if (k > 0) v0 = *reinterpret_cast<const lm_u4u *>(src + b);
  if (k > 1) v1 = *reinterpret_cast<const lm_u4u *>(src + b + 16);
  if (k > 2) v2 = *reinterpret_cast<const lm_u4u *>(src + b + 32);
  const uint32_t t8 = b + 16 * k;
  const bool h8 = t8 + 8 <= n;
  const uint64_t w8 = h8 ? *reinterpret_cast<const lm_u8u *>(src + t8) : 0;
  const uint32_t t4 = t8 + (h8 ? 8 : 0);
  const bool h4 = t4 + 4 <= n;
  const uint32_t w4 = h4 ? *reinterpret_cast<const lm_u32u *>(src + t4) : 0;
  const uint32_t t1 = t4 + (h4 ? 4 : 0);
  const uint8_t c0 = t1 < n ? src[t1] : 0, c1 = t1 + 1 < n ? src[t1 + 1] : 0, c2 = t1 + 2 < n ? src[t1 + 2] : 0;
  if (k > 0) *reinterpret_cast<lm_u4u *>(dst + b) = v0;
  if (k > 1) *reinterpret_cast<lm_u4u *>(dst + b + 16) = v1;
  if (k > 2) *reinterpret_cast<lm_u4u *>(dst + b + 32) = v2;
  if (h8) *reinterpret_cast<lm_u8u *>(dst + t8) = w8;
  if (h4) *reinterpret_cast<lm_u32u *>(dst + t4) = w4;
  if (t1 < n) dst[t1] = c0;
  if (t1 + 1 < n) dst[t1 + 1] = c1;
  if (t1 + 2 < n) dst[t1 + 2] = c2;
}

enum { K_UOPT = 0, K_IDIF = 1, K_RLE = 2 };
// lib0 RLE column encoder over n values get(i), tiled (IT consecutive entries per thread): returns the
// byte size; writes at dst when wr.  Runs from neighbour compares (of diffs for IntDiffOptRle), run
// lengths from a carried running max of the run-start positions, run bytes placed by a carried scan.
template <int K, class Get>
__device__ uint32_t col_rle(Shm &S, Get get, uint32_t n, bool wr, uint8_t *dst, bool &bad) {
  constexpr uint32_t IT = 4, TILE = BT * IT;
  uint64_t carry_sp = 0;
  uint32_t carry_b = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += TILE) {
    const uint32_t i0 = t0 + threadIdx.x * IT;
    int64_t val[IT + 3];  // values of entries i0 - 2 .. i0 + IT (0 outside [0, n): the IntDiff base)
#pragma unroll
    for (uint32_t k = 0; k < IT + 3; k++) {
      const int64_t e = (int64_t)i0 + k - 2;
      val[k] = e >= 0 && e < (int64_t)n ? (int64_t)get((uint32_t)e) : 0;
    }
    int64_t cv[IT + 2];   // compared value (diff for IntDiffOptRle) of entries i0 - 1 .. i0 + IT
#pragma unroll
    for (uint32_t k = 0; k < IT + 2; k++) cv[k] = K == K_IDIF ? val[k + 1] - val[k] : val[k + 1];
    bool st[IT], en[IT];
    uint32_t last = 0;
#pragma unroll
    for (uint32_t t = 0; t < IT; t++) {
      const uint32_t e = i0 + t;
      const bool v = e < n;
      st[t] = v && (e == 0 || cv[t + 1] != cv[t]);
      en[t] = v && (e + 1 == n || cv[t + 2] != cv[t + 1]);
      if (st[t]) last = e;
    }
    uint64_t tmax, ex;
    bmax(S, last, carry_sp, tmax, &ex);
    uint32_t sp = (uint32_t)ex, rb[IT], cnt[IT], tb = 0;
#pragma unroll
    for (uint32_t t = 0; t < IT; t++) {
      const uint32_t e = i0 + t;
      if (st[t]) sp = e;
      cnt[t] = e - sp + 1;
      rb[t] = 0;
      if (!en[t]) continue;
      const int64_t cur = cv[t + 1];
      if (K == K_UOPT) {
        rb[t] = vszi((uint32_t)cur) + (cnt[t] > 1 ? gvsz(cnt[t] - 2) : 0);
      } else if (K == K_IDIF) {
        bad |= cur <= -(1ll << 30) || cur >= (1ll << 30);
        const int32_t x = (int32_t)((uint32_t)(int32_t)cur << 1) | (cnt[t] > 1 ? 1 : 0);
        rb[t] = vszi(x < 0 ? 0u - (uint32_t)x : (uint32_t)x) + (cnt[t] > 1 ? gvsz(cnt[t] - 2) : 0);
      } else {
        rb[t] = 1 + (e + 1 == n ? 0 : gvsz(cnt[t] - 1));
      }
      tb += rb[t];
    }
    uint32_t x1[1] = {tb}, t1[1];
    bscan<1>(S, x1, t1);
    if (wr) {
      uint32_t q = carry_b + x1[0];
#pragma unroll
      for (uint32_t t = 0; t < IT; t++) {
        if (!en[t]) continue;
        const int64_t cur = cv[t + 1];
        uint32_t o = q;
        if (K == K_UOPT) {
          o = gput_vi(dst, o, cnt[t] > 1, (uint32_t)cur);
          if (cnt[t] > 1) gput_vu(dst, o, cnt[t] - 2);
        } else if (K == K_IDIF) {
          const int32_t x = (int32_t)((uint32_t)(int32_t)cur << 1) | (cnt[t] > 1 ? 1 : 0);
          o = gput_vi(dst, o, x < 0, x < 0 ? 0u - (uint32_t)x : (uint32_t)x);
          if (cnt[t] > 1) gput_vu(dst, o, cnt[t] - 2);
        } else {
          dst[o++] = (uint8_t)cur;
          if (i0 + t + 1 != n) gput_vu(dst, o, cnt[t] - 1);
        }
        q += rb[t];
      }
    }
    carry_b += t1[0];
    carry_sp = tmax;
  }
  return carry_b;
}

// the document's bases in the record / run / range arrays
struct DocB {
  uint32_t d, rb, ns, runb, nr, dsb, nds;
  uint64_t b0, bytes;
};
__device__ __forceinline__ DocB doc_bases(const LMJob &J, uint32_t i) {
  DocB B;
  B.d = J.bdoc[i];
  const uint32_t u0 = J.doc_upd[B.d], k = J.doc_upd[B.d + 1] - u0;
  B.b0 = J.upd_off[u0];
  B.bytes = J.upd_off[u0 + k] - B.b0;
  const uint32_t bu0 = J.bu_off[i], bu1 = J.bu_off[i + 1];
  B.rb = J.u_off[bu0];
  B.ns = J.u_off[bu1] - B.rb;
  B.runb = J.u_off[J.stride + bu0];
  B.nr = J.u_off[J.stride + bu1] - B.runb;
  B.dsb = J.u_off[2 * J.stride + bu0];
  B.nds = J.u_off[2 * J.stride + bu1] - B.dsb;
  return B;
}

// ---- 3b. V2 columns: one workgroup per (document, column); WR = false sizes, WR = true writes ------
template <bool WR>
__global__ void __launch_bounds__(BT) k_lm_col(LMJob J) {
  __shared__ Shm S;
  const uint32_t i = blockIdx.x, c = blockIdx.y;
  if (J.bad[i]) return;
  const DocB D = doc_bases(J, i);
  uint32_t *const info = J.dinfo + (uint64_t)DI_N * i;
  const uint32_t rb = D.rb;
  const uint64_t cb = 3ull * rb, ib = 2ull * rb;
  const uint32_t n = info[DI_NCOL + c];
  uint8_t *dst = nullptr;
  if (WR) dst = J.out + *(const uint64_t *)(info + DI_SLOT) + info[DI_CBASE + c];
  bool bad = false;
  uint32_t sz = 0;
  switch (c) {
    case 0: sz = col_rle<K_IDIF>(S, [&](uint32_t x) { return x; }, n, WR, dst, bad); break;
    case 1: sz = col_rle<K_UOPT>(S, [&](uint32_t x) { return J.c_cl[cb + x]; }, n, WR, dst, bad); break;
    case 2: sz = col_rle<K_IDIF>(S, [&](uint32_t x) { return J.c_lc[rb + x]; }, n, WR, dst, bad); break;
    case 3: sz = col_rle<K_IDIF>(S, [&](uint32_t x) { return J.c_rc[rb + x]; }, n, WR, dst, bad); break;
    case 4: sz = col_rle<K_RLE>(S, [&](uint32_t x) { return (uint32_t)J.c_in[ib + x]; }, n, WR, dst, bad); break;
    case 5: {  // StringEncoder: varString(bodies) | UintOptRle(lengths); ASCII, so lengths are bytes
      const uint32_t sbody = info[DI_SBODY];
      const uint32_t hb = gvsz(sbody);
      if (WR) {
        if (threadIdx.x == 0) gput_vu(dst, 0, sbody);
        for (uint32_t e = threadIdx.x; e < n; e += BT) {
          const uint64_t s = J.c_st[cb + e];
          copy_bytes(dst + hb + J.c_sbo[cb + e], J.A + (s >> 24), (uint32_t)(s & 0xffffff));
        }
      }
      sz = hb + sbody + col_rle<K_UOPT>(S, [&](uint32_t x) { return (uint32_t)(J.c_st[cb + x] & 0xffffff); }, n, WR,
                                        WR ? dst + hb + sbody : nullptr, bad);
      break;
    }
    case 6: sz = col_rle<K_RLE>(S, [&](uint32_t x) { return (uint32_t)J.c_pi[rb + x]; }, n, WR, dst, bad); break;
    case 7: sz = col_rle<K_UOPT>(S, [&](uint32_t x) { return (uint32_t)J.c_tr[rb + x]; }, n, WR, dst, bad); break;
    default: sz = col_rle<K_UOPT>(S, [&](uint32_t x) { return J.c_ln[rb + x]; }, n, WR, dst, bad); break;
  }
  if (!WR && threadIdx.x == 0) info[DI_CSZ + c] = sz;
  if (!WR && bor(S, bad) && threadIdx.x == 0) J.bad[i] = 1;  // (diffs outside +-2^30: general path)
}

// ---- 3a. per document: runs, output order, struct sizes / column entries, delete set --------------
template <bool V2>
__global__ void __launch_bounds__(BT) k_lm_doc1(LMJob J) {
  __shared__ Shm S;
  const uint32_t i = blockIdx.x, tid = threadIdx.x;
  if (J.bad[i]) return;
  const DocB D = doc_bases(J, i);
  const uint32_t rb = D.rb, ns = D.ns, runb = D.runb, nr = D.nr, dsb = D.dsb, nds = D.nds;
  auto decline = [&]() {
    if (tid == 0) J.bad[i] = 1;  // status stays ST_PENDING: the general path takes the document
  };
  if (ns == 0) { decline(); return; }

  // ---- A. runs in key order: overlaps, gaps, parts, bases
  uint32_t nparts = 0;
  {
    uint32_t cs = 0, cu = 0, cp = 0;
    bool bad = false;
    for (uint32_t t0 = 0; t0 < nr; t0 += BT) {
      const uint32_t r = t0 + tid;
      const bool v = r < nr;
      uint64_t key = 0, pkey = 0;
      uint32_t cnt = 0, pend = 0, gap = 0;
      bool same = false, plast = false;
      if (v) {
        key = J.srunkey[runb + r];
        const uint32_t ri = J.srunidx[runb + r];
        cnt = J.runcnt[ri];
        if (r > 0) {
          pkey = J.srunkey[runb + r - 1];
          pend = J.runend[J.srunidx[runb + r - 1]];
          same = (pkey >> 32) == (key >> 32);
        }
        const uint32_t clock = (uint32_t)key;
        bad |= same && pend > clock;
        gap = same && pend < clock ? clock - pend : 0;
        plast = r + 1 >= nr || (J.srunkey[runb + r + 1] >> 32) != (key >> 32);
      }
      const uint32_t pst = v && !same;
      uint32_t x[3] = {cnt, v ? cnt + (gap != 0) : 0, pst}, tot[3];
      const uint32_t units = x[1];
      bscan<3>(S, x, tot);
      if (v) {
        const uint32_t pid = cp + x[2] + pst - 1;
        J.a_sbase[runb + r] = cs + x[0];
        J.a_gap[runb + r] = gap;
        J.a_pid[runb + r] = pid | (pst << 31);
        if (pst) J.p_uf[runb + pid] = cu + x[1];
        if (plast) J.p_ul[runb + pid] = cu + x[1] + units;
      }
      cs += tot[0];
      cu += tot[1];
      cp += tot[2];
    }
    if (bor(S, bad)) { decline(); return; }
    nparts = cp;
  }
  // ---- B. expand runs to the output struct order
  for (uint32_t t0 = 0; t0 < nr; t0 += BT) {
    const uint32_t r = t0 + tid;
    if (r < nr) {
      const uint32_t ri = J.srunidx[runb + r];
      const uint32_t first = J.runfirst[ri], cnt = J.runcnt[ri];
      const uint32_t sbase = J.a_sbase[runb + r], gap = J.a_gap[runb + r], pp = J.a_pid[runb + r];
      const uint32_t pid = pp & 0x7fffffffu;
      const uint32_t pw = (pp >> 31) ? J.p_ul[runb + pid] - J.p_uf[runb + pid] : 0;
      for (uint32_t t = 0; t < cnt; t++) {
        const uint32_t pos = rb + sbase + t;
        J.ord[pos] = first + t;
        J.o_gap[pos] = t == 0 ? gap : 0;
        J.o_pw[pos] = t == 0 ? pw : 0;
      }
    }
  }
  __syncthreads();
  // ---- C. per-struct sizes (V1 rows) / V2 column entries and rest bytes
  uint32_t sect = 0;           // V1: struct bytes after vu(nparts); V2: rest bytes after vu(nparts)
  uint32_t ncol[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, sbody = 0;  // V2: kc cl lc rc in st pi tr ln
  {
    bool bad = false;
    for (uint32_t t0 = 0; t0 < ns; t0 += BT) {
      const uint32_t p = t0 + tid;
      const bool v = p < ns;
      uint32_t q = 0, gap = 0, pw = 0, info = 0, aux = 0;
      uint64_t key = 0;
      if (v) {
        q = J.ord[rb + p];
        gap = J.o_gap[rb + p];
        pw = J.o_pw[rb + p];
        key = J.rkey[q];
        aux = J.raux[q];
        info = aux & 0xff;
      }
      const uint32_t client = ~(uint32_t)(key >> 32), clock = (uint32_t)key;
      if (!V2) {
        uint32_t x[1] = {v ? (pw ? gvsz(pw) + gvsz(client) + gvsz(clock) : 0) + (gap ? 1 + gvsz(gap) : 0) + J.rbn[q] : 0}, tot[1];
        bscan<1>(S, x, tot);
        if (v) J.o_off[rb + p] = sect + x[0];
        sect += tot[0];
      } else {
        const uint32_t pi = (aux >> 8) & 0xff, t = aux >> 16, ref = info & 31;
        const bool ho = info & 0x80, hr = info & 0x40, noo = (info & 0xC0) == 0;
        const bool kk = ref == 6 || (ref == 7 && (t == 3 || t == 5));
        uint64_t s[3] = {0, 0, 0};
        uint4 f = make_uint4(0, 0, 0, 0);
        uint32_t spn = 0;
        if (v) {
          s[0] = J.rs[3 * (uint64_t)q];
          s[1] = J.rs[3 * (uint64_t)q + 1];
          s[2] = J.rs[3 * (uint64_t)q + 2];
          f = J.rf[q];
          spn = J.rbn[q];
        }
        const bool e0 = v && noo && pi, e1 = v && noo && (info & 0x20), e2 = v && (ref == 4 || kk);
        uint32_t x[11], tot[11];
        x[0] = v && kk;
        x[1] = v ? (pw != 0) + ho + hr + (noo && !pi) : 0;
        x[2] = v && (ho || (noo && !pi));
        x[3] = v && hr;
        x[4] = v ? 1 + (gap != 0) : 0;
        x[5] = (uint32_t)e0 + e1 + e2;
        x[6] = v && noo;
        x[7] = v && ref == 7;
        x[8] = v && (ref == 1 || ref == 8);
        x[9] = v ? (pw ? gvsz(pw) + gvsz(clock) : 0) + (gap ? gvsz(gap) : 0) + spn : 0;
        x[10] = (e0 ? (uint32_t)(s[0] & 0xffffff) : 0) + (e1 ? (uint32_t)(s[1] & 0xffffff) : 0) + (e2 ? (uint32_t)(s[2] & 0xffffff) : 0);
        bscan<11>(S, x, tot);
        if (v) {
          uint32_t icl = ncol[1] + x[1], iin = ncol[4] + x[4], ist = ncol[5] + x[5], sbo = sbody + x[10];
          const uint64_t cb = 3ull * rb, ib = 2ull * rb;
          if (pw) J.c_cl[cb + icl++] = client;  // writeClient at a part start
          if (ho) { J.c_cl[cb + icl++] = f.x; J.c_lc[rb + ncol[2] + x[2]] = f.y; }
          if (hr) { J.c_cl[cb + icl++] = f.z; J.c_rc[rb + ncol[3] + x[3]] = f.w; }
          if (gap) J.c_in[ib + iin++] = 10;    // Skip
          J.c_in[ib + iin] = (uint8_t)(ho || hr ? info & ~0x20u : info);
          if (noo) {
            J.c_pi[rb + ncol[6] + x[6]] = (uint8_t)pi;
            if (!pi) { J.c_cl[cb + icl++] = f.x; J.c_lc[rb + ncol[2] + x[2]] = f.y; }
          }
          const bool es[3] = {e0, e1, e2};
#pragma unroll
          for (int z = 0; z < 3; z++) {
            if (!es[z]) continue;
            J.c_st[cb + ist] = s[z];
            J.c_sbo[cb + ist] = sbo;
            ist++;
            sbo += (uint32_t)(s[z] & 0xffffff);
          }
          if (ref == 7) J.c_tr[rb + ncol[7] + x[7]] = (uint8_t)t;
          if (ref == 1 || ref == 8) J.c_ln[rb + ncol[8] + x[8]] = J.rlen[q];
          J.o_off[rb + p] = sect + x[9];
        }
#pragma unroll
        for (int z = 0; z < 9; z++) ncol[z] += tot[z];
        sect += tot[9];
        sbody += tot[10];
      }
    }
    (void)bad;
  }
  __syncthreads();
  // ---- E. delete set: union per client (>= touching rule, max end), groups by first appearance
  uint32_t ngroups = 0, nranges = 0, qtot = 0;
  {
    uint32_t cg = 0, cr = 0;
    uint64_t cmx = 0, cmn = 0;
    bool bad = false;
    constexpr uint64_t M33 = (1ull << 33) - 1;
    for (uint32_t t0 = 0; t0 < nds; t0 += BT) {
      const uint32_t e = t0 + tid;
      const bool v = e < nds;
      uint64_t key = 0, pkey = 0, nkey = 0;
      uint32_t len = 0, idx = 0, nlen = 0;
      if (v) {
        const uint32_t gi = J.sdidx[dsb + e];
        key = J.sdkey[dsb + e];
        idx = gi - dsb;  // emission index = first-appearance order (update, position)
        len = J.dlen[gi];
        if (e > 0) pkey = J.sdkey[dsb + e - 1];
        if (e + 1 < nds) {
          nkey = J.sdkey[dsb + e + 1];
          nlen = J.dlen[J.sdidx[dsb + e + 1]];
        }
      }
      (void)nlen;
      const uint32_t cli = (uint32_t)(key >> 32), clk = (uint32_t)key;
      const uint64_t end = (uint64_t)clk + len;
      const bool segst = v && (e == 0 || (uint32_t)(pkey >> 32) != cli);
      const bool seglast = v && (e + 1 >= nds || (uint32_t)(nkey >> 32) != cli);
      uint32_t xs[1] = {segst}, ts[1];
      bscan<1>(S, xs, ts);
      const uint32_t segid = cg + xs[0] + segst - 1;
      uint64_t tmx, tmn, exm;
      const uint64_t mx = bmax(S, v ? ((uint64_t)segid << 33) | end : 0, cmx, tmx, &exm);
      const uint64_t mn = bmax(S, v ? ((uint64_t)segid << 32) | (uint32_t)~idx : 0, cmn, tmn);
      const bool newr = v && (segst || clk > (exm & M33));
      // the next entry starts a new range when it starts a segment or lies past this running max
      const bool nnew = !v || seglast || (uint32_t)nkey > (mx & M33);
      uint32_t xr[1] = {newr}, tr_[1];
      bscan<1>(S, xr, tr_);
      const uint32_t rid = cr + xr[0] + newr - 1;
      if (v) {
        if (newr) {
          J.q_clk[dsb + rid] = clk;
          J.q_grp[dsb + rid] = segid;
        }
        if (nnew) {
          bad |= (mx & M33) > 0xffffffffull;
          J.q_end[dsb + rid] = (uint32_t)(mx & M33);
        }
        if (segst) {
          J.g_first[dsb + segid] = rid;
          J.g_cli[dsb + segid] = cli;
        }
        if (seglast) J.g_min[dsb + segid] = ~(uint32_t)mn;
      }
      cg += ts[0];
      cr += tr_[0];
      cmx = tmx;
      cmn = tmn;
    }
    if (bor(S, bad) || cg > GMAX) { decline(); return; }
    ngroups = cg;
    nranges = cr;
    // range bytes (V1: clock, len; V2: clock - previous end of the client, len - 1) -> prefix q_pre
    uint32_t cq = 0;
    for (uint32_t t0 = 0; t0 < nranges; t0 += BT) {
      const uint32_t q = t0 + tid;
      uint32_t x[1] = {0}, t[1];
      if (q < nranges) {
        const uint32_t c0 = J.q_clk[dsb + q], e0 = J.q_end[dsb + q], g = J.q_grp[dsb + q];
        const uint32_t pe = q > J.g_first[dsb + g] ? J.q_end[dsb + q - 1] : 0;
        x[0] = V2 ? gvsz(c0 - pe) + gvsz(e0 - c0 - 1) : gvsz(c0) + gvsz(e0 - c0);
      }
      bscan<1>(S, x, t);
      if (q < nranges) J.q_pre[dsb + q] = cq + x[0];
      cq += t[0];
    }
    qtot = cq;
  }
  // groups ranked by first appearance (min emission index), bytes by rank, offsets by a scan
  for (uint32_t g = tid; g < ngroups; g += BT) S.gmin[g] = J.g_min[dsb + g];
  __syncthreads();
  auto qpre = [&](uint32_t x) { return x < nranges ? J.q_pre[dsb + x] : qtot; };
  for (uint32_t g = tid; g < ngroups; g += BT) {
    const uint32_t mine = S.gmin[g];
    uint32_t rk = 0;
    for (uint32_t h = 0; h < ngroups; h++) rk += S.gmin[h] < mine;
    const uint32_t f0 = J.g_first[dsb + g], f1 = g + 1 < ngroups ? J.g_first[dsb + g + 1] : nranges;
    J.g_woff[dsb + g] = rk;
    J.g_rb[dsb + rk] = gvsz(J.g_cli[dsb + g]) + gvsz(f1 - f0) + qpre(f1) - qpre(f0);
  }
  __syncthreads();
  const uint32_t ds_hdr = gvsz(ngroups);
  uint32_t ds_bytes = ds_hdr;
  for (uint32_t t0 = 0; t0 < ngroups; t0 += BT) {
    const uint32_t r = t0 + tid;
    uint32_t x[1] = {r < ngroups ? J.g_rb[dsb + r] : 0}, t[1];
    bscan<1>(S, x, t);
    if (r < ngroups) J.g_rb[dsb + r] = ds_bytes + x[0];
    ds_bytes += t[0];
  }
  __syncthreads();
  for (uint32_t g = tid; g < ngroups; g += BT) {
    const uint32_t off = J.g_rb[dsb + J.g_woff[dsb + g]];
    const uint32_t f0 = J.g_first[dsb + g], f1 = g + 1 < ngroups ? J.g_first[dsb + g + 1] : nranges;
    J.g_woff[dsb + g] = off;
    J.g_min[dsb + g] = off + gvsz(J.g_cli[dsb + g]) + gvsz(f1 - f0) - qpre(f0);  // base of its ranges
  }
  if (tid == 0) {
    uint32_t *const info = J.dinfo + (uint64_t)DI_N * i;
    info[DI_NPARTS] = nparts;
    for (int z = 0; z < 9; z++) info[DI_NCOL + z] = ncol[z];
    info[DI_SBODY] = sbody;
    info[DI_SECT] = sect;
    info[DI_NGROUPS] = ngroups;
    info[DI_NRANGES] = nranges;
    info[DI_DSBYTES] = ds_bytes;
  }
}

// ---- 3c. per document: placement in its slot, header, rest / rows, delete set (V2 columns: k_lm_col)
template <bool V2>
__global__ void __launch_bounds__(BT) k_lm_doc2(LMJob J) {
  const uint32_t i = blockIdx.x, tid = threadIdx.x;
  if (J.bad[i]) return;
  const DocB D = doc_bases(J, i);
  const uint32_t d = D.d, rb = D.rb, ns = D.ns, dsb = D.dsb;
  const uint64_t b0 = D.b0, bytes = D.bytes;
  uint32_t *const info = J.dinfo + (uint64_t)DI_N * i;
  const uint32_t nparts = info[DI_NPARTS], sect = info[DI_SECT], ngroups = info[DI_NGROUPS];
  const uint32_t nranges = info[DI_NRANGES], ds_bytes = info[DI_DSBYTES];
  uint32_t csz[9];
  for (int z = 0; z < 9; z++) csz[z] = V2 ? info[DI_CSZ + z] : 0;
  // ---- F. placement: the document's slot (2 * input bytes before it + 64 * d, 16-aligned)
  uint32_t cbase[9], colbytes = 0;
  {
    uint32_t p = 1;
#pragma unroll
    for (int c = 0; c < 9; c++) {
      p += gvsz(csz[c]);
      cbase[c] = p;
      p += csz[c];
    }
    colbytes = p;
  }
  const uint32_t hdr = V2 ? colbytes + gvsz(nparts) : gvsz(nparts);
  const uint64_t total = (uint64_t)hdr + sect + ds_bytes;
  const uint64_t slot = 2 * (b0 - J.upd_off[0]) + 64ull * d;
  const uint64_t slot_al = (slot + 15) & ~15ull;
  const uint64_t lim = slot + 2 * bytes + 64;
  if (slot_al + total > lim || slot_al + total > J.cap) {
    if (tid == 0) J.bad[i] = 1;  // status stays ST_PENDING: the general path takes the document
    return;
  }
  uint8_t *dst = J.out + slot_al;
  if (tid == 0) {
    *(uint64_t *)(info + DI_SLOT) = slot_al;
    for (int c = 0; c < 9; c++) info[DI_CBASE + c] = cbase[c];
  }
  // ---- G. struct section (the V2 columns themselves: k_lm_col<true>)
  if (tid == 0) {
    if (V2) {
      dst[0] = 0;
      uint32_t p = 1;
      for (int c = 0; c < 9; c++) p = gput_vu(dst, p, csz[c]) + csz[c];
      gput_vu(dst, colbytes, nparts);
    } else {
      gput_vu(dst, 0, nparts);
    }
  }
  for (uint32_t p = tid; p < ns; p += BT) {
    const uint32_t q = J.ord[rb + p], gap = J.o_gap[rb + p], pw = J.o_pw[rb + p];
    const uint64_t key = J.rkey[q];
    const uint32_t client = ~(uint32_t)(key >> 32), clock = (uint32_t)key;
    uint32_t o = hdr + J.o_off[rb + p];
    const uint64_t src = J.rsrc[q];
    const uint32_t n = J.rbn[q];
    if (V2) {  // rest: part header (written, first clock), Skip length, payload
      if (pw) { o = gput_vu(dst, o, pw); o = gput_vu(dst, o, clock); }
      if (gap) o = gput_vu(dst, o, gap);
      copy_bytes(dst + o, J.A + src, n);
    } else {   // row: part header (written, client, clock), Skip, info (0x20 only without origins), body
      if (pw) { o = gput_vu(dst, o, pw); o = gput_vu(dst, o, client); o = gput_vu(dst, o, clock); }
      if (gap) { dst[o++] = 10; o = gput_vu(dst, o, gap); }
      const uint32_t info = J.raux[q] & 0xff;
      dst[o++] = (uint8_t)(info & 0xC0 ? info & ~0x20u : info);
      copy_bytes(dst + o, J.A + src + 1, n - 1);
    }
  }
  // ---- H. delete set
  const uint32_t dsbase = hdr + sect;
  if (tid == 0) gput_vu(dst, dsbase, ngroups);
  for (uint32_t g = tid; g < ngroups; g += BT) {
    const uint32_t f0 = J.g_first[dsb + g], f1 = g + 1 < ngroups ? J.g_first[dsb + g + 1] : nranges;
    gput_vu(dst, gput_vu(dst, dsbase + J.g_woff[dsb + g], J.g_cli[dsb + g]), f1 - f0);
  }
  for (uint32_t q = tid; q < nranges; q += BT) {
    const uint32_t c0 = J.q_clk[dsb + q], e0 = J.q_end[dsb + q], g = J.q_grp[dsb + q];
    const uint32_t off = dsbase + J.g_min[dsb + g] + J.q_pre[dsb + q];
    if (V2) {
      const uint32_t pe = q > J.g_first[dsb + g] ? J.q_end[dsb + q - 1] : 0;
      gput_vu(dst, gput_vu(dst, off, c0 - pe), e0 - c0 - 1);
    } else {
      gput_vu(dst, gput_vu(dst, off, c0), e0 - c0);
    }
  }
  if (tid == 0) {
    J.out_off[d] = slot_al;
    J.out_len[d] = total;
    J.status[d] = ym::ST_OK;
  }
}

}  // namespace lm

// ---- host: the large-document pipeline over a list of documents the fast path declined -----------
namespace {
template <class T>
T *carve(uint8_t *&p, uint64_t n) {
  T *r = reinterpret_cast<T *>(p);
  p += (n * sizeof(T) + 255) & ~255ull;
  return r;
}
template <class T>
uint64_t csize(uint64_t n) { return (n * sizeof(T) + 255) & ~255ull; }
int ensure(LargeBufs &B, int k, size_t n) {
  if (n <= B.cap[k]) return 0;
  if (B.p[k]) hipFree(B.p[k]);
  B.p[k] = nullptr;
  B.cap[k] = 0;
  const size_t want = n + n / 4 + 4096;
  if (hipMalloc(&B.p[k], want) != hipSuccess) return -1;
  B.cap[k] = want;
  return 0;
}
}  // namespace

#define LMCHK(x)                                 \
  do {                                           \
    hipError_t e_ = (x);                         \
    if (e_ != hipSuccess) return -(int)e_ - 1000; \
  } while (0)

int large_run(const GeneralJob &j, const uint32_t *list, uint32_t nb, uint32_t n_upd, hipStream_t st, LargeBufs &B) {
  using namespace lm;
  if (j.op != OP_MERGE || nb == 0) return 0;
  if (!B.pinned_dev) {
    if (B.pinned) hipHostFree(B.pinned);
    B.pinned = nullptr;
    if (hipHostMalloc((void **)&B.pinned, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -2;
    if (hipHostGetDevicePointer((void **)&B.pinned_dev, B.pinned, 0) != hipSuccess) return -2;
  }
  LMJob J;
  memset(&J, 0, sizeof(J));
  J.A = j.A;
  J.upd_off = j.upd_off;
  J.doc_upd = j.doc_upd;
  J.v2 = j.v2;
  J.nb = nb;
  J.bdoc = list;
  J.status = j.status;
  J.out = j.out;
  J.cap = j.cap;
  J.out_off = j.out_off;
  J.out_len = j.out_len;
  // per-document arrays
  const uint64_t n1 = nb + 1;
  if (ensure(B, 0, 4 * csize<uint32_t>(n1) + csize<uint32_t>(nb) + csize<uint32_t>(4ull * nb) + csize<uint32_t>((uint64_t)DI_N * nb) + 512))
    return -2;
  uint8_t *p = (uint8_t *)B.p[0];
  J.bu_off = carve<uint32_t>(p, n1);
  J.ch_off = carve<uint32_t>(p, n1);
  uint32_t *kcnt = carve<uint32_t>(p, n1);
  uint32_t *ccnt = carve<uint32_t>(p, n1);
  J.bad = carve<uint32_t>(p, nb);
  uint32_t *seg = carve<uint32_t>(p, 4ull * nb);
  uint32_t *tot = carve<uint32_t>(p, 4);
  J.dinfo = carve<uint32_t>(p, (uint64_t)DI_N * nb);
  k_lm_prep<<<(nb + 256) / 256, 256, 0, st>>>(J, list, kcnt, ccnt);
  size_t tmp = 0, t2 = 0;
  scan_excl<uint32_t>(nullptr, tmp, kcnt, J.bu_off, n1, st);
  if (ensure(B, 3, tmp + 256)) return -2;
  if (scan_excl<uint32_t>(B.p[3], tmp, kcnt, J.bu_off, n1, st) || scan_excl<uint32_t>(B.p[3], tmp, ccnt, J.ch_off, n1, st)) return -3;
  LMCHK(hipMemcpyAsync(tot, J.bu_off + nb, 4, hipMemcpyDeviceToDevice, st));
  LMCHK(hipMemcpyAsync(tot + 1, J.ch_off + nb, 4, hipMemcpyDeviceToDevice, st));
  // no host round trip for the update / chunk totals: the per-update count arrays are sized by the
  // batch's update count and the walk's grid by the chunk bound (the walk reads the true total, tot[1])
  const uint32_t nbu = n_upd, nch = (uint32_t)((n_upd + 63ull * nb) / 64);  // >= sum over listed docs of ceil(k / 64)
  if (nch == 0) return 0;
  J.stride = nbu + 1;
  if (ensure(B, 1, 2 * csize<uint32_t>(3ull * J.stride))) return -2;
  p = (uint8_t *)B.p[1];
  J.u_cnt = carve<uint32_t>(p, 3ull * J.stride);
  J.u_off = carve<uint32_t>(p, 3ull * J.stride);
  // the listed documents' updates only (tot[0] of them; J.stride, the batch's update count + 1, bounds it)
  k_lm_zero<<<(J.stride + 255) / 256, 256, 0, st>>>(J, tot);
  const uint32_t grid = nch < 65536 ? nch : 65536;
  if (J.v2) k_lm_walk<false, true><<<grid, 64, WALK_LDS, st>>>(J, tot);
  else k_lm_walk<false, false><<<grid, 64, WALK_LDS, st>>>(J, tot);
  scan_excl<uint32_t>(nullptr, t2, J.u_cnt, J.u_off, J.stride, st, tot, 1);
  if (ensure(B, 3, t2 + 256)) return -2;
  for (int k = 0; k < 3; k++)
    if (scan_excl<uint32_t>(B.p[3], t2, J.u_cnt + k * J.stride, J.u_off + k * J.stride, J.stride, st, tot, 1)) return -3;
  k_lm_totals<<<1, 64, 0, st>>>(J, tot, (uint32_t *)B.pinned_dev);
  LMCHK(hipStreamSynchronize(st));
  if (((uint32_t *)B.pinned)[3] == 0) return 0;  // no listed document has a chunk: all stay pending
  const uint64_t NS = ((uint32_t *)B.pinned)[0] + 1ull, NR = ((uint32_t *)B.pinned)[1] + 1ull, ND = ((uint32_t *)B.pinned)[2] + 1ull;
  const bool v2 = J.v2;
  const uint64_t NT = NR > ND ? NR : ND;  // the sorts' scratch pair
  uint64_t need = csize<uint64_t>(NT) + csize<uint32_t>(NT) + csize<uint64_t>(NS) * 2 + csize<uint32_t>(NS) * 3 + (v2 ? csize<uint4>(NS) + csize<uint64_t>(3 * NS) : 0) +
                  csize<uint64_t>(NR) * 2 + csize<uint32_t>(NR) * 10 + csize<uint32_t>(NS) * 4 +
                  csize<uint64_t>(ND) * 2 + csize<uint32_t>(ND) * 12 +
                  (v2 ? csize<uint32_t>(3 * NS) * 2 + csize<uint32_t>(NS) * 3 + csize<uint8_t>(2 * NS) + csize<uint8_t>(NS) * 2 +
                            csize<uint64_t>(3 * NS) : 0) + 4096;
  if (ensure(B, 2, need)) return -2;
  p = (uint8_t *)B.p[2];
  J.rkey = carve<uint64_t>(p, NS);
  J.rsrc = carve<uint64_t>(p, NS);
  J.rlen = carve<uint32_t>(p, NS);
  J.raux = carve<uint32_t>(p, NS);
  J.rbn = carve<uint32_t>(p, NS);
  if (v2) {
    J.rf = carve<uint4>(p, NS);
    J.rs = carve<uint64_t>(p, 3 * NS);
  }
  J.runkey = carve<uint64_t>(p, NR);
  J.srunkey = carve<uint64_t>(p, NR);
  J.runidx = carve<uint32_t>(p, NR);
  J.srunidx = carve<uint32_t>(p, NR);
  J.runfirst = carve<uint32_t>(p, NR);
  J.runcnt = carve<uint32_t>(p, NR);
  J.runend = carve<uint32_t>(p, NR);
  J.a_sbase = carve<uint32_t>(p, NR);
  J.a_gap = carve<uint32_t>(p, NR);
  J.a_pid = carve<uint32_t>(p, NR);
  J.p_uf = carve<uint32_t>(p, NR);
  J.p_ul = carve<uint32_t>(p, NR);
  J.ord = carve<uint32_t>(p, NS);
  J.o_gap = carve<uint32_t>(p, NS);
  J.o_pw = carve<uint32_t>(p, NS);
  J.o_off = carve<uint32_t>(p, NS);
  J.dkey = carve<uint64_t>(p, ND);
  J.sdkey = carve<uint64_t>(p, ND);
  J.dlen = carve<uint32_t>(p, ND);
  J.didx = carve<uint32_t>(p, ND);
  J.sdidx = carve<uint32_t>(p, ND);
  J.q_clk = carve<uint32_t>(p, ND);
  J.q_end = carve<uint32_t>(p, ND);
  J.q_grp = carve<uint32_t>(p, ND);
  J.q_pre = carve<uint32_t>(p, ND);
  J.g_first = carve<uint32_t>(p, ND);
  J.g_cli = carve<uint32_t>(p, ND);
  J.g_min = carve<uint32_t>(p, ND);
  J.g_woff = carve<uint32_t>(p, ND);
  J.g_rb = carve<uint32_t>(p, ND);
  if (v2) {
    J.c_cl = carve<uint32_t>(p, 3 * NS);
    J.c_sbo = carve<uint32_t>(p, 3 * NS);
    J.c_lc = carve<uint32_t>(p, NS);
    J.c_rc = carve<uint32_t>(p, NS);
    J.c_ln = carve<uint32_t>(p, NS);
    J.c_in = carve<uint8_t>(p, 2 * NS);
    J.c_pi = carve<uint8_t>(p, NS);
    J.c_tr = carve<uint8_t>(p, NS);
    J.c_st = carve<uint64_t>(p, 3 * NS);
  }
  uint64_t *skt = carve<uint64_t>(p, NT);
  uint32_t *svt = carve<uint32_t>(p, NT);
  if ((uint64_t)(p - (uint8_t *)B.p[2]) > B.cap[2]) return -3;
  if (J.v2) k_lm_walk<true, true><<<grid, 64, WALK_LDS, st>>>(J, tot);
  else k_lm_walk<true, false><<<grid, 64, WALK_LDS, st>>>(J, tot);
  k_lm_segs<<<(nb + 255) / 256, 256, 0, st>>>(J, seg);
  // segmented radix sorts (ym_segsort.hip, one workgroup per document): runs by (~client << 32 | clock),
  // delete ranges by (client << 32 | clock)
  if (NR > 1 && segsort_pairs(J.runkey, J.runidx, J.srunkey, J.srunidx, skt, svt, seg, seg + nb, nb, st)) return -3;
  if (ND > 1 && segsort_pairs(J.dkey, J.didx, J.sdkey, J.sdidx, skt, svt, seg + 2 * nb, seg + 3 * nb, nb, st)) return -3;
  if (J.v2) {
    k_lm_doc1<true><<<nb, BT, 0, st>>>(J);
    k_lm_col<false><<<dim3(nb, 9), BT, 0, st>>>(J);
    k_lm_doc2<true><<<nb, BT, 0, st>>>(J);
    k_lm_col<true><<<dim3(nb, 9), BT, 0, st>>>(J);
  } else {
    k_lm_doc1<false><<<nb, BT, 0, st>>>(J);
    k_lm_doc2<false><<<nb, BT, 0, st>>>(J);
  }
  return 1;
}

}  // namespace ymk
