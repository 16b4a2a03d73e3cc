// ym_pwalk.hip -- chunk-parallel V1 diffUpdate / encodeStateVectorFromUpdate over large single updates
// (BASELINE configs[2] C3: 0.9 MB updates of ~70 k structs; configs[4] C5 diff).
//
// A V1 update is a byte stream of structs whose boundaries are only known by parsing from the start,
// which made the previous design (ym_big.hip) one sequential walk per document.  Here the walk is split:
//
//  1. k_pw_walk -- one lane per 1 KB chunk of every document (C3: 3.6 M lanes).  Each lane parses
//     structs *speculatively* from its chunk's first byte: a position where no struct parses is recorded
//     as a FAIL and the walk resumes one byte later.  V1 structs re-synchronise within a few structs, so
//     after a short garbage prefix the lane is on the document's true struct chain.  Every step is
//     recorded (position | flags, clock length), plus the chunk's exit position (>= the chunk's end).
//  2. k_pw_stitch -- one wave per document.  It follows the true chain chunk by chunk: at a chunk it
//     finds its entry position among the chunk's records (a ballot over 64 records), then consumes the
//     records 64 at a time: clocks by a wave prefix sum, the diff cut by a ballot (the segmented search of
//     SURVEY §8a), Skips and info-byte patches by ballots.  Where the entry is not a record (the lane's
//     speculative chain skipped it) or is a FAIL (a string / ContentAny longer than the speculative cap,
//     or a real error), the stitch parses that one struct itself, uncapped, and goes on; an error on the
//     true chain declines the document to the sequential walker.  Section headers and the delete set are
//     parsed by the stitch (the delete set's varuints are validated 1 KB per wave step by a ballot over
//     continuation bits).  The output is assembled as in ym_big.hip: part headers and the sliced first
//     struct written by lane 0, verbatim spans copied by the wave, then the info-byte patches.
//
// Semantics are exactly those of ym_big.hip's k_big_v1 (yjs 13.5.16 diffUpdate / encodeStateVector-
// FromUpdate): the same structs are accepted (ym_lane.h mirrors ym_scalar.h), the same
// inputs are declined.  Documents this path declines (or does not take: several updates, < PW_MIN bytes)
// go to k_big_v1, and from there to the general path.
#include <hip/hip_runtime.h>
#include "ym_scan.h"

#include "ym_fast_common.h"
#include "ym_kernels.h"
#include "ym_lane.h"
#include "ym_scalar.h"
#include "ym_wave_ds.h"
#include "ym_cmap.h"

namespace ymk {
namespace pw {
using namespace fastc;
using ln::F_FAIL;
using ln::F_PATCH;
using ln::F_SKIP;
using ln::POS_MASK;
using sc::SCur;

constexpr uint32_t CH = 1024;          // chunk bytes (one walking lane each)
constexpr uint32_t CAP = CH / 2 + 8;   // records per chunk (a struct is >= 2 bytes; FAIL runs on top: overflow)
// longest string / binary / ContentAny a speculative parse accepts: a larger length read at a position
// that does not start a struct would make the lane jump over the true chain (C3: with no cap on binaries
// 3 % of the chunks never re-synchronised; with 64 the walk meets the true chain after 7 bytes on average,
// 31 at p99).  Longer true contents are re-parsed uncapped by the stitch.
constexpr uint32_t SPEC_CAP = 64;
constexpr uint32_t NFIRST = 8;         // records per chunk descriptor (the stitch's entry lookup)
constexpr uint32_t FAIL_RUN = 8;       // failed positions in a row before the walk only tries short-cut candidates
// a chunk starts mid-struct: its first START_CHEAP bytes try short-cut candidates only (C3 meets the true
// chain there after a few bytes); a chunk still off the chain after them (structs outside the short cut,
// C5's XML items) goes back to the full parser at every position
constexpr uint32_t START_CHEAP = 48;
constexpr uint32_t PRE_ONE = 0, PRE_MANY = 512;  // k_pw_walk's pre-roll (bytes before the chunk, no records)
// longest string / binary / ContentAny the window tables accept (k_pw_ms, k_pw_small): a table entry is a
// parse at an offset that may not start a struct, and an uncapped parse there can run to the window's end
// (a garbage length read as a string to validate): the tables cost O(window x cap).  Longer true contents
// are parsed uncapped by the chain walk itself.
constexpr uint32_t TAB_CAP = 128;
constexpr uint64_t PW_MIN = 32768;     // smaller updates stay on k_big_v1
constexpr uint32_t NSEC = BS_NSEC, NSV = BS_NSV, PRE = BS_PRE, SECW = BS_SECW;
constexpr uint32_t NPATCH = 1024;
constexpr uint32_t L_PPOS = 0;                     // u32[NPATCH] patch positions (document-relative)
constexpr uint32_t L_PSEC = L_PPOS + 4 * NPATCH;   // u32[NPATCH] section of each patch
constexpr uint32_t L_PVAL = L_PSEC + 4 * NPATCH;   // u8[NPATCH]  patched info bytes
constexpr uint32_t L_REC = L_PVAL + NPATCH;        // u32[CAP] the records of the chunk being consumed
constexpr uint32_t LDS_BYTES = L_REC + 4 * CAP;
constexpr uint32_t L_DSL = (LDS_BYTES + 15) & ~15u;  // diff: wds::DsLdsS (the delete set's token tables, 1 KB windows:
                                                    // the 4 KB ones cost the stitch its occupancy -- C3 V1 diff 14 -> 24 ms)
constexpr uint32_t L_SVM = (L_DSL + (uint32_t)sizeof(wds::DsLdsS) + 15) & ~15u;  // diff, DSL: lsv's map (32 KB)
enum { S_PRELEN = 0, S_A0, S_A1, S_B0, S_B1, S_WRITTEN, S_CLIENT, S_FCLOCK, S_OUTB };
constexpr uint32_t NONE = 0xffffffffu;

struct Scr {
  uint32_t *sec, *svt, *dsc;
  uint8_t *pre;
  uint32_t *map;
};
__device__ __forceinline__ Scr scratch(const GeneralJob &j) {
  uint8_t *b = j.bscratch + (uint64_t)blockIdx.x * BS_BYTES;
  return Scr{(uint32_t *)(b + BS_SEC), (uint32_t *)(b + BS_SVT), (uint32_t *)(b + BS_DSC), b + BS_PREB, (uint32_t *)(b + BS_MAP)};
}
#define sec(ci, f) X.sec[SECW * (ci) + (f)]

// stitch path counters (build with -DYM_PW_PROF; read with ym__pw_prof): [0] chunks consumed whole from
// their entry, [1] entry found but the chunk not whole, [2] entry not among the first records, [3] record
// batches, [4] structs re-parsed by the stitch, [5] record search loads
__device__ unsigned long long pw_prof[16];
#ifdef YM_PW_PROF
#define PWP(i) do { if (threadIdx.x == 0) atomicAdd(&pw_prof[i], 1ull); } while (0)
#else
#define PWP(i) do { } while (0)
#endif
// stitch phase time (same build; ym__pw_ticks, 100 MHz ticks summed over documents): PT(i) charges the
// time since the previous PT to phase i -- [0] state vector, [1] section headers + SV lookup, [2] chunk
// descriptors + O(1) entry, [3] record staging, [4] record search, [5] consumption, [6] the cut + sliced
// head, [7] delete set, [8] sizes + allocation, [9] write, [10] patches
__device__ unsigned long long pw_ticks[16];
#if defined(YM_PW_PROF) || defined(YM_PW_TICKS)
#define PT_DECL uint64_t pt_t = __builtin_amdgcn_s_memrealtime(), pt_acc[11] = {};
#define PT(i) do { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); pt_acc[i] += t_ - pt_t; pt_t = t_; } while (0)
#define PT_FLUSH() do { if (threadIdx.x == 0) for (int i_ = 0; i_ < 11; i_++) atomicAdd(&pw_ticks[i_], pt_acc[i_]); } while (0)
#else
#define PT_DECL
#define PT(i) do { } while (0)
#define PT_FLUSH() do { } while (0)
#endif
// Record k of chunk g: chunk-major (a chunk's records are contiguous: the stitch stages them with one
// coalesced read).  The walking lane collects four records in registers and stores them as one 16-byte
// write, so a chunk's lines fill from one lane in order and leave L2 whole.  (Measured, C3 V1 diff: records
// interleaved across the wave's 64 chunks -- one 4-byte store per record, each lane of a store on another
// line -- wrote 4.2 GB per launch for 0.5 GB of records: every record cost a 32-byte partial write.)
__device__ __forceinline__ uint64_t rec_idx(uint32_t g, uint32_t k) { return (uint64_t)g * CAP + k; }
// A record is one u32: the struct's offset in its chunk (10 bits), its flags (bits 10-12: FAIL, Skip, patch)
// and its clock length (19 bits; a longer struct is recorded as a FAIL, so the stitch re-parses it).  Half
// the bytes of the (position, clock sum) pair it replaced: the walk writes, and the stitch reads, 4 bytes
// per struct.
constexpr uint32_t REC_CLEN = 1u << 19;
__device__ __forceinline__ uint32_t rec_make(uint32_t off, uint32_t fl, uint32_t clen) {
  return off | ((fl >> 18) & 0x1c00u) | (clen << 13);
}
// the record's position word (document position | F_* flags) in chunk cx
__device__ __forceinline__ uint32_t rec_pw(uint32_t w, uint32_t cx) { return (cx * CH + (w & 1023u)) | ((w & 0x1c00u) << 18); }
__device__ __forceinline__ uint32_t rec_clen(uint32_t w) { return w >> 13; }
// ---- 0. eligibility and chunk counts ---------------------------------------------------------------
// msz[d]: the section-parallel stitch's per-document area (k_pw_ms), for documents of >= ms_min sections
__host__ __device__ inline uint64_t ms_area(uint32_t nsec);
// *many: set when a chunk-walked document has > 64 client sections (the stitch then validates delete sets through
// LDS token tables; C5: ~1,000 clients)
__global__ void k_pw_prep(GeneralJob j, uint32_t *cnt, uint8_t *done, uint64_t pw_min, uint64_t *msz, uint32_t ms_min,
                          uint32_t *many) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d > j.n) return;
  uint32_t c = 0;
  uint64_t a = 0;
  if (d < j.n) {
    done[d] = 0;
    const uint32_t u0 = j.doc_upd[d];
    if (j.doc_upd[d + 1] - u0 == 1) {
      const uint64_t len = j.upd_off[u0 + 1] - j.upd_off[u0];
      if (len >= pw_min && len > 0 && len < (1ull << 28)) {
        c = (uint32_t)((len + CH - 1) / CH);
        ln::LCur h = ln::make(j.A + j.upd_off[u0], 0, (uint32_t)len);
        const uint32_t nsec = ln::rvu(h);
        if (!h.bad && nsec >= ms_min && nsec <= (1u << 16)) { a = ms_area(nsec); c = 0; }  // (the table walk: no chunks)
        if (c && !h.bad && nsec > 64) atomicOr(many, 1u);
      }
    }
  }
  cnt[d] = c;  // cnt[n] = 0: the exclusive scan's last entry is the total
  msz[d] = a;
  // the totals the host sizes the record buffers by (only large documents add: no contention otherwise)
  if (c) atomicAdd(many + 2, c);
  if (a) atomicAdd((unsigned long long *)(many + 4), (unsigned long long)a);
}

// the prep's totals (six words) straight into the coherent pinned host words pw_finish reads
__global__ void k_pw_totals(const uint32_t *many, uint32_t *host) {
  if (threadIdx.x < 6) host[threadIdx.x] = many[threadIdx.x];
}

// ---- 1. speculative chunk walk ----------------------------------------------------------------------
// Records: one u32 per step (offset in the chunk | flags | clock length, rec_make).  Chunk descriptor
// (5 x 16 B): {nrec | lastfail << 16, lastpatch | lastskip << 16, exit, clock sum at exit}, then the
// first NFIRST records' position words and clock sums (the stitch's entry lookup needs no record load).
// last* = index + 1 of the last FAIL / patched / Skip record (0: none); a struct of >= 2^19 clocks is
// recorded as a FAIL (its length does not fit the record): the stitch takes such records one by one.
// pre_one / pre_many: bytes walked before the chunk's first byte, without records (documents of <= 16 / > 16
// client sections), so that the chain is met before the chunk starts: the stitch then finds its entry among
// the chunk's first records instead of re-parsing structs in lockstep until the chain meets it (round 6)
__global__ void __launch_bounds__(256) k_pw_walk(GeneralJob j, const uint32_t *cbase, uint32_t nd, uint32_t total,
                                                 uint4 *desc, uint32_t *recs, uint32_t pre_one, uint32_t pre_many) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  uint32_t lo = 0, hi = nd - 1;  // the document: largest d with cbase[d] <= g
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (cbase[mid] <= g) lo = mid; else hi = mid - 1;
  }
  const uint32_t d = lo, ci = g - cbase[d];
  const uint32_t u0 = j.doc_upd[d];
  const uint64_t ub = j.upd_off[u0];
  const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
  const uint8_t *D = j.A + ub;
  const uint32_t c0 = ci * CH, c1 = c0 + CH < len ? c0 + CH : len;
  // documents of many client sections (C5) try a section header where the chain falls off (below)
  bool many = false;
  {
    ln::LCur h = ln::make(D, 0, len);
    many = ln::rvu(h) > 16 && !h.bad;
  }
  uint32_t nrec = 0, cum = 0, lastfail = 0, lastpatch = 0, lastskip = 0, fails = FAIL_RUN, okrun = 0;  // the chunk start is mid-struct: only short-cut candidates until two structs in a row
  bool frun = false, ovf = false, start = true;
  const uint32_t pre = many ? pre_many : pre_one;
  const uint32_t w0 = c0 > pre ? c0 - pre : 0;  // the walk's start (records from c0 on)
  uint32_t p = w0;
  // the descriptor's first-record words (position | flags, clock sum) are stored as the records come
  uint4 *Q = desc + 5ull * g;
  uint4 rq = make_uint4(0, 0, 0, 0);  // the records of the current group of four
  uint32_t *fpw = reinterpret_cast<uint32_t *>(Q + 1), *fcum = reinterpret_cast<uint32_t *>(Q + 3);
  Q[1] = Q[2] = make_uint4(POS_MASK, POS_MASK, POS_MASK, POS_MASK);
  Q[3] = Q[4] = make_uint4(0, 0, 0, 0);
  while (p < c1) {
    if (start && p >= w0 + START_CHEAP) {
      start = false;
      if (fails >= FAIL_RUN) fails = 0;
    }
    uint32_t cl, fl, nx;
    bool ok = ln::parse_fast(D, p, len, nx, cl, fl);  // branch-free short cut (most structs)
#ifdef YM_PW_PROF
    atomicAdd(&pw_prof[ok ? 6 : fails < FAIL_RUN ? 7 : 5], 1ull);
#endif
    if (!ok && fails < FAIL_RUN) {
      ln::LCur c = ln::make(D, p, len, SPEC_CAP);
      ok = ln::parse_at(c, cl, fl);
      nx = c.p;
    }
    // The chain just fell off at p after a struct: most often a section header (C5: ~1,000 per document).
    // Three varuints (#structs > 0, client, clock) followed by a struct that parses: the chain goes on past
    // the header (the FAIL recorded at p ends the previous section's last struct there), so the stitch finds
    // the section's first struct among the records instead of re-parsing until the chain meets it again.
    uint32_t hjump = 0;
    if (many && !ok && okrun >= 2 && p > w0) {  // (after >= 2 structs in a row: not inside a delete set's varuints)
      ln::LCur h = ln::make(D, p, len);
      const uint32_t ns = ln::rvu(h);
      ln::rvu(h);
      ln::rvu(h);
      if (!h.bad && ns > 0 && h.p < len) {
        uint32_t cl2, fl2, nx2;
        bool ok2 = ln::parse_fast(D, h.p, len, nx2, cl2, fl2);
        if (!ok2) {
          ln::LCur c2 = ln::make(D, h.p, len, SPEC_CAP);
          ok2 = ln::parse_at(c2, cl2, fl2);
        }
        if (ok2) hjump = h.p;
      }
    }
    const bool rec = p >= c0;  // (the pre-roll records nothing)
    if (rec && (ok || !frun)) {
      if (nrec == CAP) { ovf = true; break; }  // overflow: the stitch re-parses this chunk
      // a struct of >= 2^19 clocks is recorded as a FAIL (its length does not fit the record; clock sums
      // over the chunk could wrap): the stitch takes the records from the entry up to here one by one and
      // re-parses that struct
      const bool big = ok && cl >= REC_CLEN;
      const uint32_t rfl = ok && !big ? fl : F_FAIL;
      const uint32_t w = rec_make(p - c0, rfl, ok && !big ? cl : 0), sl = nrec & 3;
      rq.x = sl == 0 ? w : rq.x;
      rq.y = sl == 1 ? w : rq.y;
      rq.z = sl == 2 ? w : rq.z;
      rq.w = w;
      if (sl == 3) *reinterpret_cast<uint4 *>(recs + rec_idx(g, nrec - 3)) = rq;
      if (nrec < NFIRST) { fpw[nrec] = p | rfl; fcum[nrec] = cum; }
      nrec++;
      if (!ok || big) lastfail = nrec;
      if (ok && (fl & F_PATCH)) lastpatch = nrec;
      if (ok && (fl & F_SKIP)) lastskip = nrec;
    }
    cum += ok && rec ? cl : 0;
    // back to trying every position only after two structs in a row (a lone garbage GC in a delete set
    // would otherwise restart the run of full parses)
    okrun = ok ? okrun + 1 : 0;
    fails = ok ? (okrun >= 2 ? 0 : fails) : fails + 1;
    // a long run of non-struct bytes (the delete set, a long content): only positions the short cut could
    // accept are tried from there on -- the full parser at every byte of a 100 KB delete set cost more
    // than the whole struct section
    p = ok ? nx : hjump ? hjump : fails < FAIL_RUN ? p + 1 : ln::next_cand(D, p + 1, c1);
    frun = !ok && !hjump;
  }
  if (ovf) nrec = 0;
  if (nrec & 3) *reinterpret_cast<uint4 *>(recs + rec_idx(g, nrec & ~3u)) = rq;  // the last group (its tail: don't-care)
  Q[0] = make_uint4(nrec | (lastfail << 16), lastpatch | (lastskip << 16), p, cum);
}

// ---- 2. stitch ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sv_lookup(const uint32_t *svt, uint32_t nsv, uint32_t client) {
  int best = -1;
  for (uint32_t i0 = 0; i0 < nsv; i0 += 64) {
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t m = __ballot(i < nsv && svt[2 * i] == client);
    if (m) best = (int)(i0 + 63 - __builtin_clzll(m));
  }
  return best >= 0 ? svt[2 * best + 1] : 0;
}
__device__ __forceinline__ bool seen_before(const uint32_t *dsc, uint32_t n, uint32_t client) {
  bool hit = false;
  for (uint32_t h0 = 0; h0 < n; h0 += 64) {
    const uint32_t h = h0 + threadIdx.x;
    hit |= __any(h < n && dsc[h] == client);
  }
  return hit;
}
typedef uint4 __attribute__((aligned(1))) u4u;
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t n) {  // (one wave)
  const uint32_t nv = n >> 4;
  uint32_t v = threadIdx.x & 63;
  for (; v + 192 < nv; v += 256) {  // four 16-byte loads in flight per lane
    const uint4 a = reinterpret_cast<const u4u *>(src)[v], b = reinterpret_cast<const u4u *>(src)[v + 64];
    const uint4 c = reinterpret_cast<const u4u *>(src)[v + 128], e = reinterpret_cast<const u4u *>(src)[v + 192];
    reinterpret_cast<u4u *>(dst)[v] = a;
    reinterpret_cast<u4u *>(dst)[v + 64] = b;
    reinterpret_cast<u4u *>(dst)[v + 128] = c;
    reinterpret_cast<u4u *>(dst)[v + 192] = e;
  }
  for (; v < nv; v += 64) reinterpret_cast<u4u *>(dst)[v] = reinterpret_cast<const u4u *>(src)[v];
  for (uint32_t i = (nv << 4) + (threadIdx.x & 63); i < n; i += 64) dst[i] = src[i];
}
__device__ __forceinline__ uint32_t put_vu_g(uint8_t *o, uint32_t p, uint32_t v) {
  while (v > 127) { o[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
  o[p++] = (uint8_t)v;
  return p;
}

// Item.write / GC.write with offset `off` (> 0) of the struct at document position s0 (ending at s1):
// the re-encoded head goes to `pre` (lane 0), the content tail to span [a0, a1).  Returns SH_OK; SH_DECLINE
// (the content kind cannot be sliced here, a head longer than PRE); SH_URI when `off` splits a surrogate pair
// of a ContentString: ContentString.write(encoder, off) writes str.slice(off), which starts with a lone low
// surrogate, and V1 writeVarString (encodeURIComponent) throws URIError there -- yjs's diffUpdate throws it
// as it writes that struct, before reading anything after it (the lazy reader).
enum : uint32_t { SH_DECLINE = 0, SH_OK = 1, SH_URI = 2 };
__device__ __forceinline__ uint32_t slice_head_body(sc::cu32 *B, uint32_t adj, uint32_t s0, uint32_t s1, uint32_t client,
                                                   uint64_t clock, uint32_t len, uint32_t off, uint8_t *pre, uint32_t &prelen,
                                                   uint32_t &a0, uint32_t &a1) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t info = sc::byte(B, s0 + adj);
  const bool gc = (info & 31) == 0;
  uint8_t h[PRE + 16];
  uint32_t q = 0;
  auto put = [&](uint32_t v) { while (v > 127) { h[q++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } h[q++] = (uint8_t)v; };
  a0 = a1 = 0;
  if (gc) {
    h[q++] = 0;
    put(len - off);
  } else {
    const uint32_t ref = info & 31;
    if (ref != 1 && ref != 4 && ref != 8) return SH_DECLINE;
    SCur e = sc::make(B, s0 + adj + 1, s1 + adj);
    const uint32_t ni = ref | 0x80 | (info & 0x40) | ((info & 0xC0) == 0 ? (info & 0x20) : 0);
    if (info & 0x80) { sc::skvu(e); sc::skvu(e); }
    uint32_t ro0 = 0, ro1 = 0;
    if (info & 0x40) { ro0 = e.p; sc::skvu(e); sc::skvu(e); ro1 = e.p; }
    if ((info & 0xC0) == 0) {
      const uint32_t pi = sc::rvu(e);
      if (pi == 1) { const uint32_t n = sc::rvu(e); sc::skip(e, n); }
      else { sc::skvu(e); sc::skvu(e); }
      if (info & 0x20) { const uint32_t n = sc::rvu(e); sc::skip(e, n); }
    }
    h[q++] = (uint8_t)ni;
    put(client);
    put((uint32_t)(clock + off - 1));
    if (ro1 - ro0 > 10) return SH_DECLINE;
    for (uint32_t b = ro0; b < ro1; b++) h[q++] = (uint8_t)sc::byte(B, b);
    if (ref == 1) {
      sc::rvu(e);
      put(len - off);
    } else if (ref == 8) {
      sc::rvu(e);
      for (uint32_t i = 0; i < off; i++) sc::any_scalar(e);  // ContentAny.splice: drop `off` values
      put(len - off);
      a0 = e.p - adj;
      a1 = s1;
    } else {  // ContentString: str.slice(off) in UTF-16 units; a split surrogate pair throws in yjs
      const uint32_t n = sc::rvu(e);
      uint32_t bi = 0, u = 0;
      while (u < off && bi < n) {
        const uint32_t b = sc::byte(B, e.p + bi);
        const uint32_t l = b < 0x80 ? 1 : b < 0xE0 ? 2 : b < 0xF0 ? 3 : 4;
        u += l == 4 ? 2 : 1;
        bi += l;
      }
      if (e.bad || n > e.e - e.p) return SH_DECLINE;
      if (u == off + 1) return SH_URI;  // a 4-byte character split (the struct's bytes were validated)
      if (u != off) return SH_DECLINE;
      put(n - bi);
      a0 = e.p - adj + bi;
      a1 = e.p - adj + n;
    }
    if (e.bad) return SH_DECLINE;
  }
  if (q > PRE) return SH_DECLINE;
  if (lane == 0)
    for (uint32_t b = 0; b < q; b++) pre[b] = h[b];
  prelen = q;
  return SH_OK;
}
// out of line (k_pw_small, k_pw_ms, the many-section stitch: inlined, its registers cost them occupancy -- diff_c2_v1
// 0.70 -> 0.78 ms); the single-section stitch inlines slice_head_body (C3 V1 diff 14.9 -> 14.1 ms: the call saved
// and restored the stitch's live registers through scratch)
__device__ __noinline__ uint32_t slice_head(sc::cu32 *B, uint32_t adj, uint32_t s0, uint32_t s1, uint32_t client, uint64_t clock,
                                           uint32_t len, uint32_t off, uint8_t *pre, uint32_t &prelen, uint32_t &a0, uint32_t &a1) {
  return slice_head_body(B, adj, s0, s1, client, clock, len, off, pre, prelen, a0, a1);
}

// a declined document keeps done[d] != 1 (k_big_v1 takes it); the value says why (ym__pw_reasons)
#define PW_DECLINE_R(r)                  \
  {                                      \
    if (lane == 0) done[d] = (uint8_t)(r); \
    __syncthreads();                     \
    continue;                            \
  }
#define PW_DECLINE() PW_DECLINE_R(why ? why : 2)
// the document's result is yjs's URIError (slice_head SH_URI): completed here with that status
// ---- LDS state-vector map of the DSL variant (many-section documents: C5's ~1,000-entry state vectors): sv[client]
// from one probe round of LDS reads instead of cmap's three dependent device-scope loads per section (round 6).
// Keys client + 1 (0 = empty) over 4,096 slots (load factor <= 1/2 at BS_NSV entries); a slot's value is first the
// largest entry index mapped to it (decodeStateVector: a later entry for a client wins, encoding.js:536-545), then
// that entry's clock.  Client 0xFFFFFFFF (whose key would be 0) keeps its index / clock in the two words after.
namespace lsv {
constexpr uint32_t SLOTS = 4096, MASK = SLOTS - 1, BYTES = 8 * SLOTS + 16;
static_assert(SLOTS == BS_MAP_SLOTS && SLOTS >= 2 * NSV, "cmap::hash; load factor <= 1/2");
__device__ __forceinline__ void build(uint32_t base, const uint32_t *svt, uint32_t nsv) {
  const uint32_t lane = threadIdx.x;
  uint32_t *K = reinterpret_cast<uint32_t *>(sm + base), *V = K + SLOTS;
  for (uint32_t i = lane; i < (2 * SLOTS + 4) / 4; i += 64) reinterpret_cast<uint4 *>(K)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (uint32_t i = lane; i < nsv; i += 64) {
    const uint32_t c = svt[2 * i];
    if (c == cmap::XCLIENT) {
      atomicMax(&K[2 * SLOTS], i + 1);
      continue;
    }
    uint32_t sl = cmap::hash(c);
    for (uint32_t probe = 0; probe < SLOTS; probe++, sl = (sl + 1) & MASK) {
      const uint32_t old = atomicCAS(&K[sl], 0u, c + 1);
      if (old == 0 || old == c + 1) {
        atomicMax(&V[sl], i + 1);
        break;
      }
    }
  }
  __syncthreads();
  for (uint32_t sl = lane; sl < SLOTS; sl += 64) {
    const uint32_t v = V[sl];
    if (v) V[sl] = svt[2 * (v - 1) + 1];
  }
  if (lane == 0 && K[2 * SLOTS]) K[2 * SLOTS + 1] = svt[2 * (K[2 * SLOTS] - 1) + 1];
  __syncthreads();
}
// sv[client] (0 when absent), wave-uniform client
__device__ __forceinline__ uint32_t get(uint32_t base, uint32_t client) {
  const uint32_t *K = reinterpret_cast<const uint32_t *>(sm + base), *V = K + SLOTS;
  if (client == cmap::XCLIENT) return K[2 * SLOTS] ? K[2 * SLOTS + 1] : 0;
  const uint32_t key = client + 1, s0 = cmap::hash(client);
  for (uint32_t b = 0; b < SLOTS; b += 64) {
    const uint32_t sl = (s0 + b + threadIdx.x) & MASK;
    const uint32_t kv = K[sl];
    const uint64_t hit = __ballot(kv == key), emp = __ballot(kv == 0);
    if (hit | emp) {
      const uint32_t fh = hit ? (uint32_t)__builtin_ctzll(hit) : 64, fe = emp ? (uint32_t)__builtin_ctzll(emp) : 64;
      if (fh > fe) return 0;
      return V[(s0 + b + fh) & MASK];
    }
  }
  return 0;
}
}  // namespace lsv

// A section header (#structs, client, clock: three lib0 varuints, <= 15 bytes) from one 24-byte window whose
// three loads are issued together.  ln::rvu refills its cursor after each varint: three dependent global loads
// per section, ~2 of the stitch's ~8 ms per C5 document (~1,000 sections).  Same checks as ln::rvu.
__device__ __forceinline__ uint64_t win8(uint64_t a, uint64_t b, uint64_t c, uint32_t o) {  // bytes [o, o + 8), o < 16
  const uint64_t lo = o < 8 ? a : b, hi = o < 8 ? b : c;
  const uint32_t sh = 8 * (o & 7);
  return sh == 0 ? lo : (lo >> sh) | (hi << (64 - sh));
}
__device__ __forceinline__ bool hdr3(const uint8_t *D, uint32_t &x, uint32_t len, uint32_t &v0, uint32_t &v1, uint64_t &v2) {
  if (x + 24 > len) {
    ln::LCur c = ln::make(D, x, len);
    v0 = ln::rvu(c);
    v1 = ln::rvu(c);
    v2 = ln::rvu(c);
    x = c.p;
    return !c.bad;
  }
  const uint64_t a = ln::ld8(D, x), b = ln::ld8(D, x + 8), c = ln::ld8(D, x + 16);
  uint32_t o = 0, v[3];
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint64_t w = win8(a, b, c, o);
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const uint32_t nb = ln::vu_nb(lo, hi);
    const uint32_t val = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u) | (hi << 28);
    bad |= ln::vu_bad(lo, hi, nb, x + o, len);
    v[k] = val & (uint32_t)((1ull << (7 * (nb < 5 ? nb : 5))) - 1);
    o += nb < 6 ? nb : 0;
  }
  v0 = v[0];
  v1 = v[1];
  v2 = v[2];
  x += o;
  return !bad;
}

constexpr uint32_t WHY_URI = 99;
#define PW_URIERR()                                                                  \
  {                                                                                  \
    if (lane == 0) {                                                                 \
      j.status[d] = ym::ST_URI;                                                      \
      j.out_len[d] = 0;                                                              \
      j.out_off[d] = 0;                                                              \
      done[d] = 1;                                                                   \
      atomicAdd((unsigned long long *)j.pw_count, 1ull);                             \
    }                                                                                \
    __syncthreads();                                                                 \
    continue;                                                                        \
  }

// OP = OP_DIFF, OP_SV or OP_META (parseUpdateMeta: from = a section's first clock, to = its end clock)
// DSL: the delete set validated through LDS token tables (ym_wave_ds.h) first -- batches with many-client
// documents only: the tables' 17 KB of LDS cost the stitch occupancy (C3 V1 diff 14.3 -> 17.5 ms)
template <int OP, bool DSL = false>
__global__ void __launch_bounds__(64) k_pw_stitch(GeneralJob j, const uint32_t *cbase, const uint4 *desc, const uint32_t *recs,
                                                  uint8_t *done, const uint64_t *msz) {
  const uint32_t lane = threadIdx.x;
  const Scr X = scratch(j);
  PT_DECL
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    const uint32_t cb = cbase[d], nch = cbase[d + 1] - cb;
    if (nch == 0 || msz[d]) continue;  // (many sections: k_pw_ms)
    const uint32_t u0 = j.doc_upd[d];
    const uint64_t ub = j.upd_off[u0];
    const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
    const uint8_t *D = j.A + ub;
    uint32_t why = 0;  // decline reason
    sc::cu32 *const B = sc::base_of(D);
    const uint32_t adj = (uint32_t)(ub & 3);
    // ---- state vector (diff): decodeStateVector, later entries win (encoding.js:536-545)
    uint32_t nsv = 0;
    if (OP == OP_DIFF) {
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      if (s1 - s0 > 16ull * NSV) PW_DECLINE_R(3)
      bool bad;
      {
        SCur c = sc::make(sc::base_of(j.sv + s0), (uint32_t)(s0 & 3), (uint32_t)(s0 & 3) + (uint32_t)(s1 - s0));
        const uint32_t n = sc::rvu(c);
        for (uint32_t i = 0; i < n && !c.bad; i++) {
          const uint32_t cl = sc::rvu(c), ck = sc::rvu(c);
          if (nsv >= NSV) { c.bad = true; break; }
          if (lane == 0) { X.svt[2 * nsv] = cl; X.svt[2 * nsv + 1] = ck; }
          nsv++;
        }
        bad = c.bad;
      }
      __syncthreads();
      if (bad) PW_DECLINE_R(3)
      if (nsv > 64) {
        if constexpr (DSL) lsv::build(L_SVM, X.svt, nsv);
        else cmap::build_sv(X.map, X.svt, nsv);
      }
    }
    PT(0);
    // ---- struct section: headers parsed here, structs from the walk's records
    uint32_t x = 0;
    bool declined = false;
    uint32_t nclients;
    {
      ln::LCur c = ln::make(D, x, len);
      nclients = ln::rvu(c);
      declined = c.bad;
      x = c.p;
    }
    if (declined || nclients > NSEC) PW_DECLINE_R(4)
    uint32_t nparts = 0, npatch = 0;
    uint32_t sv_client = 0, sv_clock = 0, sv_n = 0;
    bool sv_stop = false, sv_any = false;
    uint32_t prev_client = 0;
    // chunk cursor: the current chunk and the next record index in it; descriptors of chunks [wb, wb + 64)
    uint32_t cc = NONE, s = 0, wb = NONE - 64;
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0, q4 = q0;
    uint32_t staged = NONE;  // the chunk whose records (and exit sentinel) sit in LDS at L_REC
    for (uint32_t ci = 0; ci < nclients && !declined; ci++) {
      uint32_t nstructs, client;
      uint64_t clock;
      if (!hdr3(D, x, len, nstructs, client, clock)) { declined = true; why = 5; break; }
      if (ci > 0 && client == prev_client) { declined = true; why = 6; break; }
      // meta: taken only when the clients descend (a repeated client would keep its first Map slot)
      if (OP == OP_META && ci > 0 && client > prev_client) { declined = true; why = 6; break; }
      const uint32_t first_clock = (uint32_t)clock;
      prev_client = client;
      const uint32_t k = OP != OP_DIFF ? 0
                         : nsv > 64 ? (DSL ? lsv::get(L_SVM, client) : cmap::sv_get(X.map, X.svt, client))
                                    : sv_lookup(X.svt, nsv, client);
      if (OP == OP_SV && nstructs > 0 && sv_any && client != sv_client) {
        if (sv_clock != 0) {
          if (sv_n >= NSV) { declined = true; why = 13; break; }
          if (lane == 0) { X.svt[2 * sv_n] = sv_client; X.svt[2 * sv_n + 1] = sv_clock; }
          sv_n++;
        }
        sv_client = client; sv_clock = 0; sv_stop = clock != 0;
      }
      bool copying = false;
      uint32_t written = 0;
      uint32_t rem = nstructs;
      PT(1);
      while (rem > 0) {
        if (x >= len) { declined = true; why = 7; break; }
        const uint32_t cx = x / CH;
        // ---- chunk descriptors, 64 chunks per load (one lane each)
        if (cx < wb || cx >= wb + 64) {
          wb = cx;
          if (wb + lane < nch) {
            const uint4 *Q = desc + 5ull * (cb + wb + lane);
            q0 = Q[0]; q1 = Q[1]; q2 = Q[2]; q3 = Q[3]; q4 = Q[4];
          }
        }
        const int di = (int)(cx - wb);
        const uint32_t w0 = lane_read(q0.x, di), w1 = lane_read(q0.y, di);
        const uint32_t nrec = w0 & 0xffffu, lfe = w0 >> 16, lpe = w1 & 0xffffu, lse = w1 >> 16;
        const uint32_t cexit = lane_read(q0.z, di), cumx = lane_read(q0.w, di);
        if (cx != cc) { cc = cx; s = 0; }
        const uint32_t gc = cb + cx;
        PT(2);
        // ---- chunk entry: x among the descriptor's first records -> the rest of the chunk in O(1)
        if (s == 0) {
          uint32_t fs = NONE, fcum = 0;
#pragma unroll
          for (int kf = NFIRST - 1; kf >= 0; kf--) {
            const uint32_t pwk = lane_read(kf < 4 ? (&q1.x)[kf] : (&q2.x)[kf - 4], di);
            if ((uint32_t)kf < nrec && (pwk & POS_MASK) == x && !(pwk & F_FAIL)) {
              fs = (uint32_t)kf;
              fcum = lane_read(kf < 4 ? (&q3.x)[kf] : (&q4.x)[kf - 4], di);
            }
          }
          if (fs != NONE) {
            const uint32_t avail = nrec - fs;
            const uint32_t delta = cumx - fcum;  // clocks of records fs .. nrec-1 (no wrap when lfe <= fs)
            bool whole = rem >= avail && lfe <= fs;
            if (OP == OP_DIFF) whole = whole && (copying ? lpe <= fs : clock + delta <= k);
            if (OP == OP_SV) whole = whole && sv_any && lse <= fs;
            if (whole) {
              PWP(0);
              if (clock + delta > 0xffffffffull) { declined = true; why = 10; break; }
              if (OP == OP_SV && !sv_stop) sv_clock = (uint32_t)(clock + delta);
              if (OP == OP_DIFF && copying) written += avail;
              clock += delta;
              rem -= avail;
              x = cexit;
              s = nrec;
              PT(5);
              continue;
            }
            PWP(1);
            s = fs;
          } else PWP(2);
        }
        // ---- record by record.  The chunk's records are staged into LDS first, all loads in flight at
        // once (one memory round trip per chunk instead of one per 64-record batch, twice: the search and
        // the consumption): C5 sections end inside chunks and cut mid-chunk, so most chunks go this way.
        if (staged != gc && s < nrec) {
          __syncthreads();
          for (uint32_t k = lane; k < nrec; k += 64) at<uint32_t>(L_REC + 4 * k) = recs[rec_idx(gc, k)];
          __syncthreads();
          staged = gc;
        }
        PT(3);
        // locate x among the chunk's records (a ballot over 64 per step)
        bool found = false;
        for (;;) {
          if (s >= nrec) break;
          PWP(5);
          const uint32_t kk = s + lane;
          const uint32_t pw = kk < nrec ? rec_pw(at<uint32_t>(L_REC + 4 * kk), cx) : POS_MASK;
          const uint64_t lt = __ballot(kk < nrec && (pw & POS_MASK) < x);
          const uint32_t nlt = __popcll(lt);
          if (nlt == 64) { s += 64; continue; }
          s += nlt;
          if (s < nrec) {
            const uint32_t cand = lane_read(pw, nlt);
            found = (cand & POS_MASK) == x && !(cand & F_FAIL);
          }
          break;
        }
        PT(4);
        uint32_t n, pos = 0, end = 0, clen = 0, fl = 0;
        bool valid;
        if (found) {
          PWP(3);
          n = nrec - s < 64 ? nrec - s : 64;
          if (rem < n) n = rem;
          const uint32_t kk = s + lane;
          valid = lane < n;
          if (valid) {
            const uint32_t w = at<uint32_t>(L_REC + 4 * kk);
            fl = rec_pw(w, cx);
            pos = fl & POS_MASK;
            clen = rec_clen(w);
            // a struct ends where the next record starts (the chunk's last one at the walk's exit)
            end = kk + 1 < nrec ? rec_pw(at<uint32_t>(L_REC + 4 * (kk + 1)), cx) & POS_MASK : cexit;
          }
          const uint64_t fm = __ballot(valid && (fl & F_FAIL));
          if (fm) {  // a FAIL inside: consume up to it, the next round re-parses that struct uncapped
            n = (uint32_t)__builtin_ctzll(fm);
            valid = lane < n;
          }
          s += n;
        } else {
          // the walk's chain does not pass x (or failed there under its cap): the structs are parsed here, in
          // lockstep, one batch up to the first that starts at a usable record of the chain (C5: ~5 after each
          // section header), the section's or the chunk's end, or 64 -- one consumption round for them all
          uint32_t y = x, t = 0, sp = s;
          bool bad = false;
          for (;;) {
            uint32_t nx, cl, f2;
            PWP(4);
            if (!ln::parse_struct(D, y, len, nx, cl, f2)) { bad = t == 0; break; }  // (t > 0: the next round declines)
            if (lane == t) { pos = y; end = nx; clen = cl; fl = f2; }
            t++;
            y = nx;
            if (t >= rem || t >= 64 || y / CH != cx) break;
            if (staged == gc) {  // does the chain's record list pass y?
              uint32_t rp = NONE;
              while (sp < nrec && ((rp = rec_pw(at<uint32_t>(L_REC + 4 * sp), cx)) & POS_MASK) < y) sp++;
              if (sp < nrec && (rp & POS_MASK) == y && !(rp & F_FAIL)) break;
            }
          }
          if (bad) { declined = true; why = 8; break; }
          n = t;
          valid = lane < n;
        }
        // ---- consume n structs: clocks by a wave prefix sum
        if (__any(valid && clen >= (1u << 24))) { declined = true; why = 9; break; }
        const uint32_t cl = valid ? clen : 0;
        const uint32_t incl = wave_incl_add(cl), excl = incl - cl;
        const uint32_t tot = lane_read(incl, 63);
        if (clock + tot > 0xffffffffull) { declined = true; why = 10; break; }
        const bool skip = valid && (fl & F_SKIP);
        const uint64_t eclk = clock + incl;  // end clock of this lane's struct
        if (OP == OP_SV) {
          if (!sv_any) {  // the update's first struct initialises the state
            sv_any = true;
            sv_client = client;
            sv_stop = clock != 0;
            sv_clock = sv_stop ? 0 : (uint32_t)(clock + lane_read(cl, 0));
          }
          const uint64_t skm = __ballot(skip);
          const uint32_t fs = skm ? (uint32_t)__builtin_ctzll(skm) : n;  // first Skip
          if (!sv_stop && fs > 0) sv_clock = (uint32_t)(clock + lane_read(incl, fs - 1));
          if (skm) sv_stop = true;
        } else if (OP == OP_DIFF) {
          PT(5);
          uint32_t first = 0;  // first struct of this batch written verbatim (patch range start)
          bool pend = false;
          if (!copying) {
            const uint64_t cm = __ballot(valid && !skip && eclk > k);
            if (cm) {
              const uint32_t f = (uint32_t)__builtin_ctzll(cm);
              copying = true;
              written = n - f;
              const uint64_t fclk = clock + lane_read(excl, f);
              const uint32_t off = k > fclk ? (uint32_t)(k - fclk) : 0;
              const uint32_t fpos = lane_read(pos, f), fend = lane_read(end, f), flen = lane_read(cl, f);
              uint32_t prelen = 0, a0 = 0, a1 = 0, b0;
              if (off == 0) {
                b0 = fpos;
                first = f;
              } else {
                const uint32_t sh = DSL ? slice_head(B, adj, fpos, fend, client, fclk, flen, off, X.pre + ci * PRE, prelen, a0, a1)
                                        : slice_head_body(B, adj, fpos, fend, client, fclk, flen, off, X.pre + ci * PRE, prelen, a0, a1);
                if (sh != SH_OK) {
                  declined = true;
                  why = sh == SH_URI ? WHY_URI : 11;
                  break;
                }
                b0 = fend;
                first = f + 1;
              }
              if (lane == 0) {
                sec(ci, S_PRELEN) = prelen;
                sec(ci, S_A0) = a0;
                sec(ci, S_A1) = a1;
                sec(ci, S_B0) = b0;
                sec(ci, S_FCLOCK) = (uint32_t)(fclk + off);
                sec(ci, S_CLIENT) = client;
              }
              pend = true;
            }
          } else {
            written += n;
            pend = true;
          }
          if (pend) {  // info-byte patches of the verbatim structs
            const bool pl = valid && lane >= first && (fl & F_PATCH);
            const uint64_t pm = __ballot(pl);
            if (pm) {
              const uint32_t np = __popcll(pm);
              if (npatch + np > NPATCH) { declined = true; why = 12; break; }
              if (pl) {
                const uint32_t slot = npatch + __popcll(pm & ((1ull << lane) - 1));
                const uint32_t info = D[pos];
                const bool gc = (info & 31) == 0;
                at<uint32_t>(L_PPOS + 4 * slot) = pos;
                at<uint32_t>(L_PSEC + 4 * slot) = ci;
                sm[L_PVAL + slot] = (uint8_t)(gc ? 0 : info & ~0x20u);
              }
              npatch += np;
            }
          }
        }
        clock += tot;
        x = lane_read(end, n - 1);
        rem -= n;
        PT(OP == OP_DIFF ? 6 : 5);
      }
      if (declined) break;
      if (OP == OP_META && nstructs > 0) {
        if (sv_n >= NSV) { declined = true; why = 13; break; }
        if (lane == 0) { X.svt[2 * sv_n] = client; X.svt[2 * sv_n + 1] = first_clock; X.sec[sv_n] = (uint32_t)clock; }
        sv_n++;
      }
      if (OP == OP_DIFF) {
        if (lane == 0) {
          sec(ci, S_B1) = copying ? x : 0;
          sec(ci, S_WRITTEN) = written;
          if (!copying) sec(ci, S_PRELEN) = NONE;
        }
        nparts += copying;
      }
    }
    if (declined && why == WHY_URI) PW_URIERR()
    if (declined) PW_DECLINE()
    __syncthreads();
    if (OP == OP_META) {  // from then to, each vu(n) | (client, clock)*
      __threadfence_block();
      __syncthreads();
      uint32_t tl = 0;
      for (uint32_t i = lane; i < sv_n; i += 64) tl += 2 * vsz(X.svt[2 * i]) + vsz(X.svt[2 * i + 1]) + vsz(X.sec[i]);
      const uint32_t total = 2 * vsz(sv_n) + lane_read(wave_incl_add(tl), 63);
      uint64_t base = 0;
      if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
      base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
      if (lane == 0) { done[d] = 1; atomicAdd((unsigned long long *)j.pw_count, 1ull); }
      if (base + total > j.cap) {
        if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
        __syncthreads();
        continue;
      }
      if (lane == 0) {
        uint8_t *o = j.out + base;
        uint32_t p = put_vu_g(o, 0, sv_n);
        for (uint32_t i = 0; i < sv_n; i++) { p = put_vu_g(o, p, X.svt[2 * i]); p = put_vu_g(o, p, X.svt[2 * i + 1]); }
        p = put_vu_g(o, p, sv_n);
        for (uint32_t i = 0; i < sv_n; i++) { p = put_vu_g(o, p, X.svt[2 * i]); p = put_vu_g(o, p, X.sec[i]); }
        j.out_off[d] = base;
        j.out_len[d] = total;
        j.status[d] = ym::ST_OK;
      }
      __syncthreads();
      continue;
    }
    if (OP == OP_SV) {
      if (sv_any && sv_clock != 0) {
        if (sv_n >= NSV) PW_DECLINE_R(13)
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
      if (lane == 0) { done[d] = 1; atomicAdd((unsigned long long *)j.pw_count, 1ull); }
      if (base + total > j.cap) {
        if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
        __syncthreads();
        continue;
      }
      if (lane == 0) {
        uint8_t *o = j.out + base;
        uint32_t p = put_vu_g(o, 0, sv_n);
        for (uint32_t i = 0; i < sv_n; i++) { p = put_vu_g(o, p, X.svt[2 * i]); p = put_vu_g(o, p, X.svt[2 * i + 1]); }
        j.out_off[d] = base;
        j.out_len[d] = total;
        j.status[d] = ym::ST_OK;
      }
      __syncthreads();
      continue;
    }
    // ---- delete set: validated (readDeleteSet), then copied verbatim -- through the LDS token tables
    // (ym_wave_ds.h; C5: ~1,000 clients, each a few dependent loads on the walk below), or the walk below
    // when those cannot decide (a client's ranges beyond a window, too many clients)
    const uint32_t ds0 = x;
    const uint32_t xds = DSL ? wds::ds_validate_lds(D, x, len, *reinterpret_cast<wds::DsLdsS *>(sm + L_DSL)) : wds::DS_BIG;
    if (xds == NONE) { why = 17; PW_DECLINE() }
    if (xds != wds::DS_BIG) {
      x = xds;
    } else {
      ln::LCur c = ln::make(D, x, len);
      const uint32_t ndc = ln::rvu(c);
      x = c.p;
      declined = c.bad;
      why = 17;
      const bool big = ndc > 64 && ndc <= BS_NDSC;
      if (big) cmap::clear(X.map);
      for (uint32_t i = 0; i < ndc && !declined; i++) {
        ln::LCur h = ln::make(D, x, len);
        const uint32_t client = ln::rvu(h);
        const uint32_t m = ln::rvu(h);
        x = h.p;
        // readDeleteSet drops clients without ranges and merges a repeated client into its first
        // occurrence: either makes the re-written set differ from the input bytes
        if (h.bad || m == 0 || i >= BS_NDSC) { declined = true; why = 14; break; }
        if (big ? cmap::seen_insert(X.map, client) : seen_before(X.dsc, i, client)) { declined = true; why = 15; break; }
        if (lane == 0) X.dsc[i] = client;
        __threadfence_block();
        x = wds::skip_varuints(D, x, len, 2ull * m);
        if (x == NONE) { declined = true; why = 16; break; }
      }
    }
    if (declined) PW_DECLINE()
    why = 0;
    const uint32_t ds1 = x;
    PT(7);
    __threadfence_block();
    __syncthreads();
    // ---- sizes, allocation
    uint32_t tl = 0;
    for (uint32_t ci = lane; ci < nclients; ci += 64) {
      const uint32_t pl = sec(ci, S_PRELEN);
      if (pl == NONE) continue;
      tl += vsz(sec(ci, S_WRITTEN)) + vsz(sec(ci, S_CLIENT)) + vsz(sec(ci, S_FCLOCK)) + pl + (sec(ci, S_A1) - sec(ci, S_A0)) +
            (sec(ci, S_B1) - sec(ci, S_B0));
    }
    const uint64_t total = vsz(nparts) + (uint64_t)(ds1 - ds0) + lane_read(wave_incl_add(tl), 63);
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
    if (lane == 0) { done[d] = 1; atomicAdd((unsigned long long *)j.pw_count, 1ull); }
    if (base + total > j.cap) {
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    PT(8);
    // ---- write: 64 sections per round, one per lane for the section table reads, the header and the
    // sliced head (placed by a wave prefix sum of the section sizes), then the wave copies the spans
    // section by section -- a C5 document's ~1,000 sections no longer cost ~5 dependent loads each
    uint8_t *const o = j.out + base;
    if (lane == 0) put_vu_g(o, 0, nparts);
    uint32_t p = vsz(nparts);
    for (uint32_t c0 = 0; c0 < nclients; c0 += 64) {
      const uint32_t ci = c0 + lane;
      const uint32_t pl = ci < nclients ? sec(ci, S_PRELEN) : NONE;
      uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0, hb = 0, written = 0, client = 0, fclock = 0;
      if (pl != NONE) {
        written = sec(ci, S_WRITTEN);
        client = sec(ci, S_CLIENT);
        fclock = sec(ci, S_FCLOCK);
        a0 = sec(ci, S_A0);
        a1 = sec(ci, S_A1);
        b0 = sec(ci, S_B0);
        b1 = sec(ci, S_B1);
        hb = vsz(written) + vsz(client) + vsz(fclock) + pl;
      }
      const uint32_t sz = hb + (a1 - a0) + (b1 - b0);
      const uint32_t incl = wave_incl_add(sz), q = p + incl - sz + hb;  // q: the section's first span byte
      if (pl != NONE) {
        uint32_t t = put_vu_g(o, q - hb, written);
        t = put_vu_g(o, t, client);
        t = put_vu_g(o, t, fclock);
        for (uint32_t b = 0; b < pl; b++) o[t + b] = X.pre[ci * PRE + b];
        sec(ci, S_OUTB) = q + (a1 - a0) - b0;  // output position = document position + S_OUTB
      }
      for (uint64_t live = __ballot(sz > hb); live; live &= live - 1) {
        const uint32_t k = (uint32_t)__builtin_ctzll(live);
        const uint32_t kq = lane_read(q, k), ka0 = lane_read(a0, k), kna = lane_read(a1 - a0, k);
        copy_bytes(o + kq, D + ka0, kna);
        copy_bytes(o + kq + kna, D + lane_read(b0, k), lane_read(b1 - b0, k));
      }
      p += lane_read(incl, 63);
    }
    copy_bytes(o + p, D + ds0, ds1 - ds0);
    __threadfence();  // the patches below overwrite bytes other lanes stored
    __syncthreads();
    PT(9);
    for (uint32_t i = lane; i < npatch; i += 64) {
      const uint32_t pos = at<uint32_t>(L_PPOS + 4 * i);
      const uint32_t ci = at<uint32_t>(L_PSEC + 4 * i);
      o[sec(ci, S_OUTB) + pos] = sm[L_PVAL + i];
    }
    if (lane == 0) {
      j.out_off[d] = base;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
    PT(10);
  }
  PT_FLUSH();
}


// ---- 3. multi-section documents (configs[4] C5: ~1,000 client sections, ~30 k structs) -------------------
// k_pw_stitch follows the chain one section after the other: a C5 section costs ~10 dependent global loads
// (header, state vector, descriptors, records, the cut) plus ~5 structs re-parsed after its header, where
// the walk's speculative chain lost step (round 3: ~25 us per section, 28 ms per call).  Here one 512-thread
// block per document and no chunk walk:
//   A+B  the chain through LDS windows of 4 KB: the block parses a struct at EVERY byte offset of the window
//        (next position, clock length, Skip / patch flags: tables), then thread 0 follows the true chain --
//        section headers parsed, each struct one table lookup -- and does the stitch's per-section work on
//        the way: clocks, the state-vector entry, the cut and its sliced head, the info-byte patches.
//   C    the delete set validated through LDS token tables (ym_wave_ds.h), sizes by a block scan over the
//        sections, then every wave writes its sections' pieces in place.
// The same documents are accepted, with the same bytes, as k_pw_stitch / k_big_v1 would (the golden vectors
// run through this path with YMERGE_PWMS_MIN=2, tests/test_gpu_golden.py).
constexpr uint32_t MS_WAVES = 8, MS_T = 64 * MS_WAVES;
// sections from which a document takes this path (YMERGE_PWMS_MIN; off by default: measured on C5 V1 diff,
// 57 ms against k_pw_stitch's 27.6 -- the tables parse every byte offset of a 700 KB document with the full
// divergent struct parser, ~13 ms per document, and the lockstep chain costs ~2,000 cycles per struct)
constexpr uint32_t MS_MIN = 0xffffffffu;
constexpr uint32_t MSPATCH = 4096;     // info-byte patches per document
constexpr uint32_t MSVMAX = 2048, MSVSLOTS = 4096;
enum { M_X0 = 0, M_W, M_CLIENT, M_CLOCK, M_X1, M_PRELEN, M_A0, M_A1, M_B0, M_WRITTEN, M_FCLOCK, M_VAL, M_END, M_OUT, NMF = 16 };
__host__ __device__ inline uint64_t ms_area(uint32_t nsec) { return (((uint64_t)nsec * (4 * NMF + PRE) + 15) & ~15ull) + 9ull * MSPATCH + 256; }
struct MsDoc {
  uint32_t *sec;    // [nsec][NMF]
  uint8_t *pre;     // [nsec][PRE]
  uint32_t *ppos, *psec;
  uint8_t *pval;
};
__device__ __forceinline__ MsDoc ms_doc(uint8_t *area, uint64_t off, uint32_t nsec) {
  uint8_t *b = area + off;
  MsDoc m;
  m.sec = reinterpret_cast<uint32_t *>(b);
  m.pre = b + 4ull * NMF * nsec;
  uint8_t *p = b + (((uint64_t)nsec * (4 * NMF + PRE) + 15) & ~15ull);
  m.ppos = reinterpret_cast<uint32_t *>(p);
  m.psec = m.ppos + MSPATCH;
  m.pval = reinterpret_cast<uint8_t *>(m.psec + MSPATCH);
  return m;
}
#define msec(ci, f) M.sec[NMF * (ci) + (f)]

// the walk's tables over one LDS window: per byte offset the struct a parse there would give (next
// position, clock length, flags; TV: decided), computed by the whole block
constexpr uint32_t TW = 4096, TMARG = 256;
constexpr uint32_t TV = 0x80;
struct TabLds {
  uint8_t b[TW + TMARG + 16];
  uint16_t nx[TW];
  uint32_t len[TW];
  uint8_t fl[TW];
};
union MsLds {
  TabLds tab;
  wds::DsLds ds;
};
// lane 0's value to the whole wave, as a scalar
__device__ __forceinline__ uint32_t RF(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
// lib0 readVarUint (canonical, u32) at o of the LDS bytes b (valid [0, lim)), advancing o
__device__ __forceinline__ uint32_t tab_vu(const uint8_t *b, uint32_t &o, uint32_t lim, bool &bad) {
  uint32_t v = 0, nb = 0, x = 0x80;
  while ((x & 0x80) && nb < 5) {
    x = o + nb < lim ? b[o + nb] : 0x80;
    v |= (x & 0x7f) << (7 * nb);
    nb++;
  }
  bad |= (x & 0x80) || (nb > 1 && x == 0) || (nb == 5 && (x & 0x70) != 0);
  o += nb;
  return v;
}

template <int OP>
__global__ void __launch_bounds__(MS_T) k_pw_ms(GeneralJob j, uint8_t *done, const uint64_t *msz, const uint64_t *moff,
                                                uint8_t *area) {
  const uint32_t t = threadIdx.x, lane = t % 64, wv = t / 64;
  __shared__ uint32_t mkey[OP == OP_DIFF ? MSVSLOTS : 1], mval[OP == OP_DIFF ? MSVSLOTS : 1], svclk[OP == OP_DIFF ? MSVMAX : 1];
  __shared__ uint32_t s_bad, s_why, s_nsec, s_ds0, s_npatch, s_sum[MS_WAVES + 1];
  __shared__ uint32_t s_p, s_done;
  __shared__ MsLds U;
  TabLds &T = U.tab;
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    if (msz[d] == 0) continue;
    const uint32_t u0 = j.doc_upd[d];
    const uint64_t ub = j.upd_off[u0];
    const uint32_t len = (uint32_t)(j.upd_off[u0 + 1] - ub);
    const uint8_t *D = j.A + ub;
    sc::cu32 *const B = sc::base_of(D);
    const uint32_t adj = (uint32_t)(ub & 3);
    if (t == 0) { s_bad = 0; s_why = 0; s_npatch = 0; s_done = 0; }
    if (OP == OP_DIFF)
      for (uint32_t q = t; q < MSVSLOTS; q += MS_T) mval[q] = 0;
    __syncthreads();
    const uint64_t tm0 = __builtin_amdgcn_s_memrealtime();
    // ---- the state vector (diff): its bytes staged into LDS, decodeStateVector by thread 0 into the hash
    // map (a later entry wins)
    if (OP == OP_DIFF) {
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      const uint32_t sl = s1 - s0 > TW + TMARG ? NONE : (uint32_t)(s1 - s0);
      if (sl != NONE)
        for (uint32_t q = t; q < sl; q += MS_T) T.b[q] = j.sv[s0 + q];
      __syncthreads();
      if (t == 0) {
        bool bad = sl == NONE;
        uint32_t o = 0;
        const uint32_t ns = bad ? 0 : tab_vu(T.b, o, sl, bad);
        bad |= ns > MSVMAX;
        for (uint32_t q = 0; q < ns && !bad; q++) {
          const uint32_t cl = tab_vu(T.b, o, sl, bad), ck = tab_vu(T.b, o, sl, bad);
          svclk[q] = ck;
          uint32_t h = (cl * 0x9E3779B1u) >> 20;
          while (mval[h] != 0 && mkey[h] != cl) h = (h + 1) & (MSVSLOTS - 1);
          mkey[h] = cl;
          mval[h] = q + 1;
        }
        if (bad) { s_bad = 1; s_why = 3; }
      }
    }
    uint32_t nsec = 0;
    {
      ln::LCur c = ln::make(D, 0, len);
      nsec = ln::rvu(c);
      if (t == 0) s_p = c.p;
    }
    const MsDoc M = ms_doc(area, moff[d], nsec);
    // ---- A + B: the struct chain, window by window: the block computes the tables, thread 0 follows the
    // chain (section headers parsed, each struct a table lookup; a struct the window cannot decide -- one
    // that runs past it, a string longer than the margin -- parsed by thread 0 from the document)
    // thread 0's walk state, carried across windows
    uint32_t ci = 0, rem = 0, client = 0, k = 0, prev = 0, written = 0, sv_clock = 0, npatch = 0;
    uint64_t clock = 0;
    bool insec = false, copying = false, sv_stop = false, first = false;
    uint64_t t_tab = 0, t_walk = 0, n_win = 0, n_str = 0;
    __syncthreads();
    while (!s_bad && !s_done) {
      const uint64_t tw0 = __builtin_amdgcn_s_memrealtime();
      const uint32_t wb = s_p & ~15u;
      const uint32_t wl = wb + TW + TMARG < len ? wb + TW + TMARG : len;
      const uint32_t lim = wl - wb, wn = lim < TW ? lim : TW;
      __syncthreads();
      for (uint32_t q = 16 * t; q < lim; q += 16 * MS_T) {
        const uint4 v = wds::load16m(D, wb + q, len);
        __builtin_memcpy(T.b + q, &v, 16);
      }
      __syncthreads();
      for (uint32_t o = t; o < wn; o += MS_T) {
        uint32_t nx, cl, fl;
        const bool ok = ln::parse_fast(T.b, o, lim, nx, cl, fl) || ln::parse_struct(T.b, o, lim, nx, cl, fl, TAB_CAP);
        T.nx[o] = (uint16_t)(ok ? nx - o : 0);
        T.len[o] = cl;
        T.fl[o] = (uint8_t)(ok ? TV | ((fl & F_SKIP) ? 1 : 0) | ((fl & F_PATCH) ? 2 : 0) : 0);
      }
      __syncthreads();
      const uint64_t tw1 = __builtin_amdgcn_s_memrealtime();
      t_tab += tw1 - tw0;
      n_win++;
      if (wv == 0) {  // wave 0 in lockstep: every lane the same values (LDS reads made uniform), state in SGPRs
        uint32_t p = RF(s_p), why = 0;
        bool fin = false;
        const uint32_t wend = wb + wn;
        for (;;) {
          if (!insec) {  // a section header: vu(#structs) vu(client) vu(clock)
            if (ci == nsec) { fin = true; break; }
            if (p >= wend) { if (wend >= len) why = 7; break; }
            bool bad = false;
            uint32_t ns, first_clock;
            if (p + 16 <= wl) {
              uint32_t o = p - wb;
              ns = RF(tab_vu(T.b, o, lim, bad));
              client = RF(tab_vu(T.b, o, lim, bad));
              first_clock = RF(tab_vu(T.b, o, lim, bad));
              p = wb + RF(o);
              bad = RF(bad ? 1u : 0u) != 0;
            } else {
              ln::LCur c = ln::make(D, p, len);
              ns = RF(ln::rvu(c));
              client = RF(ln::rvu(c));
              first_clock = RF(ln::rvu(c));
              p = RF(c.p);
              bad = RF(c.bad ? 1u : 0u) != 0;
            }
            if (bad) { why = 5; break; }
            // each section a new client (the writer merges consecutive parts of one client); meta: descending
            if (ns == 0 || (ci > 0 && client == prev) || (OP == OP_META && ci > 0 && client > prev)) { why = 6; break; }
            prev = client;
            if (lane == 0) { msec(ci, M_X0) = p; msec(ci, M_W) = ns; msec(ci, M_CLIENT) = client; msec(ci, M_CLOCK) = first_clock; }
            k = 0;
            if (OP == OP_DIFF) {
              uint32_t h = (client * 0x9E3779B1u) >> 20;
              while (RF(mval[h]) != 0) {
                if (RF(mkey[h]) == client) { k = RF(svclk[RF(mval[h]) - 1]); break; }
                h = (h + 1) & (MSVSLOTS - 1);
              }
            }
            clock = first_clock;
            sv_stop = clock != 0;
            first = ci == 0;  // the state vector: the first section's first struct counts even as a Skip (os@37724)
            sv_clock = 0;
            copying = false;
            written = 0;
            rem = ns;
            insec = true;
            continue;
          }
          if (rem == 0) {  // the section's end
            if (lane == 0) {
              msec(ci, M_END) = (uint32_t)clock;
              msec(ci, M_VAL) = sv_clock;
              if (OP == OP_DIFF) {
                msec(ci, M_WRITTEN) = copying ? written : 0;
                if (!copying) msec(ci, M_PRELEN) = NONE;
              }
              msec(ci, M_X1) = p;
            }
            ci++;
            insec = false;
            continue;
          }
          // one struct
          if (p >= wend) { if (wend >= len) why = 7; break; }
          const uint32_t o = p - wb;
          uint32_t fl = RF(T.fl[o]), nx, cl;
          if (fl & TV) {
            nx = p + RF(T.nx[o]);
            cl = RF(T.len[o]);
          } else {
            uint32_t f2;
            if (RF(ln::parse_fast(D, p, len, nx, cl, f2) || ln::parse_struct(D, p, len, nx, cl, f2) ? 1u : 0u) == 0) { why = 8; break; }
            nx = RF(nx);
            cl = RF(cl);
            f2 = RF(f2);
            fl = TV | ((f2 & F_SKIP) ? 1 : 0) | ((f2 & F_PATCH) ? 2 : 0);
          }
          if (cl >= (1u << 24)) { why = 9; break; }
          if (clock + cl > 0xffffffffull) { why = 10; break; }
          const bool skip = fl & 1;
          const uint64_t end = clock + cl;
          if (OP == OP_SV) {
            if (first) {
              first = false;
              if (!sv_stop) sv_clock = (uint32_t)end;
              if (skip) sv_stop = true;
            } else if (!sv_stop) {
              if (skip) sv_stop = true;
              else sv_clock = (uint32_t)end;
            }
          } else if (OP == OP_DIFF) {
            bool patch = false;
            if (!copying) {
              if (!skip && end > k) {  // the cut: the first struct that ends past sv[client]
                copying = true;
                written = 1;
                const uint32_t off = k > clock ? (uint32_t)(k - clock) : 0;
                uint32_t prelen = 0, a0 = 0, a1 = 0, b0;
                if (off == 0) {
                  b0 = p;
                  patch = true;
                } else {
                  // (every lane computes the head; the lanes store the same bytes)
                  // (a split surrogate pair, SH_URI, declines here: the streamed walker / general path report it)
                  if (RF(slice_head(B, adj, p, nx, client, clock, cl, off, M.pre + (uint64_t)ci * PRE, prelen, a0, a1)) != SH_OK) { why = 11; break; }
                  prelen = RF(prelen); a0 = RF(a0); a1 = RF(a1);
                  b0 = nx;
                }
                if (lane == 0) {
                  msec(ci, M_PRELEN) = prelen;
                  msec(ci, M_A0) = a0;
                  msec(ci, M_A1) = a1;
                  msec(ci, M_B0) = b0;
                  msec(ci, M_FCLOCK) = (uint32_t)(clock + off);
                }
              }
            } else {
              written++;
              patch = true;
            }
            if (patch && (fl & 2)) {  // the info byte re-encoded: 0x20 cleared with an origin, GC := 0
              if (npatch >= MSPATCH) { why = 12; break; }
              const uint32_t info = RF(o < lim ? T.b[o] : D[p]);
              if (lane == 0) {
                M.ppos[npatch] = p;
                M.psec[npatch] = ci;
                M.pval[npatch] = (uint8_t)((info & 31) == 0 ? 0 : info & ~0x20u);
              }
              npatch++;
            }
          }
          clock = end;
          p = nx;
          rem--;
          n_str++;
        }
        t_walk += __builtin_amdgcn_s_memrealtime() - tw1;
        if (lane == 0) {
          s_p = p;
          if (why) { s_bad = 1; s_why = why; }
          if (fin) { s_done = 1; s_ds0 = p; s_npatch = npatch; }
        }
      }
      __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    if (s_bad) {
      if (t == 0) done[d] = (uint8_t)s_why;
      __syncthreads();
      continue;
    }
    const uint64_t tm1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t tm2 = tm1;
    if (t == 0) {
      atomicAdd(&pw_prof[0], tm1 - tm0);
      atomicAdd(&pw_prof[8], t_tab); atomicAdd(&pw_prof[9], t_walk); atomicAdd(&pw_prof[10], n_win); atomicAdd(&pw_prof[11], n_str);
    }
    // ---- C
    if (OP != OP_DIFF) {  // state vector / meta: one entry per section, written by one thread
      if (t == 0) {
        uint32_t total = 0, cnt = 0;
        for (uint32_t ci = 0; ci < nsec; ci++) {
          if (OP == OP_SV) {
            const uint32_t v = msec(ci, M_VAL);
            if (v) { cnt++; total += vsz(msec(ci, M_CLIENT)) + vsz(v); }
          } else {
            total += 2 * vsz(msec(ci, M_CLIENT)) + vsz(msec(ci, M_CLOCK)) + vsz(msec(ci, M_END));
          }
        }
        total += OP == OP_SV ? vsz(cnt) : 2 * vsz(nsec);
        const uint64_t base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
        done[d] = 1;
        atomicAdd((unsigned long long *)j.pw_count, 1ull);
        if (base + total > j.cap) {
          j.status[d] = ym::ST_CAPACITY;
          j.out_len[d] = 0;
        } else {
          uint8_t *o = j.out + base;
          uint32_t p = put_vu_g(o, 0, OP == OP_SV ? cnt : nsec);
          for (uint32_t ci = 0; ci < nsec; ci++) {
            if (OP == OP_SV && !msec(ci, M_VAL)) continue;
            p = put_vu_g(o, p, msec(ci, M_CLIENT));
            p = put_vu_g(o, p, OP == OP_SV ? msec(ci, M_VAL) : msec(ci, M_CLOCK));
          }
          if (OP == OP_META) {
            p = put_vu_g(o, p, nsec);
            for (uint32_t ci = 0; ci < nsec; ci++) { p = put_vu_g(o, p, msec(ci, M_CLIENT)); p = put_vu_g(o, p, msec(ci, M_END)); }
          }
          j.out_off[d] = base;
          j.out_len[d] = total;
          j.status[d] = ym::ST_OK;
        }
      }
      __syncthreads();
      continue;
    }
    // delete set: validated (readDeleteSet: no empty and no repeated client) through the LDS token tables
    // (ym_wave_ds.h), then copied verbatim
    {
      const uint32_t x = wds::ds_validate_lds(D, s_ds0, len, U.ds);
      if (t == 0) {
        if (x == NONE || x == wds::DS_BIG) { s_bad = 1; s_why = 17; }
        s_sum[MS_WAVES] = x;
      }
    }
    __syncthreads();
    if (s_bad) {
      if (t == 0) done[d] = (uint8_t)s_why;
      __syncthreads();
      continue;
    }
    const uint32_t ds1 = s_sum[MS_WAVES];
    const uint32_t ds0 = s_ds0;
    // sizes: each section's part, offsets by a block scan (sections in chunks of MS_T)
    uint32_t acc = 0, nparts = 0;
    for (uint32_t c0 = 0; c0 < nsec; c0 += MS_T) {
      const uint32_t ci = c0 + t;
      uint32_t sz = 0, kept = 0;
      if (ci < nsec && msec(ci, M_PRELEN) != NONE) {
        kept = 1;
        sz = vsz(msec(ci, M_WRITTEN)) + vsz(msec(ci, M_CLIENT)) + vsz(msec(ci, M_FCLOCK)) + msec(ci, M_PRELEN) +
             (msec(ci, M_A1) - msec(ci, M_A0)) + (msec(ci, M_X1) - msec(ci, M_B0));
      }
      const uint32_t wi = wave_incl_add(sz), wk = wave_incl_add(kept);
      if (lane == 63) { s_sum[wv] = wi; }
      __syncthreads();
      uint32_t pre = 0, all = 0;
      for (uint32_t q = 0; q < MS_WAVES; q++) { pre += q < wv ? s_sum[q] : 0; all += s_sum[q]; }
      if (ci < nsec && kept) msec(ci, M_OUT) = acc + pre + wi - sz;
      acc += all;
      __syncthreads();
      if (lane == 63) s_sum[wv] = wk;
      __syncthreads();
      for (uint32_t q = 0; q < MS_WAVES; q++) nparts += s_sum[q];
      __syncthreads();
    }
    const uint64_t total = vsz(nparts) + (uint64_t)acc + (ds1 - ds0);
    __shared__ unsigned long long s_base;
    if (t == 0) {
      s_base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
      done[d] = 1;
      atomicAdd((unsigned long long *)j.pw_count, 1ull);
    }
    __threadfence_block();
    __syncthreads();
    const uint64_t base = s_base;
    if (base + total > j.cap) {
      if (t == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    uint8_t *const o = j.out + base;
    const uint32_t p0 = vsz(nparts);
    if (t == 0) put_vu_g(o, 0, nparts);
    for (uint32_t ci = wv; ci < nsec; ci += MS_WAVES) {
      const uint32_t pl = msec(ci, M_PRELEN);
      if (pl == NONE) continue;
      const uint32_t written = msec(ci, M_WRITTEN), client = msec(ci, M_CLIENT), fclock = msec(ci, M_FCLOCK);
      uint32_t p = p0 + msec(ci, M_OUT);
      if (lane == 0) {
        uint32_t q = put_vu_g(o, p, written);
        q = put_vu_g(o, q, client);
        q = put_vu_g(o, q, fclock);
        for (uint32_t b = 0; b < pl; b++) o[q + b] = M.pre[(uint64_t)ci * PRE + b];
      }
      p += vsz(written) + vsz(client) + vsz(fclock) + pl;
      const uint32_t a0 = msec(ci, M_A0), a1 = msec(ci, M_A1);
      copy_bytes(o + p, D + a0, a1 - a0);
      p += a1 - a0;
      const uint32_t b0 = msec(ci, M_B0), b1 = msec(ci, M_X1);
      copy_bytes(o + p, D + b0, b1 - b0);
      if (lane == 0) msec(ci, M_OUT) = p - b0;  // output position = document position + this
    }
    if (wv == MS_WAVES - 1) copy_bytes(o + p0 + acc, D + ds0, ds1 - ds0);
    __threadfence();  // the patches below overwrite bytes other waves stored
    __syncthreads();
    const uint32_t np = s_npatch;
    for (uint32_t i = t; i < np; i += MS_T) o[msec(M.psec[i], M_OUT) + M.ppos[i]] = M.pval[i];
    if (t == 0) {
      atomicAdd(&pw_prof[2], __builtin_amdgcn_s_memrealtime() - tm2);
      atomicAdd(&pw_prof[3], (unsigned long long)np);
      j.out_off[d] = base;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}
#undef msec

// ---- 4. small documents: one wave per document, the whole update in one LDS window ---------------------
// The sync server's SyncStep1 -> SyncStep2 load: diffUpdate / encodeStateVectorFromUpdate / parseUpdateMeta
// over merged C2-size documents (~1-2 KB, a few to tens of client sections, ~100 structs).  k_pw_ms's table
// walk at one wave: the wave stages the update (<= 2 KB, or <= 4 KB) and parses a struct at every byte offset
// (one packed word per offset: next delta, Skip / patch flags, clock length); the wave then follows the
// chain in lockstep (every lane the same values, LDS reads made uniform: the chain's state in SGPRs), one
// table lookup per struct, doing the per-section work on the way (state-vector rules, the diff's cut and
// sliced head, info-byte patches) into LDS section records; the delete set is validated by the same
// lockstep walk (canonical varuints, no empty or repeated client); then lane ci sizes / writes section ci
// (wave prefix sums place them) and the wave copies the spans.  Same acceptance and bytes as k_pw_ms /
// k_big_v1 (a document this declines keeps done[d] == 0: the lane-per-document kernels and k_big_v1 follow).
// SW_NPRE: sliced first structs (one per section the diff cuts inside a struct) a document may have; more
// and the document goes to the streamed walker (the pool instead of one per section: 20.0 KB of LDS per
// diff wave instead of 22.3, 8 waves per CU instead of 7)
constexpr uint32_t SW_MIN = 80, SW_NSEC = 64, SW_NSV = 128, SW_SVS = 256, SW_NPATCH = 512, SW_DHS = 256, SW_NPRE = 16;
constexpr uint32_t SW_PROBE = 4;  // structs of the first section parsed before the tables (rich content declines; sv / meta: 2)
constexpr uint32_t SW_TV = 1u << 14, SW_CLEN = 1u << 17;  // table word: delta (12 bits) | skip << 12 | patch << 13 | TV | clen << 15
// section record fields: the first NQ_SV are what the state vector / meta walks keep, the rest the diff's
enum { Q_W = 0, Q_CLIENT, Q_CLOCK, Q_X1, Q_VAL, Q_END, NQ_SV, Q_PRELEN = NQ_SV, Q_A0, Q_A1, Q_B0, Q_WRITTEN, Q_FCLOCK, Q_OUT, NQ };
// DF: the diff's arrays (sliced heads, info-byte patches, the target state vector's hash, the delete set's
// client set) and section fields; the state vector / meta walks leave them out: 11.9 KB instead of 22.3 KB
// per wave at the 2 KB window, 13 waves per CU instead of 7 (their 58 VGPRs allow more; the diff's 173 do not)
template <uint32_t SWB, bool DF>
struct SwLds {
  static constexpr uint32_t NP = DF ? SW_NPATCH : 1, NS = DF ? SW_NPRE : 1, NH = DF ? SW_SVS : 1;
  uint8_t b[SWB + 48];
  uint32_t tab[SWB];
  uint32_t sec[SW_NSEC][DF ? NQ : NQ_SV];
  uint8_t pre[NS][PRE];
  uint16_t ppos[NP];
  uint8_t psec[NP], pval[NP];
  uint32_t mkey[NH], mval[NH], svclk[DF ? SW_NSV : 1];
  uint32_t dhs[DF ? SW_DHS : 1];
};
// lockstep lib0 readVarUint over the LDS bytes (uniform o): canonical, u32
__device__ __forceinline__ uint32_t sw_vu(const uint8_t *b, uint32_t &o, uint32_t lim, bool &bad) {
  uint32_t v = 0, nb = 0, x = 0x80;
  while ((x & 0x80) && nb < 5) {
    x = o + nb < lim ? RF(b[o + nb]) : 0x80;
    v |= (x & 0x7f) << (7 * nb);
    nb++;
  }
  bad |= (x & 0x80) || (nb > 1 && x == 0) || (nb == 5 && (x & 0x70) != 0);
  o += nb;
  return v;
}

#define SW_DECLINE_R(r)                                    \
  {                                                        \
    if (lane == 0) { done[d] = (uint8_t)(r); atomicAdd(tally, 1u); } \
    __syncthreads();                                       \
    continue;                                              \
  }
#define SW_URIERR() PW_URIERR()  // (the same completion: URIError status, done, counted)
// documents of (SWMIN, SWB] bytes.  tally[0]: documents this kernel's launches of the call declined so far
// (completions: j.pw_count, with the chunk walk's).  Rich content (nested `any` values, JSON objects / numbers: C2R / C4R) is declined to
// k_big_v1 after the table pass and part of the walk; once a batch has shown mostly such documents (more than
// 256 declines, 8 per completion), the blocks that start later leave their documents to k_big_v1 untried
// (the results are the same either way: only the wasted work goes).
template <int OP, uint32_t SWMIN, uint32_t SWB>
__global__ void __launch_bounds__(64) k_pw_small(GeneralJob j, uint8_t *done, uint64_t pw_min, uint32_t *tally) {
  __shared__ SwLds<SWB, OP == OP_DIFF> L;
  const uint32_t lane = threadIdx.x;
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    const uint32_t u0 = j.doc_upd[d];
    if (j.doc_upd[d + 1] - u0 != 1 || done[d]) continue;
    {
      const uint32_t dec = __builtin_nontemporal_load(tally);
      const uint64_t acc = __builtin_nontemporal_load(j.pw_count);
      if (dec > 256 && dec > 8 * acc) continue;
    }
    const uint64_t ub = j.upd_off[u0];
    const uint64_t len64 = j.upd_off[u0 + 1] - ub;
    // (tiny updates: the lane-per-document kernel; from pw_min on: the chunk walk / k_pw_ms)
    if (len64 <= SWMIN || len64 > SWB || len64 >= pw_min) continue;
    const uint32_t len = (uint32_t)len64;
    const uint8_t *D = j.A + ub;
    sc::cu32 *const B = sc::base_of(D);
    const uint32_t adj = (uint32_t)(ub & 3);
    __syncthreads();
    {  // the bytes (all loads in flight before the stores; the vector crossing the end re-loads the last 16
       // bytes) and 48 bytes of 0x80 past them (no stop byte)
      constexpr uint32_t NQ = (SWB + 1023) / 1024;
      uint32_t qs[NQ];
      uint4 xv[NQ];
#pragma unroll
      for (uint32_t t = 0; t < NQ; t++) {
        const uint32_t q = 16 * lane + 1024 * t;
        qs[t] = q + 16 <= len ? q : len - 16;
        xv[t] = *reinterpret_cast<const wds::u4u *>(D + qs[t]);
      }
#pragma unroll
      for (uint32_t t = 0; t < NQ; t++) __builtin_memcpy(L.b + qs[t], &xv[t], 16);
      if (lane < 48) L.b[len + lane] = 0x80;
    }
    uint32_t why = 0;
    bool bad = false;
    // the state vector (diff): decodeStateVector into the LDS hash map (a later entry wins), in lockstep
    if (OP == OP_DIFF) {
      for (uint32_t q = lane; q < SW_SVS; q += 64) L.mval[q] = 0;
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      __syncthreads();
      if (s1 - s0 > (1u << 20)) {
        why = 3;
      } else {
        ln::LCur sv = ln::make(j.sv + s0, 0, (uint32_t)(s1 - s0));
        const uint32_t ns = RF(ln::rvu(sv));
        if (RF(sv.bad ? 1u : 0u) || ns > SW_NSV) why = 3;
        for (uint32_t q = 0; q < ns && !why; q++) {
          const uint32_t cl = RF(ln::rvu(sv)), ck = RF(ln::rvu(sv));
          if (RF(sv.bad ? 1u : 0u)) { why = 3; break; }
          if (lane == 0) L.svclk[q] = ck;
          uint32_t h = (cl * 0x9E3779B1u) >> 24;
          while (RF(L.mval[h]) != 0 && RF(L.mkey[h]) != cl) h = (h + 1) & (SW_SVS - 1);
          if (lane == 0) { L.mkey[h] = cl; L.mval[h] = q + 1; }
          __syncthreads();
        }
      }
      if (why) SW_DECLINE_R(why ? why : 2)
    }
    __syncthreads();
    // probe: the chain's first structs with the full (non-nested) parser, in lockstep.  Rich content (nested
    // `any` values, JSON objects / numbers) usually shows there, and declines before the table pass that
    // makes up most of a document's cost here (C2R diff / C4R sv: every document declines to k_big_v1).
    {
      uint32_t q = 0;
      bool pb = false;
      const uint32_t nsec0 = sw_vu(L.b, q, len, pb);
      const uint32_t ns0 = nsec0 ? sw_vu(L.b, q, len, pb) : 0;
      sw_vu(L.b, q, len, pb);  // client
      sw_vu(L.b, q, len, pb);  // first clock
      for (uint32_t r = 0; r < ns0 && r < (OP == OP_DIFF ? SW_PROBE : 2u) && !pb; r++) {
        uint32_t nx, cl, f2;
        if (RF(ln::parse_struct(L.b, q, len, nx, cl, f2, len) ? 1u : 0u) == 0) { why = 8; break; }
        q = RF(nx);
      }
    }
    if (why) SW_DECLINE_R(why)
    // the tables: the branch-free short cut at every offset (most offsets start no struct, and the full
    // parser's divergent union over 64 garbage offsets costs ~5x the whole lockstep walk); a struct it does
    // not decide is parsed by the walk itself
    for (uint32_t o = lane; o < len; o += 64) {
      uint32_t nx, cl, fl;
      const bool ok = ln::parse_fast(L.b, o, len, nx, cl, fl);
      L.tab[o] = ok && cl < SW_CLEN && nx - o < 4096 ? (nx - o) | ((fl & F_SKIP) ? 1u << 12 : 0) | ((fl & F_PATCH) ? 1u << 13 : 0) | SW_TV | (cl << 15) : 0;
    }
    __syncthreads();
    // the chain, in lockstep
    uint32_t o = 0;
    const uint32_t nsec = sw_vu(L.b, o, len, bad);
    uint32_t p = o, npatch = 0, prev = 0;
    if (bad || nsec > SW_NSEC) SW_DECLINE_R(2)
    uint32_t npre = 0;  // sliced heads in the pool (diff)
    for (uint32_t ci = 0; ci < nsec && !why; ci++) {
      uint32_t q = p;
      const uint32_t ns = sw_vu(L.b, q, len, bad), client = sw_vu(L.b, q, len, bad), first_clock = sw_vu(L.b, q, len, bad);
      p = q;
      if (bad) { why = 5; break; }
      if (ns == 0 || (ci > 0 && client == prev) || (OP == OP_META && ci > 0 && client > prev)) { why = 6; break; }
      prev = client;
      uint32_t k = 0;
      if (OP == OP_DIFF) {
        uint32_t h = (client * 0x9E3779B1u) >> 24;
        while (RF(L.mval[h]) != 0) {
          if (RF(L.mkey[h]) == client) { k = RF(L.svclk[RF(L.mval[h]) - 1]); break; }
          h = (h + 1) & (SW_SVS - 1);
        }
      }
      uint64_t clock = first_clock;
      bool sv_stop = clock != 0, first = ci == 0, copying = false;
      uint32_t sv_clock = 0, written = 0;
      for (uint32_t r = 0; r < ns; r++) {
        if (p >= len) { why = 7; break; }
        const uint32_t w = RF(L.tab[p]);
        uint32_t nx, cl, fl;
        if (w & SW_TV) {
          nx = p + (w & 4095u);
          cl = w >> 15;
          fl = (w >> 12) & 3;
        } else {
          uint32_t f2;
          if (RF(ln::parse_struct(L.b, p, len, nx, cl, f2, len) ? 1u : 0u) == 0) { why = 8; break; }
          nx = RF(nx);
          cl = RF(cl);
          f2 = RF(f2);
          fl = ((f2 & F_SKIP) ? 1 : 0) | ((f2 & F_PATCH) ? 2 : 0);
        }
        if (cl >= (1u << 24)) { why = 9; break; }
        if (clock + cl > 0xffffffffull) { why = 10; break; }
        const bool skip = fl & 1;
        const uint64_t end = clock + cl;
        if (OP == OP_SV) {
          if (first) {
            first = false;
            if (!sv_stop) sv_clock = (uint32_t)end;
            if (skip) sv_stop = true;
          } else if (!sv_stop) {
            if (skip) sv_stop = true;
            else sv_clock = (uint32_t)end;
          }
        } else if (OP == OP_DIFF) {
          bool patch = false;
          if (!copying) {
            if (!skip && end > k) {  // the cut: the first struct that ends past sv[client]
              copying = true;
              written = 1;
              const uint32_t off = k > clock ? (uint32_t)(k - clock) : 0;
              uint32_t prelen = 0, a0 = 0, a1 = 0, b0, slot = 0;
              if (off == 0) {
                b0 = p;
                patch = true;
              } else {
                if (npre >= SW_NPRE) { why = 12; break; }
                slot = npre++;
                const uint32_t sh = RF(slice_head(B, adj, p, nx, client, clock, cl, off, L.pre[slot], prelen, a0, a1));
                if (sh != SH_OK) { why = sh == SH_URI ? WHY_URI : 11; break; }
                prelen = RF(prelen); a0 = RF(a0); a1 = RF(a1);
                b0 = nx;
              }
              if (lane == 0) {
                L.sec[ci][Q_PRELEN] = prelen | slot << 8;  // (prelen <= PRE < 256)
                L.sec[ci][Q_A0] = a0;
                L.sec[ci][Q_A1] = a1;
                L.sec[ci][Q_B0] = b0;
                L.sec[ci][Q_FCLOCK] = (uint32_t)(clock + off);
              }
            }
          } else {
            written++;
            patch = true;
          }
          if (patch && (fl & 2)) {  // the info byte re-encoded: 0x20 cleared with an origin, GC := 0
            if (npatch >= SW_NPATCH) { why = 12; break; }
            const uint32_t info = RF(L.b[p]);
            if (lane == 0) {
              L.ppos[npatch] = (uint16_t)p;
              L.psec[npatch] = (uint8_t)ci;
              L.pval[npatch] = (uint8_t)((info & 31) == 0 ? 0 : info & ~0x20u);
            }
            npatch++;
          }
        }
        clock = end;
        p = nx;
      }
      if (why) break;
      if (lane == 0) {
        L.sec[ci][Q_W] = ns;
        L.sec[ci][Q_CLIENT] = client;
        L.sec[ci][Q_CLOCK] = first_clock;
        L.sec[ci][Q_END] = (uint32_t)clock;
        L.sec[ci][Q_VAL] = sv_clock;
        L.sec[ci][Q_X1] = p;
        if (OP == OP_DIFF) {
          L.sec[ci][Q_WRITTEN] = copying ? written : 0;
          if (!copying) L.sec[ci][Q_PRELEN] = NONE;
        }
      }
    }
    if (why == WHY_URI) SW_URIERR()
    if (why) SW_DECLINE_R(why ? why : 2)
    const uint32_t ds0 = p;
    uint32_t ds1 = 0;
    if (OP == OP_DIFF) {  // the delete set: readDeleteSet's varuints canonical, no empty and no repeated client
      for (uint32_t q = lane; q < SW_DHS; q += 64) L.dhs[q] = NONE;
      __syncthreads();
      uint32_t q = p;
      const uint32_t ndc = sw_vu(L.b, q, len, bad);
      bool seen_max = false;
      if (bad || ndc > SW_DHS / 2) why = 17;
      for (uint32_t c = 0; c < ndc && !why; c++) {
        const uint32_t client = sw_vu(L.b, q, len, bad), m = sw_vu(L.b, q, len, bad);
        if (bad || m == 0) { why = 17; break; }
        if (client == NONE) {
          if (seen_max) { why = 17; break; }
          seen_max = true;
        } else {
          uint32_t h = (client * 0x9E3779B1u) >> 24;
          for (;;) {
            const uint32_t x = RF(L.dhs[h]);
            if (x == client) { why = 17; break; }
            if (x == NONE) break;
            h = (h + 1) & (SW_DHS - 1);
          }
          if (why) break;
          if (lane == 0) L.dhs[h] = client;
          __syncthreads();
        }
        for (uint32_t r = 0; r < 2 * m && !bad; r++) sw_vu(L.b, q, len, bad);
        if (bad) { why = 17; break; }
      }
      ds1 = q;
      if (why) SW_DECLINE_R(why ? why : 2)
    }
    __syncthreads();
    // outputs
    const uint32_t ci = lane;
    const bool live = ci < nsec;
    if (OP != OP_DIFF) {
      // state vector: vu(#entries) | per section with a value: client, value; meta: vu(nsec) | client, first
      // clock ... | vu(nsec) | client, end ...
      uint32_t sz = 0, sz2 = 0, cnt = 0;
      if (live) {
        if (OP == OP_SV) {
          const uint32_t v = L.sec[ci][Q_VAL];
          cnt = v != 0;
          sz = v ? vsz(L.sec[ci][Q_CLIENT]) + vsz(v) : 0;
        } else {
          sz = vsz(L.sec[ci][Q_CLIENT]) + vsz(L.sec[ci][Q_CLOCK]);
          sz2 = vsz(L.sec[ci][Q_CLIENT]) + vsz(L.sec[ci][Q_END]);
        }
      }
      const uint32_t i1 = wave_incl_add(sz), i2 = wave_incl_add(sz2), ic = wave_incl_add(cnt);
      const uint32_t t1 = lane_read(i1, 63), t2 = lane_read(i2, 63), tc = lane_read(ic, 63);
      const uint32_t h1 = vsz(OP == OP_SV ? tc : nsec), h2 = OP == OP_META ? vsz(nsec) : 0;
      const uint32_t total = h1 + t1 + h2 + t2;
      uint64_t base = 0;
      if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
      base = ((uint64_t)RF((uint32_t)(base >> 32)) << 32) | RF((uint32_t)base);
      if (lane == 0) { done[d] = 1; atomicAdd((unsigned long long *)j.pw_count, 1ull); }
      if (base + total > j.cap) {
        if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
        continue;
      }
      uint8_t *o = j.out + base;
      if (lane == 0) put_vu_g(o, 0, OP == OP_SV ? tc : nsec);
      if (live && sz) {
        const uint32_t q = put_vu_g(o, h1 + i1 - sz, L.sec[ci][Q_CLIENT]);
        put_vu_g(o, q, OP == OP_SV ? L.sec[ci][Q_VAL] : L.sec[ci][Q_CLOCK]);
      }
      if (OP == OP_META) {
        if (lane == 0) put_vu_g(o, h1 + t1, nsec);
        if (live) put_vu_g(o, put_vu_g(o, h1 + t1 + h2 + i2 - sz2, L.sec[ci][Q_CLIENT]), L.sec[ci][Q_END]);
      }
      if (lane == 0) {
        j.out_off[d] = base;
        j.out_len[d] = total;
        j.status[d] = ym::ST_OK;
      }
      continue;
    }
    // diff: kept sections' parts (header, sliced head, spans), then the delete set verbatim
    uint32_t sz = 0, kept = 0;
    if (live && L.sec[ci][Q_PRELEN] != NONE) {
      kept = 1;
      sz = vsz(L.sec[ci][Q_WRITTEN]) + vsz(L.sec[ci][Q_CLIENT]) + vsz(L.sec[ci][Q_FCLOCK]) + (L.sec[ci][Q_PRELEN] & 0xffu) +
           (L.sec[ci][Q_A1] - L.sec[ci][Q_A0]) + (L.sec[ci][Q_X1] - L.sec[ci][Q_B0]);
    }
    const uint32_t wi = wave_incl_add(sz), wk = wave_incl_add(kept);
    const uint32_t acc = lane_read(wi, 63), nparts = lane_read(wk, 63);
    const uint32_t p0 = vsz(nparts);
    const uint64_t total = p0 + (uint64_t)acc + (ds1 - ds0);
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    base = ((uint64_t)RF((uint32_t)(base >> 32)) << 32) | RF((uint32_t)base);
    if (lane == 0) { done[d] = 1; atomicAdd((unsigned long long *)j.pw_count, 1ull); }
    if (base + total > j.cap) {
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      continue;
    }
    uint8_t *const out = j.out + base;
    if (lane == 0) put_vu_g(out, 0, nparts);
    if (kept) {  // header and sliced head; the section's span placement for the patches
      const uint32_t pl = L.sec[ci][Q_PRELEN] & 0xffu, slot = L.sec[ci][Q_PRELEN] >> 8;
      uint32_t q = put_vu_g(out, p0 + wi - sz, L.sec[ci][Q_WRITTEN]);
      q = put_vu_g(out, q, L.sec[ci][Q_CLIENT]);
      q = put_vu_g(out, q, L.sec[ci][Q_FCLOCK]);
      for (uint32_t x = 0; x < pl; x++) out[q + x] = L.pre[slot][x];
      q += pl;
      L.sec[ci][Q_OUT] = q;
    }
    __syncthreads();
    // the spans, section by section, 64 bytes per step from LDS
    for (uint32_t c = 0; c < nsec; c++) {
      const uint32_t pl = RF(L.sec[c][Q_PRELEN]);
      if (pl == NONE) continue;
      uint32_t q = RF(L.sec[c][Q_OUT]);
      const uint32_t a0 = RF(L.sec[c][Q_A0]), a1 = RF(L.sec[c][Q_A1]), b0 = RF(L.sec[c][Q_B0]), x1 = RF(L.sec[c][Q_X1]);
      for (uint32_t x = lane; x < a1 - a0; x += 64) out[q + x] = L.b[a0 + x];
      q += a1 - a0;
      for (uint32_t x = lane; x < x1 - b0; x += 64) out[q + x] = L.b[b0 + x];
      if (lane == 0) L.sec[c][Q_OUT] = q - b0;  // output position = document position + this
    }
    for (uint32_t x = lane; x < ds1 - ds0; x += 64) out[p0 + acc + x] = L.b[ds0 + x];
    __syncthreads();
    for (uint32_t i = lane; i < npatch; i += 64) out[L.sec[L.psec[i]][Q_OUT] + L.ppos[i]] = L.pval[i];
    if (lane == 0) {
      j.out_off[d] = base;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
  }
}

}  // namespace pw

#define PWCHK(x)                                  \
  do {                                            \
    hipError_t e_ = (x);                          \
    if (e_ != hipSuccess) return -(int)e_ - 1000; \
  } while (0)

namespace {
int pw_ensure(PwBufs &B, int k, size_t n) {
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

// The chunk-parallel walk + stitch over the large single-update documents of a V1 diff / sv call (ym_kernels.h
// pw_prepare / pw_finish).  Documents it completes are marked in `*done_out` (k_big_v1 skips them).
const uint8_t *pw_last_done = nullptr;
namespace {
// the prep kernel's outputs after `done`: many[0] (a chunk-walked document of > 64 sections), many[1]
// (k_pw_small's tally), many[2] (chunks in all), many[4..5] (u64: bytes of the table-walked documents' areas)
uint32_t *pw_many(const GeneralJob &j, uint8_t *done) { return (uint32_t *)(((uintptr_t)(done + j.n) + 15) & ~(uintptr_t)15); }
}  // namespace
int pw_prepare(uint32_t op, const GeneralJob &j, hipStream_t st, PwBufs &B, const uint8_t **done_out) {
  using namespace pw;
  *done_out = nullptr;
  B.pending = false;
  if (j.v2 || (op != OP_DIFF && op != OP_SV && op != OP_META) || j.n == 0 || !j.pw_count || getenv("YMERGE_NO_PW")) return 0;
  // YMERGE_PW_MIN: smallest update taken (tests push small golden cases through this path)
  uint64_t pw_min = PW_MIN;
  if (const char *e = getenv("YMERGE_PW_MIN")) pw_min = strtoull(e, nullptr, 10);
  if (!B.pinned_dev) {
    if (B.pinned) hipHostFree(B.pinned);
    B.pinned = nullptr;
    if (hipHostMalloc((void **)&B.pinned, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return -2;
    if (hipHostGetDevicePointer((void **)&B.pinned_dev, B.pinned, 0) != hipSuccess) return -2;
  }
  if (!B.ev && hipEventCreateWithFlags(&B.ev, hipEventDisableTiming) != hipSuccess) return -2;
  uint32_t ms_min = MS_MIN;
  if (const char *e = getenv("YMERGE_PWMS_MIN")) ms_min = (uint32_t)strtoul(e, nullptr, 10);
  const uint32_t n1 = j.n + 1;
  if (pw_ensure(B, 0, 24ull * n1 + 64 + j.n)) return -2;
  uint64_t *msz = (uint64_t *)B.p[0];
  uint32_t *cnt = (uint32_t *)(msz + 2 * n1);
  uint8_t *done = (uint8_t *)(cnt + 2 * n1);
  uint32_t *many = pw_many(j, done);
  PWCHK(hipMemsetAsync(many, 0, 24, st));
  k_pw_prep<<<(n1 + 255) / 256, 256, 0, st>>>(j, cnt, done, pw_min, msz, ms_min, many);
  k_pw_totals<<<1, 64, 0, st>>>(many, B.pinned_dev);  // (a copy op would hold the stream ~25 us)
  PWCHK(hipEventRecord(B.ev, st));
  *done_out = done;  // every document is marked (0 = not taken) from here on
  pw_last_done = done;
  B.pending = true;
  B.op = op;
  return 1;
}
int pw_finish(const GeneralJob &j, hipStream_t st, PwBufs &B) {
  using namespace pw;
  if (!B.pending) return 0;
  B.pending = false;
  const uint32_t op = B.op, n1 = j.n + 1;
  uint64_t *msz = (uint64_t *)B.p[0], *moff = msz + n1;
  uint32_t *cnt = (uint32_t *)(msz + 2 * n1), *cbase = cnt + n1;
  uint8_t *done = (uint8_t *)(cnt + 2 * n1);
  PWCHK(hipEventSynchronize(B.ev));  // (the small documents' kernels keep the device busy meanwhile)
  const bool dsl = B.pinned[0] != 0;
  const uint32_t total = B.pinned[2];
  uint64_t mtotal;
  __builtin_memcpy(&mtotal, B.pinned + 4, 8);
  if (total == 0 && mtotal == 0) return 1;
  size_t tmp = 0, tmp2 = 0;
  if (total) scan_excl<uint32_t>(nullptr, tmp, cnt, cbase, n1, st);
  if (mtotal) scan_excl<uint64_t>(nullptr, tmp2, msz, moff, n1, st);
  if (tmp2 > tmp) tmp = tmp2;
  if (pw_ensure(B, 1, tmp + 16)) return -2;
  if (total && scan_excl<uint32_t>(B.p[1], tmp, cnt, cbase, n1, st)) return -3;
  if (mtotal && scan_excl<uint64_t>(B.p[1], tmp, msz, moff, n1, st)) return -3;
  const uint32_t grid = j.n < BS_GRID ? j.n : BS_GRID;
  // many-section documents: the table walk (no chunk records)
  if (mtotal > 0) {
    if (pw_ensure(B, 4, mtotal + 256)) {  // no room for the section tables: k_big_v1 takes those documents
      hipMemsetAsync(msz, 0, 8ull * n1, st);
    } else {
      uint8_t *area = (uint8_t *)B.p[4];
      if (op == OP_DIFF) k_pw_ms<OP_DIFF><<<grid, MS_T, 0, st>>>(j, done, msz, moff, area);
      else if (op == OP_SV) k_pw_ms<OP_SV><<<grid, MS_T, 0, st>>>(j, done, msz, moff, area);
      else k_pw_ms<OP_META><<<grid, MS_T, 0, st>>>(j, done, msz, moff, area);
    }
  }
  if (total == 0) return 1;
  if (pw_ensure(B, 2, 80ull * total) || pw_ensure(B, 3, 4ull * CAP * ((total + 63) & ~63u))) {
    // no room for the records: the chunk-walked documents go to k_big_v1 (the table-walked ones are done)
    return 1;
  }
  uint4 *desc = (uint4 *)B.p[2];
  uint32_t *recs = (uint32_t *)B.p[3];
  static int pre_one = -1, pre_many = -1;
  if (pre_one < 0) {  // (YMERGE_PW_PRE: both; YMERGE_PW_PRE_MANY: many-section documents only)
    const char *e = getenv("YMERGE_PW_PRE"), *em = getenv("YMERGE_PW_PRE_MANY");
    pre_one = e ? atoi(e) : (int)PRE_ONE;
    pre_many = em ? atoi(em) : e ? atoi(e) : (int)PRE_MANY;
  }
  k_pw_walk<<<(total + 255) / 256, 256, 0, st>>>(j, cbase, j.n, total, desc, recs, (uint32_t)pre_one, (uint32_t)pre_many);
  if (op == OP_DIFF && dsl) k_pw_stitch<OP_DIFF, true><<<grid, 64, L_SVM + lsv::BYTES, st>>>(j, cbase, desc, recs, done, msz);
  else if (op == OP_DIFF) k_pw_stitch<OP_DIFF><<<grid, 64, LDS_BYTES, st>>>(j, cbase, desc, recs, done, msz);
  else if (op == OP_SV) k_pw_stitch<OP_SV><<<grid, 64, LDS_BYTES, st>>>(j, cbase, desc, recs, done, msz);
  else k_pw_stitch<OP_META><<<grid, 64, LDS_BYTES, st>>>(j, cbase, desc, recs, done, msz);
  return 1;
}

}  // namespace ymk

// Small single updates of a V1 diff / sv / meta call that the lane-per-document kernels (ym_small.hip) left:
// one wave per document (k_pw_small; YMERGE_NO_PWSMALL: off).  After pw_prepare (done marked), before pw_finish.
namespace ymk {
int pw_small_launch(uint32_t op, const GeneralJob &j, uint8_t *done, hipStream_t st) {
  using namespace pw;
  static const bool no_small = getenv("YMERGE_NO_PWSMALL") != nullptr;
  if (!done || no_small || j.v2 || (op != OP_DIFF && op != OP_SV && op != OP_META) || j.n == 0) return 0;
  uint64_t pw_min = PW_MIN;
  if (const char *e = getenv("YMERGE_PW_MIN")) pw_min = strtoull(e, nullptr, 10);
  const uint32_t gs = j.n < 65536 ? j.n : 65536;
  uint32_t *tally = (uint32_t *)(((uintptr_t)(done + j.n) + 15) & ~(uintptr_t)15) + 1;  // (pw_prepare's `many` + 1)
// (the first window at 1,536 B: merged C2 documents, ~1 KB, fit it, and its 2.6 KB less LDS than a 2 KB window
// let more waves in -- diff_c2_v1 0.76 -> 0.71 ms, sv_c2_v1 0.49 -> 0.46; 1,280 B sends too many to the 4 KB
// launch: 0.95 / 0.56)
#define PW_SMALL(O)                                                          \
  k_pw_small<O, SW_MIN, 1536><<<gs, 64, 0, st>>>(j, done, pw_min, tally);    \
  k_pw_small<O, 1536, 4096><<<gs, 64, 0, st>>>(j, done, pw_min, tally);
  if (op == OP_DIFF) { PW_SMALL(OP_DIFF) }
  else if (op == OP_SV) { PW_SMALL(OP_SV) }
  else { PW_SMALL(OP_META) }
#undef PW_SMALL
  return 1;
}
}  // namespace ymk

// debugging aid (not part of include/ymerge.h): the last chunk-walk call's per-document outcome on the
// calling thread's device, 1 = completed, >= 2 = the decline reason (k_pw_stitch's `why`)
extern "C" int ym__pw_reasons(uint8_t *host, uint32_t n) {
  return ymk::pw_last_done ? (int)hipMemcpy(host, ymk::pw_last_done, n, hipMemcpyDeviceToHost) : -1;
}
namespace ymk {
namespace pw {
// parse_fast against parse_struct (uncapped) at every byte position of a buffer: [0] positions the short
// cut decided, [1] of them disagreeing with the full parser (next, length, flags or acceptance)
__global__ void k_lane_selftest(const uint8_t *b, uint32_t n, unsigned long long *cnt) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint32_t nx, cl, fl, nx2, cl2, fl2;
  if (!ln::parse_fast(b, p, n, nx, cl, fl)) return;
  atomicAdd(&cnt[0], 1ull);
  const bool ok = ln::parse_struct(b, p, n, nx2, cl2, fl2);
  if (!ok || nx != nx2 || cl != cl2 || fl != fl2) atomicAdd(&cnt[1], 1ull);
}
}  // namespace pw
}  // namespace ymk
// test hook (not part of include/ymerge.h): runs k_lane_selftest over a host buffer on the current device
extern "C" int ym__lane_selftest(const uint8_t *host, uint32_t n, unsigned long long *out) {
  uint8_t *d = nullptr;
  unsigned long long *c = nullptr;
  if (hipMalloc(&d, n + 64) != hipSuccess || hipMalloc(&c, 16) != hipSuccess) return -1;
  hipMemset(d, 0, n + 64);
  hipMemcpy(d, host, n, hipMemcpyHostToDevice);
  hipMemset(c, 0, 16);
  ymk::pw::k_lane_selftest<<<(n + 255) / 256, 256>>>(d, n, c);
  const int r = (int)hipMemcpy(out, c, 16, hipMemcpyDeviceToHost);
  hipFree(d);
  hipFree(c);
  return r;
}
extern "C" int ym__pw_ticks(unsigned long long *host, int reset) {  // 16 words
  int r = (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ymk::pw::pw_ticks), 128);
  if (reset) { unsigned long long z[16] = {}; hipMemcpyToSymbol(HIP_SYMBOL(ymk::pw::pw_ticks), z, 128); }
  return r;
}
extern "C" int ym__pw_prof(unsigned long long *host, int reset) {
  int r = (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ymk::pw::pw_prof), 128);
  if (reset) { unsigned long long z[16] = {}; hipMemcpyToSymbol(HIP_SYMBOL(ymk::pw::pw_prof), z, 128); }
  return r;
}
