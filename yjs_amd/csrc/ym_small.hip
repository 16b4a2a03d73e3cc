// ym_small.hip -- V1 diffUpdate / encodeStateVectorFromUpdate / parseUpdateMeta over SMALL single updates,
// one document per LANE (the sync server's SyncStep1 -> SyncStep2 load: merged C2 / C4 documents of
// ~1-2 KB, and parseUpdateMeta over every ~17-byte update of a log).
//
// k_big_v1 (ym_big.hip) runs one document per wave in lockstep: the walk of a 2 KB document is ~85
// dependent struct parses on one wave (~28 k instructions) whatever its size, and 1 M tiny updates are
// 1 M waves.  Here a 64-thread block takes ND documents: the wave stages their bytes into LDS with
// coalesced 16-byte loads (document l at slot l), then lane l walks document l on its own, the structs
// parsed by the chunk walk's lane parsers (ym_lane.h: the branch-free short cut parse_fast, parse_at for
// the rest), so a wave's instruction stream serves ND documents at once:
//   diff  pass 1 walks every section: sv[client] (a per-lane LDS copy of the decoded state vector, later
//         entries win), the cut (first non-Skip struct ending past it), the count written, the delete set
//         validated; then the document's output is bump-allocated; pass 2 writes each kept section: part
//         header, the cut struct (Item.write / GC.write with offset, or as is), the following structs
//         as is (info byte normalised: 0x20 cleared with an origin, GC := 0), then the delete set verbatim.
//   sv    the state-vector rules of k_big_v1 (13.5.16 os@37724), one pass.
//   meta  per section with structs: its first clock and the end of its last struct.
// Semantics and declines are exactly k_big_v1's (the same checks in the same order of effect); a lane
// that declines leaves its document to k_big_v1 (done[d] stays 0), which declines it further to the
// general path.  Documents of other sizes are left untouched.
#include <hip/hip_runtime.h>

#include "ym_fast_common.h"
#include "ym_kernels.h"
#include "ym_lane.h"

namespace ymk {
namespace smallv1 {
using namespace fastc;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t PREMAX = 64;  // bytes of a re-encoded head (the cut struct's fields before its content tail)

// LDS: ND slots of SLOT bytes (the document at offset b0 & 15, 32 bytes of slack for the parsers' window
// reads), per document NSEC section records (5 u32: diff's kept sections, sv / meta entries) and NSVE
// decoded state-vector entries (2 u32; then the delete set's clients)
template <uint32_t ND, uint32_t SLOT, uint32_t NSEC, uint32_t NSVE>
struct Lay {
  static constexpr uint32_t REC = ND * SLOT;
  static constexpr uint32_t SV = REC + ND * NSEC * 20;
  static constexpr uint32_t BYTES = SV + ND * NSVE * 8;
};

// Output stores go through a buffer resource (the document's output range, ym_fast_common.h Slot): vector
// memory stores at byte offsets.  (A generic pointer's store would also count against the LDS counter, so
// every later LDS read of the lane's walk would wait for that store's round trip to HBM.)
__device__ __forceinline__ void put_u64s(Slot o, uint32_t p, uint64_t v) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 w = {(unsigned int)v, (unsigned int)(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(w, o, (int)p, 0, 0);
}
__device__ __forceinline__ uint32_t gput(Slot o, uint32_t p, uint32_t v) { return put_vu(o, p, v); }
// n bytes from LDS offset s to output offset p
__device__ __forceinline__ void gcopy(Slot o, uint32_t p, uint32_t s, uint32_t n) {
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) put_u64s(o, p + i, ld8(s + i));
  for (; i < n; i++) ob8(o, p + i, sm[s + i]);
}
// one struct at LDS offset p (document end e): next position, clock length, info byte; false: k_big_v1's
// decline.  The parsers of the LDS merge kernels (ym_fast_common.h), nested payloads included.
__device__ __forceinline__ bool one(uint32_t p, uint32_t e, uint32_t &nx, uint32_t &len, uint32_t &info) {
  info = sm[p];
  // the branch-free short cut first (ym_lane.h: GC / Skip, Items with an origin and ContentDeleted or an
  // ASCII string -- the lanes of a wave stay converged on the structs of text documents), else the parsers
  uint32_t fl;
  if (ln::parse_fast(sm, p, e, nx, len, fl)) return true;
  Cur c = {p + 1, e, false};
  const bool skip = info == 10, gc = !skip && (info & 31) == 0;
  if (skip || gc) {
    len = rvu(c);
  } else if (!item_body<true>(c, info, len)) {
    return false;
  }
  nx = c.p;
  return !c.bad && c.p <= e;
}
__device__ __forceinline__ uint32_t norm_info(uint32_t info) {
  const bool skip = info == 10, gc = !skip && (info & 31) == 0;
  return skip ? info : gc ? 0 : ((info & 0xC0) ? info & ~0x20u : info);
}
// Item.write / GC.write with offset off (> 0) of the struct [s0, s1) (LDS offsets, info byte at s0) of client
// `client` at `clock`: writes the head to o (when o != nullptr) and returns its bytes, with the content tail
// [a0, a1) of the input that follows it; NONE: k_big_v1 declines (a kind it does not slice, a cut inside a
// surrogate pair: the general path raises yjs's error)
__device__ __forceinline__ uint32_t head(uint32_t s0, uint32_t s1, uint32_t info, uint32_t client, uint32_t clock,
                                         uint32_t len, uint32_t off, bool wr, Slot o, uint32_t p, uint32_t &a0, uint32_t &a1) {
  a0 = a1 = 0;
  const bool gc = info != 10 && (info & 31) == 0;
  if (gc) {
    if (wr) { ob8(o, p, 0); gput(o, p + 1, len - off); }
    return 1 + vsz(len - off);
  }
  const uint32_t ref = info & 31;
  if (ref != 1 && ref != 4 && ref != 8) return NONE;
  Cur e = {s0 + 1, s1, false};
  const uint32_t ni = ref | 0x80 | (info & 0x40) | ((info & 0xC0) == 0 ? (info & 0x20) : 0);
  if (info & 0x80) { skvu(e); skvu(e); }
  uint32_t ro0 = 0, ro1 = 0;
  if (info & 0x40) { ro0 = e.p; skvu(e); skvu(e); ro1 = e.p; }
  if ((info & 0xC0) == 0) {
    const uint32_t pi = rvu(e);
    if (pi == 1) { const uint32_t n = rvu(e); e.p += n; }
    else { skvu(e); skvu(e); }
    if (info & 0x20) { const uint32_t n = rvu(e); e.p += n; }
  }
  uint32_t q = 1 + vsz(client) + vsz(clock + off - 1) + (ro1 - ro0);
  if (wr) {
    ob8(o, p, ni);
    uint32_t t = gput(o, p + 1, client);
    t = gput(o, t, clock + off - 1);
    for (uint32_t x = ro0; x < ro1; x++) ob8(o, t++, sm[x]);
  }
  if (ref == 1) {
    rvu(e);
    if (wr) gput(o, p + q, len - off);
    q += vsz(len - off);
  } else if (ref == 8) {
    rvu(e);
    for (uint32_t i = 0; i < off; i++) any_canon<true>(e);  // ContentAny.splice: drop `off` values
    if (wr) gput(o, p + q, len - off);
    q += vsz(len - off);
    a0 = e.p;
    a1 = s1;
  } else {  // ContentString: str.slice(off) in UTF-16 units
    const uint32_t n = rvu(e);
    uint32_t bi = 0, u = 0;
    while (u < off && bi < n) {
      const uint32_t x = sm[e.p + bi];
      const uint32_t l = x < 0x80 ? 1 : x < 0xE0 ? 2 : x < 0xF0 ? 3 : 4;
      u += l == 4 ? 2 : 1;
      bi += l;
    }
    if (u != off) return NONE;
    if (wr) gput(o, p + q, n - bi);
    q += vsz(n - bi);
    a0 = e.p + bi;
    a1 = e.p + n;
  }
  if (e.bad || q > PREMAX) return NONE;
  return q;
}

// OP_DIFF / OP_SV / OP_META over documents [blockIdx.x * ND, + ND) that are one update of <= SLOT - 48 bytes
template <int OP, uint32_t ND, uint32_t SLOT, uint32_t NSEC, uint32_t NSVE>
__global__ void __launch_bounds__(64) k_small_v1(GeneralJob j, uint8_t *done, uint64_t pw_min) {
  using L = Lay<ND, SLOT, NSEC, NSVE>;
  const uint32_t lane = threadIdx.x;
  const uint32_t d0 = blockIdx.x * ND;
  // ---- staging: document l's bytes at slot l (byte b0 at offset b0 & 15): tiny documents by their own
  // lane (a few independent 16-byte loads each), small ones by the whole wave, 1 KB per step
  auto stage = [&](uint32_t l, uint32_t v0, uint32_t dv) {
    const uint32_t d = d0 + l;
    if (d >= j.n) return;
    const uint32_t u0 = j.doc_upd[d];
    if (j.doc_upd[d + 1] - u0 != 1 || done[d]) return;
    const uint64_t b0 = j.upd_off[u0], len = j.upd_off[u0 + 1] - b0;
    if (len == 0 || len + 48 > SLOT || len >= pw_min) return;
    const uint4 *src = reinterpret_cast<const uint4 *>(j.A + (b0 & ~15ull));
    const uint32_t nvec = (uint32_t)(((b0 & 15) + len + 15) >> 4);
    if (ND == 64) {  // a lane's own document: every load in flight before the first store
      constexpr uint32_t MV = (SLOT - 48 + 30) / 16;
      uint4 x[MV];
#pragma unroll
      for (uint32_t t = 0; t < MV; t++) x[t] = src[t < nvec ? t : nvec - 1];
#pragma unroll
      for (uint32_t t = 0; t < MV; t++) at<uint4>(l * SLOT + 16 * (t < nvec ? t : nvec - 1)) = x[t];
      return;
    }
    for (uint32_t v = v0; v < nvec; v += dv) at<uint4>(l * SLOT + 16 * v) = src[v];
  };
  if (ND == 64) stage(lane, 0, 1);
  else for (uint32_t l = 0; l < ND; l++) stage(l, lane, 64);
  __syncthreads();
  if (lane >= ND) return;
  const uint32_t d = d0 + lane;
  if (d >= j.n) return;
  const uint32_t u0 = j.doc_upd[d];
  if (j.doc_upd[d + 1] - u0 != 1 || done[d]) return;
  const uint64_t ub = j.upd_off[u0], len64 = j.upd_off[u0 + 1] - ub;
  // (from pw_min on the document is the chunk walk's: the two sets stay disjoint, as k_pw_small's)
  if (len64 == 0 || len64 + 48 > SLOT || len64 >= pw_min) return;
  const uint32_t len = (uint32_t)len64;
  const uint32_t B = lane * SLOT + (uint32_t)(ub & 15), E = B + len;  // the update's bytes: LDS [B, E)
  const uint32_t REC = L::REC + lane * NSEC * 20;                      // u32[NSEC][5]
  const uint32_t SVT = L::SV + lane * NSVE * 8;                        // u32[NSVE][2]
  auto rec = [&](uint32_t i) -> uint32_t & { return at<uint32_t>(REC + 4 * i); };
  auto svt = [&](uint32_t i) -> uint32_t & { return at<uint32_t>(SVT + 4 * i); };
  // ---- the state vector (diff): decodeStateVector, a later entry for a client wins
  uint32_t nsv = 0;
  if (OP == OP_DIFF) {
    const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
    if (s1 - s0 > 16ull * NSVE) return;
    ln::LCur c = ln::make(j.sv + s0, 0, (uint32_t)(s1 - s0));
    const uint32_t n = ln::rvu(c);
    if (c.bad || n > NSVE) return;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t cl = ln::rvu(c), ck = ln::rvu(c);
      svt(2 * i) = cl;
      svt(2 * i + 1) = ck;
    }
    if (c.bad) return;
    nsv = n;
  }
  auto sv_get = [&](uint32_t client) -> uint32_t {
    uint32_t k = 0;
    for (uint32_t i = 0; i < nsv; i++)
      if (svt(2 * i) == client) k = svt(2 * i + 1);
    return k;
  };
  // ---- pass 1: the struct section
  Cur c = {B, E, false};
  const uint32_t nclients = rvu(c);
  if (c.bad || nclients > NSEC) return;
  uint32_t p = c.p;
  uint32_t nparts = 0, body = 0;  // diff: kept sections, their bytes (headers included)
  uint32_t sv_client = 0, sv_clock = 0, sv_n = 0, prev_client = 0;
  bool sv_stop = false, sv_any = false;
  for (uint32_t ci = 0; ci < nclients; ci++) {
    Cur h = {p, E, false};
    const uint32_t nstructs = rvu(h), client = rvu(h);
    uint64_t clock = rvu(h);
    if (h.bad) return;
    p = h.p;
    if (ci > 0 && client == prev_client) return;                  // the writer would not start a part
    if (OP == OP_META && ci > 0 && client > prev_client) return;  // a repeated client keeps its first position
    const uint32_t first_clock = (uint32_t)clock;
    prev_client = client;
    const uint32_t k = OP == OP_DIFF ? sv_get(client) : 0;
    if (OP == OP_SV && nstructs > 0 && sv_any && client != sv_client) {  // client change (os@37724)
      if (sv_clock != 0) {
        if (sv_n >= NSEC) return;
        rec(2 * sv_n) = sv_client;
        rec(2 * sv_n + 1) = sv_clock;
        sv_n++;
      }
      sv_client = client; sv_clock = 0; sv_stop = clock != 0;
    }
    bool copying = false;
    uint32_t written = 0, sbytes = 0;
    for (uint32_t si = 0; si < nstructs; si++) {
      uint32_t nx, l, info;
      if (p >= E || !one(p, E, nx, l, info)) return;
      const bool skip = info == 10;
      if (clock + l > 0xffffffffull) return;
      if (OP == OP_SV) {
        if (!sv_any) {
          sv_any = true;
          sv_client = client;
          sv_stop = clock != 0;
          sv_clock = sv_stop ? 0 : (uint32_t)(clock + l);
        }
        if (skip) sv_stop = true;
        if (!sv_stop) sv_clock = (uint32_t)(clock + l);
      } else if (OP == OP_DIFF) {
        if (!copying) {
          if (!skip && clock + l > k) {  // the cut
            copying = true;
            written = 1;
            const uint32_t off = k > clock ? (uint32_t)(k - clock) : 0;
            if (nparts >= NSEC) return;
            uint32_t hb = nx - p;
            if (off > 0) {
              uint32_t a0, a1;
              hb = head(p, nx, info, client, (uint32_t)clock, l, off, false, make_slot(j.out, 0), 0, a0, a1);
              if (hb == NONE) return;
              hb += a1 - a0;
            }
            rec(5 * nparts) = p;
            rec(5 * nparts + 1) = off;
            rec(5 * nparts + 3) = (uint32_t)(clock + off);
            rec(5 * nparts + 4) = client;
            sbytes = hb;
          }
        } else {
          written++;
          sbytes += nx - p;
        }
      }
      clock += l;
      p = nx;
    }
    if (OP == OP_META && nstructs > 0) {
      if (sv_n >= NSEC) return;
      rec(3 * sv_n) = client;
      rec(3 * sv_n + 1) = first_clock;
      rec(3 * sv_n + 2) = (uint32_t)clock;
      sv_n++;
    }
    if (OP == OP_DIFF && copying) {
      rec(5 * nparts + 2) = written;
      body += vsz(written) + vsz(client) + vsz(rec(5 * nparts + 3)) + sbytes;
      nparts++;
    }
  }
  uint32_t total = 0;
  if (OP == OP_META) {
    uint32_t tl = 2 * vsz(sv_n);
    for (uint32_t i = 0; i < sv_n; i++) tl += 2 * vsz(rec(3 * i)) + vsz(rec(3 * i + 1)) + vsz(rec(3 * i + 2));
    total = tl;
  } else if (OP == OP_SV) {
    if (sv_any && sv_clock != 0) {
      if (sv_n >= NSEC) return;
      rec(2 * sv_n) = sv_client;
      rec(2 * sv_n + 1) = sv_clock;
      sv_n++;
    }
    uint32_t tl = vsz(sv_n);
    for (uint32_t i = 0; i < sv_n; i++) tl += vsz(rec(2 * i)) + vsz(rec(2 * i + 1));
    total = tl;
  }
  // ---- delete set (diff): validated, copied verbatim (readDeleteSet + writeDeleteSet round trip)
  const uint32_t ds0 = p;
  if (OP == OP_DIFF) {
    Cur e = {p, E, false};
    const uint32_t ndc = rvu(e);
    if (e.bad || ndc > 2 * NSVE) return;
    // repeated clients: checked against the clients seen so far (the sv table's space is free now)
    for (uint32_t i = 0; i < ndc; i++) {
      const uint32_t client = rvu(e), m = rvu(e);
      if (e.bad || m == 0) return;
      for (uint32_t h = 0; h < i; h++)
        if (svt(h) == client) return;
      svt(i) = client;
      for (uint32_t q = 0; q < m && !e.bad; q++) { skvu(e); skvu(e); }
    }
    if (e.bad) return;
    p = e.p;
    total = vsz(nparts) + body + (p - ds0);
  }
  // ---- allocation, then the output (buffer stores into the document's output range)
  const uint64_t base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
  done[d] = 1;
  if (base + total > j.cap) {
    j.status[d] = ym::ST_CAPACITY;
    j.out_len[d] = 0;
    return;
  }
  const Slot o = make_slot(j.out + base, total);
  if (OP == OP_META) {  // from then to: vu(n) | (client, clock)*
    uint32_t q = gput(o, 0, sv_n);
    for (uint32_t i = 0; i < sv_n; i++) { q = gput(o, q, rec(3 * i)); q = gput(o, q, rec(3 * i + 1)); }
    q = gput(o, q, sv_n);
    for (uint32_t i = 0; i < sv_n; i++) { q = gput(o, q, rec(3 * i)); q = gput(o, q, rec(3 * i + 2)); }
  } else if (OP == OP_SV) {
    uint32_t q = gput(o, 0, sv_n);
    for (uint32_t i = 0; i < sv_n; i++) { q = gput(o, q, rec(2 * i)); q = gput(o, q, rec(2 * i + 1)); }
  } else {
    // ---- pass 2 (diff): each kept section from its cut struct
    uint32_t q = gput(o, 0, nparts);
    for (uint32_t s = 0; s < nparts; s++) {
      const uint32_t written = rec(5 * s + 2), off = rec(5 * s + 1), fclock = rec(5 * s + 3), client = rec(5 * s + 4);
      q = gput(o, q, written);
      q = gput(o, q, client);
      q = gput(o, q, fclock);
      uint32_t x = rec(5 * s);
      for (uint32_t w = 0; w < written; w++) {
        uint32_t nx, l, info;
        one(x, E, nx, l, info);  // (parsed in pass 1)
        if (w == 0 && off > 0) {
          uint32_t a0, a1;
          q += head(x, nx, info, client, fclock - off, l, off, true, o, q, a0, a1);
          gcopy(o, q, a0, a1 - a0);
          q += a1 - a0;
        } else {
          ob8(o, q, norm_info(info));
          gcopy(o, q + 1, x + 1, nx - x - 1);
          q += nx - x;
        }
        x = nx;
      }
    }
    gcopy(o, q, ds0, p - ds0);
  }
  j.out_off[d] = base;
  j.out_len[d] = total;
  j.status[d] = ym::ST_OK;
}

}  // namespace smallv1

// The lane-per-document pass over the small single-update documents of a V1 diff / sv / meta call (after the
// chunk walk, before k_big_v1, which skips what this marks done).  Two shapes: tiny updates (<= 80 bytes:
// 64 per block, e.g. parseUpdateMeta over an update log) and small documents (<= 2 KB: 16 per block).
int small_launch(uint32_t op, const GeneralJob &j, uint8_t *done, hipStream_t st, bool tiny_only) {
  using namespace smallv1;
  if (!done || j.v2 || getenv("YMERGE_NO_SMALL")) return 0;
  const uint32_t g64 = (j.n + 63) / 64, g16 = (j.n + 15) / 16;
  uint64_t pw_min = 32768;  // ym_pwalk.hip PW_MIN: the chunk walk's documents (YMERGE_PW_MIN, as pw_prepare)
  if (const char *e = getenv("YMERGE_PW_MIN")) pw_min = strtoull(e, nullptr, 10);
  // tiny: 64 documents of <= 80 bytes (2 sections, 16 state-vector entries); small: 16 of <= 2 KB (32 each;
  // more: k_pw_small)
  // (the 2 KB shape for meta only: measured on C2 / C2r / C4r merged documents, diff and state vector run
  // faster as one wave per document, k_pw_small -- a rich document's lanes diverge in the parsers)
#define YS_LAUNCH(O)                                                                                         \
  k_small_v1<O, 64, 128, 8, 16><<<g64, 64, Lay<64, 128, 8, 16>::BYTES, st>>>(j, done, pw_min);                    \
  if (O == OP_META && !tiny_only) k_small_v1<O, 16, 2112, 32, 32><<<g16, 64, Lay<16, 2112, 32, 32>::BYTES, st>>>(j, done, pw_min);
  if (op == OP_DIFF) { YS_LAUNCH(OP_DIFF) }
  else if (op == OP_SV) { YS_LAUNCH(OP_SV) }
  else if (op == OP_META) { YS_LAUNCH(OP_META) }
  else return 0;
#undef YS_LAUNCH
  return 1;
}

}  // namespace ymk
