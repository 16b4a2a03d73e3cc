// ym_big.hip -- V1 diffUpdate / encodeStateVectorFromUpdate over single updates of any size: one wave
// per document, the update streamed through an LDS window, the struct walk run by the whole wave in
// lockstep (uniform control flow, no divergence), output assembled from small LDS pieces plus
// verbatim input spans copied by all 64 lanes.
//
// Semantics are yjs 13.5.16's:
//   diffUpdate (bundle fs / us@40707): per client section, structs whose end <= sv[client] are dropped,
//     Skips before the cut are dropped, the first struct past the cut is written with offset
//     max(sv - clock, 0) (Item.write with offset: origin := (client, clock + offset - 1), content
//     sliced -- ContentString.js:94-96, ContentDeleted.js:83-85, ContentAny.js:80-87, GC.js:45-48),
//     every following struct of the section is written as is (LazyStructWriter, rs/gs/ps/ws), the
//     delete set is re-written unchanged (readDeleteSet + writeDeleteSet, DeleteSet.js:219-256).
//   encodeStateVectorFromUpdate (cs / os@37724): per client, the end of its last struct while its
//     first struct starts at 0 and no Skip has been seen; clients with clock 0 are omitted.
// "As is" = the input bytes with the info byte normalised (0x20 cleared when an origin is present,
// GC info := 0), which the kernel applies as patches after the bulk copy.  Inputs this path does not
// verify (JSON/Doc content, non-canonical encodings, repeated clients, oversized structs, ...) are
// declined to the exact general path (ym_general.hip), as in ym_fast.hip.
#include <hip/hip_runtime.h>

#include "ym_fast_common.h"
#include "ym_kernels.h"
#include "ym_scalar.h"
#include "ym_cmap.h"

namespace ymk {
namespace big {
using namespace fastc;
using sc::SCur;
constexpr uint32_t NSEC = BS_NSEC;  // client sections per update (HBM scratch, per block)
constexpr uint32_t NSV = BS_NSV;    // state-vector entries (HBM scratch)
constexpr uint32_t NPATCH = 512;
constexpr uint32_t PRE = BS_PRE;    // sliced-struct prefix bytes per section

constexpr uint32_t SECW = BS_SECW;  // u32 fields per section record
constexpr uint32_t L_PRE = 0;                        // u8[PRE] the current section's sliced-struct head
constexpr uint32_t L_PPOS = L_PRE + PRE;             // u32[NPATCH] patch positions (update-relative)
constexpr uint32_t L_PVAL = L_PPOS + 4 * NPATCH;     // u8[NPATCH]  patched info bytes
constexpr uint32_t L_PSEC = L_PVAL + NPATCH;         // u32[NPATCH] section of each patch
constexpr uint32_t LDS_BYTES = L_PSEC + 4 * NPATCH;
// section record fields: head bytes (or NONE: nothing written), span A (content tail of a sliced
// struct), span B (the following structs, as is), part header (written, client, first clock), and
// the output position of update byte 0 within span B (for the patches)
enum { S_PRELEN = 0, S_A0, S_A1, S_B0, S_B1, S_WRITTEN, S_CLIENT, S_FCLOCK, S_OUTB };
constexpr uint32_t NONE = 0xffffffffu;
// per-block HBM scratch (ym_kernels.h BS_*): section records, their sliced heads, state vector,
// delete-set clients
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
// sv[client] (decodeStateVector: a later entry for the same client wins), wave-parallel
__device__ __forceinline__ uint32_t sv_lookup(const uint32_t *svt, uint32_t nsv, uint32_t client) {
  int best = -1;
  for (uint32_t i0 = 0; i0 < nsv; i0 += 64) {
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t m = __ballot(i < nsv && svt[2 * i] == client);
    if (m) best = (int)(i0 + 63 - __builtin_clzll(m));
  }
  return best >= 0 ? svt[2 * best + 1] : 0;
}
// was `client` among the first n delete-set clients? (wave-parallel)
__device__ __forceinline__ bool seen_before(const uint32_t *dsc, uint32_t n, uint32_t client) {
  bool hit = false;
  for (uint32_t h0 = 0; h0 < n; h0 += 64) {
    const uint32_t h = h0 + threadIdx.x;
    hit |= __any(h < n && dsc[h] == client);
  }
  return hit;
}

// wave copy of n bytes (any alignment): 16-byte unaligned vector accesses, then the tail bytes
typedef uint4 __attribute__((aligned(1))) u4u;
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t n) {
  const uint32_t nv = n >> 4;
  for (uint32_t v = threadIdx.x; v < nv; v += 64) reinterpret_cast<u4u *>(dst)[v] = reinterpret_cast<const u4u *>(src)[v];
  for (uint32_t i = (nv << 4) + threadIdx.x; i < n; i += 64) dst[i] = src[i];
}
__device__ __forceinline__ uint32_t put_vu_lds(uint32_t p, uint32_t v) {
  while (v > 127) { sm[p++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
  sm[p++] = (uint8_t)v;
  return p;
}

#define YB_DECLINE()                                        \
  {                                                         \
    if (threadIdx.x == 0) {                                 \
      j.status[d] = ST_PENDING;                             \
      const uint32_t q_ = atomicAdd(j.pend_count, 1u);      \
      if (j.pend_list) j.pend_list[q_] = d;                 \
    }                                                       \
    __syncthreads();                                        \
    continue;                                               \
  }

// OP = OP_DIFF, OP_SV or OP_META (parseUpdateMeta: per client section with structs, the first clock
// (`from`) and the end of its last struct, Skips included (`to`); V1 only)
template <int OP>
__global__ void __launch_bounds__(64) k_big_v1(GeneralJob j) {
  const uint32_t lane = threadIdx.x;
  const Scr X = scratch(j);
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    if (j.pw_done && j.pw_done[d] == 1) continue;  // completed by the chunk-parallel walk
    const uint32_t u0 = j.doc_upd[d];
    if (j.doc_upd[d + 1] - u0 != 1) YB_DECLINE()
    // the update, read by scalar loads (ym_scalar.h): byte offsets from a dword-aligned base
    const uint64_t ub = j.upd_off[u0];
    const uint64_t len64 = j.upd_off[u0 + 1] - ub;
    if (len64 == 0 || len64 > 0xfffffff0ull) YB_DECLINE()
    sc::cu32 *const B = sc::base_of(j.A + ub);
    const uint32_t adj = (uint32_t)(ub & 3);
    auto rel = [&](uint32_t x) { return x - adj; };  // base offset -> update-relative
    // ---- state vector (diff): decodeStateVector, later entries win (encoding.js:536-545)
    uint32_t nsv = 0;
    bool bad = false;
    if (OP == OP_DIFF) {
      const uint64_t s0 = j.sv_off[d], s1 = j.sv_off[d + 1];
      if (s1 - s0 > 16ull * NSV) YB_DECLINE()
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
      if (bad) YB_DECLINE()
      if (nsv > 64) cmap::build_sv(X.map, X.svt, nsv);
    }
    // ---- struct section (encoding.js:127-198 layout; 13.5.16 LazyStructReader)
    SCur c = sc::make(B, adj, adj + (uint32_t)len64);
    const uint32_t nclients = rvu(c);
    if (nclients > NSEC) YB_DECLINE()
    uint32_t nparts = 0, npatch = 0, body_bytes = 0;
    // state-vector op state (os@37724), carried across sections
    uint32_t sv_client = 0, sv_clock = 0, sv_n = 0;
    bool sv_stop = false, sv_any = false;
    uint32_t prev_client = 0;
    bool declined = false;
    for (uint32_t ci = 0; ci < nclients && !c.bad && !declined; ci++) {
      sc::uni(c);
      const uint32_t nstructs = rvu(c);
      const uint32_t client = rvu(c);
      uint64_t clock = rvu(c);
      if (ci > 0 && client == prev_client) { declined = true; break; }  // writer would not start a part
      // meta: a client met again would keep its first Map position -- taken only when every section's
      // client is below the previous one (yjs writes clients in descending order), so none repeats
      if (OP == OP_META && ci > 0 && client > prev_client) { declined = true; break; }
      const uint32_t first_clock = (uint32_t)clock;
      prev_client = client;
      const uint32_t k = OP != OP_DIFF ? 0 : nsv > 64 ? cmap::sv_get(X.map, X.svt, client) : sv_lookup(X.svt, nsv, client);
      if (OP == OP_SV && nstructs > 0 && sv_any && client != sv_client) {  // client change (os@37724)
        if (sv_clock != 0) {
          if (sv_n >= NSV) { declined = true; break; }
          if (lane == 0) { X.svt[2 * sv_n] = sv_client; X.svt[2 * sv_n + 1] = sv_clock; }
          sv_n++;
        }
        sv_client = client; sv_clock = 0; sv_stop = clock != 0;
      }
      bool copying = false;
      uint32_t written = 0, b0r = 0;
      for (uint32_t si = 0; si < nstructs && !c.bad; si++) {
        sc::uni(c);
        clock = sc::rfl64(clock);
        const uint32_t s0 = c.p;
        const uint32_t info = rdb(c);
        uint32_t len;
        const bool skip = info == 10, gc = !skip && (info & 31) == 0;
        if (skip || gc) len = rvu(c);
        else if (!item_body(c, info, len)) { declined = true; break; }
        if (c.bad || c.p > c.e) { declined = true; break; }
        if (clock + len > 0xffffffffull) { declined = true; break; }
        if (OP == OP_SV) {
          if (!sv_any) {  // the update's first struct initialises the state
            sv_any = true;
            sv_client = client;
            sv_stop = clock != 0;
            sv_clock = sv_stop ? 0 : (uint32_t)(clock + len);
          }
          if (skip) sv_stop = true;
          if (!sv_stop) sv_clock = (uint32_t)(clock + len);
        } else if (OP == OP_META) {
          // parseUpdateMeta only measures the section: nothing is cut or copied
        } else if (!copying) {
          if (!skip && clock + len > k) {  // the cut: first struct that ends past sv[client]
            copying = true;
            written = 1;
            const uint32_t off = k > clock ? (uint32_t)(k - clock) : 0;
            const uint32_t pre = L_PRE;
            uint32_t q = pre, a0 = 0, a1 = 0;
            if (off == 0) {
              b0r = rel(s0);
              const uint32_t ni = gc ? 0 : ((info & 0xC0) ? info & ~0x20u : info);
              if (ni != info) {
                if (npatch >= NPATCH) { declined = true; break; }
                if (lane == 0) { at<uint32_t>(L_PPOS + 4 * npatch) = b0r; sm[L_PVAL + npatch] = (uint8_t)ni; at<uint32_t>(L_PSEC + 4 * npatch) = ci; }
                npatch++;
              }
            } else {
              // Item.write / GC.write with offset: re-encode the head, copy the content's tail
              SCur e = sc::make(B, s0 + 1, c.p);
              const uint32_t ref = info & 31;
              if (gc) {
                if (lane == 0) { sm[q] = 0; put_vu_lds(q + 1, len - off); }
                q += 1 + vsz(len - off);
              } else {
                if (ref != 1 && ref != 4 && ref != 8) { declined = true; break; }
                // parentSub was read iff there were no origins; Item.write keeps its info bit even
                // though the new origin suppresses writing it (E9)
                const uint32_t ni = ref | 0x80 | (info & 0x40) | ((info & 0xC0) == 0 ? (info & 0x20) : 0);
                if (info & 0x80) { skvu(e); skvu(e); }
                uint32_t ro0 = 0, ro1 = 0;
                if (info & 0x40) { ro0 = e.p; skvu(e); skvu(e); ro1 = e.p; }
                if ((info & 0xC0) == 0) {
                  const uint32_t pi = rvu(e);
                  if (pi == 1) { const uint32_t n = rvu(e); sc::skip(e, n); }
                  else { skvu(e); skvu(e); }
                  if (info & 0x20) { const uint32_t n = rvu(e); sc::skip(e, n); }
                }
                if (lane == 0) {
                  sm[q] = (uint8_t)ni;
                  uint32_t t = put_vu_lds(q + 1, client);
                  t = put_vu_lds(t, (uint32_t)(clock + off - 1));
                  for (uint32_t b = ro0; b < ro1; b++) sm[t++] = (uint8_t)sc::byte(B, b);
                }
                q += 1 + vsz(client) + vsz((uint32_t)(clock + off - 1)) + (ro1 - ro0);
                if (ref == 1) {
                  rvu(e);
                  if (lane == 0) put_vu_lds(q, len - off);
                  q += vsz(len - off);
                } else if (ref == 8) {
                  rvu(e);
                  for (uint32_t i = 0; i < off; i++) any_canon(e);  // ContentAny.splice: drop `off` values
                  if (lane == 0) put_vu_lds(q, len - off);
                  q += vsz(len - off);
                  a0 = rel(e.p);
                  a1 = rel(c.p);
                } else {  // ContentString: str.slice(off) in UTF-16 units; a split surrogate throws in yjs
                  const uint32_t n = rvu(e);
                  uint32_t bi = 0, u = 0;
                  while (u < off && bi < n) {
                    const uint32_t b = sc::byte(B, e.p + bi);
                    const uint32_t l = b < 0x80 ? 1 : b < 0xE0 ? 2 : b < 0xF0 ? 3 : 4;
                    u += l == 4 ? 2 : 1;
                    bi += l;
                  }
                  if (u != off) { declined = true; break; }  // cut inside a surrogate pair: URIError path
                  if (lane == 0) put_vu_lds(q, n - bi);
                  q += vsz(n - bi);
                  a0 = rel(e.p + bi);
                  a1 = rel(e.p + n);
                }
                if (e.bad) { declined = true; break; }
              }
              b0r = rel(c.p);
              if (q - pre > PRE) { declined = true; break; }
            }
            if (lane == 0) {
              for (uint32_t b = 0; b < q - pre; b++) X.pre[ci * PRE + b] = sm[pre + b];
              sec(ci, S_PRELEN) = q - pre;
              sec(ci, S_A0) = a0;
              sec(ci, S_A1) = a1;
              sec(ci, S_B0) = b0r;
              sec(ci, S_FCLOCK) = (uint32_t)(clock + off);
              sec(ci, S_CLIENT) = client;
            }
          }
        } else {
          written++;
          const uint32_t ni = skip ? info : gc ? 0 : ((info & 0xC0) ? info & ~0x20u : info);
          if (ni != info) {
            if (npatch >= NPATCH) { declined = true; break; }
            if (lane == 0) { at<uint32_t>(L_PPOS + 4 * npatch) = rel(s0); sm[L_PVAL + npatch] = (uint8_t)ni; at<uint32_t>(L_PSEC + 4 * npatch) = ci; }
            npatch++;
          }
        }
        clock += len;
      }
      if (declined || c.bad) break;
      if (OP == OP_META && nstructs > 0) {
        if (sv_n >= NSV) { declined = true; break; }
        if (lane == 0) { X.svt[2 * sv_n] = client; X.svt[2 * sv_n + 1] = first_clock; X.sec[sv_n] = (uint32_t)clock; }
        sv_n++;
      }
      if (OP == OP_DIFF) {
        if (lane == 0) {
          sec(ci, S_B1) = copying ? rel(c.p) : 0;
          sec(ci, S_WRITTEN) = written;
          if (!copying) sec(ci, S_PRELEN) = NONE;
        }
        nparts += copying;
      }
    }
    if (declined || c.bad) YB_DECLINE()
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
        for (uint32_t i = 0; i < sv_n; i++) { put(X.svt[2 * i]); put(X.sec[i]); }
        j.out_off[d] = base;
        j.out_len[d] = total;
        j.status[d] = ym::ST_OK;
      }
      __syncthreads();
      continue;
    }
    if (OP == OP_SV) {
      if (sv_any && sv_clock != 0) {
        if (sv_n >= NSV) YB_DECLINE()
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
    // ---- delete set: validated, then copied verbatim (readDeleteSet + writeDeleteSet round trip)
    const uint32_t ds0 = rel(c.p);
    {
      const uint32_t ndc = rvu(c);
      const bool big = ndc > 64 && ndc <= BS_NDSC && !c.bad;
      if (big) cmap::clear(X.map);
      for (uint32_t i = 0; i < ndc && !c.bad && !declined; i++) {
        const uint32_t client = rvu(c);
        const uint32_t m = rvu(c);
        // readDeleteSet drops clients without ranges and merges a repeated client into its first
        // occurrence: either makes the re-written set differ from the input bytes
        if (m == 0 || i >= BS_NDSC) { declined = true; break; }
        if (big ? cmap::seen_insert(X.map, client) : seen_before(X.dsc, i, client)) { declined = true; break; }
        if (lane == 0) X.dsc[i] = client;
        __threadfence_block();
        for (uint32_t q = 0; q < m && !c.bad; q++) {
          rvu(c);
          rvu(c);
        }
      }
    }
    if (declined || c.bad) YB_DECLINE()
    const uint32_t ds1 = rel(c.p);
    __syncthreads();
    // ---- sizes, allocation
    __threadfence_block();
    __syncthreads();
    uint32_t tl = 0;
    for (uint32_t ci = lane; ci < nclients; ci += 64) {
      const uint32_t pl = sec(ci, S_PRELEN);
      if (pl == NONE) continue;
      tl += vsz(sec(ci, S_WRITTEN)) + vsz(sec(ci, S_CLIENT)) + vsz(sec(ci, S_FCLOCK)) + pl +
            (sec(ci, S_A1) - sec(ci, S_A0)) + (sec(ci, S_B1) - sec(ci, S_B0));
    }
    const uint32_t total = vsz(nparts) + (ds1 - ds0) + lane_read(wave_incl_add(tl), 63);
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd((unsigned long long *)j.used, (unsigned long long)total);
    base = ((uint64_t)lane_read((uint32_t)(base >> 32), 0) << 32) | lane_read((uint32_t)base, 0);
    if (base + total > j.cap) {
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      __syncthreads();
      continue;
    }
    // ---- write: small pieces by lane 0, spans by the wave, then the info patches
    uint8_t *const o = j.out + base;
    const uint8_t *const src = j.A + ub;
    auto copy_span = [&](uint32_t dst, uint32_t s0_, uint32_t s1_) { copy_bytes(o + dst, src + s0_, s1_ - s0_); };
    uint32_t p = 0;
    if (lane == 0) {
      uint32_t t = 0;
      uint32_t v = nparts;
      while (v > 127) { o[t++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
      o[t++] = (uint8_t)v;
    }
    p = vsz(nparts);
    for (uint32_t ci = 0; ci < nclients; ci++) {
      const uint32_t pl = sec(ci, S_PRELEN);
      if (pl == NONE) continue;
      const uint32_t written = sec(ci, S_WRITTEN), client = sec(ci, S_CLIENT), fclock = sec(ci, S_FCLOCK);
      if (lane == 0) {  // part header (LazyStructWriter: written, client, first clock) + sliced head
        uint32_t t = p;
        for (uint32_t v : {written, client, fclock}) {
          while (v > 127) { o[t++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
          o[t++] = (uint8_t)v;
        }
        for (uint32_t b = 0; b < pl; b++) o[t + b] = X.pre[ci * PRE + b];
      }
      p += vsz(written) + vsz(client) + vsz(fclock) + pl;
      const uint32_t a0 = sec(ci, S_A0), a1 = sec(ci, S_A1);
      copy_span(p, a0, a1);
      p += a1 - a0;
      const uint32_t b0r = sec(ci, S_B0), b1r = sec(ci, S_B1);
      copy_span(p, b0r, b1r);
      if (lane == 0) sec(ci, S_OUTB) = p - b0r;  // output position = update position + S_OUTB
      p += b1r - b0r;
    }
    copy_span(p, ds0, ds1);
    __threadfence();  // the patches below overwrite bytes other lanes stored
    __syncthreads();
    // patches: each lies in the B span of exactly one section (sections are disjoint, in order)
    for (uint32_t i = lane; i < npatch; i += 64) {
      const uint32_t pos = at<uint32_t>(L_PPOS + 4 * i);
      const uint32_t ci = at<uint32_t>(L_PSEC + 4 * i);
      if (pos >= sec(ci, S_B0) && pos < sec(ci, S_B1)) o[sec(ci, S_OUTB) + pos] = sm[L_PVAL + i];
    }
    if (lane == 0) {
      j.out_off[d] = base;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    __syncthreads();
  }
}

}  // namespace big

// the general path's bump allocator starts at 0; empty work list
__global__ void k_big_init(GeneralJob j) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *j.used = 0;
    *j.pend_count = 0;
  }
}

int big_launch(uint32_t op, const GeneralJob &j0, hipStream_t st, PwBufs &pwb) {
  if (j0.v2 || (op != OP_DIFF && op != OP_SV && op != OP_META)) return 0;
  k_big_init<<<1, 64, 0, st>>>(j0);
  GeneralJob j = j0;
  // large single updates: the chunk-parallel walk first (ym_pwalk.hip); small ones one per lane
  // (ym_small.hip); k_big_v1 takes the rest (it skips what those completed)
  if (int r = pw_prepare(op, j0, st, pwb, &j.pw_done); r < 0) return r;
  // an update log (parseUpdateMeta over > 65,536 single updates, nearly all <= 80 B): the tiny lane-per-update
  // shape alone; the 2 KB shape and k_pw_small would each spend ~0.15-0.28 ms stepping over a million
  // documents to find none of theirs, so the rare larger update goes to k_big_v1
  const bool log = op == OP_META && j0.n > 8 * BS_GRID;
  small_launch(op, j, const_cast<uint8_t *>(j.pw_done), st, log);
  if (!log) pw_small_launch(op, j, const_cast<uint8_t *>(j.pw_done), st);
  if (int r = pw_finish(j0, st, pwb); r < 0) return r;  // (waits for the prep's totals: the kernels above run)
  const uint32_t grid = j.n < BS_GRID ? j.n : BS_GRID;
  if (op == OP_DIFF) big::k_big_v1<OP_DIFF><<<grid, 64, big::LDS_BYTES, st>>>(j);
  else if (op == OP_META) big::k_big_v1<OP_META><<<grid, 64, big::LDS_BYTES, st>>>(j);
  else big::k_big_v1<OP_SV><<<grid, 64, big::LDS_BYTES, st>>>(j);
  return 1;
}

// The asynchronous form (ym_diff_async / ym_sv_async): the same kernels without the chunk-parallel walk
// (it sizes its records on the host) -- small documents one per lane, up to 4 KB one per wave, k_big_v1 the
// rest over a grid of at most grid_max blocks.  done: n zeroed bytes, followed at the next 16-byte boundary
// by 32 zeroed bytes (k_pw_small's tally).
int big_async_launch(uint32_t op, const GeneralJob &j0, uint8_t *done, uint32_t grid_max, hipStream_t st) {
  if (j0.v2 || (op != OP_DIFF && op != OP_SV)) return 0;
  GeneralJob j = j0;
  j.pw_done = done;
  small_launch(op, j, done, st);
  pw_small_launch(op, j, done, st);
  const uint32_t grid = j.n < grid_max ? j.n : grid_max;
  if (op == OP_DIFF) big::k_big_v1<OP_DIFF><<<grid, 64, big::LDS_BYTES, st>>>(j);
  else big::k_big_v1<OP_SV><<<grid, 64, big::LDS_BYTES, st>>>(j);
  return 1;
}

}  // namespace ymk
