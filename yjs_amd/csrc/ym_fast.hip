// ym_fast.hip -- LDS fast path for batched mergeUpdates (V1): one 64-lane wave per document.
//
// Takes documents whose inputs are "simple": every update's client sections increase in (client desc,
// clock asc), no two sections overlap, no GC/Skip structs, canonical encodings, payloads of the kinds
// yjs writes (strings, formats/embeds with literal JSON, scalar `any` values).  For such documents
// yjs 13.5.16's k-way merge (bundle ds@39007) reduces to: the client sections of all
// updates sorted by (client desc, clock asc), a Skip (info 10, 13.5.16 ui.write) before every clock
// gap, consecutive same-client sections grouped into one part (encoding.js:94-116 writeClientsStructs
// layout); the delete set is the per-client union of all inputs' ranges (13.5.16 le@10242: `>=`
// touching rule, max end) with clients in first-appearance order (DeleteSet.js:141-161
// mergeDeleteSets, 13.5.16 he@10482).  Anything else is declined (status ST_PENDING) and handled
// exactly by the general path (ym_general.hip) -- never approximated.
//
// The unit of work is the CLIENT SECTION (the structs of one client inside one update: contiguous
// clocks, contiguous bytes), not the struct: a section is copied to the output as one byte range, so
// sorting, layout and emission scale with the ~1 section per update of real traffic.  Per document,
// all in LDS (~7.9 KB, no scratch), every phase data-parallel across the wave:
//   1. 16-B loads of the document's bytes into LDS (update offsets u64, or u32 with YM_OFF32).
//   2. W1: one lane per update walks its V1 struct section (varints from one unaligned 8-byte LDS read,
//      SWAR ASCII/JSON checks), appends one record per client section via an LDS atomic and clears the
//      parentSub bit of Items with an origin in place (13.5.16 drops it on re-write, E8).  W2: one lane
//      per update with a non-empty delete set appends its ranges.
//   3. rank sort of the section keys (each lane counts the keys <= its own: broadcast reads, no barriers
//      inside), scatter, duplicate check.
//   4. layout by DPP wave scans: Skips at clock gaps, part headers, byte offsets; each lane then writes
//      its sections (part header, Skip, the section's bytes with 8-byte stores) straight into the slot.
//   5. delete set: rank sort of (client, clock), segmented running-max scan = interval union, groups
//      ranked by first appearance, byte offsets by scans, written after the struct section.
// Output slot of doc d: 2 * (input bytes before d) + 64 * d, rounded up to 64 bytes (a bound the kernel
// checks), so the fast path needs no global atomics; the general path appends after that region.
// Documents are mapped to blocks XCD-contiguously (block b runs on XCD b % 8): neighbouring documents
// share their boundary cache lines (input bytes, offsets, per-document results) inside one L2.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ym_fast_common.h"
#include "ym_kernels.h"

namespace ymk {
namespace fastv1 {

constexpr uint32_t UPD = 128;    // max updates per document
constexpr uint32_t E = 2;        // records per lane
constexpr uint32_t SEC = 64 * E; // max client sections per document
constexpr uint32_t DSN = 64 * E; // max delete ranges per document (before the union)
constexpr uint32_t IN_HOT = 2432;     // max document bytes, hot pass (C2 / C4 documents: <= 2.2 KB)
constexpr uint32_t IN_NESTED = 3328;  // ... retry pass over rich content (C2R documents: <= 3.2 KB)

// ---- LDS map (byte offsets; every array 16-aligned) ----------------------------------------------
// IN_ + 2,688 B per one-wave workgroup: 5,120 B for the hot pass = 32 workgroups per CU, 8 waves per SIMD.
// The delete set is walked after the struct section is written, so its ranges reuse the section records'
// region and its merge arrays the (then dead) document bytes; the walk lists are read into registers before
// their walks and live in the record region too.
template <uint32_t IN_>
struct Map {
  static constexpr uint32_t IN = IN_;
  static constexpr uint32_t L_IN = 0;                    // u8[IN + 16]   document bytes (+ slack for 8-B reads)
  static constexpr uint32_t L_UOFF = IN + 16;            // u16[UPD + 1]  update start (absolute LDS offsets)
  static constexpr uint32_t L_MISC = L_UOFF + 272;       // u32[4]        counters: sections, delete ranges
  static constexpr uint32_t L_DUP = L_MISC + 16;         // u32[4]        section ranks seen (duplicate check)
  static constexpr uint32_t L_HIST = L_DUP + 16;         // u32[16]       update-length histogram -> bucket offsets
  static constexpr uint32_t L_UDS = L_HIST + 64;         // u16[UPD]      LDS offset of each update's delete set
  static constexpr uint32_t R = L_UDS + 2 * UPD;         // record region
  // client sections (walk order, then rank order in place)
  static constexpr uint32_t L_SKEY = R;                  // u64[SEC]  (~client << 32 | clock)
  static constexpr uint32_t L_SLN = L_SKEY + 8 * SEC;    // u32[SEC]  clock length (21 bits) | structs << 21
  static constexpr uint32_t L_SB = L_SLN + 4 * SEC;      // u16[SEC]  LDS offset of its first struct
  static constexpr uint32_t L_SE = L_SB + 2 * SEC;       // u16[SEC]  ... and of its end
  static constexpr uint32_t L_END = L_SE + 2 * SEC;
  static constexpr uint32_t L_UORD = L_SE;               // u8[UPD]   struct walk list (updates with structs, by
                                                         //           length), in registers before the walk
  static constexpr uint32_t L_UORD2 = L_SE;              // u8[UPD]   delete-set walk list (after the section phase)
  // the layout holds the rank-ordered records in registers: parts over the clock lengths
  static constexpr uint32_t L_PFIRST = L_SLN;            // u16[SEC]  part -> units before it
  static constexpr uint32_t L_PLAST = L_SLN + 2 * SEC;   // u16[SEC]  part -> units through it
  // after the struct section is written: delete ranges over the section records
  static constexpr uint32_t L_DKEY = R;                  // u64[DSN]  (client << 32 | clock << 7 | slot)
  static constexpr uint32_t L_DLEN = L_DKEY + 8 * DSN;   // u32[DSN]
  static constexpr uint32_t L_DSEQ = L_DLEN + 4 * DSN;   // u16[DSN]  update << 8 | position (first appearance)
  // ... merged ranges and groups over the document bytes and the walk tables (dead once the delete sets are
  // walked)
  static constexpr uint32_t L_QCLK = L_IN;               // u32[DSN]  merged range start
  static constexpr uint32_t L_QEND = L_QCLK + 4 * DSN;   // u32[DSN]  merged range end
  static constexpr uint32_t L_QGRP = L_QEND + 4 * DSN;   // u8[DSN]   merged range -> group
  static constexpr uint32_t L_QPRE = L_QGRP + DSN;       // u16[DSN + 1] exclusive byte prefix over ranges
  static constexpr uint32_t L_GFIRST = L_QPRE + 272;     // u16[DSN + 1] group -> first range
  static constexpr uint32_t L_GCLI = L_GFIRST + 272;     // u32[DSN]  group client
  static constexpr uint32_t L_GMIN = L_GCLI + 4 * DSN;   // u32[DSN]  group first appearance, then group base
  static constexpr uint32_t L_GBYR = L_DKEY;             // u16[DSN]  bytes by rank, then offsets by rank (sorted keys
                                                         //           are dead)
  static constexpr uint32_t L_GB2 = L_DKEY + 512;        // u32[DSN]  group -> base offset of its ranges
  static constexpr uint32_t LDS_BYTES = L_END;
  static_assert(IN % 16 == 0, "16-B staging");
  static_assert(L_GMIN + 4 * DSN <= R, "phase-5 arrays fit below the record region");
  static_assert(L_DSEQ + 2 * DSN <= L_END, "delete ranges fit in the section region");
  static_assert(L_GB2 + 4 * DSN <= L_DSEQ + 2 * DSN && L_GB2 >= L_GBYR + 2 * DSN, "rank arrays fit over the sorted keys");
  static_assert(L_PLAST + 2 * SEC <= L_SB, "part arrays fit over the clock lengths");
  static_assert(L_UORD + UPD <= L_END, "walk lists fit in the record region");
};
using MapHot = Map<IN_HOT>;
using MapNested = Map<IN_NESTED>;
static_assert(MapHot::LDS_BYTES * 32 <= 160 * 1024, "8 one-wave workgroups per SIMD (160 KB LDS per CU)");

using namespace fastc;

// update offset i of the batch (u64, or u32 with YM_OFF32)
__device__ __forceinline__ uint64_t uoff_g(const GeneralJob &j, uint64_t i) {
  return j.upd_off32 ? (uint64_t)j.upd_off32[i] : j.upd_off[i];
}
__device__ __forceinline__ void put_u64(Slot o, uint32_t p, uint64_t v) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 w = {(unsigned int)v, (unsigned int)(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(w, o, (int)p, 0, 0);
}

// ---- short-cut Item parser (the shapes yjs writes for text, formats and map values) --------------------
// Each helper is branch-free: a wave whose lanes sit at different Items runs one straight copy of each
// instead of item_body's per-kind regions.  Any shape or check the short-cut does not decide clears `ok`;
// the caller then re-parses that Item with item_body (same checks, so both agree on every Item they take).
// An ID (client, clock): two canonical varuints < 2^32 inside one 8-byte window (ID_SKIP of skvu2)
__device__ __forceinline__ void fast_id(uint32_t &p, bool &ok) {
  const uint64_t x = ld8(p);
  const uint64_t st = ~x & 0x8080808080808080ull, st2 = st & (st - 1);
  const uint32_t i1 = ctz64(st) >> 3, i2r = ctz64(st2) >> 3, i2 = i2r < 7 ? i2r : 7;
  const uint32_t b1 = (uint32_t)(x >> (8 * (i1 < 7 ? i1 : 7))) & 0xffu, b2 = (uint32_t)(x >> (8 * i2)) & 0xffu;
  const uint32_t n1 = i1 + 1, n2 = i2r - i1;
  ok &= (st2 != 0) & (n1 <= 5) & (n2 <= 5) & !((n1 > 1) & (b1 == 0)) & !((n2 > 1) & (b2 == 0)) &
        !((n1 == 5) & ((b1 & 0x70u) != 0)) & !((n2 == 5) & ((b2 & 0x70u) != 0));
  p += i2 + 1;
}
// a varString of at most 7 ASCII bytes with a one-byte length: its length (= UTF-16 length)
__device__ __forceinline__ uint32_t fast_str(uint32_t &p, bool &ok) {
  const uint64_t x = ld8(p);
  const uint32_t n = (uint32_t)x & 0xffu, nn = n < 7 ? n : 7;
  const uint64_t body = (x >> 8) & ((1ull << (8 * nn)) - 1);
  ok &= (n <= 7) & ((body & 0x8080808080808080ull) == 0);
  p += 1 + nn;
  return nn;
}
// UTF-16 length of the strict UTF-8 in the low n (1..7) bytes of w, or ~0 (out of line: inlined, its registers
// spill in the hot kernel)
__device__ __attribute__((noinline)) uint32_t utf8_short(uint64_t w, uint32_t n) {
  utf8::State s;
  utf8::word<uint32_t>(s, (uint32_t)w, n < 4 ? n : 4);
  if (n > 4) utf8::word<uint32_t>(s, (uint32_t)(w >> 32), n - 4);
  return s.bad || s.owe != 0 ? 0xffffffffu : s.units;
}
// ContentString: a varString of at most 7 bytes with a one-byte length, any strict UTF-8 (CJK / emoji / accented
// text, checked by ym_utf8.h on the window's two halves): its UTF-16 length
__device__ __forceinline__ uint32_t fast_ustr(uint32_t &p, bool &ok) {
  const uint64_t x = ld8(p);
  const uint32_t n = (uint32_t)x & 0xffu, nn = n < 7 ? n : 7;
  const uint64_t body = (x >> 8) & ((1ull << (8 * nn)) - 1);
  uint32_t units = nn;
  ok &= n <= 7;
  if (body & 0x8080808080808080ull) {
    units = utf8_short(body, nn);
    ok &= units != 0xffffffffu;
  }
  p += 1 + nn;
  return units;
}
// JSON text of a format / embed: "true", "null" or "false"
__device__ __forceinline__ void fast_json(uint32_t &p, bool &ok) {
  const uint64_t x = ld8(p);
  const uint32_t n = (uint32_t)x & 0xffu;
  const uint32_t w4 = (uint32_t)(x >> 8);
  const uint64_t w5 = (x >> 8) & 0xffffffffffull;
  ok &= ((n == 4) & ((w4 == 0x65757274u) | (w4 == 0x6c6c756eu))) | ((n == 5) & (w5 == 0x65736c6166ull));
  p += 1 + (n < 5 ? n : 5);
}
// one `any` value: undefined / null / booleans, a varInt (canonical, int32 range), a short ASCII string
__device__ __forceinline__ void fast_any(uint32_t &p, bool &ok) {
  const uint64_t x = ld8(p);
  const uint32_t tag = (uint32_t)x & 0xffu;
  const uint32_t lit = (tag == 127) | (tag == 126) | (tag == 121) | (tag == 120);
  // varInt: sign in bit 6 of the first byte, 6 + 7k value bits, minimal, magnitude <= 2^31 - 1 when positive
  const uint64_t v = x >> 8;
  const uint64_t st = ~v & 0x8080808080808080ull;
  const uint32_t i = ctz64(st) >> 3, ni = i < 4 ? i : 4;  // last byte index (<= 4: 34 bits)
  const uint32_t lo = (uint32_t)v;
  const uint64_t mag = (uint64_t)(lo & 0x3fu) | ((uint64_t)((lo >> 8) & 0x7fu) << 6) | ((uint64_t)((lo >> 16) & 0x7fu) << 13) |
                       ((uint64_t)((lo >> 24) & 0x7fu) << 20) | ((uint64_t)((uint32_t)(v >> 32) & 0x7fu) << 27);
  const uint64_t magm = mag & ((1ull << (6 + 7 * ni)) - 1);
  const uint32_t lastb = (uint32_t)(v >> (8 * ni)) & 0xffu;
  const bool neg = (lo & 0x40u) != 0;
  const bool vint = (tag == 125) & (i <= 4) & !((ni > 0) & (lastb == 0)) & (neg | (magm <= 2147483647ull)) &
                    (magm <= 0xffffffffull);
  uint32_t q = p + 1;
  const bool str = tag == 119;
  bool sok = true;
  fast_str(q, sok);
  ok &= lit | vint | (str & sok);
  p = str ? q : p + 1 + (tag == 125 ? ni + 1 : 0);
}
// value of the canonical varuint at the start of window w, nb bytes (1..5)
__device__ __forceinline__ uint32_t vu_value(uint64_t w, uint32_t nb) {
  const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
  const uint32_t v = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u) | (hi << 28);
  return nb >= 5 ? v : v & ((1u << (7 * nb)) - 1);
}
// the Item after its info byte at c.p; false: not a short-cut shape (c untouched)
__device__ __forceinline__ bool item_fast(Cur &c, uint32_t info, uint32_t &len) {
  uint32_t p = c.p;
  bool ok = true;
  const uint32_t kind = info & 31;
  if (info & 0x80) fast_id(p, ok);
  if (info & 0x40) fast_id(p, ok);
  if ((info & 0xC0) == 0) {  // parentInfo 1: the root type's key, then the parentSub
    ok &= sm[p] == 1;
    p++;
    fast_str(p, ok);
    if (info & 0x20) fast_str(p, ok);
  }
  len = 1;
  if (kind == 4) {
    len = fast_ustr(p, ok);
    ok &= len != 0;
  } else if (kind == 6) {
    fast_str(p, ok);
    fast_json(p, ok);
  } else if (kind == 8) {
    ok &= sm[p] == 1;  // one value
    p++;
    fast_any(p, ok);
  } else {
    ok = false;
  }
  ok &= p <= c.e;
  if (ok) c.p = p;
  return ok;
}

// Walks the struct section of update u and appends one record per client section (slot from an LDS
// atomic counter, misc[0]); records where its delete set starts.  Item info bytes with an origin and
// the parentSub bit get the bit cleared in place (13.5.16's lazy reader reads parentSub only without
// origins and writes the info byte back without it, E8), so sections copy verbatim afterwards.
// Returns false to decline.  NESTED: nested payloads (any objects / arrays, JSON texts) are checked too
// (the retry pass over the documents the hot kernel declined; ym_canon_chk.h).
template <class M, bool NESTED = false>
__device__ __forceinline__ bool walk_sections(uint32_t u) {
  Cur c = {at<uint16_t>(M::L_UOFF + 2 * u), at<uint16_t>(M::L_UOFF + 2 * u + 2), false};
  const uint32_t nclients = rvu(c);
  uint64_t next_min = 0;  // sections of one update in merge order: each key > the previous one's last unit
  for (uint32_t ci = 0; ci < nclients && !c.bad; ci++) {
    const uint32_t nstructs = rvu(c);
    const uint32_t client = rvu(c);
    const uint32_t clock = rvu(c);
    const uint32_t b = c.p;
    uint64_t len = 0;
    for (uint32_t si = 0; si < nstructs && !c.bad; si++) {
      // declines set c.bad (one exit edge per loop instead of one per check)
      const uint32_t s0 = c.p;
      const uint32_t info = rdb(c);
      c.bad |= info == 10 || (info & 31) == 0;  // Skip / GC -> general path
      uint32_t l = 1;
      if (!c.bad && !item_fast(c, info, l)) c.bad |= !item_body<NESTED, M::L_HIST, M::L_MISC + 8>(c, info, l);
      if ((info & 0xC0) != 0 && (info & 0x20) != 0) sm[s0] = (uint8_t)(info & ~0x20u);
      len += l;
    }
    const uint64_t key = ((uint64_t)(~client) << 32) | clock;
    c.bad |= (nstructs == 0) | (nstructs >= (1u << 11)) | (len >= (1u << 21)) | (key < next_min);
    next_min = key + len;
    if (!c.bad) {
      const uint32_t q = atomicAdd(&at<uint32_t>(M::L_MISC), 1u);
      c.bad |= q >= SEC;
      if (q < SEC) {
        at<uint64_t>(M::L_SKEY + 8 * q) = key;
        at<uint32_t>(M::L_SLN + 4 * q) = (uint32_t)len | (nstructs << 21);
        at<uint16_t>(M::L_SB + 2 * q) = (uint16_t)b;
        at<uint16_t>(M::L_SE + 2 * q) = (uint16_t)c.p;
      }
    }
  }
  at<uint16_t>(M::L_UDS + 2 * u) = (uint16_t)c.p;
  return !c.bad;
}
// Walks the delete set of update u (DeleteSet.js:219-256) and appends its ranges (slots from misc[1]);
// a range's payload (u << 8 | position) keeps yjs's first-appearance order.
// V2: DSDecoderV2 (UpdateDecoder.js:258-267): clock delta-coded against the running value, which each
// client resets; length stored as len - 1.
template <class M, bool V2 = false>
__device__ __forceinline__ bool walk_ds(uint32_t u) {
  Cur c = {at<uint16_t>(M::L_UDS + 2 * u), at<uint16_t>(M::L_UOFF + 2 * u + 2), false};
  const uint32_t ndc = rvu(c);
  uint32_t pos = 0;
  for (uint32_t i = 0; i < ndc && !c.bad; i++) {
    const uint32_t client = rvu(c);
    const uint32_t m = rvu(c);
    uint64_t cur = 0;
    for (uint32_t q = 0; q < m && !c.bad; q++, pos++) {
      uint32_t clock, len;
      if constexpr (V2) {
        const uint64_t c64 = cur + rvu(c);
        const uint64_t l64 = (uint64_t)rvu(c) + 1;
        cur = c64 + l64;
        c.bad |= (c64 >= (1u << 25)) | (l64 > 0xffffffffull);
        clock = (uint32_t)c64;
        len = (uint32_t)l64;
      } else {
        clock = rvu(c);
        len = rvu(c);
      }
      c.bad |= (pos > 255) | (clock >= (1u << 25));
      if (!c.bad) {
        const uint32_t x = atomicAdd(&at<uint32_t>(M::L_MISC + 4), 1u);
        c.bad |= x >= DSN;
        // the slot in the low bits makes every key distinct (ranks are a permutation without a
        // tie-break pass: equal (client, clock) ranges from several inputs are the common case)
        if (x < DSN) {
          at<uint64_t>(M::L_DKEY + 8 * x) = ((uint64_t)client << 32) | (clock << 7) | x;
          at<uint32_t>(M::L_DLEN + 4 * x) = len;
          at<uint16_t>(M::L_DSEQ + 2 * x) = (uint16_t)((u << 8) | pos);
        }
      }
    }
  }
  return !c.bad;
}

#ifdef YM_FAST_TIMELINE
__device__ unsigned g_fast_ph[131072][8];  // per block: s_memrealtime (low 32 bits) after each phase
#define YM_TS(i) \
  if (threadIdx.x == 0 && blockIdx.x < 131072) g_fast_ph[blockIdx.x][i] = (unsigned)__builtin_amdgcn_s_memrealtime();
#else
#define YM_TS(i)
#endif
#define YM_DECLINE()                                 \
  {                                                  \
    if (lane == 0) decline(j, d);                    \
    __syncthreads();                                 \
    return;                                          \
  }
// STOP > 0 builds a timing-only variant that ends every document after phase STOP (profiling the
// phases by ablation); outputs of such builds are not meaningful.
#define YM_STOP(n)                                                      \
  if (STOP == (n)) {                                                    \
    if (lane == 0) { j.status[d] = ym::ST_OK; j.out_len[d] = 0; }       \
    __syncthreads();                                                    \
    return;                                                             \
  }

// ---- 3/4. client sections of document d: rank sort, layout, struct section written (EE per lane) -------
enum : int { SP_DONE = 0, SP_DECLINE = 1, SP_STOP = 2, SP_CAP = 3 };
template <class M, uint32_t EE, int STOP>
__device__ __forceinline__ int sec_phase(const GeneralJob &j, uint32_t d, uint32_t nsec, uint64_t slot, uint64_t slot_al,
                                         uint64_t slot_end, uint64_t bytes, Slot dst, uint32_t &hdr, uint32_t &struct_bytes) {
  const uint32_t lane = threadIdx.x;
  bool bad = false;
    // ---- 3. section rank sort
    uint64_t rk[EE];
    uint32_t rl[EE], rb[EE], re[EE], rr[EE];
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      const uint32_t i = lane + 64 * s;
      const bool v = i < nsec;
      rk[s] = v ? at<uint64_t>(M::L_SKEY + 8 * i) : ~0ull;
      rl[s] = v ? at<uint32_t>(M::L_SLN + 4 * i) : 0;
      rb[s] = v ? at<uint16_t>(M::L_SB + 2 * i) : 0;
      re[s] = v ? at<uint16_t>(M::L_SE + 2 * i) : 0;
    }
    bool ranked = false;
    if constexpr (EE == 1) {
      // One section per lane: rank by client groups.  A group (one client) is picked per iteration by
      // its lowest lane; its lanes take their position within the group in lane (= walk = update) order
      // and every lane of a larger key (smaller client) adds the group's size.  Valid when each group is
      // clock-sorted in walk order (the updates of one client arrive in clock order: the common case),
      // checked against the previous lane of the group; otherwise, or beyond 16 clients, rank_le4.
      const uint64_t lt = (1ull << lane) - 1;
      const bool v = lane < nsec;
      const uint32_t hi = (uint32_t)(rk[0] >> 32), lo = (uint32_t)rk[0];
      uint64_t rem = __ballot(v), grp = 0;
      uint32_t base = 0, pos = 0;
      for (uint32_t g = 0; rem != 0 && g < 16; g++) {
        const uint32_t f = (uint32_t)__builtin_ctzll(rem);
        const uint32_t h = lane_read(hi, (int)f);
        const bool in = v && hi == h;
        const uint64_t m = __ballot(in);
        if (in) { pos = (uint32_t)__popcll(m & lt); grp = m; }
        base += (v && hi > h) ? (uint32_t)__popcll(m) : 0u;
        rem &= ~m;
      }
      if (rem == 0) {
        const uint64_t pm = grp & lt;
        const int prev = pm ? 63 - __builtin_clzll(pm) : (int)lane;
        const uint32_t plo = (uint32_t)__shfl((int)lo, prev, 64);
        if (__all(!v || pm == 0 || plo < lo)) {
          rr[0] = base + pos;
          ranked = true;
        }
      }
    }
    if (!ranked) rank_le4(M::L_SKEY, nsec, rk, rr);
    __syncthreads();
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      const uint32_t i = lane + 64 * s;
      if (i < nsec) {
        const uint32_t r = rr[s];
        at<uint64_t>(M::L_SKEY + 8 * r) = rk[s];
        at<uint32_t>(M::L_SLN + 4 * r) = rl[s];
        at<uint16_t>(M::L_SB + 2 * r) = (uint16_t)rb[s];
        at<uint16_t>(M::L_SE + 2 * r) = (uint16_t)re[s];
        atomicOr(&at<uint32_t>(M::L_DUP + 4 * (r >> 5)), 1u << (r & 31));
      }
    }
    __syncthreads();
    {
      // equal (client, clock) keys share a rank: the ranks seen must be all nsec of them (else overlapping
      // inputs)
      const uint4 w = at<uint4>(M::L_DUP);
      const uint32_t seen = __popc(__builtin_amdgcn_readfirstlane(w.x)) + __popc(__builtin_amdgcn_readfirstlane(w.y)) +
                            __popc(__builtin_amdgcn_readfirstlane(w.z)) + __popc(__builtin_amdgcn_readfirstlane(w.w));
      if (seen != nsec) return SP_DECLINE;
    }
    YM_TS(2)
    if (STOP == 3) return SP_STOP;
    // ---- 4. layout over rank order; lane owns positions r = E*lane + s
    uint64_t sk[EE];
    uint32_t sl[EE], sns[EE], sb[EE], se[EE], units[EE], pstart[EE], plastf[EE], gapv[EE];
    {
      const uint32_t r0 = EE * lane;
      uint64_t kp = r0 > 0 && r0 - 1 < nsec ? at<uint64_t>(M::L_SKEY + 8 * (r0 - 1)) : ~0ull;
      uint32_t lp = r0 > 0 && r0 - 1 < nsec ? at<uint32_t>(M::L_SLN + 4 * (r0 - 1)) & 0x1fffffu : 0;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t r = r0 + s;
        const bool v = r < nsec;
        sk[s] = v ? at<uint64_t>(M::L_SKEY + 8 * r) : ~0ull;
        const uint32_t ln = v ? at<uint32_t>(M::L_SLN + 4 * r) : 0;
        sl[s] = ln & 0x1fffffu;
        sns[s] = ln >> 21;
        sb[s] = v ? at<uint16_t>(M::L_SB + 2 * r) : 0;
        se[s] = v ? at<uint16_t>(M::L_SE + 2 * r) : 0;
        const uint64_t kn = r + 1 < nsec ? at<uint64_t>(M::L_SKEY + 8 * (r + 1)) : ~0ull;
        const bool same = v && r > 0 && (kp >> 32) == (sk[s] >> 32);
        const uint64_t pend = (kp & 0xffffffffull) + lp;
        const uint64_t cl = sk[s] & 0xffffffffull;
        bad |= same && pend > cl;  // overlapping inputs: general path
        gapv[s] = same && pend < cl ? (uint32_t)(cl - pend) : 0;
        units[s] = v ? sns[s] + (gapv[s] != 0) : 0;
        pstart[s] = v && !same;
        plastf[s] = v && (r + 1 >= nsec || (kn >> 32) != (sk[s] >> 32));
        kp = sk[s];
        lp = sl[s];
      }
    }
    if (__any(bad)) return SP_DECLINE;
    // one scan for (parts << 16 | units)
    uint32_t pu[EE], pu_lane = 0, nparts;
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) pu_lane += (pstart[s] << 16) | units[s];
    {
      const uint32_t incl = wave_incl_add(pu_lane);
      nparts = lane_read(incl, 63) >> 16;
      uint32_t run = incl - pu_lane;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        pu[s] = run;  // exclusive (parts, units) before position r
        run += (pstart[s] << 16) | units[s];
        const uint32_t pid = (run >> 16) - 1;
        if (pstart[s]) at<uint16_t>(M::L_PFIRST + 2 * pid) = (uint16_t)(pu[s] & 0xffff);
        if (plastf[s]) at<uint16_t>(M::L_PLAST + 2 * pid) = (uint16_t)(run & 0xffff);
      }
    }
    __syncthreads();
    uint32_t runu[EE], soff[EE], sbytes_lane = 0;
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      runu[s] = 0;
      uint32_t b = se[s] - sb[s];
      if (pstart[s]) {
        const uint32_t pid = pu[s] >> 16;
        runu[s] = at<uint16_t>(M::L_PLAST + 2 * pid) - at<uint16_t>(M::L_PFIRST + 2 * pid);
        b += vsz(runu[s]) + vsz(~(uint32_t)(sk[s] >> 32)) + vsz((uint32_t)sk[s]);
      }
      if (gapv[s]) b += 1 + vsz(gapv[s]);
      soff[s] = b;
      sbytes_lane += b;
    }
    {
      const uint32_t incl = wave_incl_add(sbytes_lane);
      struct_bytes = lane_read(incl, 63);
      uint32_t run = incl - sbytes_lane;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) { const uint32_t b = soff[s]; soff[s] = run; run += b; }
    }
    hdr = vsz(nparts);
    if (slot_al + hdr + struct_bytes > slot_end) {
      if (slot_al + hdr + struct_bytes > slot + 2 * bytes + 64) return SP_DECLINE;
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }  // caller's arena too small
      return SP_CAP;
    }
    YM_TS(3)
    if (STOP == 4) return SP_STOP;
    // ---- 4b. write the struct section: per section its part header, its Skip, then its bytes verbatim
    if (lane == 0) put_vu(dst, 0, nparts);
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      if (EE * lane + s >= nsec) break;
      uint32_t p = hdr + soff[s];
      if (pstart[s]) {  // part header: vu(#structs incl. skips) vu(client) vu(clock)
        p = put_vu(dst, p, runu[s]);
        p = put_vu(dst, p, ~(uint32_t)(sk[s] >> 32));
        p = put_vu(dst, p, sk[s] & 0xffffffffull);
      }
      if (gapv[s]) {  // Skip: info 10 + varuint length (13.5.16 ui.write)
        ob8(dst, p++, 10);
        p = put_vu(dst, p, gapv[s]);
      }
      const uint32_t n = se[s] - sb[s], src = sb[s];
      uint32_t o = 0;
      for (; o + 8 <= n; o += 8) put_u64(dst, p + o, ld8(src + o));
      if (o + 4 <= n) { ob32(dst, p + o, ld4(src + o)); o += 4; }
      for (; o < n; o++) ob8(dst, p + o, sm[src + o]);
    }
  return SP_DONE;
}

// ---- 5/6. delete set of document d (EE delete ranges per lane: 1 when they fit one wave) --------------
enum : int { DS_DONE = 0, DS_DECLINE = 1, DS_STOP = 2 };
template <class M, uint32_t EE, int STOP, bool DSV2>
__device__ __forceinline__ int ds_phase(const GeneralJob &j, uint32_t d, uint32_t nds, uint32_t hdr, uint32_t struct_bytes,
                                        uint64_t slot, uint64_t slot_al, uint64_t slot_end, uint64_t bytes, Slot dst) {
  const uint32_t lane = threadIdx.x;
  bool bad = false;
    // ---- 5. delete set
    {
      uint64_t dk[EE];
      uint32_t dl[EE], dq[EE], dr[EE];
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t i = lane + 64 * s;
        const bool v = i < nds;
        dk[s] = v ? at<uint64_t>(M::L_DKEY + 8 * i) : ~0ull;
        dl[s] = v ? at<uint32_t>(M::L_DLEN + 4 * i) : 0;
        dq[s] = v ? at<uint16_t>(M::L_DSEQ + 2 * i) : 0;
      }
      rank_le4(M::L_DKEY, nds, dk, dr);  // distinct keys: a permutation
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        if (lane + 64 * s < nds) {
          const uint32_t r = dr[s];
          at<uint64_t>(M::L_DKEY + 8 * r) = dk[s];
          at<uint32_t>(M::L_DLEN + 4 * r) = dl[s];
          at<uint16_t>(M::L_DSEQ + 2 * r) = (uint16_t)dq[s];
        }
      }
      __syncthreads();
    }
    // sorted positions r = E*lane + s: client segments (= groups), running max end of the union,
    // merged ranges.  Per position only its key, end, segment flag and id stay in registers.
    uint32_t ngroups, nranges;
    {
      uint32_t ecl[EE], ecli[EE], segst[EE], segid[EE], eseq[EE];
      uint64_t eend[EE];
      uint32_t seg_lane = 0;
      const uint32_t r0 = EE * lane;
      uint32_t cprev = r0 > 0 && r0 - 1 < nds ? (uint32_t)(at<uint64_t>(M::L_DKEY + 8 * (r0 - 1)) >> 32) : 0;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t r = r0 + s;
        const bool v = r < nds;
        const uint64_t k = v ? at<uint64_t>(M::L_DKEY + 8 * r) : 0;
        ecl[s] = (uint32_t)k >> 7;
        ecli[s] = (uint32_t)(k >> 32);
        eend[s] = v ? (uint64_t)ecl[s] + at<uint32_t>(M::L_DLEN + 4 * r) : 0;
        eseq[s] = v ? at<uint16_t>(M::L_DSEQ + 2 * r) : 0xffff;
        segst[s] = v && (r == 0 || cprev != ecli[s]);
        seg_lane += segst[s];
        cprev = ecli[s];
      }
      {
        const uint32_t incl = wave_incl_add(seg_lane);
        ngroups = lane_read(incl, 63);
        uint32_t run = incl - seg_lane;
#pragma unroll
        for (uint32_t s = 0; s < EE; s++) { run += segst[s]; segid[s] = run - 1; }
      }
      // running max of (segment << 33 | end): within a segment it is the max end so far
      uint64_t m = 0, rmax[EE];
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint64_t x = r0 + s < nds ? ((uint64_t)segid[s] << 33) | eend[s] : 0;
        m = x > m ? x : m;
        rmax[s] = m;
      }
      const uint64_t incl = wave_incl_max64(m);
      uint64_t ex = ((uint64_t)from_prev_lane((uint32_t)(incl >> 32)) << 32) | from_prev_lane((uint32_t)incl);
      uint32_t newr[EE], nr_lane = 0;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint64_t before = ex;  // running max through position r - 1
        rmax[s] = rmax[s] > ex ? rmax[s] : ex;
        ex = rmax[s];
        newr[s] = r0 + s < nds && (segst[s] || ecl[s] > (before & 0x1ffffffffull));
        nr_lane += newr[s];
      }
      const uint32_t incl_r = wave_incl_add(nr_lane);
      nranges = lane_read(incl_r, 63);
      uint32_t run = incl_r - nr_lane;
      const uint32_t next_first = from_next_lane(newr[0]);  // newr of position E*(lane+1)
      __syncthreads();  // the sorted delete ranges are in registers (the phase-5 arrays overlay the document bytes)
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t r = r0 + s;
        if (r >= nds) break;
        run += newr[s];
        const uint32_t rid = run - 1;
        if (newr[s]) {
          at<uint32_t>(M::L_QCLK + 4 * rid) = ecl[s];
          at<uint8_t>(M::L_QGRP + rid) = (uint8_t)segid[s];
        }
        const bool nxt_new = s + 1 < EE ? newr[s + 1] != 0 : next_first != 0;
        if (r + 1 >= nds || nxt_new) {
          const uint64_t en = rmax[s] & 0x1ffffffffull;
          bad |= en > 0xffffffffull;
          at<uint32_t>(M::L_QEND + 4 * rid) = (uint32_t)en;
        }
        if (segst[s]) {
          at<uint16_t>(M::L_GFIRST + 2 * segid[s]) = (uint16_t)rid;
          at<uint32_t>(M::L_GCLI + 4 * segid[s]) = ecli[s];
          at<uint32_t>(M::L_GMIN + 4 * segid[s]) = 0xffffffffu;
        }
      }
      if (lane == 0) at<uint16_t>(M::L_GFIRST + 2 * ngroups) = (uint16_t)nranges;
      if (__any(bad)) return DS_DECLINE;
      __syncthreads();
      // first appearance of each client: min over its entries' (update << 8 | position)
#pragma unroll
      for (uint32_t s = 0; s < EE; s++)
        if (r0 + s < nds) atomicMin(&at<uint32_t>(M::L_GMIN + 4 * segid[s]), eseq[s]);
    }
    // merged ranges q = E*lane + s: exclusive byte prefix over range ids
    {
      uint32_t qb[EE], t = 0;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t q = EE * lane + s;
        const uint32_t c0 = q < nranges ? at<uint32_t>(M::L_QCLK + 4 * q) : 0;
        if constexpr (DSV2) {
          const bool first = q < nranges && at<uint16_t>(M::L_GFIRST + 2 * at<uint8_t>(M::L_QGRP + q)) == q;
          const uint32_t pe = q < nranges && !first ? at<uint32_t>(M::L_QEND + 4 * (q - 1)) : 0;
          qb[s] = q < nranges ? vsz(c0 - pe) + vsz(at<uint32_t>(M::L_QEND + 4 * q) - c0 - 1) : 0;
        } else {
          qb[s] = q < nranges ? vsz(c0) + vsz(at<uint32_t>(M::L_QEND + 4 * q) - c0) : 0;
        }
        t += qb[s];
      }
      const uint32_t incl = wave_incl_add(t);
      uint32_t run = incl - t;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t q = EE * lane + s;
        if (q < nranges) at<uint16_t>(M::L_QPRE + 2 * q) = (uint16_t)run;
        run += qb[s];
      }
      if (lane == 63) at<uint16_t>(M::L_QPRE + 2 * nranges) = (uint16_t)incl;
    }
    __syncthreads();
    // groups g = lane + 64 s: bytes and rank by first appearance
    uint32_t grk[EE], gbytes[EE];
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      const uint32_t g = lane + 64 * s;
      const bool v = g < ngroups;
      const uint32_t f0 = v ? at<uint16_t>(M::L_GFIRST + 2 * g) : 0, f1 = v ? at<uint16_t>(M::L_GFIRST + 2 * g + 2) : 0;
      gbytes[s] = v ? vsz(at<uint32_t>(M::L_GCLI + 4 * g)) + vsz(f1 - f0) + at<uint16_t>(M::L_QPRE + 2 * f1) -
                          at<uint16_t>(M::L_QPRE + 2 * f0)
                    : 0;
      const uint32_t mine = v ? at<uint32_t>(M::L_GMIN + 4 * g) : 0;
      uint32_t rk_ = 0;
      for (uint32_t h = 0; h < ngroups; h++) rk_ += at<uint32_t>(M::L_GMIN + 4 * h) < mine;
      grk[s] = rk_;
    }
#pragma unroll
    for (uint32_t s = 0; s < EE; s++)
      if (lane + 64 * s < ngroups) at<uint16_t>(M::L_GBYR + 2 * grk[s]) = (uint16_t)gbytes[s];
    __syncthreads();
    const uint32_t ds_hdr = vsz(ngroups);
    const uint32_t dsb = hdr + struct_bytes;
    uint32_t ds_groups_bytes;
    {  // exclusive prefix over ranks (ranks E*lane + s)
      uint32_t v[EE], t = 0;
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) { const uint32_t r = EE * lane + s; v[s] = r < ngroups ? at<uint16_t>(M::L_GBYR + 2 * r) : 0; t += v[s]; }
      const uint32_t incl = wave_incl_add(t);
      ds_groups_bytes = lane_read(incl, 63);
      uint32_t run = incl - t;
      __syncthreads();
#pragma unroll
      for (uint32_t s = 0; s < EE; s++) {
        const uint32_t r = EE * lane + s;
        if (r < ngroups) at<uint16_t>(M::L_GBYR + 2 * r) = (uint16_t)run;
        run += v[s];
      }
    }
    __syncthreads();
    // group g's output offset; its ranges' base = offset + header - prefix of its first range
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      const uint32_t g = lane + 64 * s;
      if (g < ngroups) {
        const uint32_t f0 = at<uint16_t>(M::L_GFIRST + 2 * g), f1 = at<uint16_t>(M::L_GFIRST + 2 * g + 2);
        const uint32_t off = dsb + ds_hdr + at<uint16_t>(M::L_GBYR + 2 * grk[s]);
        at<uint32_t>(M::L_GMIN + 4 * g) = off;  // first appearance is no longer needed
        at<uint32_t>(M::L_GB2 + 4 * g) = off + vsz(at<uint32_t>(M::L_GCLI + 4 * g)) + vsz(f1 - f0) - at<uint16_t>(M::L_QPRE + 2 * f0);
      }
    }
    __syncthreads();
    const uint32_t total = dsb + ds_hdr + ds_groups_bytes;
    if (slot_al + total > slot_end) {
      if (slot_al + total > slot + 2 * bytes + 64) return DS_DECLINE;
      if (lane == 0) { j.status[d] = ym::ST_CAPACITY; j.out_len[d] = 0; }
      return DS_DONE;
    }
    YM_TS(6)
    if (STOP == 5) return DS_STOP;
    // ---- 6. write the delete set: vu(#clients) | per client (first-appearance order): client, count, ranges
    if (lane == 0) put_vu(dst, dsb, ngroups);
#pragma unroll
    for (uint32_t s = 0; s < EE; s++) {
      const uint32_t g = lane + 64 * s;
      if (g < ngroups)
        put_vu(dst, put_vu(dst, at<uint32_t>(M::L_GMIN + 4 * g), at<uint32_t>(M::L_GCLI + 4 * g)),
               at<uint16_t>(M::L_GFIRST + 2 * g + 2) - at<uint16_t>(M::L_GFIRST + 2 * g));
      const uint32_t q = EE * lane + s;
      if (q < nranges) {
        const uint32_t c0 = at<uint32_t>(M::L_QCLK + 4 * q);
        const uint32_t off = at<uint32_t>(M::L_GB2 + 4 * at<uint8_t>(M::L_QGRP + q)) + at<uint16_t>(M::L_QPRE + 2 * q);
        if constexpr (DSV2) {
          const bool first = at<uint16_t>(M::L_GFIRST + 2 * at<uint8_t>(M::L_QGRP + q)) == q;
          const uint32_t pe = first ? 0 : at<uint32_t>(M::L_QEND + 4 * (q - 1));
          put_vu(dst, put_vu(dst, off, c0 - pe), at<uint32_t>(M::L_QEND + 4 * q) - c0 - 1);
        } else {
          put_vu(dst, put_vu(dst, off, c0), at<uint32_t>(M::L_QEND + 4 * q) - c0);
        }
      }
    }
    if (lane == 0) {
      j.out_off[d] = slot_al;
      j.out_len[d] = total;
      j.status[d] = ym::ST_OK;
    }
    return DS_DONE;
}

// ---- 1. stage: every load of document d in flight at once (round 6: the loops issued one 16-byte load per
// lane, waited for it, stored it, then issued the next): its update offsets (<= 129: three per lane) with the
// offsets of its first and last byte, then its 16-byte vectors covering [b0, b0 + bytes) (byte b0 lands at LDS
// offset b0 & 15), then the LDS stores.  False: the document is outside this kernel's shape (declined).
template <class M, bool DSONLY, class T>
__device__ __forceinline__ bool stage_doc(const GeneralJob &j, const T *off, uint32_t u0, uint32_t k, uint64_t &b0,
                                          uint64_t &bytes, uint64_t &arena0) {
  const uint32_t lane = threadIdx.x;
  arena0 = off[0];  // (the slot's origin, needed after the walk: loaded with the rest, not in the middle of the wave)
  constexpr uint32_t NO = (UPD + 1 + 63) / 64, NV = (M::IN + 31) / 16 / 64 + 1;
  // (the loads are unconditional, at clamped indices: exec-masked loads made the compiler wait for each one)
  const uint32_t kc = k <= UPD ? k : 0;
  uint64_t ov[NO];
#pragma unroll
  for (uint32_t t = 0; t < NO; t++) ov[t] = off[u0 + (lane + 64 * t < kc ? lane + 64 * t : kc)];
#ifdef YM_STAGE_SCALAR_B0
  b0 = off[u0];
  bytes = (uint64_t)off[u0 + k] - b0;
#else
  // the document's first and last offsets from those loads (lane 0 / the lane holding index kc): one memory
  // round trip for all of them instead of a scalar one first
  {
    uint64_t ve = ov[0];
#pragma unroll
    for (uint32_t t = 1; t < NO; t++) ve = (kc >> 6) == t ? ov[t] : ve;
    b0 = lane_read64(ov[0], 0);
    bytes = lane_read64(ve, (int)(kc & 63)) - b0;
  }
#endif
  if ((DSONLY ? k == 0 : k <= 1) || k > UPD || bytes > M::IN) return false;
  const uint32_t base = (uint32_t)(b0 & 15);
  const uint4 *src = reinterpret_cast<const uint4 *>(j.A + (b0 - base));
  const uint32_t nvec = (uint32_t)((base + bytes + 15) >> 4);
  // (stores at the same clamped indices, unconditionally: a lane past the end writes the last vector / offset
  // again, the same bytes; a conditional store let the compiler sink each load into its branch and wait there)
  // (no bytes at all -- empty inputs: a delete-set merge of one empty set, a merge of empty updates -- loads
  // nothing: the clamped index nvec - 1 would wrap to 2^32 - 1)
  if (nvec != 0) {
    uint32_t vi[NV];
    uint4 vv[NV];
#pragma unroll
    for (uint32_t t = 0; t < NV; t++) {
      vi[t] = lane + 64 * t < nvec ? lane + 64 * t : nvec - 1;
      vv[t] = src[vi[t]];
    }
#pragma unroll
    for (uint32_t t = 0; t < NV; t++) at<uint4>(M::L_IN + 16 * vi[t]) = vv[t];
  }
#pragma unroll
  for (uint32_t t = 0; t < NO; t++)
    at<uint16_t>(M::L_UOFF + 2 * (lane + 64 * t < kc ? lane + 64 * t : kc)) = (uint16_t)(ov[t] - b0 + base);
  return true;
}

// DSONLY: PermanentUserData's delete-set merge (ym_ds_merge): every input is an encoded delete set (no
// struct section); the walk is W2 only and the output is the merged delete set alone, in the DSEncoderV1
// format, or DSEncoderV2's (DSV2: clocks delta-coded within a client, lengths minus one).
// Grid: a multiple of 8 blocks; block b takes documents (b % 8) * G/8 + b / 8 + k * G.
// NESTED: the retry pass over the `nd` documents listed in j.list (those the first pass declined), with
// nested payload checks; its declines go to j.pend_list as before.
template <class M, int STOP, bool DSONLY, bool DSV2, bool NESTED>
__device__ __forceinline__ void merge_doc_v1(const GeneralJob &j, uint32_t di) {
  const uint32_t lane = threadIdx.x;
  {
    const uint32_t d = NESTED && j.list ? j.list[di] : di;  // (NESTED without a list: every document)
    const uint32_t u0 = j.doc_upd[d], k = j.doc_upd[d + 1] - u0;
    // ---- 1. stage (stage_doc): the offsets' width is a wave-uniform branch here, not one per load
    uint64_t b0 = 0, bytes = 0, arena0 = 0;
    const bool staged = j.upd_off32 ? stage_doc<M, DSONLY>(j, j.upd_off32, u0, k, b0, bytes, arena0)
                                    : stage_doc<M, DSONLY>(j, j.upd_off, u0, k, b0, bytes, arena0);
    if (!staged) {
      if (lane == 0) decline(j, d);
      return;
    }
    if (lane < 8) at<uint32_t>(M::L_MISC + 4 * lane) = 0;  // counters, duplicate-check bitmap
    if (lane < 16) at<uint32_t>(M::L_HIST + 4 * lane) = 0;
    __syncthreads();
    YM_TS(0)
    YM_STOP(1)
    // ---- 2. walk.  W1: one lane per update that has structs, updates ordered by length bucket so
    // that the lanes of one round take updates of similar shape; W2: one lane per update whose delete
    // set is not empty.  Splitting the two keeps every lane of a round busy with the same kind of work.
    {
      uint32_t ulen[UPD / 64], has[UPD / 64];
      bool empty = false;
#pragma unroll
      for (uint32_t s = 0; s < UPD / 64; s++) {
        const uint32_t u = lane + 64 * s;
        has[s] = 0;
        ulen[s] = 0;
        if (u < k) {
          const uint32_t u0_ = at<uint16_t>(M::L_UOFF + 2 * u), len = at<uint16_t>(M::L_UOFF + 2 * u + 2) - u0_;
          empty |= len == 0;
          ulen[s] = len;
          if (len > 0 && (DSONLY || sm[u0_] == 0)) {
            // no structs: the delete set follows (DSONLY: the input is the delete set)
            at<uint16_t>(M::L_UDS + 2 * u) = (uint16_t)(DSONLY ? u0_ : u0_ + 1);
          } else {
            has[s] = 1;
          }
        }
      }
      if (__any(empty)) YM_DECLINE()
      uint32_t n1 = 0;
#pragma unroll
      for (uint32_t s = 0; s < UPD / 64; s++) n1 += __popcll(__ballot(has[s]));
      if (n1 <= 64) {
        // one round: lane i walks the i-th update with structs (ballot compaction)
        uint32_t base = 0;
#pragma unroll
        for (uint32_t s = 0; s < UPD / 64; s++) {
          const uint64_t m = __ballot(has[s]);
          if (has[s]) at<uint8_t>(M::L_UORD + base + __popcll(m & ((1ull << lane) - 1))) = (uint8_t)(lane + 64 * s);
          base += __popcll(m);
        }
      } else {
        // two rounds: updates ordered by length bucket, so that the lanes of a round take updates of
        // similar shape (counting sort: bucket histogram, scan, scatter)
        uint32_t ub[UPD / 64], up[UPD / 64];
#pragma unroll
        for (uint32_t s = 0; s < UPD / 64; s++) {
          ub[s] = 16;
          if (has[s]) {
            ub[s] = ulen[s] >> 3 < 15 ? ulen[s] >> 3 : 15;
            up[s] = atomicAdd(&at<uint32_t>(M::L_HIST + 4 * ub[s]), 1u);
          }
        }
        __syncthreads();
        const uint32_t h = lane < 16 ? at<uint32_t>(M::L_HIST + 4 * lane) : 0;
        const uint32_t hincl = wave_incl_add(h);
        __syncthreads();
        if (lane < 16) at<uint32_t>(M::L_HIST + 4 * lane) = hincl - h;
        __syncthreads();
#pragma unroll
        for (uint32_t s = 0; s < UPD / 64; s++)
          if (ub[s] < 16) at<uint8_t>(M::L_UORD + at<uint32_t>(M::L_HIST + 4 * ub[s]) + up[s]) = (uint8_t)(lane + 64 * s);
      }
      __syncthreads();
      // the list lives in the record region: read into registers before the walk appends records
      const uint32_t w0 = at<uint8_t>(M::L_UORD + lane), w1 = at<uint8_t>(M::L_UORD + 64 + lane);
      __syncthreads();
      bool ok = true;
#pragma unroll 1
      for (uint32_t i = lane, w = w0; i < n1; i += 64, w = w1) ok &= walk_sections<M, NESTED>(w);
      if (__any(!ok)) YM_DECLINE()
    }
    __syncthreads();
    // long non-ASCII strings the walk listed (L_HIST is free during the walk): validated by the whole wave
    if (!deferred_ok<M::L_HIST, M::L_MISC + 8>()) YM_DECLINE()
    YM_TS(1)
    YM_STOP(8)
    const uint32_t nsec = at<uint32_t>(M::L_MISC);
    if ((DSONLY ? nsec != 0 : nsec == 0) || nsec > SEC) YM_DECLINE()
    // pad the key array to a multiple of 4 (rank loops read quads; SEC is a multiple of 4)
    if (lane < 3 && nsec + lane < ((nsec + 3) & ~3u)) at<uint64_t>(M::L_SKEY + 8 * (nsec + lane)) = ~0ull;
    __syncthreads();
    // output slot: 64-aligned inside the bound 2 * in + 64 per doc (no global atomics)
    const uint64_t slot = 2 * (b0 - arena0) + 64ull * (d + j.doc_base);
    const uint64_t slot_al = (slot + 63) & ~63ull;
    const uint64_t slot_end = slot + 2 * bytes + 64 < j.cap ? slot + 2 * bytes + 64 : j.cap;
    if (slot_al >= slot_end) YM_DECLINE()
    const Slot dst = make_slot(j.out + slot_al, (uint32_t)(slot_end - slot_al));
    uint32_t hdr = 0, struct_bytes = 0;
    if constexpr (!DSONLY) {
      const int r = nsec <= 64 ? sec_phase<M, 1, STOP>(j, d, nsec, slot, slot_al, slot_end, bytes, dst, hdr, struct_bytes)
                               : sec_phase<M, 2, STOP>(j, d, nsec, slot, slot_al, slot_end, bytes, dst, hdr, struct_bytes);
      if (r == SP_DECLINE) YM_DECLINE()
      if (r == SP_STOP && lane == 0) { j.status[d] = ym::ST_OK; j.out_len[d] = 0; }
      if (r != SP_DONE) {
        __syncthreads();
        return;
      }
    }  // !DSONLY
    __syncthreads();
    YM_TS(4)
    YM_STOP(7)
    // ---- W2 (after the struct section is written: the ranges reuse the section records' LDS): one lane per
    // update whose delete set has clients (first byte != 0), compacted by ballots
    {
      uint32_t n2 = 0;
#pragma unroll
      for (uint32_t s = 0; s < UPD / 64; s++) {
        const uint32_t u = lane + 64 * s;
        bool has = false;
        if (u < k) {
          const uint32_t p = at<uint16_t>(M::L_UDS + 2 * u);
          has = p >= at<uint16_t>(M::L_UOFF + 2 * u + 2) || sm[p] != 0;  // (a missing delete set: W2 declines)
        }
        const uint64_t m = __ballot(has);
        if (has) at<uint8_t>(M::L_UORD2 + n2 + __popcll(m & ((1ull << lane) - 1))) = (uint8_t)u;
        n2 += __popcll(m);
      }
      __syncthreads();
      const uint32_t w0 = at<uint8_t>(M::L_UORD2 + lane), w1 = at<uint8_t>(M::L_UORD2 + 64 + lane);
      __syncthreads();
      bool ok = true;
#pragma unroll 1
      for (uint32_t i = lane, w = w0; i < n2; i += 64, w = w1) ok &= walk_ds<M, DSV2>(w);
      if (__any(!ok)) YM_DECLINE()
    }
    __syncthreads();
    const uint32_t nds = at<uint32_t>(M::L_MISC + 4);
    if (nds > DSN) YM_DECLINE()
    if (lane < 3 && nds + lane < ((nds + 3) & ~3u)) at<uint64_t>(M::L_DKEY + 8 * (nds + lane)) = ~0ull;
    __syncthreads();
    YM_TS(5)
    YM_STOP(2)
    {
      const int r = nds <= 64 ? ds_phase<M, 1, STOP, DSV2>(j, d, nds, hdr, struct_bytes, slot, slot_al, slot_end, bytes, dst)
                              : ds_phase<M, 2, STOP, DSV2>(j, d, nds, hdr, struct_bytes, slot, slot_al, slot_end, bytes, dst);
      if (r == DS_DECLINE) YM_DECLINE()
      if (r == DS_STOP && lane == 0) { j.status[d] = ym::ST_OK; j.out_len[d] = 0; }
    }
    __syncthreads();
  }
}
// ONE: the grid covers every document (one per block, no loop: nothing is hoisted across documents, so
// the per-document values are not kept live -- and spilled -- for the whole kernel); otherwise a
// grid-stride loop.  Grid: a multiple of 8 blocks; block b takes documents (b % 8) * G/8 + b / 8 + k * G.
#ifdef YM_FAST_TIMELINE
// diagnostics build: per block of the last launch, its start / end (s_memrealtime, 100 MHz), the hardware ids
// (HW_ID: wave, SIMD, CU, SE; XCC_ID) and its document (read with ym__fast_timeline)
__device__ unsigned long long g_fast_tl[131072][4];
#endif
template <int STOP, int OCC, bool DSONLY = false, bool DSV2 = false, bool NESTED = false, bool ONE = true>
__global__ void __launch_bounds__(64, OCC) k_fast_merge_v1(GeneralJob j, uint32_t nd) {
  const uint32_t d0 = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if constexpr (ONE) {
#ifdef YM_FAST_TIMELINE
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (d0 < nd) merge_doc_v1<Map<NESTED ? IN_NESTED : IN_HOT>, STOP, DSONLY, DSV2, NESTED>(j, d0);
#ifdef YM_FAST_TIMELINE
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 131072) {
      g_fast_tl[blockIdx.x][0] = t0;
      g_fast_tl[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
      g_fast_tl[blockIdx.x][2] = ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) << 32) |
                                 (unsigned)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
      g_fast_tl[blockIdx.x][3] = d0;
    }
#endif
  } else {
    for (uint32_t di = d0; di < nd; di += gridDim.x) merge_doc_v1<Map<NESTED ? IN_NESTED : IN_HOT>, STOP, DSONLY, DSV2, NESTED>(j, di);
  }
}

}  // namespace fastv1

// merges: the general path's bump allocator starts after the fast paths' slot region (launched by
// the host only when documents were declined)
__global__ void k_fast_region(GeneralJob j, uint32_t n_upd) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *j.used = 2 * (j.upd_off[n_upd] - j.upd_off[0]) + 64ull * j.n + 64;
}

// grid: a multiple of 8 one-wave blocks (the kernel's XCD-contiguous document mapping); one block per
// document up to FAST_ONE_MAX documents (the ONE form), a grid-stride loop above
constexpr uint32_t FAST_ONE_MAX = 1u << 24;
static uint32_t fast_grid(uint32_t n) { return ((n < FAST_ONE_MAX ? n : FAST_ONE_MAX) + 7) & ~7u; }

int fast_launch(uint32_t op, const GeneralJob &j, uint32_t n_upd, hipStream_t st) {
  using namespace fastv1;
  if (op == OP_DSMERGE) {  // delete-set merges: the same kernel, delete sets only
    if (j.dsref) return 0;  // the reference's adjacency-only coalescing: general path
    const uint32_t grid = fast_grid(j.n);
    const bool one = j.n <= FAST_ONE_MAX;
    if (j.v2) {
      if (one) k_fast_merge_v1<0, 8, true, true><<<grid, 64, MapHot::LDS_BYTES, st>>>(j, j.n);
      else k_fast_merge_v1<0, 5, true, true, false, false><<<grid, 64, MapHot::LDS_BYTES, st>>>(j, j.n);
    } else {
      if (one) k_fast_merge_v1<0, 8, true, false><<<grid, 64, MapHot::LDS_BYTES, st>>>(j, j.n);
      else k_fast_merge_v1<0, 5, true, false, false, false><<<grid, 64, MapHot::LDS_BYTES, st>>>(j, j.n);
    }
    return 1;
  }
  if (op != OP_MERGE || j.v2) return 0;  // fast path: V1 merges (the C2/C4 headline configs)
  (void)n_upd;  // the work-list counter is zero on entry (ym_api.hip k_finish); `used` is set later
  const uint32_t grid = fast_grid(j.n);
  static int stop = -1, pad = 0;
  if (stop < 0) {
    const char *e = getenv("YMERGE_FAST_STOP");
    stop = e ? atoi(e) : 0;
    e = getenv("YMERGE_FAST_LDS_PAD");  // occupancy experiments: extra dynamic LDS per wave
    pad = e ? atoi(e) : 0;
  }
  const uint32_t LDS_BYTES = MapHot::LDS_BYTES + pad;
  static int occ = -1;
  // (the launch bound steers register allocation: 8 keeps the kernel within 8 waves' SGPRs and VGPRs per SIMD,
  // what the 5 KB LDS map allows; 5 lets it use more registers, 7 waves by SGPRs)
  if (occ < 0) { const char *e = getenv("YMERGE_FAST_OCC"); occ = e ? atoi(e) : 8; }
#define YM_LAUNCH(S, O) k_fast_merge_v1<S, O><<<grid, 64, LDS_BYTES, st>>>(j, j.n)
  if (j.n > FAST_ONE_MAX) {
    k_fast_merge_v1<0, 5, false, false, false, false><<<grid, 64, LDS_BYTES, st>>>(j, j.n);
  } else if (occ == 5) {
    YM_LAUNCH(0, 5);
  } else if (occ == 6) {
    YM_LAUNCH(0, 6);
  } else if (occ == 7) {
    YM_LAUNCH(0, 7);
  } else {
    switch (stop) {
      case 1: YM_LAUNCH(1, 8); break;
      case 2: YM_LAUNCH(2, 8); break;
      case 3: YM_LAUNCH(3, 8); break;
      case 4: YM_LAUNCH(4, 8); break;
      case 5: YM_LAUNCH(5, 8); break;
      case 7: YM_LAUNCH(7, 8); break;
      case 8: YM_LAUNCH(8, 8); break;
      default: YM_LAUNCH(0, 8); break;
    }
  }
#undef YM_LAUNCH
  return 1;
}

// The retry pass: V1 merges the hot kernel declined (j.list, n documents), now with nested payload checks
// (rich content: any objects / arrays, JSON texts); what this pass declines goes on to the large-document
// pipeline / general path through j.pend_list.
int fast_nested_launch(const GeneralJob &j, uint32_t n, hipStream_t st) {
  using namespace fastv1;
  if (j.op != OP_MERGE || j.v2 || n == 0) return 0;
  static int off = -1;
  if (off < 0) { const char *e = getenv("YMERGE_FAST_NESTED"); off = e && atoi(e) == 0 ? 1 : 0; }
  if (off) return 0;
  if (n <= FAST_ONE_MAX) k_fast_merge_v1<0, 6, false, false, true><<<fast_grid(n), 64, MapNested::LDS_BYTES, st>>>(j, n);
  else k_fast_merge_v1<0, 5, false, false, true, false><<<fast_grid(n), 64, MapNested::LDS_BYTES, st>>>(j, n);
  return 1;
}

}  // namespace ymk

#ifdef YM_FAST_TIMELINE
extern "C" int ym__fast_timeline(unsigned long long *host, int n) {  // n blocks x 4 words
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ymk::fastv1::g_fast_tl), (size_t)n * 32);
}
extern "C" int ym__fast_phases(unsigned *host, int n) {  // n blocks x 8 words
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ymk::fastv1::g_fast_ph), (size_t)n * 32);
}
#endif
