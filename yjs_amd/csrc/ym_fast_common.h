// ym_fast_common.h -- device helpers shared by the LDS kernels (ym_fast.hip: batched V1 merge;
// ym_big.hip: V1 diff / state vector over single large updates): LDS accessors, DPP wave scans,
// lib0 varuint / varString / any readers with the canonical-form checks the verbatim copy relies on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ym_canon_chk.h"
#include "ym_kernels.h"
#include "ym_utf8.h"

namespace ymk {
namespace fastc {

extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
template <class T>
__device__ __forceinline__ T &at(uint32_t off) { return *reinterpret_cast<T *>(sm + off); }
// unaligned LDS accesses (gfx950 runs them in hardware: tools/probe/lds_unaligned.hip)
#ifdef YM_LD8_ALIGNED
// 8 bytes at any offset from two 8-aligned LDS reads (one ds_read2_b64) and byte funnel shifts: unaligned
// ds_read_b64s stall the CU's LDS pipeline (SQ_LDS_UNALIGNED_STALL) for every wave on it.  Reads up to 15
// bytes past p.
__device__ __forceinline__ uint64_t ld8(uint32_t p) {
  const uint32_t a = p & ~7u;
  const uint64_t q0 = *reinterpret_cast<const uint64_t *>(sm + a), q1 = *reinterpret_cast<const uint64_t *>(sm + a + 8);
  const uint32_t d0 = (uint32_t)q0, d1 = (uint32_t)(q0 >> 32), d2 = (uint32_t)q1, d3 = (uint32_t)(q1 >> 32);
  const bool k = (p & 4u) != 0;
  const uint32_t x0 = k ? d1 : d0, x1 = k ? d2 : d1, x2 = k ? d3 : d2, s = p & 3u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(x1, x0, s), hi = __builtin_amdgcn_alignbyte(x2, x1, s);
  return ((uint64_t)hi << 32) | lo;
}
#else
__device__ __forceinline__ uint64_t ld8(uint32_t p) { uint64_t x; __builtin_memcpy(&x, sm + p, 8); return x; }
#endif
__device__ __forceinline__ uint32_t ld4(uint32_t p) { uint32_t x; __builtin_memcpy(&x, sm + p, 4); return x; }
__device__ __forceinline__ void st4(uint32_t p, uint32_t x) { __builtin_memcpy(sm + p, &x, 4); }

// ---- wave primitives (DPP row shifts + row broadcasts: no LDS traffic) ---------------------------
#define YM_DPP(x, ctl, rm) (uint32_t) __builtin_amdgcn_update_dpp(0, (int)(x), ctl, rm, 0xf, false)
// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  x += YM_DPP(x, 0x111, 0xf);  // row_shr:1
  x += YM_DPP(x, 0x112, 0xf);  // row_shr:2
  x += YM_DPP(x, 0x114, 0xf);  // row_shr:4
  x += YM_DPP(x, 0x118, 0xf);  // row_shr:8
  x += YM_DPP(x, 0x142, 0xa);  // row_bcast:15 -> rows 1, 3
  x += YM_DPP(x, 0x143, 0xc);  // row_bcast:31 -> rows 2, 3
  return x;
}
__device__ __forceinline__ uint32_t lane_read(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
// inclusive prefix max over the 64 lanes, u64
template <int CTL, int RM>
__device__ __forceinline__ uint64_t max_step(uint64_t x) {
  const uint32_t lo = YM_DPP((uint32_t)x, CTL, RM), hi = YM_DPP((uint32_t)(x >> 32), CTL, RM);
  const uint64_t y = ((uint64_t)hi << 32) | lo;
  return y > x ? y : x;
}
__device__ __forceinline__ uint64_t wave_incl_max64(uint64_t x) {
  x = max_step<0x111, 0xf>(x);
  x = max_step<0x112, 0xf>(x);
  x = max_step<0x114, 0xf>(x);
  x = max_step<0x118, 0xf>(x);
  x = max_step<0x142, 0xa>(x);
  x = max_step<0x143, 0xc>(x);
  return x;
}
__device__ __forceinline__ uint64_t lane_read64(uint64_t x, int l) {
  return ((uint64_t)lane_read((uint32_t)(x >> 32), l) << 32) | lane_read((uint32_t)x, l);
}
// value of lane-1 (0 for lane 0) / lane+1 (0 for lane 63): DPP wave_shr:1 / wave_shl:1
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false); }

// bytes of lib0 writeVarUint(v) for a u32: ceil(significant bits / 7), at least 1 (x * 37 >> 8 == x / 7
// for x <= 38)
__device__ __forceinline__ uint32_t vsz(uint32_t v) {
  const uint32_t bits = 32 - __builtin_clzg(v, 32);
  return ((bits > 0 ? bits : 1) + 6) * 37 >> 8;
}
// The document's output slot as a buffer resource: 32-bit offsets (no 64-bit address math per
// store) and a hardware bound (stores past the slot are dropped).
typedef __amdgpu_buffer_rsrc_t Slot;
__device__ __forceinline__ Slot make_slot(uint8_t *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void ob8(Slot o, uint32_t p, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b8((int8_t)v, o, (int)p, 0, 0);
}
__device__ __forceinline__ void ob32(Slot o, uint32_t p, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32((int)v, o, (int)p, 0, 0);
}
// The document's output staged in LDS at byte offset b (copied out with 16-byte stores afterwards:
// byte-wise global stores cost a memory-pipeline slot each).
struct LSlot {
  uint32_t b;
};
__device__ __forceinline__ void ob8(LSlot o, uint32_t p, uint32_t v) { sm[o.b + p] = (uint8_t)v; }
// lib0 writeVarUint straight into the output slot
template <class O>
__device__ __forceinline__ uint32_t put_vu(O o, uint32_t p, uint64_t v) {
  while (v > 127) { ob8(o, p++, 0x80 | (uint32_t)(v & 127)); v >>= 7; }
  ob8(o, p++, (uint32_t)v);
  return p;
}
// Lane-serial LDS -> LDS copy (regions do not overlap): 8-byte unaligned LDS reads and writes (gfx950's LDS
// takes unaligned b64 accesses), then the tail byte-wise.
__device__ __forceinline__ void lds_copy(uint32_t dst, uint32_t src, uint32_t n) {
  uint32_t b = 0;
  for (; b + 8 <= n; b += 8) {
    uint64_t x;
    __builtin_memcpy(&x, sm + src + b, 8);
    __builtin_memcpy(sm + dst + b, &x, 8);
  }
  if (b + 4 <= n) {
    uint32_t x;
    __builtin_memcpy(&x, sm + src + b, 4);
    __builtin_memcpy(sm + dst + b, &x, 4);
    b += 4;
  }
  for (; b < n; b++) sm[dst + b] = sm[src + b];
}
// Copies n staged bytes from LDS offset src to g (16-aligned) with 16-byte stores; `room` bytes are
// writable at g, so the last chunk is written whole when it fits and byte-wise otherwise.
__device__ __forceinline__ void copy_out(uint8_t *g, uint32_t src, uint32_t n, uint64_t room) {
  const uint32_t lane = threadIdx.x;
  const uint32_t n16 = ((uint64_t)((n + 15) & ~15u) <= room ? n + 15 : n) >> 4;
  for (uint32_t k = lane; k < n16; k += 64)
    *reinterpret_cast<uint4 *>(g + 16 * k) = *reinterpret_cast<const uint4 *>(sm + src + 16 * k);
  for (uint32_t i = 16 * n16 + lane; i < n; i += 64) g[i] = sm[src + i];
}

// Staging (one wave): nvec 16-byte vectors from global `src` to LDS byte offset `dst`, MAXV vectors per lane per
// pass with every load of the pass in flight before its stores (round 6: a `for (v = lane; v < n; v += 64)` loop
// waits for each load before the next -- one memory round trip per 1 KB, the head of every wave's latency).
// Lanes past the end re-load and re-store the last vector (the same bytes): no branch the compiler could sink
// the loads into.
template <uint32_t MAXV>
__device__ __forceinline__ void stage16(uint32_t dst, const uint4 *src, uint32_t nvec) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t v0 = 0; v0 < nvec; v0 += 64 * MAXV) {
    uint32_t ix[MAXV];
    uint4 x[MAXV];
#pragma unroll
    for (uint32_t t = 0; t < MAXV; t++) {
      const uint32_t i = v0 + lane + 64 * t;
      ix[t] = i < nvec ? i : nvec - 1;
      x[t] = src[ix[t]];
    }
#pragma unroll
    for (uint32_t t = 0; t < MAXV; t++) at<uint4>(dst + 16 * ix[t]) = x[t];
  }
}

// ---- V1 walker over LDS bytes ---------------------------------------------------------------------
// Any anomaly (truncation, non-canonical varint, invalid UTF-8, a payload kind this path does not
// verify) sets `bad`; the general path then reproduces yjs's exact result or error.
struct Cur {
  uint32_t p, e;
  bool bad;
};
// Length of the lib0 varuint at the start of an 8-byte window (1..5; 6 = no terminator within 5 bytes).
// Branch-free: v_ffbl on the stop bits with a sentinel.
__device__ __forceinline__ uint32_t vu_nb(uint32_t lo, uint32_t hi) {
  const uint32_t s_lo = ~lo & 0x80808080u;
  const uint32_t s_hi = (~hi & 0x80u) | 0x8000u;
  const uint32_t t = __builtin_ctzg(s_lo, 32 + __builtin_ctz(s_hi));
  return (t >> 3) + 1;
}
// validity of a varuint of nb bytes: terminated within 5 bytes, inside the update, canonical (no
// zero final group), and < 2^32 (lib0 readVarUint is u32)
__device__ __forceinline__ bool vu_bad(uint32_t lo, uint32_t hi, uint32_t nb, uint32_t p, uint32_t e) {
  const uint32_t last = nb <= 4 ? (lo >> (8 * nb - 8)) & 0xffu : hi & 0xffu;
  return (nb > 5) | (p + nb > e) | ((nb > 1) & (last == 0)) | ((nb == 5) & ((hi & 0x70u) != 0));
}
// lib0 readVarUint (u32, canonical encodings only) from one unaligned 8-byte window.  When every active
// lane reads a one-byte varint (counts, lengths, small clocks: most fields) a wave-uniform branch takes
// a 3-instruction path instead of the ~40-instruction general decode.
__device__ __forceinline__ uint32_t rvu(Cur &c) {
  const uint64_t x = ld8(c.p);
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (__all((lo & 0x80u) == 0)) {
    c.bad |= c.p >= c.e;
    c.p += 1;
    return lo & 0x7fu;
  }
  const uint32_t nb = vu_nb(lo, hi);
  const uint32_t v = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u) | ((lo >> 2) & 0x1fc000u) | ((lo >> 3) & 0xfe00000u) | (hi << 28);
  const uint32_t m = (uint32_t)((1ull << (7 * (nb < 5 ? nb : 5))) - 1);
  c.bad |= vu_bad(lo, hi, nb, c.p, c.e);
  c.p += nb < 6 ? nb : 0;
  return v & m;
}
// skips a varuint whose value is not needed (origins, parent ids), with the same validity checks
__device__ __forceinline__ void skvu(Cur &c) {
  const uint64_t x = ld8(c.p);
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (__all((lo & 0x80u) == 0)) {
    c.bad |= c.p >= c.e;
    c.p += 1;
    return;
  }
  const uint32_t nb = vu_nb(lo, hi);
  c.bad |= vu_bad(lo, hi, nb, c.p, c.e);
  c.p += nb < 6 ? nb : 0;
}
// skips two consecutive varuints (an ID: client, clock) read from one 8-byte window when both end
// inside it (the common case), with the checks of two skvu calls: terminated within 5 bytes each,
// inside the update, canonical, < 2^32.  Otherwise (a lane whose pair does not fit) two skvu calls.
__device__ __forceinline__ uint32_t ctz64(uint64_t x) { return __builtin_ctzg(x, 64); }
__device__ __forceinline__ void skvu2(Cur &c) {
  const uint64_t x = ld8(c.p);
  const uint64_t st = ~x & 0x8080808080808080ull;  // stop bytes (high bit clear)
  const uint64_t st2 = st & (st - 1);                // ... without the first
  if (st2 == 0) {
    skvu(c);
    skvu(c);
    return;
  }
  const uint32_t i1 = ctz64(st) >> 3, i2 = ctz64(st2) >> 3;  // indices of the two stop bytes
  const uint32_t b1 = (uint32_t)(x >> (8 * i1)) & 0xffu, b2 = (uint32_t)(x >> (8 * i2)) & 0xffu;
  const uint32_t n1 = i1 + 1, n2 = i2 - i1;
  c.bad |= (n1 > 5) | (n2 > 5) | (c.p + i2 + 1 > c.e) | ((n1 > 1) & (b1 == 0)) | ((n2 > 1) & (b2 == 0)) |
           ((n1 == 5) & ((b1 & 0x70u) != 0)) | ((n2 == 5) & ((b2 & 0x70u) != 0));
  c.p += i2 + 1;
}
__device__ __forceinline__ uint32_t rdb(Cur &c) {
  c.bad |= c.p >= c.e;
  return sm[c.p++];
}
__device__ __forceinline__ bool room(const Cur &c, uint32_t n) { return c.p <= c.e && n <= c.e - c.p; }
// strict UTF-8 (lib0: decodeURIComponent(escape(..))) over LDS [i, e); returns the UTF-16 length (ym_utf8.h,
// 4 bytes per step; reads up to 3 bytes past e)
// Out of line: only non-ASCII strings get here, and inlined its registers cost the one-wave kernels occupancy.
__device__ __attribute__((noinline)) uint32_t utf8_lds(uint32_t i, uint32_t e) {
  bool bad = false;
  const uint32_t u = utf8::units<uint32_t>([](uint32_t p) { return ld4(p); }, i, e, bad);
  return bad ? 0xffffffffu : u;
}
__device__ __forceinline__ uint32_t utf8_slow(uint32_t i, uint32_t e, bool &bad) {
  const uint32_t u = utf8_lds(i, e);
  bad |= u == 0xffffffffu;
  return u == 0xffffffffu ? 0 : u;
}
__device__ __forceinline__ uint64_t mask_bytes(uint64_t x, uint32_t n) { return n >= 8 ? x : x & ((1ull << (8 * n)) - 1); }
// The bytes of the next n UTF-16 units of valid UTF-8 at LDS [p, e) (a StringDecoder slice of a V2 string
// column body, validated by utf8_slow beforehand); `bad` when the slice ends inside a surrogate pair (a 4-byte
// character split between two strings: the halves re-encode by context, the fast paths decline it) or runs
// past e.  ASCII runs go 8 bytes per step.
__device__ __forceinline__ uint32_t utf8_span(uint32_t p, uint32_t e, uint32_t n, bool &bad) {
  uint32_t q = p, u = 0;
  while (u < n && q < e) {
    if (n - u >= 8 && e - q >= 8 && (ld8(q) & 0x8080808080808080ull) == 0) { q += 8; u += 8; continue; }
    const uint32_t b = sm[q];
    const uint32_t len = b < 0x80 ? 1 : b < 0xE0 ? 2 : b < 0xF0 ? 3 : 4, cu = len == 4 ? 2 : 1;
    if (u + cu > n) { bad = true; return 0; }
    u += cu;
    q += len;
  }
  if (u < n || q > e) bad = true;
  return q - p;
}
__device__ __forceinline__ uint32_t utf16_len(Cur &c, uint32_t n) {
  if (!room(c, n)) { c.bad = true; return 0; }
  uint64_t hi = 0;
  for (uint32_t o = 0; o < n; o += 8) hi |= mask_bytes(ld8(c.p + o), n - o);
  uint32_t u = n;
  if (hi & 0x8080808080808080ull) u = utf8_slow(c.p, c.p + n, c.bad);
  c.p += n;
  return u;
}
__device__ __forceinline__ uint32_t rstr(Cur &c) {
  const uint32_t n = rvu(c);
  return c.bad ? 0 : utf16_len(c, n);
}
// Long non-ASCII ContentStrings in the LDS merge kernel (round 6; pasted CJK / emoji text): the lane only counts
// the UTF-16 units (bytes that are not continuation bytes + 4-byte leaders, 8 bytes per step) and lists the
// string (u32 at DL: LDS offset | bytes << 16; the count at DC) for the wave to validate together after the walk
// (deferred_ok: 4 bytes per lane, 256 bytes per step).  A lane walking a 500-byte paste byte-serially held its
// whole wave for ~10 k instructions.  The count is the UTF-16 length of any valid string; an invalid one makes
// deferred_ok decline the document.  More than DEFER_MAX strings in a document: declined too.
constexpr uint32_t DEFER_MIN = 32, DEFER_MAX = 16;
template <uint32_t DL, uint32_t DC>
__device__ __forceinline__ uint32_t rstr_defer(Cur &c) {
  const uint32_t n = rvu(c);
  if (c.bad) return 0;
  if (n < DEFER_MIN) return utf16_len(c, n);
  if (!room(c, n)) { c.bad = true; return 0; }
  uint64_t any = 0;
  uint32_t u = 0;
  // 16 bytes per step (two independent 8-byte LDS reads in flight; a 600-byte paste is 38 steps of its lane)
  auto cnt = [&](uint64_t x, uint32_t k) {
    const uint64_t hi = x & 0x8080808080808080ull, x1 = x << 1;
    any |= hi;
    u += k - (uint32_t)__popcll(hi & ~x1) + (uint32_t)__popcll(hi & x1 & (x << 2) & (x << 3));
  };
  uint32_t o = 0;
  for (; o + 16 <= n; o += 16) {
    const uint64_t x0 = ld8(c.p + o), x1 = ld8(c.p + o + 8);
    cnt(x0, 8);
    cnt(x1, 8);
  }
  for (; o < n; o += 8) {
    const uint32_t k = n - o < 8 ? n - o : 8;
    cnt(mask_bytes(ld8(c.p + o), k), k);
  }
  if (any) {
    const uint32_t q = atomicAdd(&at<uint32_t>(DC), 1u);
    if (q < DEFER_MAX) at<uint32_t>(DL + 4 * q) = c.p | (n << 16);
    else c.bad = true;
  }
  c.p += n;
  return u;
}
// The wave validates the listed strings (after a barrier; wave-uniform result).  Lane l takes bytes [4l, 4l + 4)
// of each 256-byte step; the continuation bytes and second-byte checks a word owes its successor come from the
// previous lane (DPP), across steps from lane 63.
template <uint32_t DL, uint32_t DC>
__device__ __forceinline__ bool deferred_ok() {
  const uint32_t nd = at<uint32_t>(DC);
  if (nd == 0) return true;
  if (nd > DEFER_MAX) return false;
  const uint32_t lane = threadIdx.x & 63;
  bool bad = false;
  for (uint32_t i = 0; i < nd; i++) {
    const uint32_t ent = at<uint32_t>(DL + 4 * i), p = ent & 0xffffu, n = ent >> 16;
    uint32_t co = 0, cc = 0;
    for (uint32_t o = 0; o < n; o += 256) {
      const uint32_t q = o + 4 * lane;
      const uint32_t k = q < n ? (n - q < 4 ? n - q : 4) : 0;
      const uint32_t x = ld4(p + (q < n ? q : 0));
      utf8::State own;
      utf8::word<uint32_t>(own, x, k);  // (its carries out depend on its own bytes only)
      const uint32_t po = from_prev_lane(own.owe), pc = from_prev_lane(own.chk);
      utf8::State s;
      s.owe = lane == 0 ? co : po;
      s.chk = lane == 0 ? cc : pc;
      utf8::word<uint32_t>(s, x, k);
      bad |= s.bad;
      co = lane_read(own.owe, 63);
      cc = lane_read(own.chk, 63);
    }
    bad |= co != 0;  // (a sequence cut by the string's end at a step boundary)
  }
  return !__any(bad);
}
// SWAR: bytes of x equal to b / below 0x20 (exact per byte for the masked-in bytes)
__device__ __forceinline__ uint64_t has_byte(uint64_t x, uint64_t b) {
  const uint64_t y = x ^ (0x0101010101010101ull * b);
  return (y - 0x0101010101010101ull) & ~y & 0x8080808080808080ull;
}
__device__ __forceinline__ uint64_t has_ctl(uint64_t x) {
  return (x - 0x2020202020202020ull) & ~x & 0x8080808080808080ull;
}
// JSON text as yjs writes it for formats / embeds: true | false | null | "string without escapes"; with
// NESTED also integers, arrays and objects (ym_canon_chk.h, an out-of-line call: only the kernels off the
// headline path instantiate it, the call's stack and registers would cost the LDS merge kernel occupancy)
template <bool NESTED = false>
__device__ __forceinline__ void json_lit(Cur &c) {
  const uint32_t n = rvu(c);
  if (c.bad || !room(c, n)) { c.bad = true; return; }
  const uint64_t w = ld8(c.p);
  bool ok;
  if (n == 4) ok = (uint32_t)w == 0x65757274u || (uint32_t)w == 0x6c6c756eu;  // "true" / "null"
  else if (n == 5) ok = (w & 0xffffffffffull) == 0x65736c6166ull;            // "false"
  else ok = false;
  if (!ok && n >= 2 && (w & 0xff) == '"' && sm[c.p + n - 1] == '"') {
    // interior bytes [1, n-1): no control characters, quotes or backslashes.  Bytes >= 0x80 are
    // masked out of the control test (multi-byte UTF-8 is checked by utf16_len below).
    uint64_t bad = 0;
    for (uint32_t o = 1; o + 1 < n; o += 8) {
      uint64_t x = mask_bytes(ld8(c.p + o), n - 1 - o);
      const uint64_t pad = (n - 1 - o) >= 8 ? 0 : ~0ull << (8 * (n - 1 - o));
      const uint64_t xs = x | (pad & 0x4040404040404040ull);  // padding bytes look like '@'
      bad |= has_byte(xs, '"') | has_byte(xs, '\\') | (has_ctl(xs) & ~xs);
    }
    ok = bad == 0;
  }
  // numbers, objects, arrays: JSON.stringify(JSON.parse(text)) == text (ym_canon_chk.h)
  if (NESTED && !ok) ok = cchk::json_canon_ptr(sm, c.p, n);
  if (!ok) { c.bad = true; return; }
  utf16_len(c, n);
}
// one scalar `any` value in the canonical form lib0 writeAny emits (objects/arrays: general path)
__device__ __forceinline__ void any_scalar(Cur &c) {
  const uint32_t tag = rdb(c);
  switch (tag) {
    case 127: case 126: case 121: case 120: return;  // undefined, null, false, true
    case 125: {  // varInt: minimal, and <= 2^31-1 when positive (larger is written as a float)
      uint32_t b = rdb(c);
      uint64_t mag = b & 63;
      const bool neg = b & 64;
      int s = 6, nb = 1;
      while ((b & 128) && !c.bad) {
        b = rdb(c);
        if (s > 34) { c.bad = true; return; }
        mag |= (uint64_t)(b & 127) << s;
        s += 7;
        nb++;
      }
      if ((nb > 1 && b == 0) || (!neg && mag > 2147483647ull) || mag > 0xffffffffull) c.bad = true;
      return;
    }
    case 124: {  // float32, not an integer <= 2^31-1 (those are written as varInt), not NaN
      if (!room(c, 4)) { c.bad = true; return; }
      const uint32_t u = __builtin_bswap32(ld4(c.p));
      const float f = __uint_as_float(u);
      if (f != f || (truncf(f) == f && (double)f <= 2147483647.0)) c.bad = true;
      c.p += 4;
      return;
    }
    case 123: {  // float64 that is neither a small integer nor float32-exact
      if (!room(c, 8)) { c.bad = true; return; }
      const uint64_t u = __builtin_bswap64(ld8(c.p));
      const double x = __longlong_as_double((long long)u);
      if (x == x && ((trunc(x) == x && x <= 2147483647.0) || (double)(float)x == x)) c.bad = true;
      c.p += 8;
      return;
    }
    case 119: rstr(c); return;
    default: c.bad = true; return;
  }
}

// one `any` value in the form writeAny emits: scalars; with NESTED also nested values (ym_canon_chk.h)
template <bool NESTED = false>
__device__ __forceinline__ void any_canon(Cur &c) {
  const uint32_t tag = c.p < c.e ? sm[c.p] : 0;
  if (NESTED && (tag == 116 || tag == 117 || tag == 118 || tag == 122)) {
    uint32_t q = c.p;
    c.bad |= !cchk::any_canon_ptr(sm, c.p, c.e, &q);
    c.p = q;
  } else {
    any_scalar(c);
  }
}

// The fields and content of one V1 Item after its info byte (UpdateDecoder.js:127-243 field readers,
// Item.js:665-683 content refs; lazy reader of 13.5.16: parent kept raw, parentSub only without
// origins).  Returns false (decline) for kinds this path does not verify; `len` = the Item's length.
// DL / DC (the LDS merge kernel's walk): long non-ASCII ContentStrings deferred (rstr_defer).
template <bool NESTED = false, uint32_t DL = 0, uint32_t DC = 0>
__device__ __forceinline__ bool item_body(Cur &c, uint32_t info, uint32_t &len) {
  if (info & 0x80) skvu2(c);
  if (info & 0x40) skvu2(c);
  if ((info & 0xC0) == 0) {
    const uint32_t pi = rvu(c);
    c.bad |= pi > 1;  // parentInfo re-encodes as 0/1
    if (pi == 1) rstr(c);
    else skvu2(c);
    if (info & 0x20) rstr(c);
  }
  len = 1;
  switch (info & 31) {
    case 1: len = rvu(c); break;                                      // ContentDeleted
    case 3: { const uint32_t n = rvu(c); if (!room(c, n)) c.bad = true; else c.p += n; break; }  // Binary
    case 4: len = DL ? rstr_defer<DL, DC>(c) : rstr(c); break;         // ContentString
    case 5: json_lit<NESTED>(c); break;                               // ContentEmbed
    case 6: rstr(c); json_lit<NESTED>(c); break;                      // ContentFormat
    case 7: {                                                         // ContentType
      const uint32_t t = rvu(c);
      c.bad |= t > 6;
      if (t == 3 || t == 5) rstr(c);
      break;
    }
    case 8:                                                           // ContentAny
      len = rvu(c);
      for (uint32_t i = 0; i < len && !c.bad; i++) any_canon<NESTED>(c);
      break;
    default: c.bad = true; break;  // ContentJSON, ContentDoc, invalid refs
  }
  // (no early returns: every decline sets c.bad, so the lane's loops and exits stay single-edged)
  return !c.bad && len != 0;
}

// rank of each of the lane's keys among keys[0..n): #keys <= own (own included) - 1.  Keys past n
// are ~0 (padding) and never count.  Equal keys collide; callers detect that.
// rank_le4: the same, four keys per iteration (two 16-B broadcast reads): keys[] padded with ~0 up to a
// multiple of 4
template <uint32_t E>
__device__ __forceinline__ void rank_le4(uint32_t keys, uint32_t n, const uint64_t (&k)[E], uint32_t (&rank)[E]) {
  uint32_t cnt[E];
#pragma unroll
  for (uint32_t s = 0; s < E; s++) cnt[s] = 0;
  for (uint32_t jj = 0; jj < n; jj += 4) {
    const uint64_t a = at<uint64_t>(keys + 8 * jj), b = at<uint64_t>(keys + 8 * jj + 8);
    const uint64_t c = at<uint64_t>(keys + 8 * jj + 16), d = at<uint64_t>(keys + 8 * jj + 24);
#pragma unroll
    for (uint32_t s = 0; s < E; s++)
      cnt[s] += (uint32_t)(a <= k[s]) + (uint32_t)(b <= k[s]) + (uint32_t)(c <= k[s]) + (uint32_t)(d <= k[s]);
  }
#pragma unroll
  for (uint32_t s = 0; s < E; s++) rank[s] = cnt[s] - 1;
}
template <uint32_t E>
__device__ __forceinline__ void rank_le(uint32_t keys, uint32_t n, const uint64_t (&k)[E], uint32_t (&rank)[E]) {
  uint32_t cnt[E];
#pragma unroll
  for (uint32_t s = 0; s < E; s++) cnt[s] = 0;
  for (uint32_t jj = 0; jj < n; jj += 2) {
    const uint64_t a = at<uint64_t>(keys + 8 * jj), b = at<uint64_t>(keys + 8 * jj + 8);
#pragma unroll
    for (uint32_t s = 0; s < E; s++) cnt[s] += (uint32_t)(a <= k[s]) + (uint32_t)(b <= k[s]);
  }
#pragma unroll
  for (uint32_t s = 0; s < E; s++) rank[s] = cnt[s] - 1;
}
// exact ranks with ties broken by slot index (used only when equal keys exist)
template <uint32_t E>
__device__ __forceinline__ void rank_exact(uint32_t keys, uint32_t n, const uint64_t (&k)[E], uint32_t (&rank)[E]) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t s = 0; s < E; s++) {
    const uint32_t i = lane + 64 * s;
    uint32_t cnt = 0;
    for (uint32_t jj = 0; jj < n; jj++) {
      const uint64_t a = at<uint64_t>(keys + 8 * jj);
      cnt += (a < k[s]) || (a == k[s] && jj < i);
    }
    rank[s] = cnt;
  }
}

// a declined document is appended to the general path's work list
__device__ __forceinline__ void decline(const GeneralJob &j, uint32_t d) {
  j.status[d] = ST_PENDING;
  const uint32_t q = atomicAdd(j.pend_count, 1u);
  if (j.pend_list) j.pend_list[q] = d + j.doc_base;  // (ym_merge_async: declines are only counted)
}
}  // namespace fastc
}  // namespace ymk
