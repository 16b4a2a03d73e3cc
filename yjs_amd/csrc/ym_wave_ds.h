// ym_wave_ds.h -- wave-parallel validation of a run of lib0 varuints (a delete set's ranges), shared by
// the chunk-parallel V1 walk (ym_pwalk.hip) and the column-parallel V2 path (ym_pv2.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ym_fast_common.h"

namespace ymk {
namespace wds {
using namespace fastc;
typedef uint4 __attribute__((aligned(1))) u4u;
constexpr uint32_t NONE = 0xffffffffu;

// 16 bytes at q (bytes at or past e read as 0x80: no stop byte)
__device__ __forceinline__ uint4 load16m(const uint8_t *D, uint32_t q, uint32_t e) {
  if (q + 16 <= e) return *reinterpret_cast<const u4u *>(D + q);
  uint8_t b[16];
  for (uint32_t k = 0; k < 16; k++) b[k] = q + k < e ? D[q + k] : 0x80;
  uint4 v;
  __builtin_memcpy(&v, b, 16);
  return v;
}
// Validates `cnt` canonical varuints (u32, lib0 readVarUint) starting at x, wave-parallel: 1 KB per
// step (16 bytes per lane, the next step's bytes loaded while this one is checked), stop bytes counted
// by a wave prefix sum, the continuation run entering each lane taken from its left neighbour.  Returns
// the position after the last one, or NONE (truncated / non-canonical).
__device__ __forceinline__ uint32_t skip_varuints(const uint8_t *D, uint32_t x, uint32_t e, uint64_t cnt) {
  const uint32_t lane = threadIdx.x;
  uint32_t carry = 0;  // continuation bytes at the end of the previous step (16 = at least 16)
  uint4 cur = load16m(D, x + 16 * lane, e);
  while (cnt > 0) {
    if (x >= e) return NONE;
    const uint4 nxt = x + 1024 < e ? load16m(D, x + 1024 + 16 * lane, e) : make_uint4(0, 0, 0, 0);
    const uint32_t q = x + 16 * lane;
    uint8_t b[16];
    __builtin_memcpy(b, &cur, 16);
    uint32_t nstop = 0, tr = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
      const bool stop = b[k] < 0x80 && q + k < e;
      nstop += stop;
      tr = stop ? 0 : tr + 1;
    }
    uint32_t run = from_prev_lane(tr);
    if (lane == 0) run = carry;
    const uint32_t incl = wave_incl_add(nstop), excl = incl - nstop;
    const uint32_t tot = lane_read(incl, 63);
    const uint32_t need = cnt < tot ? (uint32_t)cnt : tot;  // stops consumed by this step
    bool bad = false;
    uint32_t rank = excl, endp = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
      const bool stop = b[k] < 0x80 && q + k < e;
      if (stop && rank < need) {
        const uint32_t nb = run + 1;
        bad |= nb > 5 || (nb > 1 && b[k] == 0) || (nb == 5 && (b[k] & 0x70) != 0);
        if (rank == need - 1) endp = q + k + 1;
      }
      rank += stop;
      run = stop ? 0 : run + 1;
    }
    if (__any(bad)) return NONE;
    if (cnt <= tot) {
      const uint64_t m = __ballot(endp != 0);
      return lane_read(endp, __builtin_ctzll(m));
    }
    cnt -= tot;
    carry = lane_read(tr == 16 ? 16 + carry : tr, 63);  // a run may continue across the step boundary
    if (carry > 16) carry = 16;
    cur = nxt;
    x += 1024;
  }
  return x;
}

// ---- readDeleteSet's reads, validated with LDS token tables (one wave) -------------------------------------
// vu(#clients), then per client vu(client) vu(m) and m (clock, len) varuint pairs: every varuint canonical
// (<= 5 bytes, no overlong final group, < 2^32), m > 0, no client twice (readDeleteSet would drop an empty
// client and merge a repeated one: either makes the re-written set differ from the input bytes).  The
// streamed walkers checked it client by client, a few dependent HBM loads each (C5: ~1,000 clients, ~5 ms
// per call).  Here the bytes pass through an LDS window: the wave tokenises it (stop bytes, a prefix sum gives
// each varuint its index, the lane holding its last byte decodes and checks it) into value / end / bad-prefix
// tables, then lane 0 steps client by client in O(1): client = val[t], m = val[t + 1], the 2m range tokens are
// good iff the bad prefix does not change, t += 2 + 2m.  Repeated clients: an LDS hash set.
constexpr uint32_t DHS = 2048;    // hash-set slots (at most DHS * 3 / 4 clients; more: the caller's own walk)
constexpr uint32_t DS_BIG = 0xfffffffeu;  // not decided here (a client's ranges beyond a window, too many clients)
// DW: window bytes (a multiple of 64: each lane tokenises DW / 64 of them)
template <uint32_t DW>
struct DsLdsT {
  uint8_t b[DW + 16];
  uint32_t val[DW];
  uint16_t end[DW];       // position after token t (window-relative)
  uint16_t badp[DW + 1];  // tokens among the first t that are not canonical
  uint32_t hs[DHS];
  uint32_t ntok, wtot, lastc, hmax;
};
using DsLds = DsLdsT<4096>;   // ~45 KB
using DsLdsS = DsLdsT<1024>;  // ~17 KB (kernels that keep their occupancy)
// (Called by every thread of the block; wave 0 tokenises, thread 0 walks.)
template <uint32_t DW>
__device__ __forceinline__ uint32_t ds_validate_lds(const uint8_t *D, uint32_t x, uint32_t e, DsLdsT<DW> &L) {
  constexpr uint32_t PB = DW / 64;  // bytes per lane
  const uint32_t t = threadIdx.x, nt = blockDim.x, lane = t & 63;
  for (uint32_t i = t; i < DHS; i += nt) L.hs[i] = NONE;
  if (t == 0) { L.lastc = 0; L.hmax = 0; }
  uint32_t ndc = NONE, nseen = 0, ci = 0;
  bool started = false;
  uint32_t w0 = x;  // window start: a token (varuint) boundary
  for (;;) {
    __syncthreads();
    const uint32_t wl = e - w0 < DW ? e - w0 : DW;  // window bytes
    for (uint32_t q = 16 * t; q < DW; q += 16 * nt) {
      const uint4 v = load16m(D, w0 + q, e);
      __builtin_memcpy(L.b + q, &v, 16);
    }
    __syncthreads();
    if (t < 64) {
    // tokenise: lane l owns bytes [PB l, PB l + PB)
    const uint32_t b0 = PB * lane;
    uint64_t stops = 0;
#pragma unroll
    for (uint32_t k = 0; k < PB; k++) stops |= (uint64_t)((b0 + k < wl) && L.b[b0 + k] < 0x80) << k;
    const uint32_t nst = (uint32_t)__popcll(stops);
    const uint32_t tincl = wave_incl_add(nst), tbase = tincl - nst, ntok = lane_read(tincl, 63);
    // the last stop before this lane's bytes (the previous token's end): a max scan of each lane's last stop
    const uint32_t mylast = stops ? b0 + 63 - __builtin_clzll(stops) : 0;
    uint32_t mx = stops ? mylast + 1 : 0;  // (+1: 0 = none)
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)mx, sh, 64);
      if ((int)lane >= sh) mx = o > mx ? o : mx;
    }
    uint32_t prev = (uint32_t)__shfl_up((int)mx, 1, 64);
    if (lane == 0) prev = 0;
    uint32_t start = prev;  // first byte of this lane's first token (window-relative)
    uint32_t nbad = 0, t = tbase;
    for (uint64_t m = stops; m; m &= m - 1) {
      const uint32_t sp = b0 + (uint32_t)__builtin_ctzll(m);
      const uint32_t nb = sp - start + 1;
      const uint32_t last = L.b[sp];
      uint32_t v = 0;
      bool bad = nb > 5 || (nb > 1 && last == 0) || (nb == 5 && (last & 0x70) != 0);
      if (!bad)
        for (uint32_t q = 0; q < nb; q++) v |= (uint32_t)(L.b[start + q] & 0x7f) << (7 * q);
      L.val[t] = v;
      L.end[t] = (uint16_t)(sp + 1);
      L.badp[t] = (uint16_t)nbad;  // (bad tokens before t within the lane: the lane base is added below)
      nbad += bad;
      start = sp + 1;
      t++;
    }
    const uint32_t bincl = wave_incl_add(nbad), bbase = bincl - nbad;
    for (uint32_t q = tbase; q < tbase + nst; q++) L.badp[q] = (uint16_t)(L.badp[q] + bbase);
    if (lane == 63) { L.badp[ntok] = (uint16_t)bincl; L.ntok = ntok; }
    }
    __syncthreads();
    // thread 0 walks the clients
    uint32_t res = 0;  // 0: next window, else the answer
    if (t == 0) {
      const uint32_t ntok = L.ntok;
      uint32_t tk = 0;
      if (!started) {
        if (ntok == 0) res = NONE;
        else if (L.badp[1] != 0) res = NONE;
        else { ndc = L.val[0]; tk = 1; started = true; }
      }
      while (res == 0) {
        if (ci == ndc) { res = w0 + (tk == 0 ? 0 : L.end[tk - 1]); break; }
        if (tk + 2 > ntok) break;  // the client's header crosses the window end
        const uint32_t client = L.val[tk], m = L.val[tk + 1];
        if (L.badp[tk + 2] != L.badp[tk] || m == 0) { res = NONE; break; }
        if (2ull * m > ntok - tk - 2) {  // its ranges cross the window end
          if (tk == 0) res = DS_BIG;
          break;
        }
        if (L.badp[tk + 2 + 2 * m] != L.badp[tk + 2]) { res = NONE; break; }
        // the hash set (client 0xFFFFFFFF is the empty slot's value: a flag of its own)
        if (client == NONE) {
          if (L.hmax) { res = NONE; break; }
          L.hmax = 1;
        } else {
          uint32_t h = (client * 0x9E3779B1u) >> 21;
          for (;;) {
            const uint32_t k = L.hs[h];
            if (k == client) { res = NONE; break; }
            if (k == NONE) { L.hs[h] = client; break; }
            h = (h + 1) & (DHS - 1);
          }
          if (res) break;
          if (++nseen > DHS * 3 / 4) { res = DS_BIG; break; }
        }
        tk += 2 + 2 * m;
        ci++;
      }
      if (res == 0) {  // next window from the current client's header
        if (tk == 0 && w0 + wl >= e) res = NONE;  // nothing left to read: truncated
        else if (tk == 0) res = DS_BIG;
        else L.lastc = L.end[tk - 1];
      }
      L.wtot = res;
    }
    __syncthreads();
    const uint32_t r = L.wtot;
    if (r != 0) return r;
    w0 += L.lastc;
    if (w0 >= e) return NONE;
  }
}

}  // namespace wds
}  // namespace ymk
