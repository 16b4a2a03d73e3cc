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

}  // namespace wds
}  // namespace ymk
