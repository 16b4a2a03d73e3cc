// ym_segsort.hip -- segmented LSD radix sort of (u64 key, u32 value) pairs, one workgroup per segment.
//
// The large-document merge (ym_large.hip) sorts each document's client runs by (~client << 32 | clock) and
// its delete ranges by (client << 32 | clock), ascending and stable (equal keys keep their emission order,
// which the delete set's first-appearance ranking reads).  A C5 document has ~16 k runs: one 1024-thread
// workgroup owns the segment, so there is no device-wide pass and no inter-workgroup synchronisation.
//
//   histogram  one read of the segment counts all eight 8-bit digits at once (8 x 256 LDS counters); a
//              digit with one non-empty bin permutes nothing and is skipped (clock high bytes, the
//              complemented client's constant bytes in small documents)
//   passes     per kept digit, tiles of 1024 pairs in segment order: each wave ranks its 64 lanes by digit
//              with eight ballots (the lanes of equal digit: their mask; rank = earlier lanes in it), the
//              16 waves' counts are scanned per digit in LDS, and each pair is stored at
//              bucket base + earlier waves' count + rank -- stable by construction; the bucket bases carry
//              across tiles
//   buffers    passes ping-pong between the output and a scratch pair, ordered so the last pass lands in
//              the output; a segment of fewer than two pairs, or one whose every digit is skipped, is
//              copied
//   small      a segment of at most 4096 pairs is sorted inside LDS (one read, one write)
// The workgroup's global stores are read back by the same workgroup after a barrier (one CU, one L1: the
// workgroup-scope acquire of __syncthreads suffices).
#include <hip/hip_runtime.h>

#include "ym_kernels.h"

namespace ymk {
namespace ss {

constexpr uint32_t T = 1024, NWV = T / 64, RB = 8, NB = 1u << RB, SMALL = 4096;

struct Lds {
  uint32_t hist[8][NB];     // digit histograms of the segment
  uint32_t wcnt[NWV][NB];   // a tile's per-wave digit counts, then their exclusive prefix over waves
  uint32_t base[NB];        // bucket bases (carried across tiles)
  uint32_t ttot[NB];        // the tile's digit totals
  unsigned long long sk[2][SMALL];  // small segments: keys (ping-pong)
  uint32_t sv[2][SMALL];            //                 values
};

__device__ __forceinline__ uint32_t digit(unsigned long long k, uint32_t i) { return (uint32_t)(k >> (RB * i)) & (NB - 1); }

// stable rank of this lane's digit dg among the wave's valid lanes; returns the rank, sets the equal-digit mask
__device__ __forceinline__ uint32_t wave_rank(uint32_t dg, bool valid, unsigned long long &eq) {
  unsigned long long m = __ballot(valid);
#pragma unroll
  for (uint32_t b = 0; b < RB; b++) {
    const unsigned long long bb = __ballot((dg >> b) & 1);
    m &= ((dg >> b) & 1) ? bb : ~bb;
  }
  eq = m;
  const uint32_t lane = threadIdx.x & 63;
  return (uint32_t)__popcll(m & ((1ull << lane) - 1));
}

// one tile of up to T pairs (this thread's pair: k, v, valid) ranked by digit i and stored at dst
template <bool LDS_DST>
__device__ __forceinline__ void tile_scatter(Lds &L, unsigned long long k, uint32_t v, bool valid, uint32_t i,
                                             unsigned long long *dk, uint32_t *dv) {
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
  const uint32_t dg = valid ? digit(k, i) : 0;
  unsigned long long eq;
  const uint32_t r = wave_rank(dg, valid, eq);
  for (uint32_t q = t; q < NWV * NB; q += T) (&L.wcnt[0][0])[q] = 0;
  __syncthreads();
  if (valid && lane == (uint32_t)__builtin_ctzll(eq)) L.wcnt[w][dg] = (uint32_t)__popcll(eq);
  __syncthreads();
  if (t < NB) {  // per digit: exclusive prefix over the waves
    uint32_t s = 0;
#pragma unroll
    for (uint32_t x = 0; x < NWV; x++) { const uint32_t c = L.wcnt[x][t]; L.wcnt[x][t] = s; s += c; }
    L.ttot[t] = s;
  }
  __syncthreads();
  if (valid) {
    const uint32_t pos = L.base[dg] + L.wcnt[w][dg] + r;
    dk[pos] = k;
    dv[pos] = v;
  }
  __syncthreads();
  if (t < NB) L.base[t] += L.ttot[t];
  (void)LDS_DST;
}

__global__ void __launch_bounds__(T) k_segsort(const unsigned long long *ki, const uint32_t *vi, unsigned long long *ko,
                                               uint32_t *vo, unsigned long long *kt, uint32_t *vt, const uint32_t *seg_b,
                                               const uint32_t *seg_e) {
  __shared__ Lds L;
  const uint32_t t = threadIdx.x, s = blockIdx.x;
  const uint32_t b = seg_b[s], e = seg_e[s];
  if (e <= b) return;
  const uint32_t n = e - b;
  // histograms of all digits
  for (uint32_t q = t; q < 8 * NB; q += T) (&L.hist[0][0])[q] = 0;
  __syncthreads();
  for (uint32_t q = t; q < n; q += T) {
    const unsigned long long k = ki[b + q];
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) atomicAdd(&L.hist[i][digit(k, i)], 1u);
  }
  __syncthreads();
  // the digits that permute: a bin holding all n pairs means the digit is constant
  __shared__ uint32_t s_keep;
  if (t == 0) s_keep = 0;
  __syncthreads();
  if (t < 8) {
    bool constant = false;
    for (uint32_t x = 0; x < NB && !constant; x++) constant = L.hist[t][x] == n;
    if (!constant) atomicOr(&s_keep, 1u << t);
  }
  __syncthreads();
  const uint32_t keep = s_keep;
  const uint32_t npass = __popc(keep);
  if (npass == 0 || n < 2) {
    for (uint32_t q = t; q < n; q += T) { ko[b + q] = ki[b + q]; vo[b + q] = vi[b + q]; }
    return;
  }
  if (n <= SMALL) {  // in LDS: load, the passes between the two LDS buffers, store
    for (uint32_t q = t; q < n; q += T) { L.sk[0][q] = ki[b + q]; L.sv[0][q] = vi[b + q]; }
    uint32_t cur = 0;
    for (uint32_t i = 0; i < 8; i++) {
      if (!(keep >> i & 1)) continue;
      __syncthreads();
      if (t < NB) {  // bucket bases: exclusive scan of the digit's histogram
        uint32_t sacc = 0;
        for (uint32_t x = 0; x < t; x++) sacc += L.hist[i][x];
        L.base[t] = sacc;
      }
      __syncthreads();
      for (uint32_t q0 = 0; q0 < n; q0 += T) {
        const uint32_t q = q0 + t;
        const bool valid = q < n;
        const unsigned long long k = valid ? L.sk[cur][q] : 0;
        const uint32_t v = valid ? L.sv[cur][q] : 0;
        tile_scatter<true>(L, k, v, valid, i, L.sk[cur ^ 1], L.sv[cur ^ 1]);
      }
      cur ^= 1;
    }
    __syncthreads();
    for (uint32_t q = t; q < n; q += T) { ko[b + q] = L.sk[cur][q]; vo[b + q] = L.sv[cur][q]; }
    return;
  }
  // in HBM: pass p of npass writes to the output when (npass - 1 - p) is even, else to the scratch pair
  const unsigned long long *sk = ki + b;
  const uint32_t *sv = vi + b;
  uint32_t p = 0;
  for (uint32_t i = 0; i < 8; i++) {
    if (!(keep >> i & 1)) continue;
    unsigned long long *dk = ((npass - 1 - p) & 1) ? kt + b : ko + b;
    uint32_t *dv = ((npass - 1 - p) & 1) ? vt + b : vo + b;
    __syncthreads();
    if (t < NB) {
      uint32_t sacc = 0;
      for (uint32_t x = 0; x < t; x++) sacc += L.hist[i][x];
      L.base[t] = sacc;
    }
    __syncthreads();
    // tiles in segment order, the next tile's pair loaded before this one is ranked
    bool valid = t < n;
    unsigned long long k = valid ? sk[t] : 0;
    uint32_t v = valid ? sv[t] : 0;
    for (uint32_t q0 = 0; q0 < n; q0 += T) {
      const uint32_t qn = q0 + T + t;
      const bool vn = qn < n;
      const unsigned long long kn = vn ? sk[qn] : 0;
      const uint32_t vnn = vn ? sv[qn] : 0;
      tile_scatter<false>(L, k, v, valid, i, dk, dv);
      k = kn;
      v = vnn;
      valid = vn;
    }
    __syncthreads();
    sk = dk;
    sv = dv;
    p++;
  }
}

}  // namespace ss

// segments [seg_b[s], seg_e[s]) of (ki, vi) sorted by key, stable, into (ko, vo); (kt, vt): scratch of the
// same size; the pairs outside every segment are not written
int segsort_pairs(const uint64_t *ki, const uint32_t *vi, uint64_t *ko, uint32_t *vo, uint64_t *kt, uint32_t *vt,
                  const uint32_t *seg_b, const uint32_t *seg_e, uint32_t nseg, hipStream_t st) {
  if (nseg == 0) return 0;
  ss::k_segsort<<<nseg, ss::T, 0, st>>>(reinterpret_cast<const unsigned long long *>(ki), vi,
                                        reinterpret_cast<unsigned long long *>(ko), vo,
                                        reinterpret_cast<unsigned long long *>(kt), vt, seg_b, seg_e);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ymk

// test entry: one call of the segmented sort on device buffers (tests/test_gpu_segsort.py)
extern "C" int ym__segsort(const uint64_t *ki, const uint32_t *vi, uint64_t *ko, uint32_t *vo, uint64_t *kt, uint32_t *vt,
                           const uint32_t *seg_b, const uint32_t *seg_e, uint32_t nseg) {
  const int r = ymk::segsort_pairs(ki, vi, ko, vo, kt, vt, seg_b, seg_e, nseg, 0);
  return r != 0 ? r : (hipDeviceSynchronize() == hipSuccess ? 0 : -2);
}
