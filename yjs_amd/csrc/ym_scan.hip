// ym_scan.hip -- device-wide exclusive prefix sums and flagged selection (ym_scan.h).
#include <hip/hip_runtime.h>

#include <vector>

#include "ym_scan.h"

namespace ymk {
namespace scan {

constexpr uint32_t T_THREADS = 256, T_ITEMS = 8, TILE = T_THREADS * T_ITEMS;

__device__ __forceinline__ uint32_t count_of(uint32_t n_max, const uint32_t *n_dev, uint32_t n_add) {
  if (!n_dev) return n_max;
  const uint64_t n = (uint64_t)*n_dev + n_add;
  return n < n_max ? (uint32_t)n : n_max;
}

// exclusive sum of v over the block's 256 threads (4 waves); total = the block's sum
template <class T>
__device__ __forceinline__ T block_excl(T v, T &total) {
  __shared__ T wsum[T_THREADS / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  T base = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < T_THREADS / 64; k++) {
    const T s = wsum[k];
    base += k < w ? s : (T)0;
    tot += s;
  }
  __syncthreads();  // (wsum is reused by the next call)
  total = tot;
  return base + x - v;
}

// 1. each tile: its exclusive scan in place, its total to tot[tile]
template <class T>
__global__ void __launch_bounds__(T_THREADS) k_scan_tile(const T *in, T *out, T *tot, uint32_t n_max, const uint32_t *n_dev,
                                                         uint32_t n_add) {
  const uint32_t n = count_of(n_max, n_dev, n_add);
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  if (base >= n) {
    if (threadIdx.x == 0) tot[blockIdx.x] = 0;
    return;
  }
  const uint64_t i0 = base + (uint64_t)T_ITEMS * threadIdx.x;
  T v[T_ITEMS], s = 0;
#pragma unroll
  for (uint32_t k = 0; k < T_ITEMS; k++) {
    v[k] = i0 + k < n ? in[i0 + k] : (T)0;
    s += v[k];
  }
  T total;
  T run = block_excl<T>(s, total);
#pragma unroll
  for (uint32_t k = 0; k < T_ITEMS; k++) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = total;
}
// 2. one block: the tile totals' exclusive scan in place (carried over chunks of TILE); *grand = the sum
template <class T>
__global__ void __launch_bounds__(T_THREADS) k_scan_totals(T *tot, uint32_t ntiles, T *grand) {
  T carry = 0;
  for (uint64_t c = 0; c < ntiles; c += TILE) {
    const uint64_t i0 = c + (uint64_t)T_ITEMS * threadIdx.x;
    T v[T_ITEMS], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < T_ITEMS; k++) {
      v[k] = i0 + k < ntiles ? tot[i0 + k] : (T)0;
      s += v[k];
    }
    T total;
    T run = carry + block_excl<T>(s, total);
#pragma unroll
    for (uint32_t k = 0; k < T_ITEMS; k++) {
      if (i0 + k < ntiles) tot[i0 + k] = run;
      run += v[k];
    }
    carry += total;
  }
  if (grand && threadIdx.x == 0) *grand = carry;
}
// 3. each tile after the first: its base added
template <class T>
__global__ void __launch_bounds__(T_THREADS) k_scan_add(T *out, const T *tot, uint32_t n_max, const uint32_t *n_dev, uint32_t n_add) {
  if (blockIdx.x == 0) return;
  const uint32_t n = count_of(n_max, n_dev, n_add);
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  if (base >= n) return;
  const T add = tot[blockIdx.x];
  const uint64_t i0 = base + (uint64_t)T_ITEMS * threadIdx.x;
#pragma unroll
  for (uint32_t k = 0; k < T_ITEMS; k++)
    if (i0 + k < n) out[i0 + k] += add;
}

// selection: per tile the number of flagged elements
__global__ void __launch_bounds__(T_THREADS) k_sel_count(const uint8_t *flags, uint32_t *cnt, uint32_t n) {
  const uint64_t i0 = (uint64_t)blockIdx.x * TILE + (uint64_t)T_ITEMS * threadIdx.x;
  uint32_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < T_ITEMS; k++) s += i0 + k < n && flags[i0 + k] != 0;
  uint32_t total;
  block_excl<uint32_t>(s, total);
  if (threadIdx.x == 0) cnt[blockIdx.x] = total;
}
__global__ void __launch_bounds__(T_THREADS) k_sel_scatter(const uint32_t *list, const uint8_t *flags, uint32_t *dst,
                                                           const uint32_t *cnt, uint32_t n) {
  const uint64_t i0 = (uint64_t)blockIdx.x * TILE + (uint64_t)T_ITEMS * threadIdx.x;
  uint8_t f[T_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < T_ITEMS; k++) {
    f[k] = i0 + k < n && flags[i0 + k] != 0;
    s += f[k];
  }
  uint32_t total;
  uint32_t pos = cnt[blockIdx.x] + block_excl<uint32_t>(s, total);
#pragma unroll
  for (uint32_t k = 0; k < T_ITEMS; k++)
    if (f[k]) dst[pos++] = list ? list[i0 + k] : (uint32_t)(i0 + k);
}

}  // namespace scan

template <class T>
int scan_excl(void *tmp, size_t &tmp_bytes, const T *in, T *out, uint32_t n_max, hipStream_t st, const uint32_t *n_dev,
              uint32_t n_add) {
  using namespace scan;
  const uint32_t ntiles = (uint32_t)(((uint64_t)n_max + TILE - 1) / TILE);
  const size_t need = sizeof(T) * ((size_t)ntiles + 1) + 16;
  if (!tmp) {
    tmp_bytes = need;
    return 0;
  }
  if (tmp_bytes < need) return -1;
  if (ntiles == 0) return 0;
  T *tot = (T *)tmp;
  k_scan_tile<T><<<ntiles, T_THREADS, 0, st>>>(in, out, tot, n_max, n_dev, n_add);
  if (ntiles > 1) {
    k_scan_totals<T><<<1, T_THREADS, 0, st>>>(tot, ntiles, nullptr);
    k_scan_add<T><<<ntiles, T_THREADS, 0, st>>>(out, tot, n_max, n_dev, n_add);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
template int scan_excl<uint32_t>(void *, size_t &, const uint32_t *, uint32_t *, uint32_t, hipStream_t, const uint32_t *, uint32_t);
template int scan_excl<uint64_t>(void *, size_t &, const uint64_t *, uint64_t *, uint32_t, hipStream_t, const uint32_t *, uint32_t);

int select_flagged(void *tmp, size_t &tmp_bytes, const uint32_t *list, const uint8_t *flags, uint32_t *dst, uint32_t *d_num,
                   uint32_t n, hipStream_t st) {
  using namespace scan;
  const uint32_t ntiles = (uint32_t)(((uint64_t)n + TILE - 1) / TILE);
  const size_t need = 4 * ((size_t)ntiles + 1) + 16;
  if (!tmp) {
    tmp_bytes = need;
    return 0;
  }
  if (tmp_bytes < need) return -1;
  if (ntiles == 0) return hipMemsetAsync(d_num, 0, 4, st) == hipSuccess ? 0 : -1;
  uint32_t *cnt = (uint32_t *)tmp;
  k_sel_count<<<ntiles, T_THREADS, 0, st>>>(flags, cnt, n);
  k_scan_totals<uint32_t><<<1, T_THREADS, 0, st>>>(cnt, ntiles, d_num);
  k_sel_scatter<<<ntiles, T_THREADS, 0, st>>>(list, flags, dst, cnt, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ymk

// Test hook (tests/test_gpu_scan.py): scans and selections of n pseudo-random elements on the device against a
// host computation; also a device-side count (n_dev = n / 2).  Returns the number of mismatching outputs (< 0:
// HIP error).
extern "C" int ym__scan_check(uint32_t n, uint32_t seed) {
  using namespace ymk;
  std::vector<uint32_t> a(n + 1);
  std::vector<uint64_t> b(n + 1);
  std::vector<uint8_t> f(n + 1);
  uint32_t x = seed * 2654435761u + 12345u;
  for (uint32_t i = 0; i <= n; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    a[i] = x & 1023u;
    b[i] = ((uint64_t)x << 20) ^ i;
    f[i] = (x >> 11) % 3 == 0;
  }
  uint32_t *da, *dao, *dn, *dsel, *dnum;
  uint64_t *db, *dbo;
  uint8_t *df;
  void *tmp;
  hipMalloc(&da, 4ull * (n + 1)); hipMalloc(&dao, 4ull * (n + 1)); hipMalloc(&db, 8ull * (n + 1)); hipMalloc(&dbo, 8ull * (n + 1));
  hipMalloc(&df, n + 1); hipMalloc(&dn, 4); hipMalloc(&dsel, 4ull * (n + 1)); hipMalloc(&dnum, 4);
  hipMemcpy(da, a.data(), 4ull * (n + 1), hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 8ull * (n + 1), hipMemcpyHostToDevice);
  hipMemcpy(df, f.data(), n + 1, hipMemcpyHostToDevice);
  const uint32_t half = n / 2;
  hipMemcpy(dn, &half, 4, hipMemcpyHostToDevice);
  size_t t1 = 0, t2 = 0, t3 = 0;
  scan_excl<uint32_t>(nullptr, t1, da, dao, n, nullptr);
  scan_excl<uint64_t>(nullptr, t2, db, dbo, n, nullptr);
  select_flagged(nullptr, t3, nullptr, df, dsel, dnum, n, nullptr);
  size_t t = t1 > t2 ? t1 : t2;
  t = t > t3 ? t : t3;
  hipMalloc(&tmp, t);
  int bad = 0;
  std::vector<uint32_t> ao(n + 1), so(n + 1);
  std::vector<uint64_t> bo(n + 1);
  uint32_t num = 0;
  if (scan_excl<uint32_t>(tmp, t, da, dao, n, nullptr) || scan_excl<uint64_t>(tmp, t, db, dbo, n, nullptr)) bad = -1;
  hipMemcpy(ao.data(), dao, 4ull * n, hipMemcpyDeviceToHost);
  hipMemcpy(bo.data(), dbo, 8ull * n, hipMemcpyDeviceToHost);
  uint32_t ra = 0;
  uint64_t rb = 0;
  for (uint32_t i = 0; i < n && bad >= 0; i++) {
    bad += ao[i] != ra || bo[i] != rb;
    ra += a[i];
    rb += b[i];
  }
  // device-side count: only the first n / 2 outputs written (in place), the rest untouched
  hipMemcpy(dao, a.data(), 4ull * (n + 1), hipMemcpyHostToDevice);
  if (bad >= 0 && scan_excl<uint32_t>(tmp, t, dao, dao, n, nullptr, dn, 0)) bad = -1;
  hipMemcpy(ao.data(), dao, 4ull * n, hipMemcpyDeviceToHost);
  ra = 0;
  for (uint32_t i = 0; i < n && bad >= 0; i++) {
    bad += ao[i] != (i < half ? ra : a[i]);
    ra += a[i];
  }
  if (bad >= 0 && select_flagged(tmp, t, nullptr, df, dsel, dnum, n, nullptr)) bad = -1;
  hipMemcpy(&num, dnum, 4, hipMemcpyDeviceToHost);
  hipMemcpy(so.data(), dsel, 4ull * n, hipMemcpyDeviceToHost);
  uint32_t q = 0;
  for (uint32_t i = 0; i < n && bad >= 0; i++)
    if (f[i]) bad += q >= num || so[q++] != i;
  if (bad >= 0) bad += q != num;
  hipFree(da); hipFree(dao); hipFree(db); hipFree(dbo); hipFree(df); hipFree(dn); hipFree(dsel); hipFree(dnum); hipFree(tmp);
  return hipGetLastError() == hipSuccess ? bad : -2;
}
