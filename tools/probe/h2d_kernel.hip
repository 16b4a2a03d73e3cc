// Host-to-device rates on the box: an SDMA copy (hipMemcpyAsync) from page-locked memory against a kernel
// that reads the page-locked memory itself (16-byte loads, UNROLL in flight per thread) and writes it to HBM.
// Build: hipcc -O3 --offload-arch=gfx950 h2d_kernel.hip -o h2d_kernel
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

template <int UNROLL>
__global__ void __launch_bounds__(256) k_copy(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) dst[i + u * stride] = v[u];
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

int main() {
  const size_t bytes = 24ull << 20, n = bytes / 16;
  for (int nc = 0; nc < 2; nc++) {
    void *h;
    hipHostMalloc(&h, bytes, hipHostMallocPortable | (nc ? hipHostMallocNonCoherent : 0));
    memset(h, 1, bytes);
    void *d;
    hipMalloc(&d, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms;
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(a, 0);
      hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, 0);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("nc=%d sdma H2D %.1f GB/s\n", nc, bytes / ms / 1e6);
    }
    for (int grid : {256, 1024, 4096}) {
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(a, 0);
        k_copy<4><<<grid, 256, 0, 0>>>((const uint4 *)h, (uint4 *)d, n);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("nc=%d kernel read grid %d unroll 4: %.1f GB/s\n", nc, grid, bytes / ms / 1e6);
      }
      hipEventRecord(a, 0);
      k_copy<1><<<grid, 256, 0, 0>>>((const uint4 *)h, (uint4 *)d, n);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("nc=%d kernel read grid %d unroll 1: %.1f GB/s\n", nc, grid, bytes / ms / 1e6);
    }
    hipFree(d);
    hipHostFree(h);
  }
  return 0;
}
