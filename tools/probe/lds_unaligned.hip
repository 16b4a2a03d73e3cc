// Probe: do unaligned 4/8/16-byte LDS loads and stores behave like byte-wise accesses on gfx950?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k(uint64_t *out, uint32_t *out32, uint8_t *outb) {
  __shared__ uint8_t sm[1024];
  const uint32_t l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) sm[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  typedef uint64_t __attribute__((aligned(1))) u64u;
  typedef uint32_t __attribute__((aligned(1))) u32u;
  const uint32_t p = l * 13 + 1;                     // every alignment
  out[l] = *(const u64u *)(sm + p);
  out32[l] = *(const u32u *)(sm + p + 2);
  __syncthreads();
  if (l < 32) *(u32u *)(sm + 512 + l * 5 + 1) = 0xA1B2C3D4u + l;   // unaligned stores, disjoint
  if (l >= 32) *(u64u *)(sm + 700 + (l - 32) * 9 + 3) = 0x1122334455667788ull + l;
  __syncthreads();
  for (int i = l; i < 1024; i += 64) outb[i] = sm[i];
}
int main() {
  uint64_t *o; uint32_t *o32; uint8_t *ob;
  hipMalloc(&o, 64 * 8); hipMalloc(&o32, 64 * 4); hipMalloc(&ob, 1024);
  k<<<1, 64>>>(o, o32, ob);
  uint64_t h[64]; uint32_t h32[64]; uint8_t hb[1024];
  hipMemcpy(h, o, 512, hipMemcpyDeviceToHost); hipMemcpy(h32, o32, 256, hipMemcpyDeviceToHost); hipMemcpy(hb, ob, 1024, hipMemcpyDeviceToHost);
  uint8_t ref[1024];
  for (int i = 0; i < 1024; i++) ref[i] = (uint8_t)(i * 7 + 3);
  int bad = 0;
  for (int l = 0; l < 64; l++) {
    uint64_t e = 0; uint32_t e32 = 0; uint32_t p = l * 13 + 1;
    for (int b = 7; b >= 0; b--) e = (e << 8) | ref[p + b];
    for (int b = 3; b >= 0; b--) e32 = (e32 << 8) | ref[p + 2 + b];
    if (e != h[l] || e32 != h32[l]) bad++;
  }
  for (int l = 0; l < 32; l++) { uint32_t v = 0xA1B2C3D4u + l; for (int b = 0; b < 4; b++) ref[512 + l * 5 + 1 + b] = (uint8_t)(v >> (8 * b)); }
  for (int l = 32; l < 64; l++) { uint64_t v = 0x1122334455667788ull + l; for (int b = 0; b < 8; b++) ref[700 + (l - 32) * 9 + 3 + b] = (uint8_t)(v >> (8 * b)); }
  for (int i = 0; i < 1024; i++) bad += hb[i] != ref[i];
  printf("lds unaligned probe: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad != 0;
}
