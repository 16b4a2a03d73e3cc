// ym_api.hip -- host side of libymerge.so: the C ABI of include/ymerge.h.
//
// Per call: (1) the LDS fast path (ym_fast.hip) takes every document it can prove simple and writes
// its output; (2) the remaining documents are compacted into a list and run through the general
// path (ym_general.hip) with an HBM workspace sized by an exclusive scan; (3) outputs are bump-
// allocated in the caller's arena.  Host-memory batches are staged through device buffers.
#include <hip/hip_runtime.h>
#include "ym_scan.h"

#include <atomic>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <vector>

#include "../../include/ymerge.h"
#include "ym_kernels.h"

namespace ymk {
__global__ void k_general_ws(GeneralJob j, uint64_t *ws_size);
__global__ void k_general(GeneralJob j, int pass);
int fast_launch(uint32_t op, const GeneralJob &j, uint32_t n_upd, hipStream_t st);  // ym_fast.hip
int fast_nested_launch(const GeneralJob &j, uint32_t n, hipStream_t st);  // ym_fast.hip
int fast2_nested_launch(const GeneralJob &j, uint32_t n, hipStream_t st);  // ym_fast2.hip
int fast2_launch(uint32_t op, const GeneralJob &j, uint32_t n_upd, hipStream_t st); // ym_fast2.hip
int big_launch(uint32_t op, const GeneralJob &j, hipStream_t st, PwBufs &pw);       // ym_big.hip
int big2_launch(uint32_t op, const GeneralJob &j, hipStream_t st, PwBufs &pw);      // ym_big2.hip
int big_async_launch(uint32_t op, const GeneralJob &j, uint8_t *done, uint32_t grid_max, hipStream_t st);   // ym_big.hip
int big2_async_launch(uint32_t op, const GeneralJob &j, uint8_t *done, uint32_t grid_max, hipStream_t st);  // ym_big2.hip
__global__ void k_fast_region(GeneralJob j, uint32_t n_upd);                         // ym_fast.hip
__global__ void k_compact_ws(GeneralJob j, uint64_t *ws_size);                        // ym_compact.hip
template <int OCC> __global__ void k_compact(GeneralJob j, uint32_t lanes, uint64_t big, int part);
}  // namespace ymk

using namespace ymk;

namespace {

#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t e_ = (x);                            \
    if (e_ != hipSuccess) return -(int)e_ - 1000;   \
  } while (0)

struct DBuf {
  void *p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = n + n / 4 + 4096;
    if (hipMalloc(&p, want) != hipSuccess) return -1;
    cap = want;
    return 0;
  }
  template <class T> T *as() const { return (T *)p; }
};

struct DevState {
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evf0 = nullptr, evf1 = nullptr, evg1 = nullptr;
  DBuf ws, ws_size, ws_off, layout, counters, scan_tmp, list_a, list_b, flags, bscratch;
  DBuf in_arena, in_off, in_doc, in_sv, in_svoff, out_arena, out_off, out_len, status;  // host staging
  DBuf cmp_off, cmp_len, cmp_arena;  // host batches: outputs packed in document order before the D2H copy
  DBuf async_off;                    // ym_merge_async: its own widened offsets (not in_off: the synchronous
  hipEvent_t ev_async = nullptr;     // calls write that one on their streams), guarded by this event
  // ym_diff_async / ym_sv_async: counters + done flags, per-block walker scratch, widened offsets, guarded
  // by ev_async2 (each such call waits on the device for the previous one)
  DBuf async2_ws, async2_bs, async2_off;
  hipEvent_t ev_async2 = nullptr;
  LargeBufs large;
  PwBufs pw, pw2;
  hipEvent_t evl1 = nullptr, evn0 = nullptr, evn1 = nullptr;
  uint64_t *pinned = nullptr;   // host memory the finishing kernel writes into (no copy op)
  uint64_t *pinned_dev = nullptr;  // ... its device address
  bool dirty = true;            // device counters not known to be reset (first call, failed call)
  uint64_t seq = 0;             // call sequence number: the fast paths' completion flag (pinned[7])
  uint64_t min_stage_cap = 0;   // host batches: staging capacity learnt from an overflowing call
  // merges (per format): the last calls' batches were mostly rich content (nested payloads), so the next one
  // starts with the nested LDS pass instead of a hot pass that would decline most documents; re-probed with
  // the hot pass every NESTED_PROBE calls
  uint32_t nested_first[2] = {0, 0};
  // pipelined host merges (run_host_pipe): copy streams, per-chunk events, the u32 offsets' staging buffer and
  // the mapped host words the per-chunk scan kernels write (chunk output ranges, declined count)
  hipStream_t s_h2d = nullptr, s_h2d2 = nullptr, s_d2h = nullptr;
  hipEvent_t pev_h[16] = {}, pev_h2[16] = {}, pev_k[16] = {}, pev_p[16] = {};
  DBuf in_off32;
  uint64_t *pipe_host = nullptr, *pipe_host_dev = nullptr;
  bool pipe_skip = false;  // the pipelined call's own fallback runs the unpipelined flow
};

// Device state is per (thread, device): a thread may drive several devices in turn (ym_init switches
// its current one and keeps the others' streams and workspaces), and a thread that never called
// ym_init starts on the device the last ym_init of the process selected (else YMERGE_DEVICE, else the
// HIP current device).
constexpr int kMaxDevices = 64;
thread_local DevState *g_states[kMaxDevices] = {};
thread_local DevState *g_state = nullptr;
std::atomic<int> g_default_device{-1};
std::mutex g_mu;

DevState *state() {
  if (!g_state) {
    int dev = g_default_device.load();
    if (dev < 0) {
      const char *env = getenv("YMERGE_DEVICE");
      if (env) dev = atoi(env);
      else hipGetDevice(&dev);
    }
    if (dev < 0 || dev >= kMaxDevices) dev = 0;
    if (!g_states[dev]) { g_states[dev] = new DevState(); g_states[dev]->device = dev; }
    g_state = g_states[dev];
  }
  if (!g_state->stream) {
    hipSetDevice(g_state->device);
    hipStreamCreateWithFlags(&g_state->stream, hipStreamNonBlocking);
    hipEventCreate(&g_state->ev0);
    hipEventCreate(&g_state->ev1);
    hipEventCreate(&g_state->evf0);
    hipEventCreate(&g_state->evf1);
    hipEventCreate(&g_state->evg1);
    hipEventCreate(&g_state->evl1);
    hipEventCreate(&g_state->evn0);
    hipEventCreate(&g_state->evn1);
    // fine-grained (coherent) host memory: the finishing kernel's stores reach it directly
    hipHostMalloc((void **)&g_state->pinned, 64 * sizeof(uint64_t), hipHostMallocCoherent | hipHostMallocMapped);
    hipHostGetDevicePointer((void **)&g_state->pinned_dev, g_state->pinned, 0);
  }
  return g_state;
}

// host batches: document d's output moves to the packed offset cmp_off[d] (exclusive scan of the masked
// lengths), so the device-to-host copy carries the outputs only, not the fast paths' sparse slot region
// (k_pack_docs, one wave per document).  pack_load16: 16 bytes at any source offset from two aligned 16-byte
// loads and a byte funnel shift (reads <= 31 bytes past s, inside the arena's padding).
__device__ inline uint4 pack_load16(const uint8_t *src, uint64_t s) {
  const uint64_t a = s & ~15ull;
  const uint32_t sh = (uint32_t)(s & 15);
  const uint4 x = *reinterpret_cast<const uint4 *>(src + a);
  if (sh == 0) return x;
  const uint4 y = *reinterpret_cast<const uint4 *>(src + a + 16);
  const uint32_t d[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  const uint32_t dw = sh >> 2, bs = sh & 3;
  uint32_t r[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    uint32_t l = d[k], h = d[k + 1];
#pragma unroll
    for (uint32_t t = 1; t < 4; t++) {
      l = dw == t ? d[k + t] : l;
      h = dw == t ? d[k + t + 1] : h;
    }
    r[k] = __builtin_amdgcn_alignbyte(h, l, bs);
  }
  return make_uint4(r[0], r[1], r[2], r[3]);
}

// ---- pipelined host merges (run_host_pipe) ----------------------------------------------------------
// One block per chunk: the exclusive scan of the chunk's masked output lengths, placed after the outputs of
// the chunks before it (`running` carries the packed total from chunk to chunk in stream order).  The chunk's
// packed range goes to mapped host memory (hw[2c], hw[2c + 1]) so the host can start its device-to-host copy
// while later chunks are still being copied in or merged; the last chunk also reports the declined count
// (hw[62]) and the documents that are not YM_OK (hw[61]).
__device__ inline uint64_t blk_excl64(uint64_t x, uint64_t *s_w, uint64_t &total) {
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, nw = blockDim.x >> 6;
  uint64_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) s_w[w] = incl;
  __syncthreads();
  uint64_t before = 0;
  total = 0;
  for (uint32_t k = 0; k < nw; k++) {
    const uint64_t v = s_w[k];
    before += k < w ? v : 0;
    total += v;
  }
  __syncthreads();
  return before + incl - x;
}
__global__ void __launch_bounds__(1024) k_chunk_scan(const int32_t *status, const uint64_t *len, uint32_t n, uint64_t *cmp_off,
                                                     uint64_t *cmp_len, uint64_t *running, volatile uint64_t *hw, uint32_t c,
                                                     const uint32_t *pend, int last, uint64_t *h_off, uint64_t *h_len,
                                                     int32_t *h_st) {
  __shared__ uint64_t s_w[16];
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x;
  if (t == 0) s_bad = 0;
  __syncthreads();
  const uint64_t base = running[0];
  uint64_t carry = 0;
  uint32_t bad = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += blockDim.x) {
    const uint32_t i = t0 + t;
    const int32_t sv = i < n ? status[i] : 0;
    const uint64_t x = i < n && sv == 0 ? len[i] : 0;
    bad += i < n && sv != 0;
    uint64_t tot;
    const uint64_t ex = blk_excl64(x, s_w, tot);
    if (i < n) {
      cmp_off[i] = base + carry + ex;
      cmp_len[i] = x;
      if (h_off) { h_off[i] = base + carry + ex; h_len[i] = x; h_st[i] = sv; }  // host memory, over PCIe
    }
    carry += tot;
  }
  if (bad) atomicAdd(&s_bad, bad);
  __syncthreads();
  if (t == 0) {
    running[0] = base + carry;
    running[1] += s_bad;
    hw[2 * c] = base;
    hw[2 * c + 1] = base + carry;
    if (last) { hw[61] = running[1]; hw[62] = *pend; }
    __threadfence_system();
  }
}
// one wave per document: its output from the fast path's slot to its packed place (16-byte stores)
// (dst may be page-locked host memory: the stores then cross PCIe as 16-byte writes; a document past `cap` is
// not written, the host reports YM_ERR_CAPACITY)
// h_off / h_len / h_st (pipelined host merges with page-locked result arrays, else nullptr): document d's packed
// offset, length and status go to host memory here, one lane each, on the output stream -- written by the
// placement scan instead, these ~20 B PCIe stores per document held the compute stream ~50 us per chunk
__global__ void __launch_bounds__(256) k_pack_docs(const uint8_t *src, const uint64_t *src_off, const uint64_t *dst_off,
                                                   const uint64_t *len, uint32_t n, uint8_t *dst, uint64_t cap,
                                                   const int32_t *st = nullptr, uint64_t *h_off = nullptr,
                                                   uint64_t *h_len = nullptr, int32_t *h_st = nullptr) {
  const uint32_t lane = threadIdx.x & 63;
  // (a grid smaller than n / 4 blocks loops: the pipelined path keeps its packing waves few, so the next
  // chunk's merge kernel, running beside them, keeps its wave slots)
  for (uint32_t d = blockIdx.x * 4 + (threadIdx.x >> 6); d < n; d += gridDim.x * 4) {
    const uint64_t L = len[d];
    if (h_off) {
      if (lane == 0) h_off[d] = dst_off[d];
      else if (lane == 1) h_len[d] = L;
      else if (lane == 2) h_st[d] = st[d];
    }
    if (L == 0) continue;
    const uint64_t so = src_off[d], dof = dst_off[d];
    if (dof + L > cap) continue;
    const uint32_t head0 = (uint32_t)((16 - (dof & 15)) & 15);
    const uint64_t h = head0 < L ? head0 : L;
    if (lane < h) dst[dof + lane] = src[so + lane];
    const uint64_t body = (L - h) & ~15ull;
    for (uint64_t k = (uint64_t)lane * 16; k < body; k += 64 * 16)
      *reinterpret_cast<uint4 *>(dst + dof + h + k) = pack_load16(src, so + h + k);
    for (uint64_t i = h + body + lane; i < L; i += 64) dst[dof + i] = src[so + i];
  }
}

// Host -> HBM copy kernel (pipelined host merges with the batch in page-locked pool memory): up to three
// 16-byte-granular segments, 16-byte loads of the host memory, four in flight per thread.  On the box it moves
// 50-56 GB/s, as an SDMA copy does (tools/probe/h2d_kernel.hip), without the DMA queue's per-copy setup gaps
// and its occasional multi-millisecond stalls.
struct H2dSeg {
  const uint4 *src;
  uint4 *dst;
  uint64_t n;  // 16-byte words
};
__global__ void __launch_bounds__(256) k_h2d_copy(H2dSeg s0, H2dSeg s1, H2dSeg s2) {
  const uint64_t n01 = s0.n + s1.n, total = n01 + s2.n;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  auto at = [&](uint64_t i, const uint4 *&src, uint4 *&dst) {
    if (i < s0.n) { src = s0.src + i; dst = s0.dst + i; }
    else if (i < n01) { src = s1.src + (i - s0.n); dst = s1.dst + (i - s0.n); }
    else { src = s2.src + (i - n01); dst = s2.dst + (i - n01); }
  };
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < total; i += 4 * stride) {
    const uint4 *sp[4];
    uint4 *dp[4];
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) at(i + u * stride, sp[u], dp[u]);
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = *sp[u];
#pragma unroll
    for (int u = 0; u < 4; u++) *dp[u] = v[u];
  }
  for (; i < total; i += stride) {
    const uint4 *sp;
    uint4 *dp;
    at(i, sp, dp);
    *dp = *sp;
  }
}

// YM_OFF32 offsets widened to u64 for the kernels that read u64 offsets
__global__ void k_widen(const uint32_t *src, uint64_t *dst, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// packed lengths: a document that is not OK contributes nothing (its out_len is reported as 0)
__global__ void k_mask_len(const int32_t *status, const uint64_t *len, uint64_t *mlen, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) mlen[i] = status[i] == 0 ? len[i] : 0;
}

__global__ void k_status_flags(const uint32_t *list, uint32_t n, const int32_t *status, int want, uint8_t *flags) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t d = list ? list[i] : i;
  flags[i] = status[d] == want;
}

// The last kernel of every host round trip (no copy op): writes the bump-allocator position, the
// declined count and (stats) errors / bytes out / bytes in straight into pinned host memory, and resets
// the device counters for the next launch.  Stats: a few blocks, each summing 4,096 documents' status /
// out_len with 16 independent loads per thread (one HBM round trip), partial sums by atomics, and the
// block that finishes last writes the host words (a handful of same-address atomics, not one per doc).
// Counters: [0] used, [2] declined (u32), [8] finished blocks (u32), [9] errors, [10] bytes out,
// [11] documents done by the chunk-parallel walk (reported in host[8]).
// FIN_THREADS threads per block, 16 documents per thread: one 1,024-thread block up to 16 k documents (no
// cross-block atomics), 256-thread blocks of 4,096 documents above that
template <uint32_t FIN_THREADS>
__global__ void __launch_bounds__(FIN_THREADS) k_finish(const int32_t *status, const uint64_t *out_len, uint32_t n,
                                                        const uint64_t *upd_off, const uint32_t *upd_off32,
                                                        uint32_t n_upd, uint64_t *counters,
                                                        volatile uint64_t *host, int stats, int merge, uint64_t seq) {
  __shared__ unsigned long long red[2][FIN_THREADS / 64];
  unsigned long long *c = reinterpret_cast<unsigned long long *>(counters);
  uint64_t err = 0, bytes = 0;
  constexpr uint32_t FIN_DOCS = 16 * FIN_THREADS;
  const uint32_t i0 = blockIdx.x * FIN_DOCS;
  // the host words' inputs (written by earlier kernels, never by k_finish) are loaded first, so their
  // HBM / L2 round trips overlap the stats loads instead of following the reduction one by one
  uint64_t used = 0, in_lo = 0, in_hi = 0, chunked = 0;
  uint32_t declined = 0;
  if (threadIdx.x == 0) {
    used = __hip_atomic_load(&c[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    chunked = __hip_atomic_load(&c[11], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    declined = __hip_atomic_load(reinterpret_cast<uint32_t *>(&c[2]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    in_lo = upd_off32 ? upd_off32[0] : upd_off[0];
    in_hi = upd_off32 ? upd_off32[n_upd] : upd_off[n_upd];
  }
  if (stats) {
    int32_t sv[16];
    uint64_t lv[16];
#pragma unroll
    for (uint32_t t = 0; t < 16; t++) {
      const uint32_t i = i0 + t * FIN_THREADS + threadIdx.x;
      sv[t] = i < n ? status[i] : 0;
      lv[t] = i < n ? out_len[i] : 0;
    }
#pragma unroll
    for (uint32_t t = 0; t < 16; t++) {
      err += sv[t] != 0;
      bytes += sv[t] == 0 ? lv[t] : 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    err += __shfl_down(err, o, 64);
    bytes += __shfl_down(bytes, o, 64);
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = err; red[1][w] = bytes; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint64_t e = 0, b = 0;
  for (uint32_t k = 0; k < FIN_THREADS / 64; k++) { e += red[0][k]; b += red[1][k]; }
  if (gridDim.x > 1) {
    // device-scope atomics are performed when they return: consuming both results orders the
    // finished-block increment after them (no fence: an agent-scope release writes back the L2)
    const unsigned long long r1 = atomicAdd(&c[9], (unsigned long long)e);
    const unsigned long long r2 = atomicAdd(&c[10], (unsigned long long)b);
    asm volatile("" ::"v"(r1), "v"(r2));
    if (atomicAdd(reinterpret_cast<uint32_t *>(&c[8]), 1u) != gridDim.x - 1) return;
    e = atomicAdd(&c[9], 0ull);
    b = atomicAdd(&c[10], 0ull);
  }
  // used: the bump allocator; merges also own the fast / large paths' slot region [0, 2 in + 64 n + 64)
  const uint64_t region = merge ? 2 * (in_hi - in_lo) + 64ull * n + 64 : 0;
  host[0] = used > region ? used : region;
  host[2] = declined;  // declined documents (the work list length)
  host[4] = e;
  host[5] = b;
  host[6] = in_hi - in_lo;
  host[8] = chunked;
  c[11] = 0;
  c[0] = 0;                                     // used := 0, pend_count := 0 and the finish counters:
  reinterpret_cast<uint32_t *>(c)[4] = 0;       // the next launch starts clean (see run_op for the
  c[8] = 0;                                     // general path)
  c[9] = 0;
  c[10] = 0;
  host[7] = seq;                                // completion word (the host spins on it)
}

// Compacts the ids of listed docs whose status == want into `dst`; returns the count.
int select_docs(DevState *S, hipStream_t st, const uint32_t *list, uint32_t n, const int32_t *status, int want,
                uint32_t *dst, uint32_t *count_out) {
  if (S->flags.ensure(n + 1)) return -1;
  k_status_flags<<<(n + 255) / 256, 256, 0, st>>>(list, n, status, want, S->flags.as<uint8_t>());
  uint32_t *d_num = S->counters.as<uint32_t>() + 8;
  size_t tmp = 0;
  select_flagged(nullptr, tmp, list, S->flags.as<uint8_t>(), dst, d_num, n, st);
  if (S->scan_tmp.ensure(tmp + 16)) return -1;
  if (select_flagged(S->scan_tmp.p, tmp, list, S->flags.as<uint8_t>(), dst, d_num, n, st)) return -1;
  HIPCHK(hipMemcpyAsync(S->pinned, d_num, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  *count_out = (uint32_t)(S->pinned[0] & 0xffffffffu);
  return 0;
}

// Doc round-trip compaction (ym_compact.hip) over `list` (n docs, nullptr: all); documents whose workspace
// overflowed run again with 4x the workspace.  The workspaces of one launch are bounded by a device-memory
// budget (YMERGE_COMPACT_WS_GB, default 16 GiB): a list whose workspaces exceed it runs in chunks cut at the
// exclusive scan of the per-document sizes; a document that alone exceeds it, or whose workspace cannot be
// allocated, or that still overflows after the last growth round, reports ST_CAPACITY (the others are not
// affected).
__global__ void k_iota(uint32_t *dst, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = i;
}
__global__ void k_set_status(const uint32_t *list, uint32_t n, int32_t *status, uint64_t *out_len, int from, int to) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t d = list ? list[i] : i;
  if (from < 0 || status[d] == from) { status[d] = to; out_len[d] = 0; }
}
int run_compact(DevState *S, hipStream_t st, GeneralJob j, uint32_t *list, uint32_t n) {
  // read on every call (a process may change them between calls): active lanes (documents) per 64-wide
  // wave -- measured on C2 / C4 (10 k documents): 1: 209 / 268 ms, 8: 110 / 102, 16: 77 / 62, 32: 85 / 62,
  // 64: 89 / 63 (profiles/r03c) -- and the register-occupancy variant
  const char *el = getenv("YMERGE_COMPACT_LANES");
  int lanes = el ? atoi(el) : 16;
  if (lanes < 1 || lanes > 64) lanes = 16;
  const char *eo = getenv("YMERGE_COMPACT_OCC");
  const int occ = eo && atoi(eo) == 2 ? 2 : 1;
  // input bytes above which a document gets a wave of its own
  const char *eg = getenv("YMERGE_COMPACT_BIG");
  const uint64_t big = eg ? strtoull(eg, nullptr, 10) : 65536;
  const char *eb = getenv("YMERGE_COMPACT_WS_GB");
  const double gb = eb ? atof(eb) : 16.0;
  const uint64_t budget = gb > 0 ? (uint64_t)(gb * (double)(1ull << 30)) : (16ull << 30);
  uint32_t mul = 1;
  for (int round = 0; n > 0; round++) {
    j.parts_mul = mul;
    if (S->ws_size.ensure((size_t)(n + 1) * 8) || S->ws_off.ensure((size_t)(n + 1) * 8)) return -1;
    j.list = list;
    j.n = n;
    k_compact_ws<<<(n + 255) / 256, 256, 0, st>>>(j, S->ws_size.as<uint64_t>());
    size_t tmp = 0;
    scan_excl<uint64_t>(nullptr, tmp, S->ws_size.as<uint64_t>(), S->ws_off.as<uint64_t>(), n, st);
    if (S->scan_tmp.ensure(tmp + 16)) return -1;
    if (scan_excl<uint64_t>(S->scan_tmp.p, tmp, S->ws_size.as<uint64_t>(), S->ws_off.as<uint64_t>(), n, st)) return -1;
    HIPCHK(hipMemcpyAsync(S->pinned, S->ws_off.as<uint64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(S->pinned + 1, S->ws_size.as<uint64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t ws_total = S->pinned[0] + S->pinned[1];
    // chunks [cut[k], cut[k + 1]) of the list, each within the budget (one chunk in the common case)
    std::vector<uint32_t> cut = {0, n};
    std::vector<uint64_t> off;
    if (ws_total > budget) {
      if (!list) {  // chunks are sub-ranges of a list: the identity list of all documents
        if (S->list_a.ensure((size_t)(n + 1) * 4)) return -2;
        list = S->list_a.as<uint32_t>();
        k_iota<<<(n + 255) / 256, 256, 0, st>>>(list, n);
      }
      off.resize((size_t)n + 1);
      HIPCHK(hipMemcpyAsync(off.data(), S->ws_off.as<uint64_t>(), (size_t)n * 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      off[n] = ws_total;
      cut.assign(1, 0);
      for (uint32_t a = 0; a < n;) {
        uint32_t b = a + 1;
        while (b < n && off[b + 1] - off[a] <= budget) b++;
        cut.push_back(b);
        a = b;
      }
    }
    // one allocation serves every chunk (they run one after the other on the stream)
    uint64_t maxb = 0;
    for (size_t k = 0; k + 1 < cut.size(); k++) {
      const uint64_t bytes = off.empty() ? ws_total : off[cut[k + 1]] - off[cut[k]];
      if (bytes <= budget || cut[k + 1] - cut[k] > 1) maxb = bytes > maxb ? bytes : maxb;
    }
    if (maxb && S->ws.ensure(maxb + 64)) return -2;
    HIPCHK(hipMemsetAsync(j.counter_retry, 0, 4, st));
    for (size_t k = 0; k + 1 < cut.size(); k++) {
      const uint32_t a = cut[k], cnt = cut[k + 1] - a;
      const uint64_t base = off.empty() ? 0 : off[a];
      const uint64_t bytes = off.empty() ? ws_total : off[a + cnt] - base;
      GeneralJob jc = j;
      jc.list = list ? list + a : nullptr;
      jc.n = cnt;
      jc.ws_off = S->ws_off.as<uint64_t>() + a;
      if (bytes > maxb) {  // one document whose workspace alone exceeds the budget
        k_set_status<<<1, 64, 0, st>>>(jc.list, cnt, j.status, j.out_len, -1, ym::ST_CAPACITY);
        continue;
      }
      jc.ws = S->ws.as<uint8_t>();  // ws + (ws_off[i] - ws_base) lands in this chunk's allocation
      jc.ws_base = base;
      // documents above `big` input bytes first, one per wave; then the rest, `lanes` per wave
      const bool split = lanes > 1;
      for (int part = split ? 1 : 0; part <= (split ? 2 : 0); part++) {
        const uint32_t ln = part == 1 ? 1u : (uint32_t)lanes;
        if (occ == 2) k_compact<2><<<(cnt + ln - 1) / ln, 64, 0, st>>>(jc, ln, big, part);
        else k_compact<1><<<(cnt + ln - 1) / ln, 64, 0, st>>>(jc, ln, big, part);
      }
    }
    HIPCHK(hipMemcpyAsync(S->pinned, j.counter_retry, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint32_t nretry = (uint32_t)(S->pinned[0] & 0xffffffffu);
    if (nretry == 0) break;
    if (round >= 5) {  // still overflowing at 1024x: a public status, not the internal retry code
      k_set_status<<<(n + 255) / 256, 256, 0, st>>>(list, n, j.status, j.out_len, ym::ST_RETRY, ym::ST_CAPACITY);
      break;
    }
    uint32_t *next = list == S->list_a.as<uint32_t>() ? S->list_b.as<uint32_t>() : S->list_a.as<uint32_t>();
    uint32_t cnt = 0;
    if (select_docs(S, st, list, n, j.status, ym::ST_RETRY, next, &cnt)) return -1;
    list = next;
    n = cnt;
    mul *= 4;
  }
  return 0;
}

// Runs the general path over `list` (n docs); retries docs whose part table overflowed.
int run_general(DevState *S, hipStream_t st, GeneralJob j, uint32_t *list, uint32_t n) {
  if (j.op == OP_COMPACT) return run_compact(S, st, j, list, n);
  uint32_t parts_mul = 1;
  for (int round = 0; n > 0; round++) {
    j.list = list;
    j.n = n;
    j.parts_mul = parts_mul;
    if (S->ws_size.ensure((size_t)(n + 1) * 8) || S->ws_off.ensure((size_t)(n + 1) * 8)) return -1;
    k_general_ws<<<(n + 255) / 256, 256, 0, st>>>(j, S->ws_size.as<uint64_t>());
    size_t tmp = 0;
    scan_excl<uint64_t>(nullptr, tmp, S->ws_size.as<uint64_t>(), S->ws_off.as<uint64_t>(), n, st);
    if (S->scan_tmp.ensure(tmp + 16)) return -1;
    if (scan_excl<uint64_t>(S->scan_tmp.p, tmp, S->ws_size.as<uint64_t>(), S->ws_off.as<uint64_t>(), n, st)) return -1;
    HIPCHK(hipMemcpyAsync(S->pinned, S->ws_off.as<uint64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(S->pinned + 1, S->ws_size.as<uint64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint64_t ws_total = S->pinned[0] + S->pinned[1];
    if (S->ws.ensure(ws_total + 64)) return -2;
    j.ws = S->ws.as<uint8_t>();
    j.ws_off = S->ws_off.as<uint64_t>();
    HIPCHK(hipMemsetAsync(j.counter_retry, 0, 4, st));
    uint32_t blocks = (n + 63) / 64;
    k_general<<<blocks, 64, 0, st>>>(j, 1);
    k_general<<<blocks, 64, 0, st>>>(j, 2);
    HIPCHK(hipMemcpyAsync(S->pinned, j.counter_retry, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint32_t nretry = (uint32_t)(S->pinned[0] & 0xffffffffu);
    if (nretry == 0 || round >= 6) break;
    uint32_t *next = list == S->list_a.as<uint32_t>() ? S->list_b.as<uint32_t>() : S->list_a.as<uint32_t>();
    uint32_t cnt = 0;
    if (select_docs(S, st, list, n, j.status, ym::ST_RETRY, next, &cnt)) return -1;
    list = next;
    n = cnt;
    parts_mul *= 8;
  }
  return 0;
}

// ---- pipelined host merges ---------------------------------------------------------------------------
// A host batch of merges (u32 offsets, YM_OFF32) in document chunks of ~6 MiB of input, three streams deep:
//   copy stream   chunk c's bytes + offsets (+ the document ranges once): a copy kernel when the batch lives in
//                 the library's page-locked pool (how the Node addon packs it), else DMA copies  -> event h[c]
//   compute       (waits h[c]) the LDS fast kernel over chunk c, then k_chunk_scan (its documents' packed
//                 offsets after the previous chunks', in stream order)                            -> event k[c]
//   output        (waits k[c]) k_pack_docs: with every output array page-locked it writes the outputs,
//                 offsets, lengths and statuses straight into host memory over PCIe; else into an HBM staging
//                 arena that the host copies out chunk by chunk
// so the link carries chunk c + 1 in while chunk c's outputs go out (full duplex) and the kernels run under
// the copies.  Measured on the box (tools/pipe_sweep.sh, C2 V1 10 k documents, 17.4 MB in / 10.6 MB out): 0.79
// ms per call with the batch in pool memory (copy kernels), 0.65 ms with DMA copies but with 7-8 ms stalls in
// about one call in six (the DMA queue), 1.9 ms unpipelined.  Optimistic: the fast kernels must take every
// document; if any is declined (or not OK) the call runs again through the general flow (run_op,
// unpipelined), which handles everything exactly.
// ---- the page-locked host pool's bookkeeping (ym_host_alloc / ym_host_free, below) ----
std::mutex g_pool_mu;
std::vector<void *> g_pool_free[64];
std::vector<std::pair<void *, int>> g_pool_live;  // (pointer, class) of every buffer handed out
int pool_class(size_t n) {
  int k = 16;
  while (k < 63 && (1ull << k) < n) k++;
  return k;
}
// [p, p + bytes) lies inside one live pool buffer: the device may read it directly (and a little past it)
bool pool_holds(const void *p, size_t bytes) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  const uint8_t *q = (const uint8_t *)p;
  for (const auto &e : g_pool_live) {
    const uint8_t *b = (const uint8_t *)e.first;
    if (q >= b && q + bytes <= b + (1ull << e.second)) return true;
  }
  return false;
}

// the device address of host memory the device can reach (page-locked: hipHostMalloc / hipHostRegister), or
// nullptr (pageable memory)
uint8_t *host_dev_ptr(const void *p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // (pageable memory: not an error of the call)
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  const uint8_t *hp = a.hostPointer ? (const uint8_t *)a.hostPointer : (const uint8_t *)p;
  return (uint8_t *)a.devicePointer + ((const uint8_t *)p - hp);
}
constexpr uint32_t PIPE_MIN_DOCS = 4096, PIPE_MAX = 16;
constexpr uint32_t PIPE_PACK_GRID = 0;  // k_pack_docs blocks per chunk in the pipelined path (0: one per 4 documents)
constexpr uint64_t PIPE_CHUNK_BYTES = 6ull << 20;
int run_op(uint32_t op, const ym_batch *b, ym_out *out, void *stream, ym_stats *stats, int depth = 0);
int run_host_pipe(DevState *S, const ym_batch *b, ym_out *out, hipStream_t st, ym_stats *stats) {
  const uint32_t nd = b->n_docs, nu = b->n_upd;
  const uint32_t *o32 = reinterpret_cast<const uint32_t *>(b->upd_off);
  const uint32_t *du = b->doc_upd;
  const uint64_t A_lo = o32[0], A_hi = o32[nu], abytes = A_hi;  // arena positions are absolute
  const bool v2 = (b->format & 0xff) == YM_V2;
  if (!S->s_h2d) {
    {  // the copy-in queue at the highest priority: its copy kernels are dispatched ahead of the merges
      int lo = 0, hi = 0;
      if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
      HIPCHK(hipStreamCreateWithPriority(&S->s_h2d, hipStreamNonBlocking, getenv("YMERGE_PIPE_NOPRIO") ? 0 : hi));
    }
    HIPCHK(hipStreamCreateWithFlags(&S->s_h2d2, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&S->s_d2h, hipStreamNonBlocking));
    for (uint32_t c = 0; c < PIPE_MAX; c++) {
      HIPCHK(hipEventCreateWithFlags(&S->pev_h[c], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&S->pev_h2[c], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&S->pev_k[c], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&S->pev_p[c], hipEventDisableTiming));
    }
    HIPCHK(hipHostMalloc((void **)&S->pipe_host, 64 * sizeof(uint64_t), hipHostMallocCoherent | hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer((void **)&S->pipe_host_dev, S->pipe_host, 0));
  }
  // chunk boundaries: documents, cut at ~equal input bytes
  static const uint64_t chunk_bytes = getenv("YMERGE_PIPE_CHUNK_KB") ? strtoull(getenv("YMERGE_PIPE_CHUNK_KB"), nullptr, 10) << 10
                                                                     : PIPE_CHUNK_BYTES;
  static const int alt = getenv("YMERGE_PIPE_ALT") ? atoi(getenv("YMERGE_PIPE_ALT")) : 0;
  uint32_t nc = (uint32_t)((A_hi - A_lo + chunk_bytes - 1) / chunk_bytes);
  nc = nc < 2 ? 2 : nc > PIPE_MAX ? PIPE_MAX : nc;
  uint32_t cut[PIPE_MAX + 1];
  cut[0] = 0;
  for (uint32_t c = 1; c < nc; c++) {
    const uint64_t target = A_lo + (A_hi - A_lo) * c / nc;
    uint32_t lo = cut[c - 1], hi = nd;  // first document starting at or after target
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (o32[du[mid]] < target) lo = mid + 1; else hi = mid;
    }
    cut[c] = lo;
  }
  cut[nc] = nd;
  // device buffers
  const uint64_t bound = 4 * abytes + 128ull * nd + 8192;
  uint64_t dev_cap = out->cap > bound ? out->cap : bound;
  if (S->min_stage_cap > dev_cap) dev_cap = S->min_stage_cap;
  if (S->in_arena.ensure(abytes + 64) || S->in_off32.ensure((nu + 1) * 4ull + 64) || S->in_doc.ensure((nd + 1) * 4ull + 64) ||
      S->out_arena.ensure(dev_cap + 16) || S->out_off.ensure(nd * 8ull) || S->out_len.ensure(nd * 8ull) ||
      S->status.ensure(nd * 4ull) || S->cmp_off.ensure(nd * 8ull + 8) || S->cmp_len.ensure(nd * 8ull + 8) ||
      S->cmp_arena.ensure(dev_cap + 16) || S->counters.ensure(1024) || S->list_a.ensure((nd + 1) * 4ull) ||
      S->layout.ensure(nd * sizeof(ym::Layout) + 16) || (v2 && S->in_off.ensure((nu + 1) * 8ull)))
    return -2;
  uint8_t *dA = S->in_arena.as<uint8_t>();
  uint32_t *dO = S->in_off32.as<uint32_t>(), *dD = S->in_doc.as<uint32_t>();
  uint64_t *counters = S->counters.as<uint64_t>();
  GeneralJob j;
  memset(&j, 0, sizeof(j));
  j.A = dA;
  j.upd_off32 = v2 ? nullptr : dO;
  j.upd_off = v2 ? S->in_off.as<uint64_t>() : nullptr;
  j.op = OP_MERGE;
  j.v2 = v2;
  j.layout = S->layout.as<ym::Layout>();
  j.out = S->out_arena.as<uint8_t>();
  j.cap = dev_cap;
  j.used = counters + 0;
  j.counter_retry = (uint32_t *)(counters + 1);
  j.pend_count = (uint32_t *)(counters + 2);
  j.pend_list = S->list_a.as<uint32_t>();
  j.pw_count = counters + 11;
  // counters (declines, the running packed total [20], non-OK documents [21]) start at zero; the
  // compute stream's previous work (an earlier call) is ordered before
  HIPCHK(hipMemsetAsync(counters, 0, 1024, st));
  S->dirty = true;  // k_finish does not run here: the next unpipelined call resets the counters
  HIPCHK(hipEventRecord(S->ev0, st));
  HIPCHK(hipStreamWaitEvent(S->s_h2d, S->ev0, 0));  // staging buffers: free once the earlier work is done
  HIPCHK(hipStreamWaitEvent(S->s_h2d2, S->ev0, 0));
  volatile uint64_t *hw = S->pipe_host;
  for (uint32_t c = 0; c < nc; c++) hw[2 * c] = hw[2 * c + 1] = ~0ull;
  // outputs in page-locked memory the device can address (ym_host_alloc, hipHostMalloc / hipHostRegister):
  // the packing kernels write the outputs, offsets, lengths and statuses straight into it over PCIe (no copy
  // op at all); otherwise the packed chunks are copied out as each completes
  uint8_t *h_arena = host_dev_ptr(out->arena);
  uint64_t *h_off = (uint64_t *)host_dev_ptr(out->out_off), *h_len = (uint64_t *)host_dev_ptr(out->out_len);
  int32_t *h_st = (int32_t *)host_dev_ptr(out->status);
  const bool direct = h_arena && h_off && h_len && h_st && !getenv("YMERGE_PIPE_COPY");
  // inputs in the library's pool (the Node addon packs there): the merge kernels read them over PCIe themselves
  // (zero-copy: no DMA copy op, whose per-copy setup left the link idle between chunks); the pool's size
  // classes leave room for the 16-byte staging loads' over-read past the end
  const uint8_t *z_arena = pool_holds(b->arena, A_hi + 64) ? host_dev_ptr(b->arena) : nullptr;
  const uint32_t *z_off = pool_holds(o32, (nu + 1) * 4ull + 64) ? (const uint32_t *)host_dev_ptr(o32) : nullptr;
  const uint32_t *z_doc = pool_holds(du, (nd + 1) * 4ull + 64) ? (const uint32_t *)host_dev_ptr(du) : nullptr;
  const bool zin = z_arena && z_off && z_doc && !getenv("YMERGE_PIPE_NOZC");
  // (1) every copy in, up front: pool-resident batches by a copy kernel per chunk on the copy stream (its
  // bytes, its offsets, and with the first chunk the document ranges); otherwise DMA copies on two queues
  // running back to back without waiting for the host
  for (uint32_t c = 0; c < nc && zin; c++) {
    const uint32_t d0 = cut[c], d1 = cut[c + 1];
    if (d1 == d0) continue;
    const uint32_t u0 = du[d0], u1 = du[d1];
    const uint64_t a0 = c == 0 ? 0 : o32[u0] & ~63ull, a1e = c + 1 == nc ? A_hi : (o32[u1] + 63) & ~63ull;
    const uint64_t a1 = ((a1e < A_hi ? a1e : A_hi) + 15) & ~15ull;
    const uint32_t o0 = c == 0 ? 0 : u0 & ~15u, o1e = c + 1 == nc ? nu + 1 : ((u1 + 1 + 15) & ~15u);
    const uint32_t o1 = ((o1e < nu + 1 ? o1e : nu + 1) + 3) & ~3u;
    const H2dSeg sa = {(const uint4 *)(z_arena + a0), (uint4 *)(dA + a0), (a1 - a0) / 16};
    const H2dSeg so = {(const uint4 *)(z_off + o0), (uint4 *)(dO + o0), (o1 - o0) / 4ull};
    const H2dSeg sd = {(const uint4 *)z_doc, (uint4 *)dD, c == 0 ? (nd + 1 + 3) / 4ull : 0};
    k_h2d_copy<<<512, 256, 0, S->s_h2d>>>(sa, so, sd);
    HIPCHK(hipEventRecord(S->pev_h[c], S->s_h2d));
  }
  if (!zin) HIPCHK(hipMemcpyAsync(dD, du, (nd + 1) * 4ull, hipMemcpyHostToDevice, S->s_h2d2));  // doc_upd: one copy
  for (uint32_t c = 0; c < nc && !zin; c++) {
    const uint32_t d0 = cut[c], d1 = cut[c + 1];
    if (d1 == d0) continue;
    const uint32_t u0 = du[d0], u1 = du[d1];
    // the chunk's bytes on one copy queue and its offsets on another (two DMA engines: their per-copy setup
    // overlaps), both cut at 64-byte boundaries (an unaligned end costs a blit kernel; the few bytes a cut
    // shares with the neighbouring chunk are copied twice, the same values, in stream order)
    const uint64_t a0 = c == 0 ? 0 : o32[u0] & ~63ull, a1e = c + 1 == nc ? A_hi : (o32[u1] + 63) & ~63ull;
    const uint64_t a1 = a1e < A_hi ? a1e : A_hi;
    // (alt: chunk c's bytes and offsets both on queue c & 1, so one queue's per-copy setup overlaps the other's
    // transfer; otherwise bytes on one queue, offsets on the other)
    hipStream_t qa = alt && (c & 1) ? S->s_h2d2 : S->s_h2d, qo = alt ? qa : S->s_h2d2;
    if (a1 > a0) HIPCHK(hipMemcpyAsync(dA + a0, b->arena + a0, a1 - a0, hipMemcpyHostToDevice, qa));
    const uint32_t o0 = c == 0 ? 0 : u0 & ~15u, o1e = c + 1 == nc ? nu + 1 : ((u1 + 1 + 15) & ~15u);
    const uint32_t o1 = o1e < nu + 1 ? o1e : nu + 1;
    HIPCHK(hipMemcpyAsync(dO + o0, o32 + o0, (o1 - o0) * 4ull, hipMemcpyHostToDevice, qo));
    HIPCHK(hipEventRecord(S->pev_h[c], qa));
    HIPCHK(hipEventRecord(S->pev_h2[c], qo));
  }
  // (2) per chunk: the merge kernel and the placement scan on the compute stream, the packing on the output
  // stream (it overlaps the next chunk's merge)
  for (uint32_t c = 0; c < nc; c++) {
    const uint32_t d0 = cut[c], d1 = cut[c + 1];
    if (d1 == d0) continue;
    const uint32_t u0 = du[d0], u1 = du[d1];
    HIPCHK(hipStreamWaitEvent(st, S->pev_h[c], 0));
    if (!zin) HIPCHK(hipStreamWaitEvent(st, S->pev_h2[c], 0));
    const uint32_t o0 = c == 0 ? 0 : u0 & ~15u;
    if (v2) k_widen<<<(u1 - o0 + 256) / 256, 256, 0, st>>>(dO + o0, S->in_off.as<uint64_t>() + o0, u1 - o0 + 1);
    GeneralJob jc = j;
    jc.doc_upd = dD + d0;
    jc.n = d1 - d0;
    jc.doc_base = d0;
    jc.status = S->status.as<int32_t>() + d0;
    jc.out_off = S->out_off.as<uint64_t>() + d0;
    jc.out_len = S->out_len.as<uint64_t>() + d0;
    const int fr = v2 ? fast2_launch(OP_MERGE, jc, nu, st) : fast_launch(OP_MERGE, jc, nu, st);
    if (fr != 1) return -3;
    k_chunk_scan<<<1, 1024, 0, st>>>(jc.status, jc.out_len, jc.n, S->cmp_off.as<uint64_t>() + d0, S->cmp_len.as<uint64_t>() + d0,
                                      counters + 20, S->pipe_host_dev, c, j.pend_count, c + 1 == nc, nullptr, nullptr, nullptr);
    HIPCHK(hipEventRecord(S->pev_k[c], st));
    HIPCHK(hipStreamWaitEvent(S->s_d2h, S->pev_k[c], 0));
    static const uint32_t pack_grid = getenv("YMERGE_PACK_GRID") ? (uint32_t)atoi(getenv("YMERGE_PACK_GRID")) : PIPE_PACK_GRID;
    const uint32_t pg = (jc.n + 3) / 4 < pack_grid || pack_grid == 0 ? (jc.n + 3) / 4 : pack_grid;
    k_pack_docs<<<pg, 256, 0, S->s_d2h>>>(j.out, jc.out_off, S->cmp_off.as<uint64_t>() + d0,
                                                      S->cmp_len.as<uint64_t>() + d0, jc.n,
                                                      direct ? h_arena : S->cmp_arena.as<uint8_t>(), direct ? out->cap : ~0ull,
                                                      jc.status, direct ? h_off + d0 : nullptr, direct ? h_len + d0 : nullptr,
                                                      direct ? h_st + d0 : nullptr);
    if (!direct) HIPCHK(hipEventRecord(S->pev_p[c], S->s_d2h));
  }
  if (stats) HIPCHK(hipEventRecord(S->ev1, st));
  // (3) copy mode: each chunk's packed range as soon as it is packed
  uint64_t total = 0;
  bool over = false;
  for (uint32_t c = 0; c < nc && !direct; c++) {
    if (cut[c + 1] == cut[c]) continue;
    hipError_t q = hipEventQuery(S->pev_p[c]);
    for (uint64_t it = 0; q == hipErrorNotReady && it < (1ull << 28); it++) {
      __builtin_ia32_pause();
      q = hipEventQuery(S->pev_p[c]);
    }
    if (q != hipSuccess) HIPCHK(hipEventSynchronize(S->pev_p[c]));
    const uint64_t lo = hw[2 * c], hi = hw[2 * c + 1];
    if (lo == ~0ull || hi < lo) return -4;
    if (hi > out->cap) over = true;
    if (over) continue;
    // the range widened to 64-byte boundaries (an unaligned copy runs as a blit kernel): the bytes past hi
    // belong to the next chunk and are copied again, correctly, by its own copy later on this stream; past the
    // last chunk they are unused capacity
    const uint64_t alo = lo & ~63ull, ahe = (hi + 63) & ~63ull, ahi = ahe < out->cap ? ahe : out->cap;
    if (ahi > alo)
      HIPCHK(hipMemcpyAsync(out->arena + alo, S->cmp_arena.as<uint8_t>() + alo, ahi - alo, hipMemcpyDeviceToHost, S->s_d2h));
    const uint32_t d0 = cut[c], n = cut[c + 1] - cut[c];  // the chunk's offsets, lengths and statuses
    HIPCHK(hipMemcpyAsync(out->out_off + d0, S->cmp_off.as<uint64_t>() + d0, n * 8ull, hipMemcpyDeviceToHost, S->s_d2h));
    HIPCHK(hipMemcpyAsync(out->out_len + d0, S->cmp_len.as<uint64_t>() + d0, n * 8ull, hipMemcpyDeviceToHost, S->s_d2h));
    HIPCHK(hipMemcpyAsync(out->status + d0, S->status.as<int32_t>() + d0, n * 4ull, hipMemcpyDeviceToHost, S->s_d2h));
  }
  HIPCHK(hipStreamSynchronize(S->s_d2h));
  {
    uint32_t c = nc;
    while (c > 0 && cut[c] == cut[c - 1]) c--;
    total = c > 0 ? hw[2 * (c - 1) + 1] : 0;
    if (total > out->cap) over = true;
  }
  const uint64_t nbad = hw[61];
  if (nbad != 0) {  // a declined (or capacity) document: the whole call through the exact flow
    S->pipe_skip = true;
    const int r = run_op(OP_MERGE, b, out, st, stats);
    S->pipe_skip = false;
    return r;
  }
  out->used = total;
  if (over) return YM_ERR_CAPACITY;
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    float ms = 0;
    hipEventElapsedTime(&ms, S->ev0, S->ev1);
    stats->device_ms = ms;
    stats->docs = stats->docs_fast = nd;
    stats->bytes_in = A_hi - A_lo;
    stats->bytes_out = total;
  }
  return 0;
}

constexpr uint32_t NESTED_PROBE = 16;
int run_op(uint32_t op, const ym_batch *b, ym_out *out, void *stream, ym_stats *stats, int depth) {
  if (!b || !out) return -1;
  DevState *S = state();
  {  // the caller (e.g. torch) may have switched this thread's device
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != S->device) HIPCHK(hipSetDevice(S->device));
  }
  hipStream_t st = stream ? (hipStream_t)stream : S->stream;
  uint32_t nd = b->n_docs;
  if (stats) memset(stats, 0, sizeof(*stats));
  if (nd == 0) { out->used = 0; return 0; }
  const bool off32 = (b->format & YM_OFF32) != 0;
  // host merges of many documents with u32 offsets: the pipelined path (depth 8 = its own fallback)
  if (op == OP_MERGE && off32 && b->mem == YM_MEM_HOST && depth == 0 && !S->pipe_skip && nd >= PIPE_MIN_DOCS &&
      !getenv("YMERGE_NO_PIPE"))
    return run_host_pipe(S, b, out, st, stats);
  const uint8_t *A = b->arena;
  const uint64_t *upd_off = off32 ? nullptr : b->upd_off;
  const uint32_t *upd_off32 = off32 ? reinterpret_cast<const uint32_t *>(b->upd_off) : nullptr;  // (host or device)
  const uint32_t *doc_upd = b->doc_upd;
  const uint8_t *svp = b->sv_arena;
  const uint64_t *sv_off = b->sv_off;
  uint8_t *o_arena = out->arena;
  uint64_t *o_off = out->out_off, *o_len = out->out_len;
  int32_t *o_status = out->status;
  bool host = b->mem == YM_MEM_HOST;
  // device output capacity: the caller's (device batches); for host batches the library's own staging,
  // at least the internal bound (the caller's buffer only receives the packed outputs)
  uint64_t dev_cap = out->cap;
  if (host) {  // stage inputs (u32 offsets as they are: widened on the device where a kernel reads u64)
    uint64_t abytes = off32 ? upd_off32[b->n_upd] : upd_off[b->n_upd];
    // ym_diff's state vectors; ym_compact's optional target state vectors
    const bool stage_sv = op == OP_DIFF || (op == OP_COMPACT && svp);
    const uint64_t svb = stage_sv ? sv_off[nd] : 0;
    const uint64_t bound = 4 * abytes + 2 * svb + 128ull * nd + 8192;
    dev_cap = out->cap > bound ? out->cap : bound;
    if (S->min_stage_cap > dev_cap) dev_cap = S->min_stage_cap;
    if (S->in_arena.ensure(abytes + 16) || S->in_doc.ensure((nd + 1) * 4ull)) return -2;
    HIPCHK(hipMemcpyAsync(S->in_arena.p, A, abytes, hipMemcpyHostToDevice, st));
    if (off32) {
      if (S->in_off32.ensure((b->n_upd + 1) * 4ull)) return -2;
      HIPCHK(hipMemcpyAsync(S->in_off32.p, upd_off32, (b->n_upd + 1) * 4ull, hipMemcpyHostToDevice, st));
      upd_off32 = S->in_off32.as<uint32_t>();
    } else {
      if (S->in_off.ensure((b->n_upd + 1) * 8ull)) return -2;
      HIPCHK(hipMemcpyAsync(S->in_off.p, upd_off, (b->n_upd + 1) * 8ull, hipMemcpyHostToDevice, st));
      upd_off = S->in_off.as<uint64_t>();
    }
    HIPCHK(hipMemcpyAsync(S->in_doc.p, doc_upd, (nd + 1) * 4ull, hipMemcpyHostToDevice, st));
    A = S->in_arena.as<uint8_t>();
    doc_upd = S->in_doc.as<uint32_t>();
    if (stage_sv) {
      uint64_t sb = sv_off[nd];
      if (S->in_sv.ensure(sb + 16) || S->in_svoff.ensure((nd + 1) * 8ull)) return -2;
      HIPCHK(hipMemcpyAsync(S->in_sv.p, svp, sb, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(S->in_svoff.p, sv_off, (nd + 1) * 8ull, hipMemcpyHostToDevice, st));
      svp = S->in_sv.as<uint8_t>();
      sv_off = S->in_svoff.as<uint64_t>();
    }
    if (S->out_arena.ensure(dev_cap + 16) || S->out_off.ensure(nd * 8ull) || S->out_len.ensure(nd * 8ull) ||
        S->status.ensure(nd * 4ull))
      return -2;
    o_arena = S->out_arena.as<uint8_t>();
    o_off = S->out_off.as<uint64_t>();
    o_len = S->out_len.as<uint64_t>();
    o_status = S->status.as<int32_t>();
  }
  if (S->layout.ensure(nd * sizeof(ym::Layout) + 16) || S->counters.ensure(1024) || S->list_a.ensure((nd + 1) * 4ull) ||
      S->list_b.ensure((nd + 1) * 4ull))
    return -2;
  uint64_t *counters = S->counters.as<uint64_t>();
  // counters: [0] used (bump allocator), [1] retry count, [2] fast-path declined count (u32),
  //           [4..6] stats (errors, bytes out, bytes in)
  GeneralJob j;
  memset(&j, 0, sizeof(j));
  j.A = A;
  j.upd_off = upd_off;
  if (off32) j.upd_off32 = upd_off32;
  // device u32 offsets: the V1 fast kernel reads them as they are; every other kernel reads u64
  // offsets, widened here on first need
  auto widen = [&]() -> int {
    if (j.upd_off) return 0;
    if (S->in_off.ensure((b->n_upd + 1) * 8ull)) return -2;
    k_widen<<<(b->n_upd + 256) / 256, 256, 0, st>>>(j.upd_off32, S->in_off.as<uint64_t>(), b->n_upd + 1);
    j.upd_off = upd_off = S->in_off.as<uint64_t>();
    return 0;
  };
  j.doc_upd = doc_upd;
  j.sv = op == OP_DIFF || op == OP_COMPACT ? svp : nullptr;
  j.sv_off = j.sv ? sv_off : nullptr;
  j.op = op;
  j.v2 = (b->format & 0xff) == YM_V2;
  j.dsref = op == OP_DSMERGE && (b->format & YM_DS_REF) != 0;
  j.nogc = op == OP_COMPACT && (b->format & YM_NO_GC) != 0;
  j.svfirst = op == OP_COMPACT && (b->format & YM_SV_FIRST) != 0;
  // ym_snapshot: the output encoding (YM_OUT_V1 / YM_OUT_V2; default: the input's)
  j.v2out = op == OP_SNAP && ((b->format & YM_OUT_V2) != 0 || (j.v2 && (b->format & YM_OUT_V1) == 0));
  j.layout = S->layout.as<ym::Layout>();
  j.status = o_status;
  j.out = o_arena;
  j.cap = dev_cap;
  j.out_off = o_off;
  j.out_len = o_len;
  j.used = counters + 0;
  j.counter_retry = (uint32_t *)(counters + 1);
  j.pend_count = (uint32_t *)(counters + 2);
  j.pend_list = S->list_a.as<uint32_t>();
  j.pw_count = counters + 11;
  j.n = nd;
  const uint64_t seq = ++S->seq;
  if (op == OP_DIFF || op == OP_SV || op == OP_META) {  // per-block scratch of the streamed walkers
    if (S->bscratch.ensure((uint64_t)(nd < BS_GRID ? nd : BS_GRID) * BS_BYTES)) return -2;
    j.bscratch = S->bscratch.as<uint8_t>();
  }

  if (S->dirty) HIPCHK(hipMemsetAsync(counters, 0, 1024, st));
  S->dirty = true;
  bool slots = false;  // the fast paths wrote their outputs into the slot region (merges, delete-set merges)
  uint64_t chunked = 0;  // documents the chunk-parallel walk completed (summed over this call's round trips)
  // ends a round trip: counters and stats land in pinned host memory, then one stream sync
  auto finish = [&]() -> int {
    const bool want = stats || host;  // host batches need the bytes out (the packed size)
    const bool one = !want || nd <= 16 * 1024;
    const uint32_t fin_blocks = one ? 1 : (nd + 4095) / 4096;
    if (one)
      k_finish<1024><<<1, 1024, 0, st>>>(o_status, o_len, nd, j.upd_off, j.upd_off ? nullptr : j.upd_off32, b->n_upd, counters, S->pinned_dev,
                                        want ? 1 : 0, slots ? 1 : 0, seq);
    else
      k_finish<256><<<fin_blocks, 256, 0, st>>>(o_status, o_len, nd, j.upd_off, j.upd_off ? nullptr : j.upd_off32, b->n_upd, counters, S->pinned_dev,
                                                 want ? 1 : 0, slots ? 1 : 0, seq);
    HIPCHK(hipEventRecord(S->ev1, st));
    // spin on the completion word k_finish writes last (no interrupt wake-up of a blocking wait), then
    // the stream sync, which finds the stream drained: it is what orders every result for the host
    volatile uint64_t *hp = S->pinned;
    for (uint64_t it = 0; hp[7] != seq && it < (1ull << 26); it++) __builtin_ia32_pause();
    hipError_t q;
    for (int it = 0; (q = hipStreamQuery(st)) == hipErrorNotReady && it < 100000; it++) __builtin_ia32_pause();
    if (q != hipSuccess) HIPCHK(hipStreamSynchronize(st));
    chunked += S->pinned[8];
    return 0;
  };
  if (!((op == OP_MERGE && !j.v2) || (op == OP_DSMERGE && !j.dsref)))
    if (int r = widen()) return r;
  HIPCHK(hipEventRecord(S->ev0, st));
  // (1) fast path over every document; appends the ones it declines to list_a.  A merge batch of mostly rich
  // documents (as the previous calls saw) starts with the nested pass over every document instead
  const uint32_t fi = j.v2 ? 1 : 0;
  const bool nested_first = op == OP_MERGE && S->nested_first[fi] > 0 && S->nested_first[fi] % NESTED_PROBE != 0 &&
                            !getenv("YMERGE_NO_NESTED_FIRST");
  int fr = 0;
  if (nested_first) fr = j.v2 ? fast2_nested_launch(j, nd, st) : fast_nested_launch(j, nd, st);
  if (fr == 0) fr = fast_launch(op, j, b->n_upd, st);     // V1 merge: LDS fast path
  if (fr == 0) fr = fast2_launch(op, j, b->n_upd, st);  // V2 merge: LDS fast path
  if (fr == 0) fr = big_launch(op, j, st, S->pw);  // V1 diff / state vector: chunk walk + wave walker
  if (fr == 0) fr = big2_launch(op, j, st, S->pw2); // V2 diff / state vector: column path + wave walker
  if (fr < 0) return fr;
  slots = op == OP_MERGE || (op == OP_DSMERGE && fr == 1);
  HIPCHK(hipEventRecord(S->evf1, st));
  uint32_t ngen = nd;
  uint32_t *list = nullptr;
  if (fr == 1) {
    // one round trip: used, the declined count and (speculatively) the stats of the fast-only case
    if (int r = finish()) return r;
    ngen = (uint32_t)(S->pinned[2] & 0xffffffffu);
    list = S->list_a.as<uint32_t>();
  }
  const uint32_t ngen_hot = ngen;
  if (op == OP_MERGE && fr == 1 && (nested_first || ngen <= nd / 2)) {
    // the nested pass (first) took most documents: keep it first, with a hot-pass probe every NESTED_PROBE
    // calls; or the hot pass declined at most half of them: the batch is not rich
    S->nested_first[fi] = nested_first && ngen < nd / 2 ? S->nested_first[fi] + 1 : 0;
  }
  if (ngen > 0)
    if (int r = widen()) return r;
  // (1b) merges: the declined documents once more through the LDS kernel with nested payload checks
  // (rich content); it re-declines the rest into list_b
  bool nested = false;
  if (ngen > 0 && list && op == OP_MERGE && !nested_first) {
    GeneralJob jn = j;
    jn.list = list;
    jn.pend_list = S->list_b.as<uint32_t>();
    HIPCHK(hipEventRecord(S->evn0, st));
    if (j.v2 ? fast2_nested_launch(jn, ngen, st) : fast_nested_launch(jn, ngen, st)) {
      nested = true;
      HIPCHK(hipEventRecord(S->evn1, st));
      if (int r = finish()) return r;
      ngen = (uint32_t)(S->pinned[2] & 0xffffffffu);
      list = S->list_b.as<uint32_t>();
    }
  }
  // the hot pass declined most documents and the nested pass took most of the batch (rich content, not
  // documents too large for the LDS kernels): start the next calls with the nested pass
  if (op == OP_MERGE && fr == 1 && !nested_first && ngen_hot > nd / 2)
    S->nested_first[fi] = nested && ngen_hot - ngen > nd / 2 ? S->nested_first[fi] + 1 : 0;
  // (2) large-document merges (ym_large.hip) over the declined list; what it declines stays pending
  uint32_t nlarge = 0;
  bool large = false;
  if (ngen > 0 && list && op == OP_MERGE) {
    int lr = large_run(j, list, ngen, b->n_upd, st, S->large);
    if (lr < 0) return lr;
    if (lr == 1) {
      large = true;
      HIPCHK(hipEventRecord(S->evl1, st));
      uint32_t cnt = 0;
      uint32_t *next = list == S->list_a.as<uint32_t>() ? S->list_b.as<uint32_t>() : S->list_a.as<uint32_t>();
      if (select_docs(S, st, list, ngen, o_status, ST_PENDING, next, &cnt)) return -1;
      nlarge = ngen - cnt;
      ngen = cnt;
      list = next;
      if (ngen == 0)
        if (int r = finish()) return r;
    }
  }
  // (3) general path over the rest
  if (ngen > 0) {
    // the general path's bump allocator: merges start after the slot region; diff / sv continue after
    // what the streamed kernels allocated (k_finish reset the device counter)
    if (slots) {
      k_fast_region<<<1, 64, 0, st>>>(j, b->n_upd);
    } else if (fr == 1) {
      S->pinned[16] = S->pinned[0];
      HIPCHK(hipMemcpyAsync(counters, S->pinned + 16, 8, hipMemcpyHostToDevice, st));
    }  // else (no specialised kernel ran): the counters are zero (reset by the last k_finish / memset)
    int r = run_general(S, st, j, list, ngen);
    if (r) return r;
    HIPCHK(hipEventRecord(S->evg1, st));
    if (int r2 = finish()) return r2;
  }
  S->dirty = false;
  uint64_t used = S->pinned[0];
  out->used = used;
  if (stats) {
    float ms = 0, fms = 0, gms = 0;
    hipEventElapsedTime(&ms, S->ev0, S->ev1);
    hipEventElapsedTime(&fms, S->ev0, S->evf1);  // ev0 is recorded right before the fast kernel
    float lms = 0;
    hipEvent_t e_prev = nested ? S->evn1 : S->evf1;  // the end of the last specialised pass before
    if (large) hipEventElapsedTime(&lms, e_prev, S->evl1);
    if (ngen > 0) hipEventElapsedTime(&gms, large ? S->evl1 : e_prev, S->evg1);
    stats->docs_large = nlarge;
    stats->large_ms = lms;
    stats->device_ms = ms;
    float nms = 0;
    if (nested) hipEventElapsedTime(&nms, S->evn0, S->evn1);
    stats->fast_ms = fr == 1 ? fms + nms : 0.0;
    stats->general_ms = ngen > 0 ? gms : 0.0;
    stats->docs = nd;
    stats->docs_general = ngen;
    stats->docs_fast = nd - ngen - nlarge;
    stats->docs_error = S->pinned[4];
    stats->bytes_out = S->pinned[5];
    stats->bytes_in = S->pinned[6];
    stats->docs_chunked = chunked;
  }
  static const bool trace = getenv("YMERGE_TRACE_CAP") != nullptr;  // diagnostics: why a call reports capacity
  if (trace)
    fprintf(stderr, "ym trace op %u depth %d nd %u used %llu dev_cap %llu out_cap %llu bytes_out %llu ngen %u\n", op, depth, nd,
            (unsigned long long)used, (unsigned long long)dev_cap, (unsigned long long)out->cap,
            (unsigned long long)S->pinned[5], ngen);
  if (!host) return used > out->cap ? YM_ERR_CAPACITY : 0;
  // host batch: pack the outputs in document order (out_off[d] = bytes of the outputs before d), then
  // copy only them back.  The staging arena is the library's own: an overflow grows it and runs the
  // call again here (the caller only ever sees the packed size in out->used).
  if (used > dev_cap) {
    if (depth >= 2) return YM_ERR_CAPACITY;
    S->min_stage_cap = used + used / 4 + 4096;
    return run_op(op, b, out, stream, stats, depth + 1);
  }
  const uint64_t total = S->pinned[5];
  out->used = total;
  if (total > out->cap) return YM_ERR_CAPACITY;
  {
    size_t tmp = 0;
    if (S->cmp_off.ensure(nd * 8ull + 8) || S->cmp_len.ensure(nd * 8ull + 8) || S->cmp_arena.ensure(total + 16)) return -2;
    uint64_t *mlen = S->cmp_len.as<uint64_t>();
    k_mask_len<<<(nd + 255) / 256, 256, 0, st>>>(o_status, o_len, mlen, nd);
    scan_excl<uint64_t>(nullptr, tmp, mlen, (uint64_t *)nullptr, nd, st);
    if (S->scan_tmp.ensure(tmp + 16)) return -2;
    if (scan_excl<uint64_t>(S->scan_tmp.p, tmp, mlen, S->cmp_off.as<uint64_t>(), nd, st)) return -3;
    // one wave per document (round 6; k_pack, a search per 16 output bytes, took 38 us for 10.6 MB)
    if (total) k_pack_docs<<<(nd + 3) / 4, 256, 0, st>>>(o_arena, o_off, S->cmp_off.as<uint64_t>(), mlen, nd, S->cmp_arena.as<uint8_t>(), ~0ull);
  }
  if (total) HIPCHK(hipMemcpyAsync(out->arena, S->cmp_arena.p, total, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(out->out_off, S->cmp_off.p, nd * 8ull, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(out->out_len, S->cmp_len.p, nd * 8ull, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(out->status, o_status, nd * 4ull, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

}  // namespace

extern "C" {

int ym_init(int device) {
  std::lock_guard<std::mutex> g(g_mu);
  if (device < 0 || device >= kMaxDevices) return -1;
  if (hipSetDevice(device) != hipSuccess) return -1;
  if (!g_states[device]) { g_states[device] = new DevState(); g_states[device]->device = device; }
  g_state = g_states[device];  // other devices' states of this thread stay alive for a later switch
  g_default_device.store(device);
  state();
  return 0;
}

static void release_state(DevState *S) {
  hipSetDevice(S->device);
  if (S->stream) hipStreamSynchronize(S->stream);
  DBuf *bufs[] = {&S->ws, &S->ws_size, &S->ws_off, &S->layout, &S->counters, &S->scan_tmp, &S->list_a, &S->list_b,
                  &S->flags, &S->bscratch, &S->in_arena, &S->in_off, &S->in_doc, &S->in_sv, &S->in_svoff, &S->out_arena,
                  &S->out_off, &S->out_len, &S->status, &S->cmp_off, &S->cmp_len, &S->cmp_arena, &S->async_off,
                  &S->async2_ws, &S->async2_bs, &S->async2_off, &S->in_off32};
  for (DBuf *b : bufs) if (b->p) hipFree(b->p);
  for (hipStream_t x : {S->s_h2d, S->s_h2d2, S->s_d2h}) if (x) { hipStreamSynchronize(x); hipStreamDestroy(x); }
  for (int c = 0; c < 16; c++) {
    if (S->pev_h[c]) hipEventDestroy(S->pev_h[c]);
    if (S->pev_h2[c]) hipEventDestroy(S->pev_h2[c]);
    if (S->pev_k[c]) hipEventDestroy(S->pev_k[c]);
    if (S->pev_p[c]) hipEventDestroy(S->pev_p[c]);
  }
  if (S->pipe_host) hipHostFree(S->pipe_host);
  if (S->ev_async) hipEventDestroy(S->ev_async);
  if (S->ev_async2) hipEventDestroy(S->ev_async2);
  if (S->pinned) hipHostFree(S->pinned);
  if (S->ev0) hipEventDestroy(S->ev0);
  if (S->ev1) hipEventDestroy(S->ev1);
  if (S->evf0) hipEventDestroy(S->evf0);
  if (S->evf1) hipEventDestroy(S->evf1);
  if (S->evg1) hipEventDestroy(S->evg1);
  if (S->evl1) hipEventDestroy(S->evl1);
  if (S->evn0) hipEventDestroy(S->evn0);
  if (S->evn1) hipEventDestroy(S->evn1);
  for (int k = 0; k < 4; k++) if (S->large.p[k]) hipFree(S->large.p[k]);
  if (S->large.pinned) hipHostFree(S->large.pinned);
  for (PwBufs *pb : {&S->pw, &S->pw2}) {
    for (int k = 0; k < PW_NBUF; k++) if (pb->p[k]) hipFree(pb->p[k]);
    if (pb->pinned) hipHostFree(pb->pinned);
    if (pb->ev) hipEventDestroy(pb->ev);
  }
  if (S->stream) hipStreamDestroy(S->stream);
  delete S;
}

// releases every device state of the calling thread
int ym_shutdown(void) {
  for (int d = 0; d < kMaxDevices; d++)
    if (g_states[d]) { release_state(g_states[d]); g_states[d] = nullptr; }
  g_state = nullptr;
  return 0;
}

const char *ym_strerror(int code) {
  if (code > 0 && (code >> 8) != 0) {  // a per-document exception with its detail (ym_core.h D_*)
    static thread_local char buf[160];
    const int detail = (code >> 8) & 0xff, arg = (code >> 16) & 0x7fff;
    static const char *getters[4] = {"length", "byteLength", "byteOffset", "buffer"};
    switch (detail) {
      case 1: return "contentRefs[(info & binary.BITS5)] is not a function";
      case 2: return "typeRefs[decoder.readTypeRef(...)] is not a function";
      case 3: return "readAnyLookupTable[(127 - readUint8(...))] is not a function";
      case 4: return "Do not know how to serialize a BigInt";
      case 5: return "Method get TypedArray.prototype.byteLength called on incompatible receiver [object Object]";
      case 6:
        snprintf(buf, sizeof buf, "Cannot set property %s of [object Object] which has only a getter", getters[arg & 3]);
        return buf;
      case 7: return "Cannot assign to read only property 'BYTES_PER_ELEMENT' of object '[object Object]'";
      case 8: return "Cannot read property 'length' of undefined";
      case 9: return "Invalid code point NaN";
      case 10: return "Offset is outside the bounds of the DataView";
      case 12: return "Cannot read property 'origin' of undefined";
      case 11:
        if (arg == 0x7fff) return "Invalid typed array length";
        snprintf(buf, sizeof buf, "Invalid typed array length: %d", arg);
        return buf;
      default: break;
    }
    code &= 0xff;
  }
  switch (code) {
    case YM_OK: return "ok";
    case YM_ERR_INT_RANGE: return "Integer out of range!";
    case YM_ERR_UNEXPECTED: return "Unexpected case";
    case YM_ERR_URI: return "URI malformed";
    case YM_ERR_TYPE: return "unknown content, type or value tag";
    case YM_ERR_RANGE: return "read past the end of the update";
    case YM_ERR_SYNTAX: return "Unexpected token in JSON";
    case YM_ERR_UNSUPPORTED: return "input needs a canonicalisation the engine does not implement";
    case YM_ERR_METHOD: return "Method unimplemented";
    case YM_ERR_CAPACITY: return "output arena too small";
    default: return code < 0 ? "HIP runtime error" : "unknown status";
  }
}

// ---- pinned host memory pool (ym_host_alloc / ym_host_free) -----------------------------------------------
// Page-locked buffers in power-of-two size classes (>= 64 KiB), kept on per-class free lists when released:
// a serving loop that hands every call a fresh output arena (the Node addon's external ArrayBuffers) gets
// memory the DMA engines write directly, without first-touch page faults or the runtime's staging copy.
void *ym_host_alloc(size_t bytes) {
  const int k = pool_class(bytes ? bytes : 1);
  std::lock_guard<std::mutex> g(g_pool_mu);
  void *p = nullptr;
  if (!g_pool_free[k].empty()) {
    p = g_pool_free[k].back();
    g_pool_free[k].pop_back();
  } else if (hipHostMalloc(&p, 1ull << k, hipHostMallocPortable) != hipSuccess) {  // (coherent: kernels read it at
                                                                                   // 50-56 GB/s, non-coherent 43)
    return nullptr;
  }
  g_pool_live.emplace_back(p, k);
  return p;
}

void ym_host_free(void *p) {
  if (!p) return;
  std::lock_guard<std::mutex> g(g_pool_mu);
  for (size_t i = 0; i < g_pool_live.size(); i++) {
    if (g_pool_live[i].first != p) continue;
    g_pool_free[g_pool_live[i].second].push_back(p);
    g_pool_live[i] = g_pool_live.back();
    g_pool_live.pop_back();
    return;
  }
}

uint64_t ym_out_bound(const ym_batch *b) {
  // device batches: the fast-path slot region (2 * in + 64 per doc) followed by room for general-path
  // outputs; host batches: the packed outputs only (the library stages the slot region itself)
  if (b->mem == YM_MEM_HOST && b->upd_off) {
    const uint32_t *o32 = reinterpret_cast<const uint32_t *>(b->upd_off);
    const uint64_t in_h = (b->format & YM_OFF32) ? (uint64_t)o32[b->n_upd] - o32[0] : b->upd_off[b->n_upd] - b->upd_off[0];
    const uint64_t sv_h = b->sv_off ? b->sv_off[b->n_docs] - b->sv_off[0] : 0;
    return 2 * in_h + 2 * sv_h + 64ull * b->n_docs + 8192;
  }
  uint64_t in = 0;
  if (b->mem == YM_MEM_HOST && b->upd_off) in = b->upd_off[b->n_upd] - b->upd_off[0];
  else in = (uint64_t)b->n_upd * 64;
  uint64_t sv = 0;
  if (b->mem == YM_MEM_HOST && b->sv_off) sv = b->sv_off[b->n_docs] - b->sv_off[0];
  return 4 * in + 2 * sv + 128ull * b->n_docs + 8192;
}

int ym_merge(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_MERGE, b, out, stream, stats); }

// Asynchronous submission (include/ymerge.h): the LDS fast path alone, enqueued on the stream; no host
// round trip, no finishing kernel.  Declined documents keep status ST_PENDING (YM_PENDING) and are counted
// into *pending (device memory); the per-document capacity check of the fast kernels reports YM_ERR_CAPACITY.
int ym_merge_async(const ym_batch *b, ym_out *out, void *stream, uint32_t *pending) {
  if (!b || !out || b->mem != YM_MEM_DEVICE) return -1;
  DevState *S = state();
  {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != S->device) HIPCHK(hipSetDevice(S->device));
  }
  hipStream_t st = stream ? (hipStream_t)stream : S->stream;
  const uint32_t nd = b->n_docs;
  if (nd == 0) return 0;
  if (S->counters.ensure(1024)) return -2;
  GeneralJob j;
  memset(&j, 0, sizeof(j));
  j.A = b->arena;
  const bool off32 = (b->format & YM_OFF32) != 0;
  j.v2 = (b->format & 0xff) == YM_V2;
  if (off32) {
    j.upd_off32 = reinterpret_cast<const uint32_t *>(b->upd_off);
    if (j.v2) {
      // the V2 kernel reads u64 offsets: widened into the async path's own buffer.  The widening waits (on the
      // device, stream-ordered) for the previous async call that read the buffer, on whatever stream it ran;
      // the synchronous entry points use other buffers, so interleaving them with async calls is safe.
      if (!S->ev_async) HIPCHK(hipEventCreateWithFlags(&S->ev_async, hipEventDisableTiming));
      // growing the buffer frees the old one, which the previous async call (any stream) may still read: wait
      // for it on the host first, as run_async does for its buffers
      if ((b->n_upd + 1) * 8ull > S->async_off.cap) HIPCHK(hipEventSynchronize(S->ev_async));
      if (S->async_off.ensure((b->n_upd + 1) * 8ull)) return -2;
      HIPCHK(hipStreamWaitEvent(st, S->ev_async, 0));
      k_widen<<<(b->n_upd + 256) / 256, 256, 0, st>>>(j.upd_off32, S->async_off.as<uint64_t>(), b->n_upd + 1);
      j.upd_off = S->async_off.as<uint64_t>();
    }
  } else {
    j.upd_off = b->upd_off;
  }
  j.doc_upd = b->doc_upd;
  j.op = OP_MERGE;
  j.status = out->status;
  j.out = out->arena;
  j.cap = out->cap;
  j.out_off = out->out_off;
  j.out_len = out->out_len;
  j.n = nd;
  j.pend_list = nullptr;  // declines are only counted
  j.pend_count = pending ? pending : reinterpret_cast<uint32_t *>(S->counters.as<uint64_t>() + 15);
  int fr = fast_launch(OP_MERGE, j, b->n_upd, st);
  if (fr == 0) fr = fast2_launch(OP_MERGE, j, b->n_upd, st);
  if (fr < 0) return fr;
  if (off32 && j.v2) HIPCHK(hipEventRecord(S->ev_async, st));
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
int ym_diff(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_DIFF, b, out, stream, stats); }

// Asynchronous diff / state vector (include/ymerge.h): the streamed single-update kernels enqueued without a
// host round trip -- small documents one per lane or per wave, k_big_v1 / k_big_v2 the rest; no chunk- or
// column-parallel pass (those size their records on the host) and no general path.  The call's counters,
// done flags and walker scratch are the async path's own: each call waits (on the device) for the previous one.
static int run_async(uint32_t op, const ym_batch *b, ym_out *out, void *stream, uint32_t *pending) {
  if (!b || !out || b->mem != YM_MEM_DEVICE) return -1;
  if (op == OP_DIFF && (!b->sv_arena || !b->sv_off)) return -1;
  DevState *S = state();
  {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != S->device) HIPCHK(hipSetDevice(S->device));
  }
  hipStream_t st = stream ? (hipStream_t)stream : S->stream;
  const uint32_t nd = b->n_docs;
  if (nd == 0) return 0;
  constexpr uint32_t GRID = 2048;  // k_big_*'s blocks (BS_BYTES of scratch each)
  const uint32_t grid = nd < GRID ? nd : GRID;
  const bool off32 = (b->format & YM_OFF32) != 0;
  const uint64_t ws_bytes = 64 + ((nd + 15ull) & ~15ull) + 64;
  if (!S->ev_async2) HIPCHK(hipEventCreateWithFlags(&S->ev_async2, hipEventDisableTiming));
  // growing a buffer frees it: let the previous async call finish reading it first
  if (S->async2_ws.cap < ws_bytes || S->async2_bs.cap < grid * BS_BYTES || (off32 && S->async2_off.cap < (b->n_upd + 1) * 8ull))
    HIPCHK(hipEventSynchronize(S->ev_async2));
  if (S->async2_ws.ensure(ws_bytes) || S->async2_bs.ensure(grid * BS_BYTES) ||
      (off32 && S->async2_off.ensure((b->n_upd + 1) * 8ull)))
    return -2;
  HIPCHK(hipStreamWaitEvent(st, S->ev_async2, 0));
  uint64_t *ctr = S->async2_ws.as<uint64_t>();  // [0] used (bump allocator), [1] declined (u32), [2] completions
  uint8_t *done = S->async2_ws.as<uint8_t>() + 64;
  HIPCHK(hipMemsetAsync(ctr, 0, ws_bytes, st));
  GeneralJob j;
  memset(&j, 0, sizeof(j));
  j.A = b->arena;
  j.v2 = (b->format & 0xff) == YM_V2;
  if (off32) {
    j.upd_off32 = reinterpret_cast<const uint32_t *>(b->upd_off);
    k_widen<<<(b->n_upd + 256) / 256, 256, 0, st>>>(j.upd_off32, S->async2_off.as<uint64_t>(), b->n_upd + 1);
    j.upd_off = S->async2_off.as<uint64_t>();
  } else {
    j.upd_off = b->upd_off;
  }
  j.doc_upd = b->doc_upd;
  j.sv = op == OP_DIFF ? b->sv_arena : nullptr;
  j.sv_off = op == OP_DIFF ? b->sv_off : nullptr;
  j.op = op;
  j.status = out->status;
  j.out = out->arena;
  j.cap = out->cap;
  j.out_off = out->out_off;
  j.out_len = out->out_len;
  j.used = ctr;
  j.pend_list = nullptr;  // declines are only counted
  j.pend_count = pending ? pending : reinterpret_cast<uint32_t *>(ctr + 1);
  j.pw_count = ctr + 2;
  j.n = nd;
  j.bscratch = S->async2_bs.as<uint8_t>();
  int fr = big_async_launch(op, j, done, grid, st);
  if (fr == 0) fr = big2_async_launch(op, j, done, grid, st);
  if (fr <= 0) return fr < 0 ? fr : -1;
  HIPCHK(hipEventRecord(S->ev_async2, st));
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
int ym_diff_async(const ym_batch *b, ym_out *out, void *stream, uint32_t *pending) { return run_async(OP_DIFF, b, out, stream, pending); }
int ym_sv_async(const ym_batch *b, ym_out *out, void *stream, uint32_t *pending) { return run_async(OP_SV, b, out, stream, pending); }
int ym_sv(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_SV, b, out, stream, stats); }
int ym_convert(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_CONV, b, out, stream, stats); }
int ym_meta(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_META, b, out, stream, stats); }
int ym_ds_merge(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_DSMERGE, b, out, stream, stats); }
int ym_snapshot(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_SNAP, b, out, stream, stats); }
int ym_compact(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats) { return run_op(OP_COMPACT, b, out, stream, stats); }

}  // extern "C"
