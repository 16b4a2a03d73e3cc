// ym_cmap.h -- per-block client map of the streamed diff / state-vector walkers (ym_big.hip, ym_big2.hip,
// ym_pwalk.hip), in the block's HBM scratch (BS_MAP): open addressing over BS_MAP_SLOTS slots, key =
// client + 1 (0 = empty), value = index + 1 of the entry it maps to.  Client 0xFFFFFFFF (a valid id: a
// 5-byte varuint) has no key of that form; its value lives in the word after the table (XW, 0 = absent).
//
// Why: a diff looks up sv[client] once per client section, and the delete set checks every client
// against the ones before it.  With ~1,000 clients (C5) a ballot scan over the list is ~16 dependent
// loads per lookup and the delete-set check quadratic; the map answers both with one probe load (64
// slots per wave load).  Used only above 64 entries, where one wave load no longer covers the list.
//
// The map is written with device-scope atomics and read with device-scope atomic loads: the table is
// reused document after document by the same block, so its lines may sit stale in the CU's L1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ymk {
namespace cmap {

constexpr uint32_t SLOTS = BS_MAP_SLOTS, MASK = SLOTS - 1, XW = 2 * SLOTS, XCLIENT = 0xffffffffu;
static_assert((SLOTS & MASK) == 0 && SLOTS >= 2 * BS_NSV && SLOTS >= 2 * BS_NDSC, "map load factor <= 1/2");

__device__ __forceinline__ uint32_t hash(uint32_t client) { return (client * 0x9E3779B1u) >> (32 - __builtin_ctz(SLOTS)); }
__device__ __forceinline__ uint32_t ld(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all lanes of the (one-wave) block
__device__ __forceinline__ void clear(uint32_t *m) {
  for (uint32_t i = threadIdx.x; i <= XW; i += 64) __hip_atomic_store(m + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence();
  __syncthreads();
}

// decodeStateVector (encoding.js:536-545): entries in order, a later entry for a client wins -- each
// slot keeps the largest index mapped to it.  svt = (client, clock) pairs.
__device__ __forceinline__ void build_sv(uint32_t *m, const uint32_t *svt, uint32_t nsv) {
  clear(m);
  for (uint32_t i = threadIdx.x; i < nsv; i += 64) {
    if (svt[2 * i] == XCLIENT) {
      __hip_atomic_fetch_max(m + XW, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    const uint32_t key = svt[2 * i] + 1;
    uint32_t s = hash(key - 1);
    for (uint32_t probe = 0; probe < SLOTS; probe++, s = (s + 1) & MASK) {
      uint32_t old = 0;
      __hip_atomic_compare_exchange_strong(m + s, &old, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == 0 || old == key) {
        __hip_atomic_fetch_max(m + SLOTS + s, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __threadfence();
  __syncthreads();
}

// the slot holding `client` (wave-uniform, != XCLIENT), or NONE; *empty = the first empty slot of its
// probe sequence
__device__ __forceinline__ uint32_t find(const uint32_t *m, uint32_t client, uint32_t *empty) {
  const uint32_t key = client + 1, s0 = hash(client);
  for (uint32_t b = 0; b < SLOTS; b += 64) {
    const uint32_t s = (s0 + b + threadIdx.x) & MASK;
    const uint32_t kv = ld(m + s);
    const uint64_t hit = __ballot(kv == key), emp = __ballot(kv == 0);
    if (hit | emp) {
      const uint32_t fh = hit ? (uint32_t)__builtin_ctzll(hit) : 64, fe = emp ? (uint32_t)__builtin_ctzll(emp) : 64;
      if (empty) *empty = fe < 64 ? (s0 + b + fe) & MASK : 0xffffffffu;
      return fh < fe ? (s0 + b + fh) & MASK : 0xffffffffu;
    }
  }
  if (empty) *empty = 0xffffffffu;
  return 0xffffffffu;
}

// sv[client] (0 when absent) from a map built by build_sv
__device__ __forceinline__ uint32_t sv_get(const uint32_t *m, const uint32_t *svt, uint32_t client) {
  const uint32_t v = client == XCLIENT ? ld(m + XW) : 0;
  const uint32_t s = client == XCLIENT ? 0xffffffffu : find(m, client, nullptr);
  if (client == XCLIENT ? v == 0 : s == 0xffffffffu) return 0;
  const uint32_t i = (client == XCLIENT ? v : ld(m + SLOTS + s)) - 1;
  return svt[2 * i + 1];
}

// the delete set's client check: true when `client` was inserted before; else inserts it (map cleared
// by `clear` before the first client)
__device__ __forceinline__ bool seen_insert(uint32_t *m, uint32_t client) {
  uint32_t e = 0xffffffffu;
  if (client == XCLIENT) {
    if (ld(m + XW)) return true;
    e = XW;
  } else {
    if (find(m, client, &e) != 0xffffffffu) return true;
  }
  if (threadIdx.x == 0 && e != 0xffffffffu) __hip_atomic_store(m + e, client == XCLIENT ? 1u : client + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence();
  __syncthreads();
  return false;
}

}  // namespace cmap
}  // namespace ymk
