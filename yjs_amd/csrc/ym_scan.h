// ym_scan.h -- the library's own device-wide exclusive prefix sums and flagged selection (the two-pass
// size-then-write pipeline's offsets: per-document workspace / output / record offsets, work lists), in place
// of the hipcub primitives.  Reduce-then-scan over tiles of 2,048 elements (256 threads x 8 consecutive
// elements): a tile kernel scans its tile and writes the tile total, one block scans the tile totals (a
// carried loop, any length), a third kernel adds each tile's base.  A batch of <= 2,048 elements is one
// kernel.  The element count may be read on the device (n_dev: the listed documents' update total of the
// large-document merge, which the host does not know without a round trip), bounded by the host's n_max.
// Same calling convention as hipcub: tmp == nullptr asks for the scratch size.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ymk {

// out[i] = in[0] + ... + in[i - 1] for i < n, n = n_dev ? min(*n_dev + n_add, n_max) : n_max (in == out allowed)
template <class T>
int scan_excl(void *tmp, size_t &tmp_bytes, const T *in, T *out, uint32_t n_max, hipStream_t st,
              const uint32_t *n_dev = nullptr, uint32_t n_add = 0);
// dst[0 .. *d_num) = (list ? list[i] : i) for the i < n with flags[i] != 0, in order
int select_flagged(void *tmp, size_t &tmp_bytes, const uint32_t *list, const uint8_t *flags, uint32_t *dst,
                   uint32_t *d_num, uint32_t n, hipStream_t st);

}  // namespace ymk
