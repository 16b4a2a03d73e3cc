// ym_compact.hip -- Doc round-trip compaction kernels (ym_compact()): per document
// the reference's applyUpdate[V2] of every input into a fresh gc=true Doc followed by
// encodeStateAsUpdate[V2] (ym_compact.h).  Struct integration is sequential within a document (every
// struct's position depends on the ones integrated before it), so documents are the parallel unit: one
// document per lane, `lanes` active lanes per 64-wide wave (1: one document per wave, no divergence
// between documents and >= one wave per document to hide HBM latency; 64: one document per lane).
// The document's state lives in its HBM workspace (carved by an exclusive scan of per-document sizes);
// one launch integrates, sizes the output, bump-allocates it and writes it in place.
#include <hip/hip_runtime.h>

#include "ym_compact.h"
#include "ym_kernels.h"

namespace ymk {
using namespace ym;

__device__ __forceinline__ uint32_t cpt_doc(const GeneralJob &j, uint32_t i) { return j.list ? j.list[i] : i; }

__global__ void k_compact_ws(GeneralJob j, uint64_t *ws_size) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= j.n) return;
  const uint32_t d = cpt_doc(j, i);
  const uint32_t k = j.doc_upd[d + 1] - j.doc_upd[d];
  const uint64_t bytes = j.upd_off[j.doc_upd[d + 1]] - j.upd_off[j.doc_upd[d]];
  ws_size[i] = cpt::ws_size(k, bytes, j.parts_mul).total;
}

// OCC: waves per SIMD the register allocation targets (1: 256 VGPRs + 98 AGPRs, no spills; 2: 256 registers,
// a few spills -- twice the waves in flight to hide the workspace's memory latency)
// big: documents of more input bytes run in a launch of their own, one per wave (a wave's lanes run their
// documents' divergent code one after the other: a few large documents sharing a wave serialise).
// part 0: every document; 1: only those above `big`; 2: only those up to `big`
template <int OCC>
__global__ void __launch_bounds__(64, OCC) k_compact(GeneralJob j, uint32_t lanes, uint64_t big, int part) {
  const uint32_t lane = threadIdx.x;
  if (lane >= lanes) return;
  const uint32_t i = blockIdx.x * lanes + lane;
  if (i >= j.n) return;
  const uint32_t d = cpt_doc(j, i);
  const uint32_t u0 = j.doc_upd[d], k = j.doc_upd[d + 1] - u0;
  const uint64_t bytes = j.upd_off[u0 + k] - j.upd_off[u0];
  if ((part == 1 && bytes <= big) || (part == 2 && bytes > big)) return;
  const cpt::WsSize z = cpt::ws_size(k, bytes, j.parts_mul);
  uint8_t *ws = j.ws + (j.ws_off[i] - j.ws_base);
  Ctx c = {0, j.A};
  cpt::Result R;
  // ym_compact with sv_arena: doc d's target state vector (encodeStateAsUpdate(doc, sv))
  const uint8_t *svp = j.sv ? j.sv + j.sv_off[d] : nullptr;
  const uint64_t svlen = j.sv ? j.sv_off[d + 1] - j.sv_off[d] : 0;
  const uint32_t flags = j.v2 | (j.nogc << 1) | (j.svfirst << 2);
  cpt::compact_doc(c, ws, z, flags, j.upd_off, u0, k, svp, svlen, R, nullptr);
  if (c.err) {
    j.status[d] = c.err;
    j.out_len[d] = 0;
    if (c.err == ST_RETRY) atomicAdd(j.counter_retry, 1u);
    return;
  }
  const uint64_t off = atomicAdd((unsigned long long *)j.used, (unsigned long long)R.total);
  if (off + R.total > j.cap) {
    j.status[d] = ST_CAPACITY;
    j.out_len[d] = 0;
    return;
  }
  Ctx c2 = {0, j.A};
  cpt::compact_doc(c2, ws, z, flags, j.upd_off, u0, k, svp, svlen, R, j.out + off);
  j.status[d] = c2.err ? (c2.err == ST_RETRY ? ST_UNEXPECTED : c2.err) : ST_OK;
  j.out_off[d] = off;
  j.out_len[d] = c2.err ? 0 : R.total;
}

template __global__ void k_compact<1>(GeneralJob, uint32_t, uint64_t, int);
template __global__ void k_compact<2>(GeneralJob, uint32_t, uint64_t, int);

}  // namespace ymk
