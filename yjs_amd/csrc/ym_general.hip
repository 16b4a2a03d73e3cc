// ym_general.hip -- general-path kernels: one thread per document running ym_core.h's exact
// sequential restatement of yjs 13.5.16 mergeUpdates / diffUpdate / encodeStateVectorFromUpdate.
// Two launches per call (pass 1 sizes every output stream, pass 2 writes in place); the per-document
// workspace lives in HBM and is carved by an exclusive scan of per-document sizes.
#include <hip/hip_runtime.h>

#include "ym_core.h"
#include "ym_kernels.h"

namespace ymk {
using namespace ym;

__device__ __forceinline__ uint32_t job_doc(const GeneralJob &j, uint32_t i) { return j.list ? j.list[i] : i; }

__device__ __forceinline__ void carve(const GeneralJob &j, uint32_t i, uint32_t d, DocWS &w) {
  uint32_t k = j.doc_upd[d + 1] - j.doc_upd[d];
  uint64_t bytes = j.upd_off[j.doc_upd[d + 1]] - j.upd_off[j.doc_upd[d]];
  const uint64_t svlen = j.op == OP_DIFF ? j.sv_off[d + 1] - j.sv_off[d] : 0;
  general_carve(j.ws + j.ws_off[i], general_ws_size(k, bytes, j.parts_mul, general_sv_bytes(j.op, svlen, bytes), j.v2), w);
}

__global__ void k_general_ws(GeneralJob j, uint64_t *ws_size) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= j.n) return;
  uint32_t d = job_doc(j, i);
  uint32_t k = j.doc_upd[d + 1] - j.doc_upd[d];
  uint64_t bytes = j.upd_off[j.doc_upd[d + 1]] - j.upd_off[j.doc_upd[d]];
  const uint64_t svlen = j.op == OP_DIFF ? j.sv_off[d + 1] - j.sv_off[d] : 0;
  ws_size[i] = general_ws_size(k, bytes, j.parts_mul, general_sv_bytes(j.op, svlen, bytes), j.v2).total;
}

__global__ void __launch_bounds__(64) k_general(GeneralJob j, int pass) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= j.n) return;
  uint32_t d = job_doc(j, i);
  if (pass == 2 && j.status[d] != ST_OK) return;
  Ctx c = {0, j.A};
  DocWS w;
  carve(j, i, d, w);
  Layout &L = j.layout[d];
  uint32_t u0 = j.doc_upd[d], k = j.doc_upd[d + 1] - u0;
  uint8_t *out = pass == 2 ? j.out + j.out_off[d] : nullptr;
  const uint8_t *sv = j.op == OP_DIFF ? j.sv + j.sv_off[d] : nullptr;
  const uint64_t svlen = j.op == OP_DIFF ? j.sv_off[d + 1] - j.sv_off[d] : 0;
  general_doc(c, w, j.op, j.v2 | (j.dsref << 8) | (j.v2out << 9), j.upd_off, u0, k, sv, svlen, pass, L, out);
  if (pass == 1) {
    j.status[d] = c.err;
    if (c.err == ST_RETRY) atomicAdd(j.counter_retry, 1u);
    if (c.err == ST_OK) {
      unsigned long long off = atomicAdd((unsigned long long *)j.used, (unsigned long long)L.total);
      j.out_off[d] = off;
      j.out_len[d] = L.total;
      if (off + L.total > j.cap) j.status[d] = ST_CAPACITY;
    } else {
      j.out_len[d] = 0;
    }
  } else if (c.err) {
    j.status[d] = c.err == ST_RETRY ? ST_UNEXPECTED : c.err;  // cannot happen: pass 1 sized everything
    j.out_len[d] = 0;
  }
}

}  // namespace ymk
