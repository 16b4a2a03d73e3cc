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

// the state-vector table: diff = the decoded state vector; meta = (client, from, to) triples, at most one
// client per update byte
__device__ __forceinline__ uint64_t ws_sv_bytes(const GeneralJob &j, uint32_t d, uint64_t bytes) {
  if (j.op == OP_DIFF) return j.sv_off[d + 1] - j.sv_off[d];
  if (j.op == OP_META) return 3 * bytes + 6;
  return 0;
}

__device__ __forceinline__ void carve(const GeneralJob &j, uint32_t i, uint32_t d, DocWS &w) {
  uint32_t k = j.doc_upd[d + 1] - j.doc_upd[d];
  uint64_t bytes = j.upd_off[j.doc_upd[d + 1]] - j.upd_off[j.doc_upd[d]];
  GeneralWsSize z = general_ws_size(k, bytes, j.parts_mul, ws_sv_bytes(j, d, bytes));
  uint8_t *p = j.ws + j.ws_off[i];
  w.rs = (Reader *)p; p += z.rs;
  w.arr = (uint32_t *)p; p += z.arr;
  w.tmp = (uint32_t *)p; p += z.arr;
  w.parts = (PartRec *)p; p += z.parts; w.parts_cap = z.parts_cap;
  w.ds = (DSE *)p; p += z.ds; w.ds_cap = z.ds_cap;
  w.dsg = (DSG *)p; p += z.dsg;
  w.sv = (int64_t *)p; w.sv_cap = z.sv_cap;
}

__global__ void k_general_ws(GeneralJob j, uint64_t *ws_size) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= j.n) return;
  uint32_t d = job_doc(j, i);
  uint32_t k = j.doc_upd[d + 1] - j.doc_upd[d];
  uint64_t bytes = j.upd_off[j.doc_upd[d + 1]] - j.upd_off[j.doc_upd[d]];
  ws_size[i] = general_ws_size(k, bytes, j.parts_mul, ws_sv_bytes(j, d, bytes)).total;
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
  if (j.op == OP_MERGE) {
    if (k == 1) {  // `if (updates.length === 1) return updates[0]`
      uint64_t n = j.upd_off[u0 + 1] - j.upd_off[u0];
      if (pass == 1) { __builtin_memset(&L, 0, sizeof(Layout)); L.total = n; }
      else for (uint64_t b = 0; b < n; b++) out[b] = j.A[j.upd_off[u0] + b];
    } else {
      merge_doc(c, w, j.upd_off, u0, k, j.v2, pass, L, out);
    }
  } else if (j.op == OP_DIFF) {
    if (k != 1) c.err = ST_UNEXPECTED;
    else diff_doc(c, w, j.upd_off[u0], j.upd_off[u0 + 1] - j.upd_off[u0], j.sv + j.sv_off[d], j.sv_off[d + 1] - j.sv_off[d],
                  j.v2, pass, L, out);
  } else if (j.op == OP_DSMERGE) {
    dsmerge_doc(c, w, j.upd_off, u0, k, j.v2, pass, L, out);
  } else if (j.op == OP_META) {
    if (k != 1) c.err = ST_UNEXPECTED;
    else meta_doc(c, w, j.upd_off[u0], j.upd_off[u0 + 1] - j.upd_off[u0], j.v2, pass, L, out);
  } else if (j.op == OP_CONV) {
    if (k != 1) c.err = ST_UNEXPECTED;
    else conv_doc(c, w, j.upd_off[u0], j.upd_off[u0 + 1] - j.upd_off[u0], j.v2, pass, L, out);
  } else {
    if (k != 1) c.err = ST_UNEXPECTED;
    else sv_doc(c, w, j.upd_off[u0], j.upd_off[u0 + 1] - j.upd_off[u0], j.v2, pass, L, out);
  }
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
