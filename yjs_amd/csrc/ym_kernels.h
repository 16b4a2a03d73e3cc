// ym_kernels.h -- launch descriptors shared by the host API (ym_api.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ym_core.h"

namespace ymk {

using ym::OP_MERGE;
using ym::OP_DIFF;
using ym::OP_SV;
using ym::OP_CONV;
using ym::OP_META;
using ym::OP_DSMERGE;
using ym::OP_SNAP;
using ym::OP_COMPACT;

// internal status: document not taken by the fast path, routed to the general path
constexpr int ST_PENDING = 101;

struct GeneralJob {
  const uint8_t *A;          // update arena
  const uint64_t *upd_off;
  const uint32_t *upd_off32; // YM_OFF32 device batches: u32 offsets (read by the V1 fast kernel; the
                             // other kernels get widened u64 offsets in upd_off)
  const uint32_t *doc_upd;
  const uint8_t *sv;         // diff: state-vector arena
  const uint64_t *sv_off;
  uint32_t n;                // documents in this launch
  const uint32_t *list;      // document ids (nullptr: 0..n-1)
  uint32_t op, v2;
  uint32_t dsref;            // ym_ds_merge: the reference's adjacency-only coalescing (YM_DS_REF)
  uint32_t v2out;            // ym_snapshot: V2 output encoding
  uint32_t nogc;             // ym_compact: Doc({ gc: false }) (YM_NO_GC)
  uint32_t svfirst;          // ym_compact: the Doc's encodeStateVector before the update (YM_SV_FIRST)
  uint32_t parts_mul;        // part-table capacity multiplier (grown on ST_RETRY)
  uint8_t *ws;               // workspace
  const uint64_t *ws_off;    // per listed slot
  uint64_t ws_base;          // ws_off value at ws (ym_compact's chunked launches; 0 elsewhere)
  ym::Layout *layout;        // per doc
  int32_t *status;           // per doc
  uint8_t *out;              // output arena
  uint64_t cap;
  uint64_t *out_off, *out_len;  // per doc
  uint64_t *used;            // bump allocator over `out`
  uint32_t *counter_retry;
  uint32_t *pend_list;       // fast path: ids of the documents it declines (appended) ...
  uint32_t *pend_count;      // ... and their number
  uint8_t *bscratch;         // streamed single-update kernels: BS_BYTES per block (ym_big*.hip)
  const uint8_t *pw_done;    // V1 diff / sv: documents the chunk-parallel walk completed (ym_pwalk.hip)
  uint64_t *pw_count;        // ... and their number (a device counter k_finish reports and resets)
  uint32_t doc_base;         // merge fast paths over one chunk of a pipelined host batch (ym_api.hip run_host_pipe):
                             // doc_upd / status / out_off / out_len start at document doc_base of the batch, whose
                             // id this adds to the slot position and the declined list (0 elsewhere)
};

// Per-block HBM scratch of the streamed diff / state-vector kernels (ym_big.hip, ym_big2.hip): client
// sections (or parts), the decoded state vector and the delete set's clients.  Grid = BS_GRID blocks
// (grid-stride over documents), so the scratch is bounded whatever the batch size.
constexpr uint32_t BS_NSEC = 2048, BS_NSV = 2048, BS_NDSC = 2048, BS_PRE = 48, BS_SECW = 12;
constexpr uint64_t BS_SEC = 0;                                      // u32[BS_NSEC][BS_SECW]
constexpr uint64_t BS_PREB = BS_SEC + 4ull * BS_NSEC * BS_SECW;     // u8[BS_NSEC][BS_PRE]
constexpr uint64_t BS_SVT = BS_PREB + (uint64_t)BS_NSEC * BS_PRE;   // u32[BS_NSV][2]
constexpr uint64_t BS_DSC = BS_SVT + 8ull * BS_NSV;                 // u32[BS_NDSC]
constexpr uint32_t BS_MAP_SLOTS = 4096;                             // client map (ym_cmap.h)
constexpr uint64_t BS_MAP = BS_DSC + 4ull * BS_NDSC;                // u32[2][BS_MAP_SLOTS] keys, values
                                                                    // + u32[4] (client 0xFFFFFFFF's entry)
constexpr uint64_t BS_BYTES = BS_MAP + 8ull * BS_MAP_SLOTS + 16;
constexpr uint32_t BS_GRID = 8192;  // up to 32 one-wave blocks per CU; scratch sized by the launch's grid

// device buffers of the large-document merge pipeline (ym_large.hip), grown on demand, cached
struct LargeBufs {
  void *p[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t cap[4] = {0, 0, 0, 0};
  uint64_t *pinned = nullptr;
  uint64_t *pinned_dev = nullptr;  // (its device address: k_lm_totals writes the record totals there)
};
// Large-document merge over `list` (n documents the fast path declined).  Documents it takes get
// status OK; the rest keep ST_PENDING.  Returns 1 when launched, 0 when not applicable, < 0 on error.
int large_run(const GeneralJob &j, const uint32_t *list, uint32_t n, uint32_t n_upd, hipStream_t st, LargeBufs &B);

// device buffers of the chunk-parallel V1 walk (ym_pwalk.hip), grown on demand, cached
constexpr int PW_NBUF = 5;
struct PwBufs {
  void *p[PW_NBUF] = {};
  size_t cap[PW_NBUF] = {};
  uint32_t *pinned = nullptr;
  uint32_t *pinned_dev = nullptr;  // (its device address: a kernel writes the totals there, no copy op)
  hipEvent_t ev = nullptr;   // pw_prepare's totals have reached `pinned`
  bool pending = false;      // pw_prepare ran, pw_finish not yet
  uint32_t op = 0;
};
// Chunk-parallel walk + stitch over the large single-update documents of a V1 diff / sv call, in two steps:
// pw_prepare marks every document not done (*done) and sends the large documents' chunk / table totals to
// the host without waiting for them; the kernels of the small documents are enqueued next (their work hides
// that round trip); pw_finish then waits for the totals, sizes the record buffers and launches the walk and
// stitch (documents completed get done[d] = 1).  Return 1 when launched, 0 when not applicable, < 0 on error.
int pw_prepare(uint32_t op, const GeneralJob &j, hipStream_t st, PwBufs &B, const uint8_t **done);
int pw_finish(const GeneralJob &j, hipStream_t st, PwBufs &B);
// Small single updates of a V1 diff / sv / meta call, one document per lane (ym_small.hip); marks done[d].
int small_launch(uint32_t op, const GeneralJob &j, uint8_t *done, hipStream_t st, bool tiny_only = false);
// ... and what those left of 80 B - 4 KB: one wave per document (ym_pwalk.hip k_pw_small).
int pw_small_launch(uint32_t op, const GeneralJob &j, uint8_t *done, hipStream_t st);
// ym_segsort.hip: segments [seg_b[s], seg_e[s]) of (ki, vi) stably sorted by key into (ko, vo); (kt, vt) scratch
int segsort_pairs(const uint64_t *ki, const uint32_t *vi, uint64_t *ko, uint32_t *vo, uint64_t *kt, uint32_t *vt,
                  const uint32_t *seg_b, const uint32_t *seg_e, uint32_t nseg, hipStream_t st);
// The same for V2 (ym_pv2.hip): column-parallel diff / sv over large single-section documents.
int pv2_prepare(uint32_t op, const GeneralJob &j, hipStream_t st, PwBufs &B, const uint8_t **done);
int pv2_finish(const GeneralJob &j, hipStream_t st, PwBufs &B);

using ym::GeneralWsSize;
using ym::general_ws_size;
using ym::al16;

}  // namespace ymk
