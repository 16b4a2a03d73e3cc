/*
 * ymerge.h -- C ABI of libymerge.so, the MI355X-native batched Yjs update engine.
 *
 * Drop-in boundary for the yjs binary update layer.  Each entry point is the batched form of one
 * yjs function; the per-document semantics (bytes in, bytes out, errors) are those of yjs 13.5.16,
 * whose wire format is gaberogan/yjs@v0's (src/utils/UpdateEncoder.js, UpdateDecoder.js):
 *
 *   ym_merge(fmt=1)  <- Y.mergeUpdates(updates)            (yjs 13.5.16 `is`; public API beside
 *   ym_merge(fmt=2)  <- Y.mergeUpdatesV2(updates)           /root/reference/src/index.js:53-67)
 *   ym_diff(fmt=1)   <- Y.diffUpdate(update, stateVector)   (13.5.16 `fs`; reference composition:
 *   ym_diff(fmt=2)   <- Y.diffUpdateV2(update, sv)            src/utils/encoding.js:462-526)
 *   ym_sv(fmt=1|2)   <- Y.encodeStateVectorFromUpdate[V2]    (13.5.16 `cs`/`os`; reference composition:
 *                                                             src/utils/encoding.js:587-611)
 *
 * All pointers are plain byte/offset arrays; no framework types cross this boundary.  `mem` says
 * where every array of a batch lives: YM_MEM_HOST (the library stages it through pinned memory) or
 * YM_MEM_DEVICE (already resident in HBM on the selected device -- the throughput path).
 *
 * Batch layout: document d owns updates doc_upd[d] .. doc_upd[d+1]-1; update u is the byte range
 * arena[upd_off[u] .. upd_off[u+1]).  For ym_diff, doc d's state vector is
 * sv_arena[sv_off[d] .. sv_off[d+1]) and doc d must own exactly one update.
 *
 * Results: out_off[d] / out_len[d] locate doc d's output inside out_arena (device batches: 16-byte
 * aligned slots, not necessarily contiguous or in document order; host batches: packed back to back in
 * document order); status[d] is a status word: bits 0-7 the YM_* class (YM_STATUS_CLASS), bits 8-15
 * which of the class's exceptions yjs throws and bits 16-30 its argument -- ym_strerror(status[d])
 * renders the message yjs's exception carries under V8 (e.g. "Invalid typed array length: 7").
 * A doc whose status is not YM_OK has out_len[d] = 0.
 * Errors are per document; the batch always completes.
 * ym_out_bound() gives a capacity that normally suffices; out->used reports what was needed.
 */
#ifndef YMERGE_H
#define YMERGE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* per-document status codes (the JS wrapper rethrows the matching yjs exception) */
enum {
  YM_OK = 0,
  YM_ERR_INT_RANGE = 1,   /* Error('Integer out of range!')  (lib0 readVarUint / truncated input)  */
  YM_ERR_UNEXPECTED = 2,  /* Error('Unexpected case')                                            */
  YM_ERR_URI = 3,         /* URIError('URI malformed')       (invalid UTF-8 / split surrogate)    */
  YM_ERR_TYPE = 4,        /* TypeError                       (unknown content ref, typeRef, tag)  */
  YM_ERR_RANGE = 5,       /* RangeError                      (truncated string / typed array)     */
  YM_ERR_SYNTAX = 6,      /* SyntaxError                     (JSON.parse of a V1 JSON field)      */
  YM_ERR_UNSUPPORTED = 7, /* valid input needing a canonicalisation the engine does not implement */
  YM_ERR_METHOD = 8,      /* Error('Method unimplemented')                                       */
  YM_ERR_CAPACITY = 9,    /* output arena too small: call again with a larger cap                */
  YM_PENDING = 101,       /* ym_*_async only: declined by the async kernels, pass it to ym_merge etc. */
};

#define YM_STATUS_CLASS(s) ((s) & 0xff)

enum { YM_MEM_HOST = 0, YM_MEM_DEVICE = 1 };
enum { YM_V1 = 1, YM_V2 = 2 };
/* ym_ds_merge only, or-ed into ym_batch.format: the reference's own sortAndMergeDeleteSet
 * (gaberogan/yjs@v0 src/utils/DeleteSet.js:113-135: only exactly adjacent ranges coalesce) instead of
 * yjs 13.5.16's (touching and overlapping ranges merge) */
enum { YM_DS_REF = 0x100 };
/* or-ed into ym_batch.format: upd_off points to n_upd + 1 uint32_t offsets (an arena below 4 GiB)
 * instead of uint64_t.  Device batches: the V1 merge fast kernel reads them as they are (half the
 * offset bytes per update); other paths widen them on the device first. */
enum { YM_OFF32 = 0x200 };
/* ym_snapshot only, or-ed into ym_batch.format: the output encoding (default: the input's) */
enum { YM_OUT_V1 = 0x1000, YM_OUT_V2 = 0x2000 };
/* ym_compact only, or-ed into ym_batch.format: the document is new Y.Doc({ gc: false }) (deleted content
 * is kept and written; Doc.js:40-43, Transaction.js:302-304) */
enum { YM_NO_GC = 0x4000 };
/* ym_compact only, or-ed into ym_batch.format: each output is the compacted Doc's encodeStateVector(doc)
 * (reference src/utils/encoding.js:572-611; clients in StructStore insertion order, StructStore.js:49-56 --
 * the SyncStep1 a server that keeps Docs sends) immediately followed by the update; the state vector is
 * self-delimiting (vu(n) then n (client, clock) varuint pairs) */
enum { YM_SV_FIRST = 0x10000 };

typedef struct ym_batch {
  const uint8_t *arena;    /* concatenated update bytes                                   */
  const uint64_t *upd_off; /* n_upd + 1 byte offsets into arena (uint32_t with YM_OFF32)  */
  const uint32_t *doc_upd; /* n_docs + 1 update-index ranges                              */
  uint32_t n_docs;
  uint32_t n_upd;
  int32_t format;          /* YM_V1 | YM_V2                                               */
  int32_t mem;             /* YM_MEM_HOST | YM_MEM_DEVICE (applies to every array here)   */
  const uint8_t *sv_arena; /* ym_diff: concatenated encoded state vectors; ym_compact:     */
                           /* target state vectors (NULL: none); other ops: ignored       */
  const uint64_t *sv_off;  /* n_docs + 1 (with sv_arena)                                  */
} ym_batch;

typedef struct ym_out {
  uint8_t *arena;    /* output bytes, capacity `cap` (same memory kind as the batch)      */
  uint64_t cap;
  uint64_t *out_off; /* n_docs                                                            */
  uint64_t *out_len; /* n_docs                                                            */
  int32_t *status;   /* n_docs                                                            */
  uint64_t used;     /* filled in: bytes of `arena` used (if > cap, retry with cap=used)  */
} ym_out;

/* per-call statistics (also reduced across ranks by the benchmark over RCCL) */
typedef struct ym_stats {
  uint64_t docs, docs_fast, docs_general, docs_error;
  uint64_t bytes_in, bytes_out;
  double device_ms;  /* device time of the call (HIP events on the call's stream)          */
  double fast_ms;    /* ... of the LDS fast-path kernel alone                              */
  double general_ms; /* ... of the general path (workspace sizing + both passes)           */
  uint64_t docs_large; /* documents merged by the large-document pipeline (ym_large.hip)     */
  double large_ms;   /* ... device time of that pipeline                                   */
  uint64_t docs_chunked; /* diff / sv documents done by the chunk-parallel walk (ym_pwalk.hip) */
} ym_stats;

int ym_init(int device);           /* select the HIP device for this thread; 0 on success */
int ym_shutdown(void);
/* message of a status word / return code: for a per-document exception the text yjs's exception
 * carries (Node 12 / V8 7.x wording; thread-local buffer, valid until the thread's next call) */
const char *ym_strerror(int code);
uint64_t ym_out_bound(const ym_batch *b); /* a capacity that is normally sufficient for ym_* */
/* Page-locked host memory from the library's pool (power-of-two size classes, recycled by ym_host_free):
 * host batches whose arrays live there are copied by the DMA engines directly (no staging copy, no first-touch
 * page faults on the outputs).  Host merges of >= 4,096 documents with YM_OFF32 offsets run pipelined: the
 * batch is cut into chunks of ~3 MiB of input, and chunk c + 1 is copied in while chunk c is merged and its
 * packed outputs copied out.  Any pointer works as before; these just make the copies faster. */
void *ym_host_alloc(size_t bytes);
void ym_host_free(void *p);

/* stream: a hipStream_t (NULL = the library's stream for the device).  Return value: 0, or
 * YM_ERR_CAPACITY when out->used > out->cap (nothing useful was written), or a negative HIP error. */
int ym_merge(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
/* Asynchronous ym_merge for device batches (the serving loop: calls queue back to back on `stream` and
 * the host never waits).  Runs the LDS fast path only (small documents: <= 128 updates, <= 2,432 B V1;
 * the C2 / C4 shapes) and returns once the kernel is enqueued; the results are valid when the stream has
 * drained.  Each output lands in the slot region [0, 2 * input bytes + 64 * n_docs + 64) of out->arena
 * (out->cap below that: YM_ERR_CAPACITY for the documents that do not fit); out->used is not written.
 * A document the fast path declines (larger, rich nested content, invalid input) gets status YM_PENDING
 * and increments *pending (a uint32_t in device memory, or NULL): run those through ym_merge.
 * V2 batches with YM_OFF32 widen their offsets into a device buffer of the async path's own (the synchronous
 * entry points never touch it, so they may run on other streams at the same time); an async call of that kind
 * waits on the device for the previous one to finish reading it, whatever stream either runs on.
 * Return value: 0, or a negative error (not a device batch, HIP launch failure). */
int ym_merge_async(const ym_batch *b, ym_out *out, void *stream, uint32_t *pending);
int ym_diff(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
int ym_sv(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
/* Asynchronous ym_diff / ym_sv for device batches (a sync server answering SyncStep1 messages back to back
 * on `stream`): the single-update walkers only (small documents one per lane or per wave, the rest one wave
 * per document), enqueued without a host round trip; the results are valid when the stream has drained.
 * Outputs are bump-allocated from the start of out->arena (out->used is not written); a document that does
 * not fit gets YM_ERR_CAPACITY.  A V2 diff's walker re-encodes the columns in scratch taken from the same
 * arena: 8 x the input bytes + 2 x the state-vector bytes + (1 KB + 384 B per client section) per document
 * always suffices.  A document the walkers decline (several updates, more than 2,048 client
 * sections or state-vector entries, non-canonical or invalid input) gets YM_PENDING and increments *pending
 * (a uint32_t in device memory, or NULL): run those through ym_diff / ym_sv, which also report their
 * exceptions.  Large single updates run on the one-wave walker here (the chunk- and column-parallel passes
 * of the synchronous calls size their records on the host).  The async calls share device scratch: each
 * waits on the device for the previous one, whatever stream either runs on (the synchronous entry points
 * and ym_merge_async use other buffers).  Return value: 0, or a negative error. */
int ym_diff_async(const ym_batch *b, ym_out *out, void *stream, uint32_t *pending);
int ym_sv_async(const ym_batch *b, ym_out *out, void *stream, uint32_t *pending);
/* convertUpdateFormatV1ToV2 (b->format = YM_V1) / convertUpdateFormatV2ToV1 (b->format = YM_V2): one
 * update per document, re-encoded in the other format (yjs 13.5.x convertUpdateFormat, bundle ms@41803) */
int ym_convert(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
/* parseUpdateMeta (b->format = YM_V1) / parseUpdateMetaV2 (YM_V2), yjs 13.5.16: one update per document.
 * The two Maps it returns are written as from then to, each vu(size) | (client, clock)* in Map order
 * (the encoding of encodeStateVector, reference src/utils/encoding.js:572-579). */
int ym_meta(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
/* PermanentUserData's delete-set merge (reference src/utils/PermanentUserData.js:49-54): the "updates" of
 * document d are encoded delete sets (DSEncoderV1 bytes for YM_V1, DSEncoderV2 for YM_V2, as
 * encodeSnapshot[V2] writes them, src/utils/Snapshot.js:84-101); the output is
 * writeDeleteSet(mergeDeleteSets(readDeleteSet(each))) in the same encoding (13.5.16 union, he@10482;
 * with YM_DS_REF in b->format the reference's adjacency-only coalescing, DeleteSet.js:113-161). */
int ym_ds_merge(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
/* Snapshot codec (reference src/utils/Snapshot.js:84-124): one encoded snapshot per document (DSEncoderV1
 * for YM_V1 input, DSEncoderV2 for YM_V2), written back as encodeSnapshot / encodeSnapshotV2 (YM_OUT_V1 /
 * YM_OUT_V2 or-ed into b->format; default the input's encoding) of decodeSnapshot[V2](input): normalisation
 * (repeated clients merged in Map order) and V1 <-> V2 conversion, with decodeSnapshot's exceptions. */
int ym_snapshot(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);
/* Doc round-trip compaction: per document, the reference's own
 *   const doc = new Y.Doc()            (gc: true; with YM_NO_GC in b->format, { gc: false })
 *   updates.forEach(u => Y.applyUpdate[V2](doc, u))
 *   Y.encodeStateAsUpdate[V2](doc)      (with b->sv_arena: Y.encodeStateAsUpdate[V2](doc, sv), doc d's
 *                                        target state vector sv_arena[sv_off[d] .. sv_off[d+1]) -- only the
 *                                        structs the target lacks, the whole delete set; encoding.js:71-116)
 * (gaberogan/yjs@v0 src/utils/encoding.js:350-383 readUpdate / applyUpdate, :490-526 encodeStateAsUpdate;
 * structs integrated by Item.integrate, deletions applied, deleted content garbage-collected and runs of
 * structs merged by cleanupTransactions, src/utils/Transaction.js:244-367) in b->format.  Structs whose
 * dependencies never arrive stay pending (pendingStack / pendingClientsStructRefs, encoding.js:225-321) and
 * so do deletions of unseen clocks (pendingDeleteReaders, DeleteSet.js:270-323): like the reference, the
 * output is the integrated store and its delete set only (encoding.js:490-493).  An input on which the
 * reference throws reports that exception (class and message, ym_strerror).  A document whose workspace
 * does not fit the device-memory budget (YMERGE_COMPACT_WS_GB, default 16 GiB per launch) reports
 * YM_ERR_CAPACITY; large batches run in budget-sized chunks. */
int ym_compact(const ym_batch *b, ym_out *out, void *stream, ym_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
