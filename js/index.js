// yjs-compatible batched update API on the MI355X (libymerge.so via the N-API addon).
//
// Drop-in for yjs 13.5's update functions -- same names, same arguments, same results and the same
// exception classes -- plus *Batch variants that process many documents in one GPU call:
//   mergeUpdates(updates) / mergeUpdatesV2            (yjs: Y.mergeUpdates[V2])
//   diffUpdate(update, sv) / diffUpdateV2              (yjs: Y.diffUpdate[V2])
//   encodeStateVectorFromUpdate(update) / ...V2        (yjs: Y.encodeStateVectorFromUpdate[V2])
//   mergeUpdatesBatch(docs, {format}), diffUpdateBatch(updates, svs, {format}),
//   encodeStateVectorFromUpdateBatch(updates, {format})
//   convertUpdateFormatV1ToV2(update) / convertUpdateFormatV2ToV1(update), convertUpdateFormatBatch(updates, {format})
//                                                      (yjs 13.5.x convertUpdateFormat; format = the input's)
//   parseUpdateMeta(update) / parseUpdateMetaV2 -> {from: Map, to: Map}, parseUpdateMetaBatch(updates, {format})
//                                                      (yjs 13.5.16 parseUpdateMeta[V2])
//   mergeDeleteSetsBatch(docs, {format, reference}), mergeEncodedDeleteSets(encodedDss, {format, reference})
//                                                      (PermanentUserData.js:49-54: mergeDeleteSets over
//                                                       encoded delete sets -> one encoded delete set)
//   encodeSnapshot[V2] / decodeSnapshot[V2], encodeSnapshotBatch / decodeSnapshotBatch,
//   convertSnapshotBatch(bufs, {format, to})         (Snapshot.js:84-124 codec, V1 <-> V2)
//   every *Batch function also as *BatchAsync(...) -> Promise (the GPU call off the event loop)
// Exceptions carry yjs's class and message (V8 wording; include/ymerge.h status words).
// There is no CPU fallback: a missing addon or GPU throws.
'use strict'
const path = require('path')
const addon = require(path.join(__dirname, 'build', 'ymerge_napi.node'))

let initialised = false
function init () {
  if (!initialised) {
    const rc = addon.init(Number(process.env.YMERGE_DEVICE || 0))
    if (rc !== 0) throw new Error('ymerge: no usable MI355X/HIP device')
    initialised = true
  }
}

const OP = { merge: 0, diff: 1, sv: 2, conv: 3, meta: 4, dsmerge: 5, snapshot: 6, compact: 7 }
const fmtOf = o => (o && (o.format === 'v2' || o.format === 2)) ? 2 : 1

// status word -> the exception yjs itself throws for that input: the class from bits 0-7, the message
// (V8's wording, e.g. "Invalid typed array length: 7") rendered by the library (ym_strerror)
function toError (st) {
  const msg = addon.strerror(st)
  switch (st & 0xff) {
    case 1: case 2: case 8: return new Error(msg)
    case 3: return new URIError(msg)
    case 4: return new TypeError(msg)
    case 5: return new RangeError(msg)
    case 6: return new SyntaxError(msg)
    case 7: { const e = new Error('ymerge: ' + msg); e.code = 'YM_UNSUPPORTED'; return e }
    default: return new Error('ymerge status ' + st + ': ' + msg)
  }
}
const YM_DS_REF = 0x100 // mergeDeleteSets with the reference's adjacency-only coalescing (include/ymerge.h)
const YM_OUT_V1 = 0x1000 // ym_snapshot output encodings
const YM_OUT_V2 = 0x2000

// a large batch is packed into page-locked memory from the library's pool (addon.hostBuffer: DMA copies to the
// GPU, no per-call page pinning); small ones, or without a HIP runtime, into ordinary memory
const HOST_MIN = 1 << 20
function hostBytes (n, big) {
  const b = big ? addon.hostBuffer(n) : undefined
  return b || new Uint8Array(n)
}
function pack (docs) {
  let n = 0; let bytes = 0
  for (const d of docs) { n += d.length; for (const u of d) bytes += u.length }
  const big = bytes >= HOST_MIN
  const arena = hostBytes(bytes, big)
  // u32 offsets below 4 GiB (YM_OFF32 in the addon: half the offset bytes to copy, pipelined host merges)
  const updOff = bytes < 4294967296 ? new Uint32Array(hostBytes(4 * (n + 1), big).buffer, 0, n + 1) : new Float64Array(n + 1)
  const docUpd = new Uint32Array(hostBytes(4 * (docs.length + 1), big).buffer, 0, docs.length + 1)
  let o = 0; let u = 0
  docs.forEach((d, i) => {
    docUpd[i] = u
    for (const x of d) { arena.set(x, o); updOff[u] = o; o += x.length; u++ }
  })
  docUpd[docs.length] = u
  updOff[n] = o
  return { arena, updOff, docUpd }
}

function unpack (res, throwErrors) {
  const out = new Array(res.status.length)
  for (let d = 0; d < res.status.length; d++) {
    if (res.status[d] !== 0) {
      const e = toError(res.status[d])
      if (throwErrors) throw e
      out[d] = e
    } else {
      out[d] = res.arena.slice(res.offsets[d], res.offsets[d] + res.lengths[d])
    }
  }
  return out
}

// every batch call: run(...) synchronously, or runAsync(...) -> Promise (napi_async_work: the GPU call
// runs on a libuv worker thread and the event loop stays free)
function call (async, args, done) {
  init()
  if (!async) return done(addon.run(...args))
  return addon.runAsync(...args).then(done)
}
function mergeUpdatesBatch (docs, opts, throwErrors = false, async = false) {
  const p = pack(docs)
  return call(async, [OP.merge, fmtOf(opts), p.arena, p.updOff, p.docUpd], r => unpack(r, throwErrors))
}
function diffUpdateBatch (updates, svs, opts, throwErrors = false, async = false) {
  const p = pack(updates.map(u => [u]))
  const s = pack(svs.map(x => [x]))
  return call(async, [OP.diff, fmtOf(opts), p.arena, p.updOff, p.docUpd, s.arena, s.updOff], r => unpack(r, throwErrors))
}
function encodeStateVectorFromUpdateBatch (updates, opts, throwErrors = false, async = false) {
  const p = pack(updates.map(u => [u]))
  return call(async, [OP.sv, fmtOf(opts), p.arena, p.updOff, p.docUpd], r => unpack(r, throwErrors))
}

function convertUpdateFormatBatch (updates, opts, throwErrors = false, async = false) {
  const p = pack(updates.map(u => [u]))
  return call(async, [OP.conv, fmtOf(opts), p.arena, p.updOff, p.docUpd], r => unpack(r, throwErrors))
}

// Doc round-trip compaction (ym_compact): per document, encodeStateAsUpdate[V2] of a fresh Doc after
// applyUpdate[V2] of every update in order -- the reference's own compaction (structs merged, deleted
// content garbage-collected).  opts.gc === false: new Y.Doc({ gc: false }) (YM_NO_GC);
// opts.targetStateVectors: one encoded state vector per document, encodeStateAsUpdate[V2](doc, sv);
// opts.withStateVector: per document { stateVector: encodeStateVector(doc), update } (YM_SV_FIRST: the Doc's
// own state vector, clients in StructStore insertion order -- what a server keeping Docs sends as SyncStep1)
const YM_NO_GC = 0x4000
const YM_SV_FIRST = 0x10000
function splitStateVector (b) {
  let pos = 0
  const vu = () => { let v = 0; let m = 1; let x; do { x = b[pos++]; v += (x & 127) * m; m *= 128 } while (x & 128); return v }
  const n = vu()
  for (let i = 0; i < 2 * n; i++) vu()
  return { stateVector: b.subarray(0, pos), update: b.subarray(pos) }
}
function compactUpdatesBatch (docs, opts, throwErrors = false, async = false) {
  const p = pack(docs)
  const withSv = !!(opts && opts.withStateVector)
  const fmt = fmtOf(opts) | (opts && opts.gc === false ? YM_NO_GC : 0) | (withSv ? YM_SV_FIRST : 0)
  const args = [OP.compact, fmt, p.arena, p.updOff, p.docUpd]
  if (opts && opts.targetStateVectors) {
    if (opts.targetStateVectors.length !== docs.length) throw new RangeError('one target state vector per document')
    const s = pack(opts.targetStateVectors.map(x => [x]))
    args.push(s.arena, s.updOff)
  }
  return call(async, args, r => unpack(r, throwErrors).map(x => withSv && x instanceof Uint8Array ? splitStateVector(x) : x))
}
const compactUpdates = (updates, sv) => compactUpdatesBatch([updates], { format: 1, targetStateVectors: sv ? [sv] : null }, true)[0]
const compactUpdatesV2 = (updates, sv) => compactUpdatesBatch([updates], { format: 2, targetStateVectors: sv ? [sv] : null }, true)[0]
const compactUpdatesBatchAsync = (docs, opts, throwErrors = false) => compactUpdatesBatch(docs, opts, throwErrors, true)

// the engine writes parseUpdateMeta's two Maps as two encoded state vectors (from, then to)
function decodeMeta (b) {
  let pos = 0
  const vu = () => { let v = 0; let m = 1; for (;;) { const x = b[pos++]; v += (x & 0x7f) * m; m *= 128; if (x < 0x80) return v } }
  const res = {}
  for (const key of ['from', 'to']) {
    const m = new Map()
    for (let n = vu(); n > 0; n--) { const client = vu(); m.set(client, vu()) }
    res[key] = m
  }
  return res
}
function parseUpdateMetaBatch (updates, opts, throwErrors = false, async = false) {
  const p = pack(updates.map(u => [u]))
  return call(async, [OP.meta, fmtOf(opts), p.arena, p.updOff, p.docUpd],
    r => unpack(r, throwErrors).map(x => x instanceof Error ? x : decodeMeta(x)))
}
// opts.reference: the reference's own sortAndMergeDeleteSet (DeleteSet.js:113-135, only adjacent ranges
// coalesce) instead of yjs 13.5.16's union
function mergeDeleteSetsBatch (docs, opts, throwErrors = false, async = false) {
  const p = pack(docs)
  const fmt = fmtOf(opts) | (opts && opts.reference ? YM_DS_REF : 0)
  return call(async, [OP.dsmerge, fmt, p.arena, p.updOff, p.docUpd], r => unpack(r, throwErrors))
}
// Snapshot codec (reference src/utils/Snapshot.js:84-124) on the GPU: encodeSnapshot[V2](decodeSnapshot[V2](buf))
// per buffer -- normalisation and V1 <-> V2 conversion (opts.format: the input's, opts.to: the output's)
function convertSnapshotBatch (bufs, opts, throwErrors = false, async = false) {
  const p = pack(bufs.map(b => [b]))
  const to = opts && (opts.to === 'v2' || opts.to === 2) ? YM_OUT_V2 : (opts && (opts.to === 'v1' || opts.to === 1) ? YM_OUT_V1 : 0)
  return call(async, [OP.snapshot, fmtOf(opts) | to, p.arena, p.updOff, p.docUpd], r => unpack(r, throwErrors))
}
// the canonical V1 bytes the engine writes -> { ds: Map<client, [{clock, len}]>, sv: Map<client, clock> }
// (the shape of the reference's Snapshot: DeleteSet.clients and the state map)
function readSnapshotV1 (b) {
  let pos = 0
  const vu = () => { let v = 0; let m = 1; for (;;) { const x = b[pos++]; v += (x & 0x7f) * m; m *= 128; if (x < 0x80) return v } }
  const clients = new Map()
  for (let n = vu(); n > 0; n--) {
    const client = vu(); const items = []
    for (let m = vu(); m > 0; m--) { const clock = vu(); items.push({ clock, len: vu() }) }
    clients.set(client, items)
  }
  const sv = new Map()
  for (let n = vu(); n > 0; n--) { const client = vu(); sv.set(client, vu()) }
  return { ds: { clients }, sv }
}
// a snapshot object laid out as V1 bytes (the host only packs the values; the engine encodes)
function writeSnapshotV1 (s) {
  const out = []
  const vu = v => { while (v > 127) { out.push(128 | (v % 128)); v = Math.floor(v / 128) } out.push(v) }
  vu(s.ds.clients.size)
  s.ds.clients.forEach((items, client) => { vu(client); vu(items.length); for (const it of items) { vu(it.clock); vu(it.len) } })
  vu(s.sv.size)
  s.sv.forEach((clock, client) => { vu(client); vu(clock) })
  return Uint8Array.from(out)
}
const decodeSnapshotBatch = (bufs, opts, throwErrors = false) =>
  convertSnapshotBatch(bufs, { format: fmtOf(opts), to: 1 }, throwErrors).map(r => r instanceof Error ? r : readSnapshotV1(r))
const encodeSnapshotBatch = (snapshots, opts, throwErrors = false) =>
  convertSnapshotBatch(snapshots.map(writeSnapshotV1), { format: 1, to: fmtOf(opts) }, throwErrors)
const decodeSnapshot = buf => decodeSnapshotBatch([buf], { format: 1 }, true)[0]
const decodeSnapshotV2 = buf => decodeSnapshotBatch([buf], { format: 2 }, true)[0]
const encodeSnapshot = s => encodeSnapshotBatch([s], { format: 1 }, true)[0]
const encodeSnapshotV2 = s => encodeSnapshotBatch([s], { format: 2 }, true)[0]

// Promise-returning batch forms: reject on a device failure, resolve to per-document results (bytes
// or the Error yjs would throw for that document)
const mergeUpdatesBatchAsync = (docs, opts) => mergeUpdatesBatch(docs, opts, false, true)
const diffUpdateBatchAsync = (updates, svs, opts) => diffUpdateBatch(updates, svs, opts, false, true)
const encodeStateVectorFromUpdateBatchAsync = (updates, opts) => encodeStateVectorFromUpdateBatch(updates, opts, false, true)
const convertUpdateFormatBatchAsync = (updates, opts) => convertUpdateFormatBatch(updates, opts, false, true)
const parseUpdateMetaBatchAsync = (updates, opts) => parseUpdateMetaBatch(updates, opts, false, true)
const mergeDeleteSetsBatchAsync = (docs, opts) => mergeDeleteSetsBatch(docs, opts, false, true)
const convertSnapshotBatchAsync = (bufs, opts) => convertSnapshotBatch(bufs, opts, false, true)

// single-document yjs signatures (mergeUpdates([u]) returns the same object, like yjs)
const mergeUpdates = updates => updates.length === 1 ? updates[0] : mergeUpdatesBatch([updates], { format: 'v1' }, true)[0]
const mergeUpdatesV2 = updates => updates.length === 1 ? updates[0] : mergeUpdatesBatch([updates], { format: 'v2' }, true)[0]
const diffUpdate = (update, sv) => diffUpdateBatch([update], [sv], { format: 'v1' }, true)[0]
const diffUpdateV2 = (update, sv) => diffUpdateBatch([update], [sv], { format: 'v2' }, true)[0]
const encodeStateVectorFromUpdate = u => encodeStateVectorFromUpdateBatch([u], { format: 'v1' }, true)[0]
const encodeStateVectorFromUpdateV2 = u => encodeStateVectorFromUpdateBatch([u], { format: 'v2' }, true)[0]
const convertUpdateFormatV1ToV2 = u => convertUpdateFormatBatch([u], { format: 'v1' }, true)[0]
const convertUpdateFormatV2ToV1 = u => convertUpdateFormatBatch([u], { format: 'v2' }, true)[0]
const parseUpdateMeta = u => parseUpdateMetaBatch([u], { format: 'v1' }, true)[0]
const parseUpdateMetaV2 = u => parseUpdateMetaBatch([u], { format: 'v2' }, true)[0]
const mergeEncodedDeleteSets = (dss, opts) => mergeDeleteSetsBatch([dss], opts, true)[0]

module.exports = {
  mergeUpdates, mergeUpdatesV2, diffUpdate, diffUpdateV2, encodeStateVectorFromUpdate, encodeStateVectorFromUpdateV2,
  mergeUpdatesBatch, diffUpdateBatch, encodeStateVectorFromUpdateBatch,
  convertUpdateFormatV1ToV2, convertUpdateFormatV2ToV1, convertUpdateFormatBatch,
  parseUpdateMeta, parseUpdateMetaV2, parseUpdateMetaBatch, mergeDeleteSetsBatch, mergeEncodedDeleteSets,
  mergeUpdatesBatchAsync, diffUpdateBatchAsync, encodeStateVectorFromUpdateBatchAsync, convertUpdateFormatBatchAsync,
  parseUpdateMetaBatchAsync, mergeDeleteSetsBatchAsync,
  convertSnapshotBatch, convertSnapshotBatchAsync, decodeSnapshotBatch, encodeSnapshotBatch,
  decodeSnapshot, decodeSnapshotV2, encodeSnapshot, encodeSnapshotV2,
  compactUpdates, compactUpdatesV2, compactUpdatesBatch, compactUpdatesBatchAsync
}
