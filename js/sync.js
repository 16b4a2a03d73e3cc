// y-protocols sync over stored updates, batched on the MI355X (mirror of yjs_amd/sync.py).
//
// Same message framing and names as y-protocols 0.2.3 sync.js (messageYjsSyncStep1/2/Update,
// writeSyncStep1, writeSyncStep2, writeUpdate, readSyncMessage), with the document kept as one stored
// update instead of a Y.Doc: SyncStep1 -> SyncStep2(diffUpdate(stored, sv)), SyncStep2 / Update ->
// stored = mergeUpdates([stored, update]).  readSyncMessagesBatch answers many documents in one GPU
// call per message kind.
'use strict'
const Y = require('./index.js')

const messageYjsSyncStep1 = 0
const messageYjsSyncStep2 = 1
const messageYjsUpdate = 2

function vu (v) {
  const out = []
  while (v > 127) { out.push(0x80 | (v & 127)); v = Math.floor(v / 128) }
  out.push(v)
  return out
}
function encodeMessage (type, payload) {
  const h = vu(type).concat(vu(payload.length))
  const m = new Uint8Array(h.length + payload.length)
  m.set(h, 0)
  m.set(payload, h.length)
  return m
}
function readVu (b, pos) {
  let num = 0; let mult = 1
  for (;;) {
    const r = b[pos++]
    num += (r & 127) * mult  // past the end: undefined & 127 === 0, as lib0
    mult *= 128
    if (r < 128) return [num, pos]
    if (mult > Number.MAX_SAFE_INTEGER) throw new Error('Integer out of range!')
  }
}
function decodeMessage (m) {
  let [t, p] = readVu(m, 0)
  let n
  [n, p] = readVu(m, p)
  if (p + n > m.length) throw new RangeError('Unexpected end of array')
  return [t, m.subarray(p, p + n)]
}
const v2 = o => o && (o.format === 'v2' || o.format === 2)
const writeSyncStep1 = (stored, opts) => encodeMessage(messageYjsSyncStep1, (v2(opts) ? Y.encodeStateVectorFromUpdateV2 : Y.encodeStateVectorFromUpdate)(stored))
const writeSyncStep2 = (stored, sv, opts) => encodeMessage(messageYjsSyncStep2, (v2(opts) ? Y.diffUpdateV2 : Y.diffUpdate)(stored, sv))
const writeUpdate = update => encodeMessage(messageYjsUpdate, update)

function readSyncMessagesBatch (messages, stored, opts) {
  const types = []; const replies = messages.map(() => null); const next = stored.slice()
  const step1 = []; const apply = []
  messages.forEach((m, i) => {
    const [t, payload] = decodeMessage(m)
    types.push(t)
    if (t === messageYjsSyncStep1) step1.push([i, payload])
    else if (t === messageYjsSyncStep2 || t === messageYjsUpdate) apply.push([i, payload])
    else throw new Error('Unknown message type')
  })
  if (step1.length) {
    const d = Y.diffUpdateBatch(step1.map(([i]) => stored[i]), step1.map(([, sv]) => sv), opts, true)
    step1.forEach(([i], k) => { replies[i] = encodeMessage(messageYjsSyncStep2, d[k]) })
  }
  if (apply.length) {
    const m = Y.mergeUpdatesBatch(apply.map(([i, u]) => [stored[i], u]), opts, true)
    apply.forEach(([i], k) => { next[i] = m[k] })
  }
  return { types, replies, stored: next }
}
const readSyncMessage = (message, stored, opts) => {
  const r = readSyncMessagesBatch([message], [stored], opts)
  return { type: r.types[0], reply: r.replies[0], stored: r.stored[0] }
}

module.exports = {
  messageYjsSyncStep1, messageYjsSyncStep2, messageYjsUpdate, encodeMessage, decodeMessage,
  writeSyncStep1, writeSyncStep2, writeUpdate, readSyncMessage, readSyncMessagesBatch
}
