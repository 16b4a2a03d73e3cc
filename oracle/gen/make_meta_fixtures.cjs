// Golden vectors for parseUpdateMeta[V2] and for PermanentUserData's delete-set merge (test
// infrastructure, container-only).  Writes tests/golden/meta.json and tests/golden/dsmerge.json.
//
// meta: yjs 13.5.16's own Y.parseUpdateMeta / Y.parseUpdateMetaV2 (via yjs_bundle.cjs) over every
//   single-update input already in tests/golden/*.json and the merged outputs of the merge cases (in
//   their own format, inputs up to 64 KB).  The two Maps it returns are written as the engine encodes
//   them: from then to, each vu(size) | (client, clock)* in Map order.
// dsmerge: k encoded delete sets per case, merged the way PermanentUserData does it
//   (PermanentUserData.js:49-54: mergeDeleteSets(ds.map(encodedDs => readDeleteSet(new DSDecoderV1(..))))),
//   run by constructing a Y.PermanentUserData over a users map that holds the blobs; the merged set is
//   written with encodeSnapshot (DSEncoderV1) / encodeSnapshotV2 (DSEncoderV2) of a snapshot with an empty
//   state vector, whose trailing vu(0) is dropped.  V2 blobs are converted to V1 for PermanentUserData
//   (readDeleteSet + writeDeleteSet through decodeSnapshotV2 / encodeSnapshot keep every interval and the
//   first-appearance client order, which is all mergeDeleteSets depends on).
// Usage: node make_meta_fixtures.cjs [golden dir]
'use strict'
const fs = require('fs')
const path = require('path')
const { Y, load } = require('./yjs_bundle.cjs')
const enc = load(29194) // lib0 encoding 0.2.42

const DIR = process.argv[2] || path.join(__dirname, '../../tests/golden')
const b64 = u8 => Buffer.from(u8).toString('base64')
const u8 = s => new Uint8Array(Buffer.from(s, 'base64'))

function encodeMaps (from, to) {
  const e = enc.Mf()
  for (const m of [from, to]) {
    enc.uE(e, m.size)
    m.forEach((clock, client) => { enc.uE(e, client); enc.uE(e, clock) })
  }
  return enc._f(e)
}

// ---- meta ----
const seen = new Set()
const meta = []
function addMeta (name, fmt, input) {
  const key = fmt + ':' + input
  if (seen.has(key) || input.length > 90000) return
  seen.add(key)
  const c = { name, op: 'meta', fmt, inputs: [input] }
  try {
    const m = (fmt === 1 ? Y.parseUpdateMeta : Y.parseUpdateMetaV2)(u8(input))
    c.expect = b64(encodeMaps(m.from, m.to))
  } catch (e) {
    c.error = e.constructor.name
    c.message = String(e.message)
  }
  meta.push(c)
}
const SKIP = new Set(['conv.json', 'meta.json', 'dsmerge.json'])
for (const f of fs.readdirSync(DIR).sort()) {
  if (!f.endsWith('.json') || SKIP.has(f)) continue
  const j = JSON.parse(fs.readFileSync(path.join(DIR, f), 'utf8'))
  for (const c of j.cases) {
    if (c.op !== 'merge' && c.inputs.length === 1) addMeta(`${f}/${c.name}/${c.op}`, c.fmt, c.inputs[0])
    if (c.op === 'merge' && c.expect) addMeta(`${f}/${c.name}/merged`, c.fmt, c.expect)
  }
}

// ---- dsmerge ----
function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return { u32: next, int: (lo, hi) => lo + (next() % (hi - lo + 1)), real: () => next() / 4294967296 }
}
const dropTail = u => u.slice(0, u.length - 1) // the empty state vector's vu(0)
function encodeDs (clients, v2) { // clients: [[client, [[clock, len], ...]], ...] in write order
  const ds = Y.createDeleteSet()
  for (const [client, items] of clients) ds.clients.set(client, items.map(([clock, len]) => ({ clock, len })))
  const snap = Y.createSnapshot(ds, new Map())
  return dropTail(v2 ? Y.encodeSnapshotV2(snap) : Y.encodeSnapshot(snap))
}
function pudMerge (blobsV1) {
  const doc = new Y.Doc()
  const users = doc.getMap('users')
  const user = new Y.Map()
  users.set('u', user)
  const arr = new Y.Array()
  arr.push(blobsV1)
  user.set('ds', arr)
  user.set('ids', new Y.Array())
  const pud = new Y.PermanentUserData(doc, users)
  return pud.dss.get('u')
}
const dsm = []
function addDsm (name, fmt, blobs) {
  const c = { name, op: 'dsmerge', fmt, inputs: blobs.map(b64) }
  try {
    const v1 = fmt === 1 ? blobs : blobs.map(b => dropTail(Y.encodeSnapshot(Y.decodeSnapshotV2(Uint8Array.from([...b, 0])))))
    const merged = pudMerge(v1)
    const snap = Y.createSnapshot(merged, new Map())
    c.expect = b64(dropTail(fmt === 1 ? Y.encodeSnapshot(snap) : Y.encodeSnapshotV2(snap)))
  } catch (e) {
    c.error = e.constructor.name
    c.message = String(e.message)
  }
  dsm.push(c)
}
function randDs (r, nClients, maxItems, clockSpan, sorted) {
  const out = []
  const pool = [1, 7, 1000, 8919, 123456789, 4294967295, 0, 42]
  const used = new Set()
  for (let i = 0; i < nClients; i++) {
    let client = pool[r.int(0, pool.length - 1)]
    if (r.real() < 0.5) client = r.int(0, 2000)
    if (used.has(client) && r.real() < 0.7) continue
    used.add(client)
    const n = r.int(0, maxItems)
    let items = []
    for (let j = 0; j < n; j++) items.push([r.int(0, clockSpan), r.int(1, 6)])
    if (sorted) {
      items.sort((a, b) => a[0] - b[0])
      const dedup = []
      let end = 0
      for (const [cl, ln] of items) { if (cl >= end) { dedup.push([cl, ln]); end = cl + ln } }
      items = dedup
    }
    out.push([client, items])
  }
  return out
}
for (const fmt of [1, 2]) {
  addDsm('empty_list', fmt, [])
  addDsm('one_empty', fmt, [encodeDs([], fmt === 2)])
  addDsm('one_sorted', fmt, [encodeDs([[5, [[0, 2], [4, 1]]]], fmt === 2)])
  addDsm('touching', fmt, [encodeDs([[5, [[0, 2]]]], fmt === 2), encodeDs([[5, [[2, 3]]]], fmt === 2)])
  addDsm('overlap_contained', fmt, [encodeDs([[5, [[0, 10]]]], fmt === 2), encodeDs([[5, [[2, 3]]], [6, [[1, 1]]]], fmt === 2)])
  addDsm('gap', fmt, [encodeDs([[5, [[0, 2]]]], fmt === 2), encodeDs([[5, [[3, 1]]]], fmt === 2)])
  addDsm('client_order_first_appearance', fmt, [encodeDs([[9, [[0, 1]]], [3, [[0, 1]]]], fmt === 2), encodeDs([[3, [[5, 1]]], [1, [[0, 1]]], [9, [[1, 1]]]], fmt === 2)])
  addDsm('zero_entry_client', fmt, [encodeDs([[9, []], [3, [[0, 1]]]], fmt === 2), encodeDs([[9, [[4, 2]]]], fmt === 2)])
  addDsm('large_clocks', fmt, [encodeDs([[4294967295, [[4294967290, 3]]]], fmt === 2), encodeDs([[4294967295, [[4294967292, 4]]]], fmt === 2)])
  const blob = encodeDs([[5, [[0, 2], [9, 1]]], [6, [[3, 3]]]], fmt === 2)
  addDsm('truncated', fmt, [blob, blob.slice(0, blob.length - 2)])
  addDsm('truncated_empty', fmt, [new Uint8Array(0)])
  if (fmt === 1) addDsm('trailing_bytes', fmt, [Uint8Array.from([...blob, 7, 7, 7]), blob]) // V2: the V1 conversion would read the tail as a state vector
  addDsm('duplicate_client_groups', fmt, [Uint8Array.from([2, 5, 1, 0, 1, 5, 1, 0, 2])])
}
// V1 blobs may carry unsorted, overlapping and zero-length intervals (the reader takes any order)
addDsm('v1_unsorted_zero_len', 1, [encodeDs([[5, [[9, 1], [0, 0], [3, 2], [0, 4]]]], false), encodeDs([[5, [[2, 0]]]], false)])
for (let s = 1; s <= 60; s++) {
  const r = rng(s * 7919)
  for (const fmt of [1, 2]) {
    const k = r.int(1, s % 10 === 0 ? 40 : 8)
    const blobs = []
    for (let i = 0; i < k; i++) blobs.push(encodeDs(randDs(r, r.int(0, 6), r.int(0, 12), s % 3 === 0 ? 60 : 4000, fmt === 2 || r.real() < 0.5), fmt === 2))
    addDsm(`random_${s}`, fmt, blobs)
  }
}

const ORACLE = 'yjs 13.5.16 (JupyterLab bundle 3502.fbe0c610be82ba1360db.js) + lib0 0.2.42'
fs.writeFileSync(path.join(DIR, 'meta.json'), JSON.stringify({ generator: 'oracle/gen/make_meta_fixtures.cjs', oracle: ORACLE + ' parseUpdateMeta[V2]', cases: meta }))
fs.writeFileSync(path.join(DIR, 'dsmerge.json'), JSON.stringify({ generator: 'oracle/gen/make_meta_fixtures.cjs', oracle: ORACLE + ' PermanentUserData mergeDeleteSets + encodeSnapshot[V2]', cases: dsm }))
console.log('meta.json', meta.length, 'cases', meta.filter(c => c.error).length, 'errors')
console.log('dsmerge.json', dsm.length, 'cases', dsm.filter(c => c.error).length, 'errors')
