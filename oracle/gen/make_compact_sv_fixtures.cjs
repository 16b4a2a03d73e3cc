// Target-state-vector compaction fixtures (ym_compact with ym_batch.sv_arena), test infrastructure,
// container-only: the reference (gaberogan/yjs@v0, yjs 13.4.9, via ref_yjs.cjs) applies a document's updates
// to a fresh Doc (gc: true, and gc: false for a share of them) and writes encodeStateAsUpdate[V2](doc, sv)
// (encoding.js:490-526: writeClientsStructs from the target's clocks, encoding.js:71-116 -- the first struct
// of a client written with an offset, Item.js:625-658 and the Content*.write(encoder, offset) methods -- and
// the whole delete set) for several target state vectors per document:
//   empty (the encoding of an empty Map), full (the document's own), the state after a prefix of the inputs,
//   random clocks per client (mid-struct offsets), unknown clients / repeated entries (later entries win),
//   and malformed vectors (truncated, zero-length: decodeStateVector throws).
// Inputs: every inline case of tests/golden/compact.json (referenced by id), a few workload documents, and
// a group built here ("slice"): texts with surrogate pairs, arrays and deletions, every clock of every client
// as a target (ContentString.write's str.slice(offset) cutting a pair: V1 throws URIError, V2's string
// column pairs the halves up).  Output: tests/golden/compact_sv.json.
'use strict'
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const crypto = require('crypto')
const { loadReference } = require('./ref_yjs.cjs')

const GOLDEN = path.join(__dirname, '../../tests/golden')
const u8 = b64 => new Uint8Array(Buffer.from(b64, 'base64'))
const b64 = u => Buffer.from(u).toString('base64')
const sha = u => crypto.createHash('sha256').update(u).digest('hex')

let seed = 0x5eed5
const rnd = n => { seed = (seed * 1103515245 + 12345) >>> 0; return Math.floor((seed / 4294967296) * n) }

function loadYmb (name) {
  const b = zlib.gunzipSync(fs.readFileSync(path.join(__dirname, '../../bench_data', name + '.ymb.gz')))
  const nd = b.readUInt32LE(4); const nu = b.readUInt32LE(8)
  let o = 12
  const docUpd = []; for (let i = 0; i <= nd; i++) { docUpd.push(b.readUInt32LE(o)); o += 4 }
  const off = []; for (let i = 0; i <= nu; i++) { off.push(Number(b.readBigUInt64LE(o))); o += 8 }
  const arena = b.subarray(o)
  const docs = []
  for (let d = 0; d < nd; d++) {
    const ups = []
    for (let u = docUpd[d]; u < docUpd[d + 1]; u++) ups.push(new Uint8Array(arena.subarray(off[u], off[u + 1])))
    docs.push(ups)
  }
  return docs
}

// encodeStateVector's layout (writeStateVector, encoding.js:572-579) of a list of [client, clock] entries
function svBytes (Y, entries) {
  const out = []
  const vu = n => { while (n > 127) { out.push(128 | (n % 128)); n = Math.floor(n / 128) } out.push(n) }
  vu(entries.length)
  for (const [c, k] of entries) { vu(c); vu(k) }
  return new Uint8Array(out)
}

function build (Y, inputs, v2, gc) {
  const doc = new Y.Doc({ gc })
  for (const u of inputs) (v2 ? Y.applyUpdateV2 : Y.applyUpdate)(doc, u)
  return doc
}

function targetsFor (Y, doc, inputs, v2, gc, many) {
  const sv = Y.decodeStateVector(Y.encodeStateVector(doc))
  const ents = Array.from(sv.entries())
  const t = []
  t.push({ kind: 'empty', sv: svBytes(Y, []) })
  t.push({ kind: 'full', sv: Y.encodeStateVector(doc) })
  if (inputs.length >= 2) {
    const h = Math.max(1, inputs.length >> 1)
    try {
      t.push({ kind: 'prefix', sv: Y.encodeStateVector(build(Y, inputs.slice(0, h), v2, gc)) })
    } catch (e) {}
  }
  for (let r = 0; r < (many ? 3 : 2); r++) {
    const e = ents.filter(() => rnd(4) !== 0).map(([c, k]) => [c, rnd(k + 1)])
    t.push({ kind: 'random', sv: svBytes(Y, e) })
  }
  if (ents.length) {  // unknown clients, a repeated client (the later entry wins), a clock past the state
    const [c0, k0] = ents[rnd(ents.length)]
    t.push({ kind: 'repeat', sv: svBytes(Y, [[c0, 0], [123456789, 5], [c0, rnd(k0 + 1)]]) })
    t.push({ kind: 'past', sv: svBytes(Y, [[c0, k0 + 1000000], [2 ** 40, 1]]) })
  }
  return t
}

function run (Y, doc, v2, target) {
  const r = { kind: target.kind, sv: b64(target.sv) }
  try {
    const out = (v2 ? Y.encodeStateAsUpdateV2 : Y.encodeStateAsUpdate)(doc, target.sv)
    return [r, out]
  } catch (e) {
    r.error = { name: e.constructor.name, message: e.message }
    return [r, null]
  }
}

// documents built here: text with surrogate pairs cut by inserts and deletes, arrays, nested types
function sliceDocs (Y) {
  const docs = []
  const scripts = [
    (a, b) => { a.getText('t').insert(0, 'a\u{1F600}b\u{1F601}\u{1F602}c'); b.getText('t').insert(0, 'xy\u{1F603}') },
    (a, b) => { const t = a.getText('t'); t.insert(0, '\u{1F600}\u{1F601}\u{1F602}\u{1F603}'); t.delete(2, 2); b.getArray('a').insert(0, [1, 'two', { three: 3 }, [4], 5.5, true]) },
    (a, b) => { const t = a.getText('t'); t.insert(0, 'hello \u{1F30D} world'); t.insert(7, 'X'); t.format(0, 5, { bold: true }); b.getMap('m').set('k', 'v\u{1F600}') },
    (a, b) => { const x = a.getArray('a'); x.insert(0, ['a', 'b', 'c', 'd', 'e', 'f']); x.delete(1, 3); const t = b.getText('t'); t.insert(0, 'é中\u{10348}z'); t.delete(1, 1) },
    (a, b) => { const t = a.getText('t'); for (let i = 0; i < 6; i++) t.insert(i * 2 > t.length ? t.length : i * 2, i % 2 ? '\u{1F680}' : 'q'); const x = b.getXmlFragment('x'); const e = new Y.YXmlElement('p'); x.insert(0, [e]); e.insert(0, [new Y.YXmlText('\u{1F600}ab')]) }
  ]
  for (let s = 0; s < scripts.length; s++) {
    for (const gc of [true, false]) {
      const a = new Y.Doc({ gc }); a.clientID = 11 + s
      const b = new Y.Doc({ gc }); b.clientID = 900 + s
      const v1 = []; const v2 = []
      for (const d of [a, b]) { d.on('update', u => v1.push(u)); d.on('updateV2', u => v2.push(u)) }
      scripts[s](a, b)
      // a sees b's updates and edits on top of them (origins across clients)
      Y.applyUpdate(a, Y.encodeStateAsUpdate(b))
      const at = a.getText('t')
      if (at.length > 3) { at.insert(2, '\u{1F4A9}'); at.delete(1, 2) }
      docs.push({ s, gc, v1: v1.slice(), v2: v2.slice() })
    }
  }
  return docs
}

;(async () => {
  const Y = await loadReference()
  const src = JSON.parse(fs.readFileSync(path.join(GOLDEN, 'compact.json')))
  const ymb = {}
  const keepSrc = { c1_v1: 1, c1_v2: 1, c2_v1: 2, c2_v2: 2, c4_v1: 1, c4_v2: 1, c3_v1: 1, c3_v2: 1, c5_v1: 1, c5_v2: 1 }
  const cases = []
  const stats = {}
  const add = (r, doc, v2, targets, keepBytes) => {
    r.targets = []
    for (const t of targets) {
      const [o, out] = run(Y, doc, v2, t)
      if (out) { if (keepBytes) o.expect = b64(out); else { o.expect_sha256 = sha(out); o.expect_len = out.length } }
      r.targets.push(o)
      stats[o.error ? 'error' : o.kind] = (stats[o.error ? 'error' : o.kind] || 0) + 1
    }
    cases.push(r)
  }
  let n = 0
  for (const c of src.cases) {
    let inputs
    if (c.src) {
      if (c.src.drop || !(c.src.doc < (keepSrc[c.src.ymb] || 0))) continue
      ymb[c.src.ymb] = ymb[c.src.ymb] || loadYmb(c.src.ymb)
      inputs = ymb[c.src.ymb][c.src.doc]
    } else {
      if (c.error) continue  // the updates themselves throw: no document to write
      inputs = c.inputs.map(u8)
    }
    const v2 = c.fmt === 2
    const gc = (n++ % 4) !== 3
    let doc
    try { doc = build(Y, inputs, v2, gc) } catch (e) { continue }
    const targets = targetsFor(Y, doc, inputs, v2, gc, !!c.src)
    if (n % 50 === 1) {  // malformed target vectors: decodeStateVector throws
      const full = Y.encodeStateVector(doc)
      targets.push({ kind: 'zero_length', sv: new Uint8Array(0) })
      if (full.length > 1) targets.push({ kind: 'truncated', sv: full.subarray(0, full.length - 1) })
      targets.push({ kind: 'overlong', sv: new Uint8Array([1, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f, 0]) })
    }
    add({ ref: c.id, fmt: c.fmt, gc, group: c.group }, doc, v2, targets, false)
  }
  for (const d of sliceDocs(Y)) {
    for (const fmt of [1, 2]) {
      const inputs = fmt === 2 ? d.v2 : d.v1
      const doc = build(Y, inputs, fmt === 2, d.gc)
      const sv = Array.from(Y.decodeStateVector(Y.encodeStateVector(doc)).entries())
      const targets = []
      for (const [c, k] of sv) for (let i = 0; i <= k; i++) targets.push({ kind: 'clock', sv: svBytes(Y, [[c, i]]) })
      add({ id: `slice_${d.s}_${d.gc ? 'gc' : 'nogc'}_v${fmt}`, fmt, gc: d.gc, group: 'slice', inputs: inputs.map(b64) }, doc, fmt === 2, targets, true)
    }
  }
  fs.writeFileSync(path.join(GOLDEN, 'compact_sv.json'), JSON.stringify({
    generator: 'oracle/gen/make_compact_sv_fixtures.cjs (gaberogan/yjs@v0 = yjs 13.4.9, encodeStateAsUpdate[V2](doc, sv))',
    cases
  }))
  console.log(cases.length, 'documents', JSON.stringify(stats))
})().catch(e => { console.error(e); process.exit(1) })
