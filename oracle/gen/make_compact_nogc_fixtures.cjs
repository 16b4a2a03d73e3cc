// Doc round-trip compaction fixtures for new Y.Doc({ gc: false }) (ym_compact with YM_NO_GC), test
// infrastructure, container-only: the same inputs as tests/golden/compact.json (make_compact_fixtures.cjs) --
// every inline case and a few workload documents -- applied by the reference (gaberogan/yjs@v0, yjs 13.4.9,
// via ref_yjs.cjs) to a Doc whose gc option is false (Doc.js:40-43: cleanupTransactions skips
// tryGcDeleteSet, Transaction.js:302-304, so deleted content stays and is written), then
// encodeStateAsUpdate[V2].  Output: tests/golden/compact_nogc.json, the layout of compact.json.
'use strict'
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const crypto = require('crypto')
const { loadReference } = require('./ref_yjs.cjs')

const GOLDEN = path.join(__dirname, '../../tests/golden')
const u8 = b64 => new Uint8Array(Buffer.from(b64, 'base64'))
const b64 = u => Buffer.from(u).toString('base64')

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

;(async () => {
  const Y = await loadReference()
  const src = JSON.parse(fs.readFileSync(path.join(GOLDEN, 'compact.json')))
  const ymb = {}
  // workload documents kept: the first few of each template set (the rest of compact.json's are gc=true only)
  const keepSrc = { c1_v1: 1, c1_v2: 1, c2_v1: 4, c2_v2: 4, c4_v1: 2, c4_v2: 2, c3_v1: 1, c3_v2: 1, c5_v1: 1, c5_v2: 1 }
  const cases = []
  const stats = {}
  for (const c of src.cases) {
    let inputs
    if (c.src) {
      if (c.src.drop || !(c.src.doc < (keepSrc[c.src.ymb] || 0))) continue
      ymb[c.src.ymb] = ymb[c.src.ymb] || loadYmb(c.src.ymb)
      inputs = ymb[c.src.ymb][c.src.doc]
    } else {
      inputs = c.inputs.map(u8)
    }
    const v2 = c.fmt === 2
    const r = c.src ? { id: c.id, group: c.group, fmt: c.fmt, src: c.src } : { id: c.id, group: c.group, fmt: c.fmt, inputs: c.inputs }
    try {
      const doc = new Y.Doc({ gc: false })
      for (const u of inputs) (v2 ? Y.applyUpdateV2 : Y.applyUpdate)(doc, u)
      const p = [doc.store.pendingClientsStructRefs.size, doc.store.pendingStack.length, doc.store.pendingDeleteReaders.length]
      if (p[0] + p[1] + p[2] !== 0) r.pending = p
      const out = (v2 ? Y.encodeStateAsUpdateV2 : Y.encodeStateAsUpdate)(doc)
      if (c.src) { r.expect_sha256 = crypto.createHash('sha256').update(out).digest('hex'); r.expect_len = out.length } else r.expect = b64(out)
      r.sv = b64(Y.encodeStateVector(doc))  // the Doc's own state vector (encoding.js:572-611)
      // does gc: false change the bytes for this input? (a document without deletions is the same either way)
      r.differs_from_gc = c.error ? null : (c.expect !== undefined ? c.expect !== r.expect : c.expect_sha256 !== r.expect_sha256)
    } catch (e) {
      r.error = { name: e.constructor.name, message: e.message }
    }
    cases.push(r)
    stats[c.group] = (stats[c.group] || 0) + 1
    if (r.differs_from_gc) stats[c.group + '/differs'] = (stats[c.group + '/differs'] || 0) + 1
  }
  fs.writeFileSync(path.join(GOLDEN, 'compact_nogc.json'), JSON.stringify({
    generator: 'oracle/gen/make_compact_nogc_fixtures.cjs (gaberogan/yjs@v0 = yjs 13.4.9, new Y.Doc({ gc: false }))',
    cases
  }))
  console.log(cases.length, 'cases', JSON.stringify(stats))
})().catch(e => { console.error(e); process.exit(1) })
