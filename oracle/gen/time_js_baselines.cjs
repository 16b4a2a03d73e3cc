// Times the JavaScript implementations on the bench workloads (container-only; SURVEY.md §8(d) host
// baseline calibration): yjs 13.5.16 mergeUpdates (the byte target) and the reference's own Doc round
// trip (gaberogan/yjs@v0 = 13.4.9: applyUpdate of every update into a gc:false Doc, then
// encodeStateAsUpdate -- it has no mergeUpdates) over the same documents, one thread, V1.
// Usage: node time_js_baselines.cjs <workload: c2_v1 | c4_v1> <docs> -> one JSON line.
'use strict'
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const { Y } = require('./yjs_bundle.cjs')
const { loadReference } = require('./ref_yjs.cjs')

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
  const wl = process.argv[2] || 'c2_v1'
  const n = +(process.argv[3] || 2000)
  const tmpl = loadYmb(wl)
  const docs = []; for (let i = 0; i < n; i++) docs.push(tmpl[i % tmpl.length])
  let bytes = 0; for (const d of docs) for (const u of d) bytes += u.length
  const R = await loadReference()
  const time = f => { const t0 = process.hrtime.bigint(); let out = 0; for (const d of docs) out += f(d).length; return [Number(process.hrtime.bigint() - t0) / 1e9, out] }
  time(d => Y.mergeUpdates(d)) // warm-up (JIT)
  const [t1, o1] = time(d => Y.mergeUpdates(d))
  const canon = d => { const doc = new R.Doc({ gc: false }); for (const u of d) R.applyUpdate(doc, u); return R.encodeStateAsUpdate(doc) }
  time(canon)
  const [t2, o2] = time(canon)
  console.log(JSON.stringify({
    workload: wl, docs: n, input_bytes: bytes, threads: 1, node: process.version,
    yjs_13_5_16_mergeUpdates: { s: t1, input_gbs: bytes / t1 / 1e9, docs_per_s: n / t1, output_bytes: o1 },
    reference_13_4_9_doc_roundtrip_gc_false: { s: t2, input_gbs: bytes / t2 / 1e9, docs_per_s: n / t2, output_bytes: o2 }
  }))
})().catch(e => { console.error(e); process.exit(1) })
