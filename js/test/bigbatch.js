// A large batch through the Node drop-in: the C2 V1 workload (bench_data/c2_v1.ymb.gz, yjs-generated templates)
// replicated to 10,000 documents, merged by one mergeUpdatesBatch call -- packed into page-locked pool memory
// (addon.hostBuffer), u32 offsets, the library's pipelined host path -- and compared document by document
// with the same documents merged 100 at a time (ordinary memory, unpipelined).  Prints one JSON line with the
// mismatches and the big call's time (the rate includes the JS packing and unpacking).
'use strict'
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const Y = require(path.join(__dirname, '..', 'index.js'))

const buf = zlib.gunzipSync(fs.readFileSync(path.join(__dirname, '..', '..', 'bench_data', 'c2_v1.ymb.gz')))
const nDocs = buf.readUInt32LE(4); const nUpd = buf.readUInt32LE(8)
const docUpd = []; let o = 12
for (let i = 0; i <= nDocs; i++) { docUpd.push(buf.readUInt32LE(o)); o += 4 }
const updOff = []
for (let i = 0; i <= nUpd; i++) { updOff.push(Number(buf.readBigUInt64LE(o))); o += 8 }
const arena = buf.subarray(o)
const templates = []
for (let d = 0; d < nDocs; d++) {
  const us = []
  for (let u = docUpd[d]; u < docUpd[d + 1]; u++) us.push(arena.subarray(updOff[u], updOff[u + 1]))
  templates.push(us)
}
const N = Number(process.env.NDOCS || 10000)
const docs = []
for (let i = 0; i < N; i++) docs.push(templates[i % templates.length])
let inBytes = 0
for (const d of docs) for (const u of d) inBytes += u.length

const ref = []
for (let i = 0; i < N; i += 100) ref.push(...Y.mergeUpdatesBatch(docs.slice(i, i + 100)))
let got = Y.mergeUpdatesBatch(docs)
let bad = 0
for (let i = 0; i < N; i++) if (Buffer.compare(Buffer.from(got[i]), Buffer.from(ref[i])) !== 0) bad++
const reps = 5
const t0 = process.hrtime.bigint()
for (let r = 0; r < reps; r++) got = Y.mergeUpdatesBatch(docs)
const ms = Number(process.hrtime.bigint() - t0) / 1e6 / reps
console.log(JSON.stringify({ docs: N, bad, in_bytes: inBytes, ms_per_call: +ms.toFixed(3), gbs: +(inBytes / ms / 1e6).toFixed(3) }))
process.exit(bad === 0 ? 0 : 1)
