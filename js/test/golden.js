// Runs the golden vectors (tests/golden/*.json) through the JS API on the GPU; prints a JSON summary.
'use strict'
const fs = require('fs')
const path = require('path')
const Y = require('..')
const dir = path.join(__dirname, '..', '..', 'tests', 'golden')
const errName = { URIError: 'URIError', TypeError: 'TypeError', RangeError: 'RangeError', SyntaxError: 'SyntaxError', Error: 'Error' }
// the 13.5.16 bundle is minified: its unknown-content-ref message names the minified callee; the engine
// reports the reference's source text (src/structs/Item.js readItemContent)
const MINIFIED = { 'ai[(e & b.kr)] is not a function': 'contentRefs[(info & binary.BITS5)] is not a function' }
let ok = 0; let bad = []; let unsupported = 0
// parseUpdateMeta's Maps re-encoded the way the golden vectors hold them (from, then to; vu pairs)
function encodeMeta (m) {
  const out = []
  const vu = v => { while (v > 127) { out.push(128 | (v % 128)); v = Math.floor(v / 128) } out.push(v) }
  for (const map of [m.from, m.to]) { vu(map.size); map.forEach((clock, client) => { vu(client); vu(clock) }) }
  return Uint8Array.from(out)
}
// compact*.json hold Doc round-trip fixtures in their own layout (tests/compact_cases.py): checked below
const opFiles = () => fs.readdirSync(dir).filter(f => f.endsWith('.json') && !f.startsWith('compact')).sort()
for (const f of opFiles()) {
  const cases = JSON.parse(fs.readFileSync(path.join(dir, f))).cases
  for (const c of cases) {
    const inputs = c.inputs.map(b => new Uint8Array(Buffer.from(b, 'base64')))
    if (c.op === 'merge' && inputs.length === 0) continue
    let out; let err
    try {
      if (c.op === 'merge') out = (c.fmt === 1 ? Y.mergeUpdates : Y.mergeUpdatesV2)(inputs)
      else if (c.op === 'diff') out = (c.fmt === 1 ? Y.diffUpdate : Y.diffUpdateV2)(inputs[0], new Uint8Array(Buffer.from(c.sv, 'base64')))
      else if (c.op === 'meta') out = encodeMeta((c.fmt === 1 ? Y.parseUpdateMeta : Y.parseUpdateMetaV2)(inputs[0]))
      else if (c.op === 'dsmerge') out = Y.mergeEncodedDeleteSets(inputs, { format: c.fmt })
      else if (c.op === 'dsmerge_ref') out = Y.mergeEncodedDeleteSets(inputs, { format: c.fmt, reference: true })
      else if (c.op === 'snap_to_v1' || c.op === 'snap_to_v2') out = Y.convertSnapshotBatch([inputs[0]], { format: c.fmt, to: c.op === 'snap_to_v2' ? 2 : 1 }, true)[0]
      else if (c.op === 'conv') out = (c.fmt === 1 ? Y.convertUpdateFormatV1ToV2 : Y.convertUpdateFormatV2ToV1)(inputs[0])
      else out = (c.fmt === 1 ? Y.encodeStateVectorFromUpdate : Y.encodeStateVectorFromUpdateV2)(inputs[0])
    } catch (e) { err = e }
    const id = `${f}/${c.name}/v${c.fmt}/${c.op}`
    if (err && err.code === 'YM_UNSUPPORTED') { unsupported++; continue }
    if (c.error) {
      if (!err || err.constructor.name !== errName[c.error] || err.message !== (MINIFIED[c.message] || c.message)) bad.push([id, 'error', err && err.message, c.message])
      else ok++
    } else if (err || Buffer.compare(Buffer.from(out), Buffer.from(c.expect, 'base64')) !== 0) bad.push([id, 'bytes', err && err.message])
    else ok++
  }
}
// the Promise-returning batch forms (napi_async_work) against the golden merges, several calls in flight
const asyncCheck = async () => {
  const groups = { 1: [], 2: [] }
  for (const f of opFiles()) {
    for (const c of JSON.parse(fs.readFileSync(path.join(dir, f))).cases) {
      if (c.op === 'merge' && c.inputs.length > 1) groups[c.fmt].push(c)
    }
  }
  let n = 0
  const runs = [1, 2].map(fmt => Y.mergeUpdatesBatchAsync(groups[fmt].map(c => c.inputs.map(b => new Uint8Array(Buffer.from(b, 'base64')))), { format: fmt })
    .then(res => res.forEach((r, i) => {
      const c = groups[fmt][i]
      const good = c.error ? r instanceof Error && r.constructor.name === errName[c.error] : !(r instanceof Error) && Buffer.compare(Buffer.from(r), Buffer.from(c.expect, 'base64')) === 0
      if (good) n++; else bad.push([c.name, 'async', r instanceof Error ? r.message : r.length])
    })))
  await Promise.all(runs)
  return n
}
// Doc round-trip compaction through the JS API: the inline gc: false fixtures (opts.gc === false) and the
// target-state-vector slice documents (opts.targetStateVectors), errors by class and message
let compactOk = 0
{
  const b = x => new Uint8Array(Buffer.from(x, 'base64'))
  const check = (id, r, c) => {
    const good = c.error ? r instanceof Error && r.constructor.name === c.error.name && r.message === c.error.message
      : !(r instanceof Error) && Buffer.compare(Buffer.from(r), Buffer.from(c.expect, 'base64')) === 0
    if (good) compactOk++; else bad.push([id, 'compact', r instanceof Error ? r.message : r.length])
  }
  for (const fmt of [1, 2]) {
    const nogc = JSON.parse(fs.readFileSync(path.join(dir, 'compact_nogc.json'))).cases.filter(c => c.inputs && c.fmt === fmt)
    Y.compactUpdatesBatch(nogc.map(c => c.inputs.map(b)), { format: fmt, gc: false }).forEach((r, i) => check(nogc[i].id, r, nogc[i]))
    // opts.withStateVector: { stateVector: encodeStateVector(doc), update } per document
    Y.compactUpdatesBatch(nogc.map(c => c.inputs.map(b)), { format: fmt, gc: false, withStateVector: true }).forEach((r, i) => {
      const c = nogc[i]
      if (r instanceof Error || c.error) { check(c.id + '/sv', r, c); return }
      check(c.id + '/sv', r.update, c)
      if (Buffer.compare(Buffer.from(r.stateVector), Buffer.from(c.sv, 'base64')) !== 0) bad.push([c.id, 'compact doc sv', r.stateVector.length])
    })
    for (const c of JSON.parse(fs.readFileSync(path.join(dir, 'compact_sv.json'))).cases.filter(c => c.group === 'slice' && c.fmt === fmt)) {
      const ins = c.inputs.map(b)
      Y.compactUpdatesBatch(c.targets.map(() => ins), { format: fmt, gc: c.gc, targetStateVectors: c.targets.map(t => b(t.sv)) })
        .forEach((r, i) => check(c.id + '/' + i, r, c.targets[i]))
    }
  }
}
asyncCheck().then(asyncOk => {
  console.log(JSON.stringify({ ok, bad: bad.length, unsupported, async_ok: asyncOk, compact_ok: compactOk, first: bad.slice(0, 10) }))
  process.exit(bad.length ? 1 : 0)
}, e => { console.error(e); process.exit(1) })
