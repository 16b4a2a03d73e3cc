// Golden vectors for the delete-set merge with the REFERENCE's semantics (test infrastructure,
// container-only).  PermanentUserData (gaberogan/yjs@v0 src/utils/PermanentUserData.js:49-54) merges a
// user's encoded delete sets with mergeDeleteSets (DeleteSet.js:141-161), whose sortAndMergeDeleteSet
// (DeleteSet.js:113-135) coalesces only exactly adjacent ranges -- yjs 13.5.16 also merges overlapping
// ones.  This script runs the reference's own readDeleteSet / mergeDeleteSets / writeDeleteSet (via
// ref_yjs.cjs) over the inputs of tests/golden/dsmerge.json (which hold touching, overlapping, duplicate,
// unsorted and zero-length ranges) and writes tests/golden/dsmerge_ref.json (op "dsmerge_ref").
// Usage: node make_dsmerge_ref_fixtures.cjs
'use strict'
const fs = require('fs')
const path = require('path')
const { loadReference } = require('./ref_yjs.cjs')
const { load } = require('./yjs_bundle.cjs')
const decoding = load(64485)
const DIR = path.join(__dirname, '../../tests/golden')
const b64 = u8 => Buffer.from(u8).toString('base64')

;(async () => {
  const Y = await loadReference()
  const src = JSON.parse(fs.readFileSync(path.join(DIR, 'dsmerge.json')))
  const cases = []
  for (const c0 of src.cases) {
    const c = { name: c0.name, op: 'dsmerge_ref', fmt: c0.fmt, inputs: c0.inputs }
    try {
      const Dec = c0.fmt === 1 ? Y.DSDecoderV1 : Y.DSDecoderV2
      const Enc = c0.fmt === 1 ? Y.DSEncoderV1 : Y.DSEncoderV2
      const dss = c0.inputs.map(b => Y.readDeleteSet(new Dec(decoding.l1(new Uint8Array(Buffer.from(b, 'base64'))))))
      const e = new Enc()
      Y.writeDeleteSet(e, Y.mergeDeleteSets(dss))
      c.expect = b64(e.toUint8Array())
    } catch (e) {
      c.error = e.constructor.name
      c.message = String(e.message)
    }
    cases.push(c)
  }
  fs.writeFileSync(path.join(DIR, 'dsmerge_ref.json'), JSON.stringify({
    generator: 'oracle/gen/make_dsmerge_ref_fixtures.cjs',
    oracle: 'gaberogan/yjs@v0 (yjs 13.4.9) readDeleteSet / mergeDeleteSets / writeDeleteSet, src/utils/DeleteSet.js:113-256',
    cases
  }))
  const differ = cases.filter((c, i) => c.expect !== src.cases[i].expect).length
  console.log('dsmerge_ref.json', cases.length, 'cases', cases.filter(c => c.error).length, 'errors,', differ, 'differ from 13.5.16')
})().catch(e => { console.error(e); process.exit(1) })
