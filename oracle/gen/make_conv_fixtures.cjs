// Golden vectors for convertUpdateFormatV1ToV2 / convertUpdateFormatV2ToV1 (test infrastructure,
// container-only).  yjs 13.5.16's own convertUpdateFormat (bundle ms@41803, via yjs_bundle.cjs) is run
// over every single-update input already in tests/golden/*.json (the diff / state-vector cases, with
// their edge cases: truncation, malformed UTF-8, overlong varints, every content kind ...) and over
// the merged outputs of the merge cases, in their own format.  Writes tests/golden/conv.json.
// Usage: node make_conv_fixtures.cjs [golden dir]
'use strict'
const fs = require('fs')
const path = require('path')
const { convert } = require('./yjs_bundle.cjs')

const DIR = process.argv[2] || path.join(__dirname, '../../tests/golden')
const b64 = u8 => Buffer.from(u8).toString('base64')
const u8 = s => new Uint8Array(Buffer.from(s, 'base64'))
const seen = new Set()
const cases = []
function addConv (name, fmt, input) {
  const key = fmt + ':' + input
  if (seen.has(key)) return
  seen.add(key)
  const c = { name, op: 'conv', fmt, inputs: [input] }
  try {
    const out = (fmt === 1 ? convert.v1ToV2 : convert.v2ToV1)(u8(input))
    c.expect = b64(out)
  } catch (e) {
    c.error = e.constructor.name
    c.message = String(e.message)
  }
  cases.push(c)
}
for (const f of fs.readdirSync(DIR).sort()) {
  if (!f.endsWith('.json') || f === 'conv.json') continue
  const j = JSON.parse(fs.readFileSync(path.join(DIR, f), 'utf8'))
  for (const c of j.cases) {
    if (c.op !== 'merge' && c.inputs.length === 1) addConv(`${f}/${c.name}/${c.op}`, c.fmt, c.inputs[0])
    if (c.op === 'merge' && c.expect) addConv(`${f}/${c.name}/merged`, c.fmt, c.expect)
  }
}
fs.writeFileSync(path.join(DIR, 'conv.json'), JSON.stringify({
  generator: 'oracle/gen/make_conv_fixtures.cjs',
  oracle: 'yjs 13.5.16 convertUpdateFormat (JupyterLab bundle 3502.fbe0c610be82ba1360db.js ms@41803) + lib0 0.2.42',
  cases
}))
console.log('conv.json', cases.length, 'cases', cases.filter(c => c.error).length, 'errors')
