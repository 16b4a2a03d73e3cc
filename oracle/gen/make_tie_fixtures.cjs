// Golden vectors for mergeUpdates over many overlapping inputs (test infrastructure, container-only).
//
// 13.5.16's mergeUpdates re-sorts its readers with Array.prototype.sort on every output struct, and its
// comparator is inconsistent when a GC and an Item start at the same (client, clock) (both orders
// compare as "less").  The output then depends on V8's exact TimSort (runs, binary insertion, galloping
// merges), which only shows with 64 readers or more.  This script hand-builds V1 updates (lib0 0.2.42's
// encoder, bundle module 29194) of a few clients whose struct runs overlap at random clocks -- GC runs
// against Item runs of the same ranges -- in documents of 2 to 300 updates, converts them to V2 with
// yjs's own convertUpdateFormat, and records yjs 13.5.16's mergeUpdates[V2] output for both formats in
// tests/golden/ties.json.  Usage: node make_tie_fixtures.cjs [golden dir]
'use strict'
const fs = require('fs')
const path = require('path')
const { Y, load, convert } = require('./yjs_bundle.cjs')
const enc = load(29194)
const E = { create: enc.Mf, toU8: enc._f, u8: enc.$F, vu: enc.uE, vs: enc.uw }
const DIR = process.argv[2] || path.join(__dirname, '../../tests/golden')

function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return { int: (lo, hi) => lo + (next() % (hi - lo + 1)), chance: p => next() / 4294967296 < p }
}
// one update: a single client section of GC / Item structs starting at `clock`
function update (r, client, clock) {
  const e = E.create()
  const n = r.int(1, 3)
  E.vu(e, 1); E.vu(e, n); E.vu(e, client); E.vu(e, clock)
  let k = clock
  for (let i = 0; i < n; i++) {
    const len = r.int(1, 4)
    if (r.chance(0.45)) { E.u8(e, 0); E.vu(e, len) } else {
      if (k > 0) { E.u8(e, 0x84); E.vu(e, client); E.vu(e, k - 1) } else { E.u8(e, 0x04); E.vu(e, 1); E.vs(e, 'text') }
      E.vs(e, 'abcd'.slice(0, len))
    }
    k += len
  }
  E.vu(e, 0)
  return E.toU8(e)
}
const b64 = u8 => Buffer.from(u8).toString('base64')
const cases = []
function add (name, fmt, inputs) {
  const c = { name, op: 'merge', fmt, inputs: inputs.map(b64) }
  try { c.expect = b64(fmt === 1 ? Y.mergeUpdates(inputs) : Y.mergeUpdatesV2(inputs)) } catch (e) { c.error = e.constructor.name; c.message = String(e.message) }
  cases.push(c)
}
const N = +(process.env.TIE_DOCS || 96)
for (let d = 0; d < N; d++) {
  const r = rng(7000 + d)
  const k = d < 8 ? r.int(2, 63) : r.int(64, 300)
  const clients = r.int(1, 4)
  const ups = []
  for (let i = 0; i < k; i++) ups.push(update(r, 1 + r.int(0, clients - 1), r.int(0, 24)))
  add(`doc${d}_k${k}`, 1, ups)
  add(`doc${d}_k${k}`, 2, ups.map(u => convert.v1ToV2(u)))
}
fs.writeFileSync(path.join(DIR, 'ties.json'), JSON.stringify({
  generator: 'oracle/gen/make_tie_fixtures.cjs',
  oracle: 'yjs 13.5.16 (JupyterLab bundle 3502.fbe0c610be82ba1360db.js) mergeUpdates[V2] + lib0 0.2.42, in Node (V8 TimSort)',
  cases
}))
console.log('ties.json', cases.length, 'cases', cases.filter(c => c.error).length, 'errors')
