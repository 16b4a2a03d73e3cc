// Golden vectors for V2 string-column corner cases (test infrastructure, container-only).
//
// The V2 encoding keeps every string of an update in one string column: StringEncoder concatenates them
// and StringDecoder slices the decoded column by UTF-16 lengths (lib0 0.2.42), and readKey caches the
// element / hook names it has read (UpdateDecoder.js:382-391).  So a V2 update can carry strings that
// start or end with half of a surrogate pair (valid only as a whole column), key references to earlier
// names, and negative key references (keys[-1] is undefined).  This script hand-builds such V2 updates
// with lib0's own column encoders (bundle module 29194) -- Y.Text strings, map keys (parentSub), element
// and hook names, format keys -- and records yjs 13.5.16's mergeUpdatesV2 / diffUpdateV2 /
// encodeStateVectorFromUpdateV2 / convertUpdateFormatV2ToV1 outputs (or the thrown error) in
// tests/golden/v2str.json.  Usage: node make_v2str_fixtures.cjs [golden dir]
'use strict'
const fs = require('fs')
const path = require('path')
const { Y, load, convert } = require('./yjs_bundle.cjs')
const enc = load(29194)
const E = {
  create: enc.Mf, toU8: enc._f, u8: enc.$F, vu: enc.uE, vs: enc.uw, raw: enc.HK, any: enc.EM, vbuf: enc.mP,
  Rle: enc.GF, UintOptRle: enc.HE, IntDiffOptRle: enc.sX, Str: enc.TS
}
const DIR = process.argv[2] || path.join(__dirname, '../../tests/golden')

function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return { int: (lo, hi) => lo + (next() % (hi - lo + 1)), pick: a => a[next() % a.length], chance: p => next() / 4294967296 < p }
}
const ASTRAL = ['😀', '😎', '🎉', '𝄞', '💩']
const PLAIN = ['a', 'bc', 'é', 'xyz', '😀', 'k1', '']
// a V2 update of one client section; structs: {ref, origin, parentSub?, content}
function writeV2 (client, clock, structs, keyRefs) {
  const kc = new E.IntDiffOptRle(); const cl = new E.UintOptRle(); const lc = new E.IntDiffOptRle(); const rc = new E.IntDiffOptRle()
  const info = new E.Rle(E.u8); const str = new E.Str(); const pinfo = new E.Rle(E.u8); const tref = new E.UintOptRle()
  const len = new E.UintOptRle(); const rest = E.create()
  let keyClock = 0
  E.vu(rest, 1); E.vu(rest, structs.length); cl.write(client); E.vu(rest, clock)
  for (const st of structs) {
    const inf = st.ref | (st.origin ? 0x80 : 0) | (!st.origin && st.psub !== undefined ? 0x20 : 0)
    info.write(inf)
    if (st.origin) { cl.write(st.origin[0]); lc.write(st.origin[1]) } else {
      pinfo.write(1); str.write(st.ykey)
      if (st.psub !== undefined) str.write(st.psub)
    }
    const c = st.content
    switch (st.ref) {
      case 1: len.write(c); break
      case 4: str.write(c); break
      case 6: kc.write(keyClock++); str.write(c.key); E.any(rest, c.value); break
      case 7:
        tref.write(c.type)
        if (c.type === 3 || c.type === 5) {
          if (c.ref !== undefined) kc.write(c.ref) // a cached (or negative) key reference: no string
          else { kc.write(keyRefs.n++); str.write(c.name) }
        }
        break
    }
  }
  E.vu(rest, 0)
  const e = E.create()
  E.vu(e, 0)
  E.vbuf(e, kc.toUint8Array()); E.vbuf(e, cl.toUint8Array()); E.vbuf(e, lc.toUint8Array()); E.vbuf(e, rc.toUint8Array())
  E.vbuf(e, E.toU8(info)); E.vbuf(e, str.toUint8Array()); E.vbuf(e, E.toU8(pinfo)); E.vbuf(e, tref.toUint8Array())
  E.vbuf(e, len.toUint8Array()); E.raw(e, E.toU8(rest))
  return E.toU8(e)
}
// random structs whose strings are balanced as a column: a string may end with the high half of a
// pair whose low half starts the next string in column order
function randStructs (r, client, clock, n, split) {
  const structs = []
  let pend = null
  let names = 0
  const mk = (allowEnd = true) => {
    let s = ''
    if (pend) { s += pend; pend = null }
    s += r.pick(PLAIN)
    if (split && allowEnd && r.chance(0.35)) { const ch = r.pick(ASTRAL); s += ch[0]; pend = ch[1] }
    return s
  }
  let k = clock
  for (let i = 0; i < n; i++) {
    const st = { origin: i === 0 && k === 0 ? null : [client, k - 1] }
    if (!st.origin) { st.ykey = mk(); if (r.chance(0.5)) st.psub = mk() }
    const kind = r.pick([4, 4, 4, 7, 7, 6, 1])
    st.ref = kind
    let l = 1
    if (kind === 4) { st.content = mk(); if (st.content.length === 0) st.content = 'q'; l = st.content.length }
    else if (kind === 1) { st.content = r.int(1, 3); l = st.content }
    else if (kind === 6) st.content = { key: mk(), value: r.pick([true, 1, 'v', null]) }
    else {
      const type = r.pick([3, 3, 5, 0, 1])
      st.content = { type }
      if (type === 3 || type === 5) {
        if (names > 0 && r.chance(0.4)) st.content.ref = r.int(0, names - 1)        // cached key
        else if (r.chance(0.08)) st.content.ref = -1 - r.int(0, 2)                // keys[negative]: undefined
        else { st.content.name = mk(); names++ }
      }
    }
    structs.push(st)
    k += l
  }
  if (pend) structs.push({ origin: [client, k - 1], ref: 4, content: pend + 'z' }), k += 1 + pend.length
  return { structs, end: k }
}
const b64 = u8 => Buffer.from(u8).toString('base64')
const cases = []
function run (op, inputs, sv) {
  if (op === 'merge') return Y.mergeUpdatesV2(inputs)
  if (op === 'diff') return Y.diffUpdateV2(inputs[0], sv)
  if (op === 'sv') return Y.encodeStateVectorFromUpdateV2(inputs[0])
  if (op === 'conv') return convert.v2ToV1(inputs[0])
  throw new Error(op)
}
function add (name, op, inputs, sv) {
  const c = { name, op, fmt: 2, inputs: inputs.map(b64) }
  if (sv !== undefined) c.sv = b64(sv)
  try { c.expect = b64(run(op, inputs, sv)) } catch (e) { c.error = e.constructor.name; c.message = String(e.message) }
  cases.push(c)
}
function svBytes (pairs) { const e = E.create(); E.vu(e, pairs.length); for (const [c, k] of pairs) { E.vu(e, c); E.vu(e, k) } return E.toU8(e) }
const N = +(process.env.V2STR_DOCS || 160)
let skipped = 0
for (let d = 0; d < N; d++) {
  const r = rng(9100 + d)
  const split = d % 4 !== 3
  const a = randStructs(r, 3, 0, r.int(1, 6), split)
  const b = randStructs(r, 3, a.end, r.int(1, 4), split)
  const o = randStructs(r, 7, 0, r.int(1, 4), split)
  let ua, ub, uo, whole
  try {
    ua = writeV2(3, 0, a.structs, { n: 0 }); ub = writeV2(3, a.end, b.structs, { n: 0 }); uo = writeV2(7, 0, o.structs, { n: 0 })
    whole = writeV2(3, 0, a.structs.concat(b.structs), { n: 0 })
  } catch (e) { skipped++; continue } // a column lib0 itself cannot encode
  add(`doc${d}/merge`, 'merge', [ua, ub, uo])
  add(`doc${d}/merge_rev`, 'merge', [uo, ub, ua])
  add(`doc${d}/diff`, 'diff', [whole], svBytes([[3, r.int(0, b.end)]]))
  add(`doc${d}/conv`, 'conv', [whole])
  if (d % 4 === 0) add(`doc${d}/sv`, 'sv', [whole])
}
fs.writeFileSync(path.join(DIR, 'v2str.json'), JSON.stringify({
  generator: 'oracle/gen/make_v2str_fixtures.cjs',
  oracle: 'yjs 13.5.16 (JupyterLab bundle 3502.fbe0c610be82ba1360db.js) mergeUpdatesV2 / diffUpdateV2 / encodeStateVectorFromUpdateV2 / convertUpdateFormatV2ToV1 + lib0 0.2.42',
  cases
}))
console.log('v2str.json', cases.length, 'cases', cases.filter(c => c.error).length, 'errors', skipped, 'skipped')
