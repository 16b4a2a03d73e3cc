// Golden vectors for payload re-encoding (test infrastructure, container-only).
//
// yjs never copies payload bytes: ContentAny / V2 embed + format values go through readAny -> writeAny,
// V1 embed / format texts and ContentJSON elements through JSON.parse -> JSON.stringify, ContentDoc
// options through new Doc({guid, ...opts}).  This script hand-builds V1 and V2 updates whose payloads are
// NOT in that canonical form (whitespace, escapes, float spellings, duplicate and array-index keys,
// __proto__ keys, integers stored as floats, floats stored as float64 that fit float32, large varInts,
// overlong length prefixes, NaN / Infinity, ...) with lib0 0.2.42's own encoders (bundle module 29194,
// SURVEY.md App. C), then runs yjs 13.5.16's mergeUpdates[V2] / diffUpdate[V2] /
// encodeStateVectorFromUpdate[V2] / convertUpdateFormat over them and records inputs + outputs (or the
// thrown error) in tests/golden/canon.json.  Usage: node make_canon_fixtures.cjs [golden dir]
'use strict'
const fs = require('fs')
const path = require('path')
const { Y, load, convert } = require('./yjs_bundle.cjs')
const enc = load(29194)
const E = {
  create: enc.Mf, toU8: enc._f, u8: enc.$F, vu: enc.uE, vi: enc.pY, vs: enc.uw, any: enc.EM, vbuf: enc.mP, raw: enc.HK,
  Rle: enc.GF, UintOptRle: enc.HE, IntDiffOptRle: enc.sX, Str: enc.TS
}
const DIR = process.argv[2] || path.join(__dirname, '../../tests/golden')

function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return {
    u32: next,
    int: (lo, hi) => lo + (next() % (hi - lo + 1)),
    real: () => next() / 4294967296,
    pick: arr => arr[next() % arr.length],
    chance: p => next() / 4294967296 < p
  }
}

// ---- random non-canonical payloads --------------------------------------------------------------
const WS = ['', '', '', ' ', '\n', ' \t ', '\r\n']
const KEYS = ['a', 'b', 'bold', 'x', '0', '1', '2', '10', '01', '007', '4294967294', '4294967295', '-1', '__proto__', 'é', '😀', 'a b']
function jsonString (r) {
  const parts = ['a', 'Z', ' ', 'é', '😀', '\\"', '\\\\', '\\/', '\\n', '\\t', '\\b', '\\f', '\\r', '\\u0001', '\\u001f',
    '\\u00e9', '\\u00E9', '\\ud83d\\ude00', '\\ud800', '\\udc00x', '\\u2028', '\\u0041', 'xyz']
  let s = '"'
  const n = r.int(0, 5)
  for (let i = 0; i < n; i++) s += r.pick(parts)
  return s + '"'
}
function jsonNumber (r) {
  const forms = [
    () => String(r.int(0, 1000)), () => '-' + r.int(0, 1000), () => '-0', () => '0.5', () => '1.0', () => '1e2', () => '1E+2',
    () => '2.5e-3', () => '123456789012345678901234567890', () => '0.1', () => '1e21', () => '1e-7', () => '123.456e10',
    () => '1e400', () => '-1e400', () => '4.9e-324', () => '2.4703282292062327e-324', () => '1.7976931348623157e308',
    () => '9007199254740993', () => '0.30000000000000004', () => '3.0000', () => String(r.int(0, 99999)) + '.' + String(r.int(0, 99999)) + 'e' + r.int(-30, 30),
    () => '2147483647', () => '2147483648', () => '-2147483649', () => '4294967296', () => '1e15', () => '-1e300'
  ]
  return r.pick(forms)()
}
function jsonValue (r, depth) {
  const k = r.int(0, depth > 2 ? 4 : 7)
  const w = () => r.pick(WS)
  switch (k) {
    case 0: return r.pick(['true', 'false', 'null'])
    case 1: case 2: return jsonNumber(r)
    case 3: case 4: return jsonString(r)
    case 5: case 6: {
      const n = r.int(0, 5)
      const ents = []
      for (let i = 0; i < n; i++) ents.push(w() + JSON.stringify(r.pick(KEYS)).replace('é', r.chance(0.5) ? 'é' : '\\u00e9') + w() + ':' + w() + jsonValue(r, depth + 1) + w())
      return '{' + w() + ents.join(',') + w() + '}'
    }
    default: {
      const n = r.int(0, 4)
      const els = []
      for (let i = 0; i < n; i++) els.push(w() + jsonValue(r, depth + 1) + w())
      return '[' + els.join(',') + ']'
    }
  }
}
function jsonText (r) { return r.pick(WS) + jsonValue(r, 0) + r.pick(WS) }

const f32 = new DataView(new ArrayBuffer(4))
const f64 = new DataView(new ArrayBuffer(8))
function overlongVu (e, v) { // a varuint with one redundant continuation byte
  while (v > 127) { E.u8(e, 0x80 | (v & 127)); v >>>= 7 }
  E.u8(e, 0x80 | v); E.u8(e, 0)
}
function anyValue (r, e, depth) {
  const k = r.int(0, depth > 2 ? 11 : 14)
  switch (k) {
    case 0: E.u8(e, r.pick([127, 126, 121, 120])); return
    case 1: E.u8(e, 125); E.vi(e, r.pick([0, 5, -5, 63, 64, -64, 2147483647, -2147483648, 3000000000, 4294967295])); return
    case 2: { // overlong varInt / -0
      E.u8(e, 125)
      const v = r.int(0, 100)
      if (r.chance(0.5)) { E.u8(e, 0x80 | (v & 63) | (r.chance(0.5) ? 0x40 : 0)); E.u8(e, 0) } else E.u8(e, 0x40)
      return
    }
    case 3: { // float32 holding an integer / fraction / NaN / Infinity
      E.u8(e, 124)
      f32.setFloat32(0, r.pick([5, -7, 0, -0, 0.5, 1.25, 3e9, 16777216, NaN, Infinity, -Infinity, 2147483648, 0.1]))
      for (let i = 0; i < 4; i++) E.u8(e, f32.getUint8(i))
      return
    }
    case 4: { // float64 holding an integer / a float32 value / NaN / -0
      E.u8(e, 123)
      f64.setFloat64(0, r.pick([5, -7, 0, -0, 0.5, 1.25, 3e9, 2147483647, 2147483648, -2147483649, 1e300, NaN, Infinity, 0.1, 1 / 3, 4294967297]))
      for (let i = 0; i < 8; i++) E.u8(e, f64.getUint8(i))
      return
    }
    case 5: E.u8(e, 122); for (let i = 0; i < 8; i++) E.u8(e, r.int(0, 255)); return
    case 6: case 7: {
      E.u8(e, 119)
      const s = r.pick(['', 'abc', 'é', '😀x', 'k'])
      const b = Buffer.from(s, 'utf8')
      if (r.chance(0.3)) overlongVu(e, b.length); else E.vu(e, b.length)
      E.raw(e, b)
      return
    }
    case 8: {
      E.u8(e, 116)
      const n = r.int(0, 4)
      if (r.chance(0.3)) overlongVu(e, n); else E.vu(e, n)
      for (let i = 0; i < n; i++) E.u8(e, r.int(0, 255))
      return
    }
    case 9: case 10: case 11: E.u8(e, r.pick([127, 126, 120])); return
    case 12: case 13: { // object: duplicate / array-index / __proto__ keys
      E.u8(e, 118)
      const n = r.int(0, 5)
      E.vu(e, n)
      for (let i = 0; i < n; i++) { E.vs(e, r.pick(KEYS)); anyValue(r, e, depth + 1) }
      return
    }
    default: {
      E.u8(e, 117)
      const n = r.int(0, 4)
      E.vu(e, n)
      for (let i = 0; i < n; i++) anyValue(r, e, depth + 1)
    }
  }
}
function anyBytes (r) { const e = E.create(); anyValue(r, e, 0); return E.toU8(e) }
function docOpts (r) {
  const e = E.create()
  if (r.chance(0.15)) { anyValue(r, e, 2); return E.toU8(e) }
  const keys = []
  const n = r.int(0, 4)
  for (let i = 0; i < n; i++) keys.push(r.pick(['gc', 'autoLoad', 'meta', 'other', 'gc', 'meta', '__proto__', 'shouldLoad']))
  if (r.chance(0.1)) keys.push('guid')
  E.u8(e, 118)
  E.vu(e, keys.length)
  for (const k of keys) {
    E.vs(e, k)
    if (k === 'guid') { E.u8(e, 119); E.vs(e, 'g-' + r.int(0, 9)) } else anyValue(r, e, 1)
  }
  return E.toU8(e)
}

// ---- update writer (V1 rows / V2 columns) over lib0's encoders ----------------------------------
// struct: {ref, origin: [c,k]|null, content}
function writeUpdate (fmt, sections) {
  if (fmt === 1) {
    const e = E.create()
    E.vu(e, sections.length)
    for (const s of sections) {
      E.vu(e, s.structs.length); E.vu(e, s.client); E.vu(e, s.clock)
      for (const st of s.structs) {
        E.u8(e, st.ref | (st.origin ? 0x80 : 0))
        if (st.origin) { E.vu(e, st.origin[0]); E.vu(e, st.origin[1]) } else { E.vu(e, 1); E.vs(e, 'root') }
        const c = st.content
        switch (st.ref) {
          case 2: E.vu(e, c.length); for (const t of c) E.vs(e, t); break
          case 4: E.vs(e, c); break
          case 5: E.vs(e, c); break
          case 6: E.vs(e, c.key); E.vs(e, c.value); break
          case 8: E.vu(e, c.length); for (const a of c) E.raw(e, a); break
          case 9: E.vs(e, c.guid); E.raw(e, c.opts); break
        }
      }
    }
    E.vu(e, 0) // empty delete set
    return E.toU8(e)
  }
  const kc = new E.IntDiffOptRle(); const cl = new E.UintOptRle(); const lc = new E.IntDiffOptRle(); const rc = new E.IntDiffOptRle()
  const info = new E.Rle(E.u8); const str = new E.Str(); const pinfo = new E.Rle(E.u8); const tref = new E.UintOptRle()
  const len = new E.UintOptRle(); const rest = E.create()
  let keyClock = 0
  E.vu(rest, sections.length)
  for (const s of sections) {
    E.vu(rest, s.structs.length); cl.write(s.client); E.vu(rest, s.clock)
    for (const st of s.structs) {
      info.write(st.ref | (st.origin ? 0x80 : 0))
      if (st.origin) { cl.write(st.origin[0]); lc.write(st.origin[1]) } else { pinfo.write(1); str.write('root') }
      const c = st.content
      switch (st.ref) {
        case 2: len.write(c.length); for (const t of c) str.write(t); break
        case 4: str.write(c); break
        case 5: E.raw(rest, c); break
        case 6: kc.write(keyClock++); str.write(c.key); E.raw(rest, c.value); break
        case 8: len.write(c.length); for (const a of c) E.raw(rest, a); break
        case 9: str.write(c.guid); E.raw(rest, c.opts); break
      }
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
function randStruct (r, fmt) {
  const ref = r.pick([2, 2, 4, 5, 5, 6, 6, 8, 8, 8, 9])
  switch (ref) {
    case 2: { const n = r.int(1, 4); const a = []; for (let i = 0; i < n; i++) a.push(r.chance(0.15) ? 'undefined' : jsonText(r)); return { ref, content: a, len: n } }
    case 4: return { ref, content: r.pick(['ab', 'xyz', 'é!']), len: null }
    case 5: return { ref, content: fmt === 1 ? jsonText(r) : anyBytes(r), len: 1 }
    case 6: return { ref, content: { key: r.pick(['bold', 'color', 'x']), value: fmt === 1 ? jsonText(r) : anyBytes(r) }, len: 1 }
    case 8: { const n = r.int(1, 4); const a = []; for (let i = 0; i < n; i++) a.push(anyBytes(r)); return { ref, content: a, len: n } }
    default: return { ref, content: { guid: 'doc-' + r.int(0, 99), opts: docOpts(r) }, len: 1 }
  }
}
function strLen16 (s) { return s.length }
function randSection (r, fmt, client, clock, n) {
  const structs = []
  let k = clock
  for (let i = 0; i < n; i++) {
    const st = randStruct(r, fmt)
    st.origin = i === 0 ? null : [client, k - 1]
    structs.push(st)
    k += st.ref === 4 ? strLen16(st.content) : st.len
  }
  return { section: { client, clock, structs }, end: k }
}

// ---- cases ------------------------------------------------------------------------------------
const b64 = u8 => Buffer.from(u8).toString('base64')
const cases = []
function run (op, fmt, inputs, sv) {
  if (op === 'merge') return fmt === 1 ? Y.mergeUpdates(inputs) : Y.mergeUpdatesV2(inputs)
  if (op === 'diff') return fmt === 1 ? Y.diffUpdate(inputs[0], sv) : Y.diffUpdateV2(inputs[0], sv)
  if (op === 'sv') return fmt === 1 ? Y.encodeStateVectorFromUpdate(inputs[0]) : Y.encodeStateVectorFromUpdateV2(inputs[0])
  if (op === 'conv') return (fmt === 1 ? convert.v1ToV2 : convert.v2ToV1)(inputs[0])
  throw new Error(op)
}
function addCase (name, op, fmt, inputs, sv) {
  const c = { name, op, fmt, inputs: inputs.map(b64) }
  if (sv !== undefined) c.sv = b64(sv)
  try { c.expect = b64(run(op, fmt, inputs, sv)) } catch (e) { c.error = e.constructor.name; c.message = String(e.message) }
  cases.push(c)
}
function sv (pairs) { const e = E.create(); E.vu(e, pairs.length); for (const [c, k] of pairs) { E.vu(e, c); E.vu(e, k) } return E.toU8(e) }

const N = +(process.env.CANON_DOCS || 160)
for (let d = 0; d < N; d++) {
  const r = rng(1000 + d)
  for (const fmt of [1, 2]) {
    const client = r.int(1, 5)
    // two consecutive updates of one client + one of another client: merge, diff (cuts inside Any / JSON
    // element runs), state vector, conversion
    const a = randSection(r, fmt, client, 0, r.int(1, 4))
    const b = randSection(r, fmt, client, a.end, r.int(1, 3))
    const o = randSection(r, fmt, client + 10, 0, r.int(1, 3))
    const u1 = writeUpdate(fmt, [a.section]); const u2 = writeUpdate(fmt, [b.section]); const u3 = writeUpdate(fmt, [o.section])
    addCase(`doc${d}/merge`, 'merge', fmt, [u1, u2, u3])
    const whole = writeUpdate(fmt, [o.section, { client, clock: 0, structs: a.section.structs.concat(b.section.structs) }])
    addCase(`doc${d}/diff`, 'diff', fmt, [whole], sv([[client, r.int(0, b.end)], [client + 10, r.int(0, o.end)]]))
    addCase(`doc${d}/conv`, 'conv', fmt, [whole])
    if (d % 8 === 0) addCase(`doc${d}/sv`, 'sv', fmt, [whole])
  }
}
fs.writeFileSync(path.join(DIR, 'canon.json'), JSON.stringify({
  generator: 'oracle/gen/make_canon_fixtures.cjs',
  oracle: 'yjs 13.5.16 (JupyterLab bundle 3502.fbe0c610be82ba1360db.js) + lib0 0.2.42: mergeUpdates[V2], diffUpdate[V2], encodeStateVectorFromUpdate[V2], convertUpdateFormat',
  cases
}))
console.log('canon.json', cases.length, 'cases', cases.filter(c => c.error).length, 'errors')
