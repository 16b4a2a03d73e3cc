// Test-infrastructure loader (container-only) for gaberogan/yjs@v0 itself (yjs 13.4.9, /root/reference).
//
// The reference imports lib0 0.2.33, which is not vendored (SURVEY.md F3).  As SURVEY.md §8c / App. D
// describe, its src/ runs under Node 12 ESM against a lib0 shim whose wire modules (encoding, decoding,
// buffer, binary) re-export the offline lib0 0.2.42 of the JupyterLab bundle (yjs_bundle.cjs) and whose
// utility modules are one-liners.  Nothing is copied into the repository: the reference's src/ is copied
// to a scratch directory under /tmp at run time (ESM needs a package.json with "type": "module" next to
// it), the shims are written there, and the scratch directory is removed at exit.  The script refuses to
// run when /root/reference is absent (e.g. on the GPU box).
'use strict'
const fs = require('fs')
const os = require('os')
const path = require('path')

const REF_SRC = '/root/reference/src'
const BUNDLE = path.join(__dirname, 'yjs_bundle.cjs')

function copyDir (src, dst) {
  fs.mkdirSync(dst, { recursive: true })
  for (const e of fs.readdirSync(src, { withFileTypes: true })) {
    const s = path.join(src, e.name); const d = path.join(dst, e.name)
    if (e.isDirectory()) copyDir(s, d); else fs.copyFileSync(s, d)
  }
}

// lib0 name -> (bundle module id, {export: mangled}) for the wire modules (SURVEY.md App. C)
const WIRE = {
  encoding: [29194, {
    createEncoder: 'Mf', length: 'kE', toUint8Array: '_f', write: 'cW', writeAny: 'EM', writeUint32: 'Ep', writeUint8: '$F',
    writeUint8Array: 'HK', writeVarInt: 'pY', writeVarString: 'uw', writeVarUint: 'uE', writeVarUint8Array: 'mP',
    writeBinaryEncoder: 'mK', IntDiffOptRleEncoder: 'sX', RleEncoder: 'GF', StringEncoder: 'TS', UintOptRleEncoder: 'HE'
  }, 'export const Encoder = m.Mf().constructor\n'],
  decoding: [64485, {
    createDecoder: 'l1', hasContent: 'v3', readVarUint8Array: 'HN', readTailAsUint8Array: 'iU', readUint8: 'kj', readUint32: 'Jl',
    readVarUint: 'yg', readVarInt: 'F7', readVarString: 'kf', readAny: 'v_', RleDecoder: 'XW', UintOptRleDecoder: 'UF',
    IntDiffOptRleDecoder: 'dD', StringDecoder: 'sO'
  }, 'export const Decoder = m.l1(new Uint8Array(0)).constructor\n'],
  buffer: [65679, { createUint8ArrayViewFromArrayBuffer: 'Te', createUint8ArrayFromArrayBuffer: 'eh', toBase64: 's3', fromBase64: 'Gh', copyUint8Array: 'f9' }, ''],
  binary: [15966, { BIT1: 'Vw', BIT2: 'Qn', BIT3: 'CY', BIT4: 'Ko', BIT6: 'cq', BIT7: 'rc', BIT8: 'x1', BITS5: 'kr', BITS6: '$2', BITS7: 'jS', BITS8: 'x', BITS31: 'RP' }, '']
}
// utility modules: small restatements of the lib0 functions the reference calls
const UTIL = {
  array: 'export const last = a => a[a.length - 1]\nexport const from = Array.from\nexport const appendTo = (dest, src) => { for (let i = 0; i < src.length; i++) dest.push(src[i]) }\nexport const isArray = Array.isArray\n',
  error: "export const create = s => new Error(s)\nexport const methodUnimplemented = () => { throw create('Method unimplemented') }\nexport const unexpectedCase = () => { throw create('Unexpected case') }\n",
  function: 'export const callAll = (fs, args, i = 0) => { try { for (; i < fs.length; i++) fs[i](...args) } finally { if (i < fs.length) callAll(fs, args, i + 1) } }\nexport const nop = () => {}\n',
  iterator: 'export const iteratorMap = (it, f) => ({ [Symbol.iterator] () { return this }, next () { const r = it.next(); return { done: r.done, value: r.done ? undefined : f(r.value) } } })\nexport const iteratorFilter = (it, f) => ({ [Symbol.iterator] () { return this }, next () { let r; do { r = it.next() } while (!r.done && !f(r.value)); return r } })\nexport const next = it => it.next()\n',
  logging: "export const BOLD = ''\nexport const UNBOLD = ''\nexport const RED = ''\nexport const ORANGE = ''\nexport const GREEN = ''\nexport const print = () => {}\n",
  map: 'export const create = () => new Map()\nexport const copy = m => { const r = create(); m.forEach((v, k) => r.set(k, v)); return r }\nexport const setIfUndefined = (map, key, createT) => { let set = map.get(key); if (set === undefined) map.set(key, set = createT()); return set }\nexport const map = (m, f) => { const res = []; for (const [key, value] of m) res.push(f(value, key)); return res }\nexport const any = (m, f) => { for (const [key, value] of m) if (f(value, key)) return true; return false }\nexport const all = (m, f) => { for (const [key, value] of m) if (!f(value, key)) return false; return true }\n',
  math: 'export const floor = Math.floor\nexport const ceil = Math.ceil\nexport const abs = Math.abs\nexport const min = (a, b) => a < b ? a : b\nexport const max = (a, b) => a > b ? a : b\nexport const isNegativeZero = n => n !== 0 ? n < 0 : 1 / n < 0\n',
  object: 'export const keys = Object.keys\nexport const equalFlat = (a, b) => a === b || (Object.keys(a).length === Object.keys(b).length && Object.keys(a).every(k => (a[k] !== undefined || b.hasOwnProperty(k)) && a[k] === b[k]))\n',
  observable: 'export class Observable { constructor () { this._observers = new Map() } on (n, f) { if (!this._observers.has(n)) this._observers.set(n, new Set()); this._observers.get(n).add(f) } once (n, f) { const g = (...a) => { this.off(n, g); f(...a) }; this.on(n, g) } off (n, f) { const s = this._observers.get(n); if (s !== undefined) { s.delete(f); if (s.size === 0) this._observers.delete(n) } } emit (n, args) { return Array.from((this._observers.get(n) || new Map()).values()).forEach(f => f(...args)) } destroy () { this._observers = new Map() } }\n',
  random: "let s = 0x2545f491\nexport const uint32 = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }\nexport const uuidv4 = () => 'xxxxxxxx-xxxx-4xxx-yxxx-xxxxxxxxxxxx'.replace(/[xy]/g, c => (uint32() % 16).toString(16))\n",
  set: 'export const create = () => new Set()\n',
  time: 'export const getUnixTime = Date.now\n'
}

async function loadReference () {
  if (!fs.existsSync(REF_SRC)) throw new Error('the reference (' + REF_SRC + ') is only available in the survey container')
  const dir = fs.mkdtempSync(path.join(os.tmpdir(), 'yjs_ref_'))
  process.on('exit', () => { try { fs.rmSync ? fs.rmSync(dir, { recursive: true, force: true }) : fs.rmdirSync(dir, { recursive: true }) } catch (e) {} })
  copyDir(REF_SRC, path.join(dir, 'src'))
  fs.writeFileSync(path.join(dir, 'package.json'), '{"type": "module"}\n')
  const lib = path.join(dir, 'node_modules', 'lib0')
  fs.mkdirSync(lib, { recursive: true })
  fs.writeFileSync(path.join(lib, 'package.json'), '{"type": "module"}\n')
  for (const [name, [id, names, extra]] of Object.entries(WIRE)) {
    let src = "import { createRequire } from 'module'\nconst require = createRequire(import.meta.url)\n"
    src += `const m = require(${JSON.stringify(BUNDLE)}).load(${id})\n`
    for (const [k, v] of Object.entries(names)) src += `export const ${k} = m[${JSON.stringify(v)}]\n`
    fs.writeFileSync(path.join(lib, name + '.js'), src + extra)
  }
  for (const [name, src] of Object.entries(UTIL)) fs.writeFileSync(path.join(lib, name + '.js'), src)
  const Y = await import(path.join(dir, 'src', 'internals.js'))
  return Y
}
module.exports = { loadReference }
