// Test-infrastructure loader (container-only): exposes yjs 13.5.16 + lib0 0.2.42 from the offline
// JupyterLab webpack chunks so fixture generators can call Y.mergeUpdates / Y.diffUpdate /
// Y.encodeStateVectorFromUpdate (the byte oracle, SURVEY.md §8c, App. D).  Nothing from the bundle is
// copied into the repo: the chunks are evaluated in place and the script refuses to run without them.
'use strict'
const fs = require('fs')
const path = require('path')
const vm = require('vm')

const BUNDLE_DIR = '/opt/conda/share/jupyter/lab/static'
const CHUNKS = ['3502.fbe0c610be82ba1360db.js', '8086.1dfabaac37d971e2cc4c.js', '7616.d412fb880534d79eb96c.js']
for (const c of CHUNKS) {
  if (!fs.existsSync(path.join(BUNDLE_DIR, c))) {
    throw new Error(`oracle bundle chunk ${c} missing: fixture generation only runs in the survey container`)
  }
}
// deterministic entropy for Doc clientIDs / guids (we always set clientIDs explicitly anyway)
let seedState = 0x9e3779b9
function nextU32 () { seedState ^= seedState << 13; seedState >>>= 0; seedState ^= seedState >>> 17; seedState ^= seedState << 5; seedState >>>= 0; return seedState }
global.crypto = { getRandomValues: arr => { for (let i = 0; i < arr.length; i++) arr[i] = nextU32() & 0xff; return arr } }
Math.random = () => nextU32() / 4294967296
const KEY = 'webpackChunk_jupyterlab_application_top'
global.self = global
global[KEY] = []
// yjs 13.5.16's convertUpdateFormat (ms@41803) is not exported by the bundle: the chunk text is evaluated
// with one added statement that hands the function to the fixture generators (in memory only; the
// files on disk are untouched).  V1ToV2 = ms(u, UpdateDecoderV1 `ye`, UpdateEncoderV2 `De`), V2ToV1 = ks.
const CONVERT_ANCHOR = 'const ks=t=>ms(t,be,Se);'
for (const c of CHUNKS) {
  let src = fs.readFileSync(path.join(BUNDLE_DIR, c), 'utf8')
  if (c.startsWith('3502.')) {
    if (src.split(CONVERT_ANCHOR).length !== 2) throw new Error('convertUpdateFormat anchor not found once')
    src = src.replace(CONVERT_ANCHOR, CONVERT_ANCHOR + 'globalThis.__ymConvert={v1ToV2:t=>ms(t,ye,De),v2ToV1:ks};')
  }
  vm.runInThisContext(src, { filename: c })
}
const factories = {}
for (const entry of global[KEY]) Object.assign(factories, entry[1])
const cache = {}
function load (id) {
  if (cache[id]) return cache[id].exports
  const mod = cache[id] = { exports: {} }
  if (!factories[id]) throw new Error('bundle module not found: ' + id)
  factories[id].call(mod.exports, mod, mod.exports, load)
  return mod.exports
}
load.r = e => Object.defineProperty(e, '__esModule', { value: true })
load.d = (e, getters) => {
  for (const k in getters) if (!Object.prototype.hasOwnProperty.call(e, k)) Object.defineProperty(e, k, { enumerable: true, get: getters[k] })
}
load.o = (o, p) => Object.prototype.hasOwnProperty.call(o, p)
load.n = m => { const g = m && m.__esModule ? () => m.default : () => m; load.d(g, { a: g }); return g }
load.g = global

const Y = load(73502)
const convert = global.__ymConvert  // set when module 73502 ran
module.exports = { Y, load, convert }
