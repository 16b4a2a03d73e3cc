// Golden-vector generator (test infrastructure, container-only).
//
// Runs the byte oracle -- yjs 13.5.16 Y.mergeUpdates[V2] / Y.diffUpdate[V2] /
// Y.encodeStateVectorFromUpdate[V2], loaded from the offline JupyterLab bundle by yjs_bundle.cjs --
// over seeded synthetic workloads shaped like BASELINE.json's configs (C1 text trace, C2 multi-client
// rich text, C4 delete-heavy maps, C5 XML fragments) plus the edge cases of SURVEY.md §8c, and writes
// inputs + expected outputs (or the thrown error) to tests/golden/*.json.  The fixtures are data; this
// script is the committed recipe that made them.  Usage: node make_fixtures.cjs <outdir>
'use strict'
const fs = require('fs')
const path = require('path')
const { Y, load } = require('./yjs_bundle.cjs')
const enc = load(29194) // lib0 encoding 0.2.42 (SURVEY.md App. C name table)
const E = {
  create: enc.Mf, toU8: enc._f, u8: enc.$F, vu: enc.uE, vi: enc.pY, vs: enc.uw, any: enc.EM, vbuf: enc.mP, raw: enc.HK
}

const OUT = process.argv[2] || path.join(__dirname, '../../tests/golden')

// ---- seeded PRNG (xorshift32, as the survey's gen.mjs) ----
function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return {
    u32: next,
    int: (lo, hi) => lo + (next() % (hi - lo + 1)), // inclusive
    real: () => next() / 4294967296,
    pick: arr => arr[next() % arr.length],
    word: (lo, hi) => { const n = lo + (next() % (hi - lo + 1)); let w = ''; for (let i = 0; i < n; i++) w += String.fromCharCode(97 + next() % 26); return w }
  }
}

const b64 = u8 => Buffer.from(u8).toString('base64')
const cases = {}
function add (group, c) { (cases[group] = cases[group] || []).push(c) }

function runOp (op, fmt, inputs, sv) {
  try {
    let out
    if (op === 'merge') out = fmt === 1 ? Y.mergeUpdates(inputs) : Y.mergeUpdatesV2(inputs)
    else if (op === 'diff') out = fmt === 1 ? Y.diffUpdate(inputs[0], sv) : Y.diffUpdateV2(inputs[0], sv)
    else if (op === 'sv') out = fmt === 1 ? Y.encodeStateVectorFromUpdate(inputs[0]) : Y.encodeStateVectorFromUpdateV2(inputs[0])
    else throw new Error('bad op')
    return { out: b64(out), same: op === 'merge' && inputs.length === 1 && out === inputs[0] }
  } catch (e) {
    return { error: e.constructor.name, message: String(e.message) }
  }
}

function addCase (group, name, op, fmt, inputs, sv) {
  const r = runOp(op, fmt, inputs, sv)
  const c = { name, op, fmt, inputs: inputs.map(b64) }
  if (sv !== undefined) c.sv = b64(sv)
  if (r.error) { c.error = r.error; c.message = r.message } else { c.expect = r.out; if (r.same) c.identity = true }
  add(group, c)
  return r
}

// ---- document-shaped workload generators (13.5.16 Doc API produces the updates) ----
function capture (doc, sink1, sink2) {
  doc.on('update', (u, origin) => { if (origin !== 'remote') sink1.push(u) })
  doc.on('updateV2', (u, origin) => { if (origin !== 'remote') sink2.push(u) })
}

function syncOneWay (r, docs) {
  const a = r.pick(docs); const b = r.pick(docs)
  if (a === b) return
  Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)), 'remote')
}

// C1/C2: Y.Text, nClients, nTx transactions; 60% insert word (20% bold), 40% delete 1..3; 30% sync
function genText (seed, nClients, nTx, opts = {}) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc()
    d.clientID = opts.clientIds ? opts.clientIds[c] : 1000 + 7919 * c
    capture(d, v1, v2)
    docs.push(d)
  }
  const opsPerTx = opts.opsPerTx || 1
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const text = d.getText('text')
    d.transact(() => {
      for (let o = 0; o < opsPerTx; o++) {
        const len = text.length
        if (len === 0 || r.real() < 0.6) {
          const pos = r.int(0, len)
          let w = r.word(1, 5)
          if (opts.unicode && r.real() < 0.3) w += r.pick(['é', '中', '😀', '€', '𝄞'])
          if (opts.bold !== false && r.real() < 0.2) text.insert(pos, w, { bold: true })
          else if (opts.rich && r.real() < 0.2) text.insert(pos, w, r.pick([{ italic: true }, { italic: true, color: '#ff0' }, { bold: null }]))
          else text.insert(pos, w)
          if (opts.embed && r.real() < 0.05) text.insertEmbed(r.int(0, text.length), { image: 'img' + r.u32() % 100 })
        } else {
          const pos = r.int(0, len - 1)
          text.delete(pos, Math.min(r.int(1, 3), len - pos))
        }
      }
    })
    if (r.real() < (opts.syncP === undefined ? 0.3 : opts.syncP)) syncOneWay(r, docs)
  }
  return { v1, v2, docs }
}

// C4: Y.Map broadcast, delete-heavy
function genMap (seed, nClients, nTx, nKeys) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = 500 + 31 * c; docs.push(d)
  }
  for (const d of docs) {
    d.on('update', (u, origin) => {
      if (origin === 'remote') return
      v1.push(u)
      for (const o of docs) if (o !== d) Y.applyUpdate(o, u, 'remote')
    })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') v2.push(u) })
  }
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const m = d.getMap('map')
    const key = 'k' + (r.u32() % nKeys)
    if (m.has(key) && r.real() < 0.6) m.delete(key)
    else m.set(key, r.real() < 0.5 ? r.int(0, 1000000) : r.word(1, 6))
  }
  return { v1, v2, docs }
}

// C5: XmlFragment with elements, attributes, formatted text
function genXml (seed, nClients, nTx) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = 2000 + 13 * c; capture(d, v1, v2); docs.push(d)
  }
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const frag = d.getXmlFragment('xml')
    const p = r.real()
    if (p < 0.4 || frag.length === 0) {
      const el = new Y.XmlElement(r.pick(['p', 'h1']))
      el.setAttribute('class', 'c' + (r.u32() % 5))
      const tx = new Y.XmlText()
      el.insert(0, [tx])
      frag.insert(r.int(0, frag.length), [el])
      tx.insert(0, r.word(1, 6), r.real() < 0.5 ? { bold: true } : {})
    } else if (p < 0.75) {
      const el = frag.get(r.int(0, frag.length - 1))
      if (el instanceof Y.XmlElement && el.length > 0) {
        const tx = el.get(0)
        if (tx instanceof Y.XmlText) tx.insert(r.int(0, tx.length), r.word(1, 4), r.real() < 0.5 ? { italic: true } : {})
      }
    } else if (p < 0.8) {
      frag.insert(r.int(0, frag.length), [new Y.XmlHook('hook' + (r.u32() % 3))])
    } else {
      frag.delete(r.int(0, frag.length - 1), 1)
    }
    if (r.real() < 0.3) syncOneWay(r, docs)
  }
  return { v1, v2, docs }
}

// Y.Array with every `any` tag, binary, subdocs, nested types
function genArrayAny (seed) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const d = new Y.Doc(); d.clientID = 77; capture(d, v1, v2)
  const arr = d.getArray('array')
  const values = [null, 0, -0, 1, -1, 63, 64, -64, 2147483647, 2147483648, -2147483648, -2147483649, 4294967295, 2.5, 0.1,
    1e300, -1e-300, 3.0, true, false, '', 'str', '😀x', { a: 1, b: [1, 2, { c: 'd' }] }, { 1: 'x', b: 2, 0: 'y' },
    [1, 'two', null], new Uint8Array([1, 2, 3, 255]), 1.5e-7, 123456789012, -0.5]
  for (let i = 0; i < values.length; i++) arr.insert(arr.length, [values[i]])
  arr.insert(1, values.slice(0, 12))
  arr.insert(0, [new Uint8Array([9, 8, 7])]) // ContentBinary
  const sub = new Y.Map(); arr.insert(2, [sub]); sub.set('x', 'y'); sub.set('n', 5)
  const subdoc = new Y.Doc({ guid: 'sub-guid-1' }); arr.insert(3, [subdoc])
  const subdoc2 = new Y.Doc({ guid: 'sub-guid-2', gc: false, autoLoad: true, meta: { m: 1 } }); arr.insert(0, [subdoc2])
  const nested = new Y.Array(); arr.insert(1, [nested]); nested.insert(0, [1, 2, 3])
  const txt = new Y.Text(); arr.insert(0, [txt]); txt.insert(0, 'nested text')
  for (let i = 0; i < 10; i++) arr.delete(r.int(0, arr.length - 1), 1)
  arr.insert(arr.length, ['tail', 42])
  return { v1, v2 }
}

function hexBytes (h) { return Uint8Array.from(Buffer.from(h.replace(/\s+/g, ''), 'hex')) }

function buildV1 (fn) { const e = E.create(); fn(e); return E.toU8(e) }

function main () {
  // ---------------- C1: one client text trace (merge of all incremental updates + partial merges) ---
  {
    const { v1, v2 } = genText(12345, 1, 300, { opsPerTx: 10, bold: false, syncP: 0 })
    addCase('c1_text', 'c1_merge_all', 'merge', 1, v1)
    addCase('c1_text', 'c1_merge_all', 'merge', 2, v2)
    const half = Math.floor(v1.length / 2)
    const m1a = Y.mergeUpdates(v1.slice(0, half)); const m1b = Y.mergeUpdates(v1.slice(half))
    addCase('c1_text', 'c1_merge_of_merges', 'merge', 1, [m1a, m1b])
    const m2a = Y.mergeUpdatesV2(v2.slice(0, half)); const m2b = Y.mergeUpdatesV2(v2.slice(half))
    addCase('c1_text', 'c1_merge_of_merges', 'merge', 2, [m2a, m2b])
    addCase('c1_text', 'c1_merge_reversed', 'merge', 1, v1.slice().reverse())
    addCase('c1_text', 'c1_merge_reversed', 'merge', 2, v2.slice().reverse())
    const st1 = Y.mergeUpdates(v1); const st2 = Y.mergeUpdatesV2(v2)
    addCase('c1_text', 'c1_sv_state', 'sv', 1, [st1])
    addCase('c1_text', 'c1_sv_state', 'sv', 2, [st2])
    const r = rng(99)
    for (let k = 0; k < 6; k++) {
      const cut = r.int(0, 3000)
      const sve = E.create(); E.vu(sve, 1); E.vu(sve, 1000); E.vu(sve, cut)
      const sv = E.toU8(sve)
      addCase('c1_text', 'c1_diff_' + k, 'diff', 1, [st1], sv)
      addCase('c1_text', 'c1_diff_' + k, 'diff', 2, [st2], sv)
    }
  }
  // ---------------- C2: multi-client rich text docs ----------------
  for (let doc = 0; doc < 48; doc++) {
    const { v1, v2 } = genText(doc + 1, 4, 100, { clientIds: [1000, 8919, 16838, 24757] })
    addCase('c2_text', 'c2_doc' + doc, 'merge', 1, v1)
    addCase('c2_text', 'c2_doc' + doc, 'merge', 2, v2)
    if (doc < 12) {
      const r = rng(1000 + doc)
      const st1 = Y.mergeUpdates(v1); const st2 = Y.mergeUpdatesV2(v2)
      // random SV, empty SV, full SV
      const svFull = Y.encodeStateVectorFromUpdate(st1)
      const sve = E.create(); E.vu(sve, 3)
      for (const c of [1000, 8919, 24757]) { E.vu(sve, c); E.vu(sve, r.int(0, 200)) }
      const svRand = E.toU8(sve)
      for (const [nm, sv] of [['rand', svRand], ['empty', Uint8Array.of(0)], ['full', svFull]]) {
        addCase('c2_text', `c2_doc${doc}_diff_${nm}`, 'diff', 1, [st1], sv)
        addCase('c2_text', `c2_doc${doc}_diff_${nm}`, 'diff', 2, [st2], sv)
      }
      addCase('c2_text', `c2_doc${doc}_sv`, 'sv', 1, [st1])
      addCase('c2_text', `c2_doc${doc}_sv`, 'sv', 2, [st2])
      for (let i = 0; i < 5; i++) {
        const j = r.int(0, v1.length - 1)
        addCase('c2_text', `c2_doc${doc}_sv_upd${j}`, 'sv', 1, [v1[j]])
        addCase('c2_text', `c2_doc${doc}_sv_upd${j}`, 'sv', 2, [v2[j]])
      }
    }
  }
  // ---------------- C4: delete-heavy maps ----------------
  for (let doc = 0; doc < 24; doc++) {
    const big = doc < 4
    const { v1, v2 } = genMap(doc + 1, big ? 64 : 8, big ? 128 : 48, 8)
    addCase('c4_map', 'c4_doc' + doc, 'merge', 1, v1)
    addCase('c4_map', 'c4_doc' + doc, 'merge', 2, v2)
    if (doc < 6) {
      const st1 = Y.mergeUpdates(v1); const st2 = Y.mergeUpdatesV2(v2)
      addCase('c4_map', `c4_doc${doc}_sv`, 'sv', 1, [st1])
      addCase('c4_map', `c4_doc${doc}_sv`, 'sv', 2, [st2])
      const sve = E.create(); E.vu(sve, 2); E.vu(sve, 500); E.vu(sve, 3); E.vu(sve, 531); E.vu(sve, 1)
      addCase('c4_map', `c4_doc${doc}_diff`, 'diff', 1, [st1], E.toU8(sve))
      addCase('c4_map', `c4_doc${doc}_diff`, 'diff', 2, [st2], E.toU8(sve))
    }
  }
  // ---------------- C5: XML fragments ----------------
  for (let doc = 0; doc < 10; doc++) {
    const { v1, v2 } = genXml(doc + 7, 8, 64)
    addCase('c5_xml', 'c5_doc' + doc, 'merge', 1, v1)
    addCase('c5_xml', 'c5_doc' + doc, 'merge', 2, v2)
    const st1 = Y.mergeUpdates(v1); const st2 = Y.mergeUpdatesV2(v2)
    const r = rng(50 + doc)
    const sve = E.create(); E.vu(sve, 4)
    for (let c = 0; c < 4; c++) { E.vu(sve, 2000 + 13 * (2 * c)); E.vu(sve, r.int(0, 40)) }
    addCase('c5_xml', `c5_doc${doc}_diff`, 'diff', 1, [st1], E.toU8(sve))
    addCase('c5_xml', `c5_doc${doc}_diff`, 'diff', 2, [st2], E.toU8(sve))
    addCase('c5_xml', `c5_doc${doc}_sv`, 'sv', 1, [st1])
    addCase('c5_xml', `c5_doc${doc}_sv`, 'sv', 2, [st2])
  }
  // ---------------- content variety: any tags, binary, subdocs, nested types, embeds, unicode -------
  {
    const { v1, v2 } = genArrayAny(5)
    addCase('content', 'any_merge', 'merge', 1, v1)
    addCase('content', 'any_merge', 'merge', 2, v2)
    const st1 = Y.mergeUpdates(v1); const st2 = Y.mergeUpdatesV2(v2)
    addCase('content', 'any_sv', 'sv', 1, [st1])
    addCase('content', 'any_sv', 'sv', 2, [st2])
    for (let cut = 0; cut < 60; cut += 7) {
      const sve = E.create(); E.vu(sve, 1); E.vu(sve, 77); E.vu(sve, cut)
      addCase('content', 'any_diff_' + cut, 'diff', 1, [st1], E.toU8(sve))
      addCase('content', 'any_diff_' + cut, 'diff', 2, [st2], E.toU8(sve))
    }
    for (let seed = 1; seed <= 6; seed++) {
      const t = genText(300 + seed, 3, 60, { unicode: true, rich: true, embed: true, clientIds: [3, 1, 2] })
      addCase('content', 'unicode_rich_' + seed, 'merge', 1, t.v1)
      addCase('content', 'unicode_rich_' + seed, 'merge', 2, t.v2)
      const s1 = Y.mergeUpdates(t.v1); const s2 = Y.mergeUpdatesV2(t.v2)
      const r = rng(seed)
      for (let k = 0; k < 6; k++) {
        const sve = E.create(); E.vu(sve, 3)
        for (const c of [3, 1, 2]) { E.vu(sve, c); E.vu(sve, r.int(0, 60)) }
        addCase('content', `unicode_rich_${seed}_diff${k}`, 'diff', 1, [s1], E.toU8(sve))
        addCase('content', `unicode_rich_${seed}_diff${k}`, 'diff', 2, [s2], E.toU8(sve))
      }
    }
  }
  // ---------------- reference golden vectors (tests/compatibility.tests.js:16-46, V1) -------------
  {
    const src = fs.readFileSync('/root/reference/tests/compatibility.tests.js', 'utf8')
    const blobs = [...src.matchAll(/const oldDoc = '([A-Za-z0-9+/=]+)'/g)].map(m => Uint8Array.from(Buffer.from(m[1], 'base64')))
    blobs.forEach((u, i) => {
      addCase('refgolden', 'ref' + i + '_identity', 'merge', 1, [u])
      addCase('refgolden', 'ref' + i + '_self', 'merge', 1, [u, u])
      addCase('refgolden', 'ref' + i + '_sv', 'sv', 1, [u])
      addCase('refgolden', 'ref' + i + '_diff0', 'diff', 1, [u], Uint8Array.of(0))
      const sv = Y.encodeStateVectorFromUpdate(u)
      addCase('refgolden', 'ref' + i + '_diffsv', 'diff', 1, [u], sv)
      // half-state diffs per client
      const dec = load(64485); const d = dec.l1(sv); const n = dec.yg(d); const e2 = E.create(); E.vu(e2, n)
      for (let j = 0; j < n; j++) { const c = dec.yg(d); const k = dec.yg(d); E.vu(e2, c); E.vu(e2, Math.floor(k / 2)) }
      addCase('refgolden', 'ref' + i + '_diffhalf', 'diff', 1, [u], E.toU8(e2))
      // V2 re-encoding of the same state via a Doc round trip in 13.5.16 (decode-compatible path)
      const doc = new Y.Doc(); Y.applyUpdate(doc, u)
      const u2 = Y.encodeStateAsUpdateV2(doc)
      addCase('refgolden', 'ref' + i + '_v2_self', 'merge', 2, [u2, u2])
      addCase('refgolden', 'ref' + i + '_v2_diffhalf', 'diff', 2, [u2], E.toU8(e2))
    })
  }
  // ---------------- edge cases (SURVEY.md §8c) ----------------
  {
    const t = genText(4242, 2, 30, { clientIds: [10, 20] })
    const [a, b, c, d] = t.v1
    addCase('edge', 'single_identity', 'merge', 1, [a])
    addCase('edge', 'single_identity', 'merge', 2, [t.v2[0]])
    addCase('edge', 'empty_list_v1', 'merge', 1, [])
    addCase('edge', 'duplicate_pair', 'merge', 1, [a, a])
    addCase('edge', 'duplicate_pair', 'merge', 2, [t.v2[0], t.v2[0]])
    const full1 = Y.mergeUpdates(t.v1); const full2 = Y.mergeUpdatesV2(t.v2)
    addCase('edge', 'full_then_incr', 'merge', 1, [full1, ...t.v1.slice(0, 10)])
    addCase('edge', 'incr_then_full', 'merge', 1, [...t.v1.slice(0, 10), full1])
    addCase('edge', 'full_then_incr', 'merge', 2, [full2, ...t.v2.slice(0, 10)])
    addCase('edge', 'incr_then_full', 'merge', 2, [...t.v2.slice(0, 10), full2])
    addCase('edge', 'overlap_halves', 'merge', 1, [Y.mergeUpdates(t.v1.slice(0, 20)), Y.mergeUpdates(t.v1.slice(10))])
    addCase('edge', 'overlap_halves', 'merge', 2, [Y.mergeUpdatesV2(t.v2.slice(0, 20)), Y.mergeUpdatesV2(t.v2.slice(10))])
    // gapped inputs -> Skip structs; then merging an output that holds a Skip
    const gapped1 = addCase('edge', 'gapped', 'merge', 1, [a, c, d])
    addCase('edge', 'gapped', 'merge', 2, [t.v2[0], t.v2[2], t.v2[3]])
    const ev = t.v1.filter((_, i) => i % 3 !== 1)
    const gm = Y.mergeUpdates(ev)
    addCase('edge', 'gapped_many', 'merge', 1, ev)
    addCase('edge', 'merge_with_skip_input', 'merge', 1, [gm, ...t.v1.filter((_, i) => i % 3 === 1)])
    addCase('edge', 'sv_of_skip', 'sv', 1, [gm])
    addCase('edge', 'diff_of_skip', 'diff', 1, [gm], Uint8Array.of(0))
    const ev2 = t.v2.filter((_, i) => i % 3 !== 1)
    const gm2 = Y.mergeUpdatesV2(ev2)
    addCase('edge', 'merge_with_skip_input', 'merge', 2, [gm2, ...t.v2.filter((_, i) => i % 3 === 1)])
    addCase('edge', 'sv_of_skip', 'sv', 2, [gm2])
    addCase('edge', 'diff_of_skip', 'diff', 2, [gm2], Uint8Array.of(0))
    void gapped1; void b
    // empty updates and DS-only updates
    const emptyV1 = Uint8Array.of(0, 0)
    const dsOnly = buildV1(e => { E.vu(e, 0); E.vu(e, 2); E.vu(e, 10); E.vu(e, 2); E.vu(e, 0); E.vu(e, 3); E.vu(e, 5); E.vu(e, 2); E.vu(e, 20); E.vu(e, 1); E.vu(e, 4); E.vu(e, 1) })
    const dsOnly2 = buildV1(e => { E.vu(e, 0); E.vu(e, 2); E.vu(e, 20); E.vu(e, 1); E.vu(e, 0); E.vu(e, 4); E.vu(e, 10); E.vu(e, 1); E.vu(e, 2); E.vu(e, 9) })
    addCase('edge', 'empty_pair', 'merge', 1, [emptyV1, emptyV1])
    addCase('edge', 'empty_sv', 'sv', 1, [emptyV1])
    addCase('edge', 'empty_diff', 'diff', 1, [emptyV1], Uint8Array.of(0))
    addCase('edge', 'ds_only_union', 'merge', 1, [dsOnly, dsOnly2, a])
    addCase('edge', 'ds_only_diff', 'diff', 1, [dsOnly], Uint8Array.of(0))
    const emptyV2 = Y.mergeUpdatesV2([Y.encodeStateAsUpdateV2(new Y.Doc()), Y.encodeStateAsUpdateV2(new Y.Doc())])
    addCase('edge', 'empty_pair', 'merge', 2, [emptyV2, emptyV2])
    addCase('edge', 'empty_sv', 'sv', 2, [emptyV2])
    // map overwrite (0x20 quirk), both formats, merge + diff(empty SV)
    const mo = genMap(77, 3, 40, 2)
    addCase('edge', 'map_overwrite', 'merge', 1, mo.v1)
    addCase('edge', 'map_overwrite', 'merge', 2, mo.v2)
    for (let i = 0; i < 6; i++) {
      addCase('edge', 'map_overwrite_diff_empty_' + i, 'diff', 1, [mo.v1[i * 5]], Uint8Array.of(0))
      addCase('edge', 'map_overwrite_diff_empty_' + i, 'diff', 2, [mo.v2[i * 5]], Uint8Array.of(0))
    }
    // surrogate slicing: diff cut inside a surrogate pair throws URIError; merge of overlapping slices
    const sd = new Y.Doc(); sd.clientID = 9; const s1 = []; const s2 = []; capture(sd, s1, s2)
    sd.getText('t').insert(0, 'a😀b😀')
    sd.getText('t').insert(0, 'xyz')
    const ssv = c => { const e = E.create(); E.vu(e, 1); E.vu(e, 9); E.vu(e, c); return E.toU8(e) }
    for (let cut = 0; cut <= 6; cut++) {
      addCase('edge', 'surrogate_diff_' + cut, 'diff', 1, [s1[0]], ssv(cut))
      addCase('edge', 'surrogate_diff_' + cut, 'diff', 2, [s2[0]], ssv(cut))
    }
    // GC structs (hand-built V1, SURVEY E12)
    const gc = (client, parts) => buildV1(e => {
      E.vu(e, 1); E.vu(e, parts.length); E.vu(e, client); E.vu(e, parts[0][0])
      for (const [, len] of parts) { E.u8(e, 0); E.vu(e, len) }
      E.vu(e, 0)
    })
    const U1 = gc(5, [[0, 5]]); const U2 = gc(5, [[5, 2], [7, 2]]); const U3 = gc(9, [[0, 1]]); const U4 = gc(5, [[9, 3], [12, 1]])
    addCase('edge', 'gc_u1u2', 'merge', 1, [U1, U2])
    addCase('edge', 'gc_u2u3', 'merge', 1, [U2, U3])
    addCase('edge', 'gc_u2u4', 'merge', 1, [U2, U4])
    addCase('edge', 'gc_u1u2u4', 'merge', 1, [U1, U2, U4])
    addCase('edge', 'gc_u4u1u2u3', 'merge', 1, [U4, U1, U2, U3])
    addCase('edge', 'gc_overlap', 'merge', 1, [gc(5, [[0, 8]]), gc(5, [[3, 7]])])
    addCase('edge', 'gc_diff', 'diff', 1, [U2], ssv(6))
    // non-canonical varints (E21): clock 80 00, string length 82 00
    const over = hexBytes('01 01 05 80 00 04 00 01 74 82 00 68 69 00')
    addCase('edge', 'overlong_varint_diff', 'diff', 1, [over], Uint8Array.of(0))
    addCase('edge', 'overlong_varint_merge', 'merge', 1, [over, a])
    addCase('edge', 'overlong_varint_sv', 'sv', 1, [over])
    // malformed utf-8, unknown content ref, truncations
    const badUtf = hexBytes('01 01 05 00 04 00 01 74 03 ed a0 80 00')
    addCase('edge', 'bad_utf8_merge', 'merge', 1, [badUtf, a])
    addCase('edge', 'bad_utf8_diff', 'diff', 1, [badUtf], Uint8Array.of(0))
    addCase('edge', 'bad_utf8_sv', 'sv', 1, [badUtf])
    const ref11 = hexBytes('01 01 05 00 0b 01 01 74 00')
    addCase('edge', 'ref11_merge', 'merge', 1, [ref11, a])
    addCase('edge', 'ref11_sv', 'sv', 1, [ref11])
    const ref10 = hexBytes('01 01 05 00 0a 03 00')
    addCase('edge', 'skip_input_merge', 'merge', 1, [ref10, a])
    addCase('edge', 'skip_input_sv', 'sv', 1, [ref10])
    const full = t.v1[5]
    for (const cut of [1, 3, 8, full.length - 2, full.length - 1]) {
      if (cut <= 0 || cut >= full.length) continue
      const tr = full.slice(0, cut)
      addCase('edge', 'trunc_' + cut + '_merge', 'merge', 1, [tr, a])
      addCase('edge', 'trunc_' + cut + '_sv', 'sv', 1, [tr])
      addCase('edge', 'trunc_' + cut + '_diff', 'diff', 1, [tr], Uint8Array.of(0))
    }
    // legacy ContentJSON (ref 2) and embeds with V1 JSON text; JSON canonicalisation
    const jsonItem = (client, strs) => buildV1(e => {
      E.vu(e, 1); E.vu(e, 1); E.vu(e, client); E.vu(e, 0)
      E.u8(e, 2); E.vu(e, 1); E.vs(e, 'arr'); E.vu(e, strs.length); for (const s of strs) E.vs(e, s)
      E.vu(e, 0)
    })
    const j1 = jsonItem(3, ['1', '"two"', 'undefined', '{"b":1,"a":[true,null]}', ' 2 ', '1.50', '{"2":1,"1":2,"x":0}', '-0', '1e21', '"\\u0041\\n"'])
    addCase('edge', 'json_merge', 'merge', 1, [j1, a])
    for (let cut = 0; cut <= 10; cut += 3) addCase('edge', 'json_diff_' + cut, 'diff', 1, [j1], ssv(cut).map((x, i) => i === 1 ? 3 : x))
    // key-cache use in a V2 XmlElement name (keyClock < keys.length) -- hand-built would need a V2 writer;
    // covered by C5 fixtures where every key is written.
  }

  fs.mkdirSync(OUT, { recursive: true })
  let total = 0
  for (const [g, list] of Object.entries(cases)) {
    const file = path.join(OUT, g + '.json')
    const s = JSON.stringify({ generator: 'oracle/gen/make_fixtures.cjs', oracle: 'yjs 13.5.16 (JupyterLab bundle 3502.fbe0c610be82ba1360db.js) + lib0 0.2.42', cases: list })
    fs.writeFileSync(file, s)
    total += s.length
    console.log(g, list.length, 'cases', s.length, 'bytes')
  }
  console.log('total bytes', total)
}

main()
