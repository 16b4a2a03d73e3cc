// P-ref fixtures (SURVEY.md §0): agreement of the engine's outputs with gaberogan/yjs@v0 ITSELF (yjs
// 13.4.9, /root/reference/src run by ref_yjs.cjs), test infrastructure, container-only.
//
// The byte contract (P-bytes) is yjs 13.5.16's mergeUpdates / encodeStateVectorFromUpdate, which the
// reference predates; the golden vectors pin the engine to those bytes.  This script checks those very
// bytes against the reference's own Doc round trip, per golden merge / state-vector case:
//   P-ref-1  the struct section of canonNoGc(merged) equals that of canonNoGc applied to the inputs in
//            order, canonNoGc(x) = encodeStateAsUpdate[V2](applyUpdate[V2](new Doc({gc: false}), x))
//            (encoding.js:462-526) -- byte for byte, or unit for unit (one entry per clock: the reference
//            splits and re-merges Items depending on its transaction boundaries, and replaces a split
//            surrogate half by U+FFFD only where it happened to split);
//   P-ref-2  the clock coverage of readDeleteSet(merged) equals that of
//            mergeDeleteSets(inputs.map(readDeleteSet)) (DeleteSet.js:141-161, 241-256);
//   P-ref-3  merged applies to a fresh Doc with no pending structs or delete readers (StructStore.js:25-35);
//   P-ref-sv encodeStateVectorFromUpdate(u) equals, as a map, the reference's encodeStateVector of the
//            Doc u builds (encoding.js:587-611), when u applies completely.
//   P-ref-diff diffUpdate(u, sv) carries, unit for unit, the structs of the reference's
//            encodeStateAsUpdate(Doc(u), sv) (encoding.js:490-526: writeClientsStructs slices every client at
//            sv[client], :94-116), both decoded with the reference's readClientsStructRefs; and the same
//            delete-set coverage as the reference's (createDeleteSetFromStructStore), when u applies completely.
// Cases the reference cannot evaluate are recorded with the reason (e.g. Skip structs -- 13.5.16 output
// for gapped inputs, which 13.4.9 cannot decode, SURVEY.md F9).  Output: tests/pref/pref.json with, per
// case, the golden id, the sha256 of the bytes that were checked (the golden expectation = the engine's
// output) and the verdicts.  Usage: node make_pref_fixtures.cjs
'use strict'
const fs = require('fs')
const path = require('path')
const crypto = require('crypto')
const { loadReference } = require('./ref_yjs.cjs')
const { load } = require('./yjs_bundle.cjs')
const decoding = load(64485)

const GOLDEN = path.join(__dirname, '../../tests/golden')
const OUT = path.join(__dirname, '../../tests/pref')
const sha = u8 => crypto.createHash('sha256').update(Buffer.from(u8)).digest('hex')
const u8 = b64 => new Uint8Array(Buffer.from(b64, 'base64'))

// the store as a list of units (one per clock): splitting and merging of Items are invisible at this
// granularity, deletion is left to P-ref-2 (the reference's own YText formatting cleanup deletes
// format items depending on transaction boundaries, SURVEY.md E16)
function units (Y, doc) {
  const out = []
  const idOf = id => id ? [id.client, id.clock] : null
  const parentOf = it => {
    const p = it.parent
    if (p === null || p === undefined) return null
    if (p._item) return ['item', p._item.id.client, p._item.id.clock]
    if (p.constructor === Y.ID) return ['id', p.client, p.clock]
    if (typeof p === 'string') return ['key', p]
    for (const [k, v] of doc.share) if (v === p) return ['root', k]
    return ['?']
  }
  const clients = [...doc.store.clients.keys()].sort((a, b) => a - b)
  for (const client of clients) {
    for (const s of doc.store.clients.get(client)) {
      if (s.constructor === Y.GC) { for (let i = 0; i < s.length; i++) out.push([client, s.id.clock + i, 'GC']); continue }
      const ct = s.content
      let vals = null
      try { vals = ct.getContent() } catch (e) { vals = null }
      for (let i = 0; i < s.length; i++) {
        let v = vals && vals.length === s.length ? vals[i] : null
        if (ct.constructor === Y.ContentFormat) v = [ct.key, ct.value]
        if (ct.constructor === Y.ContentType) v = [ct.type.constructor.name, ct.type.nodeName || ct.type.hookName || null]
        if (v && typeof v === 'object' && v.constructor && v.constructor.name !== 'Object' && v.constructor.name !== 'Array' &&
            !(v instanceof Uint8Array)) v = v.constructor.name
        if (v instanceof Uint8Array) v = Array.from(v)
        // a split surrogate pair: ContentString.splice writes U+FFFD for either half (ContentString.js:55-64),
        // but only when the reference happens to split the Item there, which depends on transaction
        // boundaries -- both spellings are the same unit here
        if (typeof v === 'string' && v.length === 1 && (v === '\ufffd' || (v.charCodeAt(0) >= 0xd800 && v.charCodeAt(0) <= 0xdfff))) v = '<surrogate half or U+FFFD>'
        out.push([client, s.id.clock + i, ct.constructor.name, i === 0 ? idOf(s.origin) : [client, s.id.clock + i - 1],
          idOf(s.rightOrigin), parentOf(s), s.parentSub, v === undefined ? '<undefined>' : v])
      }
    }
  }
  return JSON.stringify(out, (k, v) => typeof v === 'bigint' ? 'bigint:' + v.toString() : v)
}

// the structs of an update as units, decoded by the reference's own reader (no integration: a diff misses
// the structs its receiver already has)
function updateUnits (Y, bytes, v2) {
  const UDec = v2 ? Y.UpdateDecoderV2 : Y.UpdateDecoderV1
  const doc = new Y.Doc()
  const refs = Y.readClientsStructRefs(new UDec(decoding.l1(bytes)), new Map(), doc)
  const out = []
  const idOf = id => id ? [id.client, id.clock] : null
  const parentOf = it => {
    const p = it.parent
    if (p === null || p === undefined) return null
    if (p.constructor === Y.ID) return ['id', p.client, p.clock]
    for (const [k, v] of doc.share) if (v === p) return ['root', k]
    return ['?']
  }
  for (const client of [...refs.keys()].sort((a, b) => a - b)) {
    for (const s of refs.get(client)) {
      if (s.constructor === Y.GC) { for (let i = 0; i < s.length; i++) out.push([client, s.id.clock + i, 'GC']); continue }
      const ct = s.content
      let vals = null
      try { vals = ct.getContent() } catch (e) { vals = null }
      for (let i = 0; i < s.length; i++) {
        let v = vals && vals.length === s.length ? vals[i] : null
        if (ct.constructor === Y.ContentFormat) v = [ct.key, ct.value]
        if (ct.constructor === Y.ContentType) v = [ct.type.constructor.name, ct.type.nodeName || ct.type.hookName || null]
        if (v && typeof v === 'object' && v.constructor && v.constructor.name !== 'Object' && v.constructor.name !== 'Array' &&
            !(v instanceof Uint8Array)) v = v.constructor.name
        if (v instanceof Uint8Array) v = Array.from(v)
        if (typeof v === 'string' && v.length === 1 && (v === '\ufffd' || (v.charCodeAt(0) >= 0xd800 && v.charCodeAt(0) <= 0xdfff))) v = '<surrogate half or U+FFFD>'
        out.push([client, s.id.clock + i, ct.constructor.name, i === 0 ? idOf(s.origin) : [client, s.id.clock + i - 1],
          idOf(s.rightOrigin), i === 0 ? parentOf(s) : null, i === 0 ? s.parentSub : null, v === undefined ? '<undefined>' : v])
      }
    }
  }
  return JSON.stringify(out, (k, v) => typeof v === 'bigint' ? 'bigint:' + v.toString() : v)
}

function covSubset (a, b) { // every [start, end) of coverage a lies inside one of b's (both merged, sorted)
  const m = new Map(b)
  return a.every(([client, iv]) => iv.every(([s, e]) => (m.get(client) || []).some(([s2, e2]) => s2 <= s && e <= e2)))
}

function coverage (ds) { // DeleteSet -> {client: [[start, end], ...]} (union of the ranges)
  const out = {}
  for (const [client, items] of ds.clients) {
    const iv = items.filter(d => d.len > 0).map(d => [d.clock, d.clock + d.len]).sort((a, b) => a[0] - b[0])
    const m = []
    for (const [s, e] of iv) { if (m.length && s <= m[m.length - 1][1]) m[m.length - 1][1] = Math.max(m[m.length - 1][1], e); else m.push([s, e]) }
    if (m.length) out[client] = m
  }
  return JSON.stringify(Object.keys(out).sort((a, b) => a - b).map(k => [+k, out[k]]))
}

;(async () => {
  const Y = await loadReference()
  const cases = []
  const stats = {}
  for (const f of fs.readdirSync(GOLDEN).filter(f => f.endsWith('.json')).sort()) {
    const g = path.basename(f, '.json')
    for (const c of JSON.parse(fs.readFileSync(path.join(GOLDEN, f))).cases) {
      if (!c.expect || (c.op !== 'merge' && c.op !== 'sv' && c.op !== 'diff')) continue
      const id = `${g}/${c.name}/v${c.fmt}/${c.op}`
      const v2 = c.fmt === 2
      const apply = v2 ? Y.applyUpdateV2 : Y.applyUpdate
      const encode = v2 ? Y.encodeStateAsUpdateV2 : Y.encodeStateAsUpdate
      const UDec = v2 ? Y.UpdateDecoderV2 : Y.UpdateDecoderV1
      const DSEnc = v2 ? Y.DSEncoderV2 : Y.DSEncoderV1
      const inputs = c.inputs.map(u8)
      const out = u8(c.expect)
      const r = { id, op: c.op, fmt: c.fmt, checked_sha256: sha(out) }
      const structPart = doc => {
        const full = encode(doc)
        const e = new DSEnc()
        Y.writeDeleteSet(e, Y.createDeleteSetFromStructStore(doc.store))
        const ds = e.toUint8Array()
        if (Buffer.compare(Buffer.from(full.slice(full.length - ds.length)), Buffer.from(ds)) !== 0) throw new Error('delete set is not the suffix')
        return full.slice(0, full.length - ds.length)
      }
      const pending = doc => doc.store.pendingClientsStructRefs.size + doc.store.pendingStack.length + doc.store.pendingDeleteReaders.length
      try {
        if (c.op === 'merge') {
          const seq = new Y.Doc({ gc: false })
          for (const u of inputs) apply(seq, u)
          const eng = new Y.Doc({ gc: false })
          apply(eng, out)
          r.pref3 = pending(eng) === 0
          const sa = structPart(seq); const sb = structPart(eng)
          r.pref1_bytes = Buffer.compare(Buffer.from(sa), Buffer.from(sb)) === 0
          const ua = units(Y, seq); const ub = units(Y, eng)
          r.pref1 = r.pref1_bytes || ua === ub
          if (!r.pref1 && process.env.PREF_DEBUG) {
            const A = JSON.parse(ua); const B = JSON.parse(ub)
            for (let i = 0; i < Math.max(A.length, B.length); i++) if (JSON.stringify(A[i]) !== JSON.stringify(B[i])) { console.log(id, i, JSON.stringify(A[i]), JSON.stringify(B[i])); break }
          }
          r.units_sha256 = sha(Buffer.from(ub))
          r.struct_sha256 = sha(sb)
          const readDs = u => { const d = new UDec(decoding.l1(u)); Y.readClientsStructRefs(d, new Map(), new Y.Doc()); return Y.readDeleteSet(d) }
          const covEng = coverage(readDs(out))
          const covIn = coverage(Y.mergeDeleteSets(inputs.map(readDs)))
          r.pref2 = covEng === covIn
          r.ds_coverage = covEng
          if (pending(seq) !== 0) { r.applicable = false; r.reason = 'the inputs leave pending structs in the reference' } else if (g === 'ties') {
            r.applicable = false
            r.reason = 'inputs of inconsistent histories (a GC and a live Item for the same ID): the Doc keeps whichever it integrates first'
          } else r.applicable = true
        } else if (c.op === 'diff') {
          const doc = new Y.Doc({ gc: false })
          apply(doc, inputs[0])
          const sv = u8(c.sv)
          const ref = encode(doc, sv)
          const ua = updateUnits(Y, ref, v2); const ub = updateUnits(Y, out, v2)
          r.pref_diff = ua === ub
          if (!r.pref_diff && process.env.PREF_DEBUG) {
            const A = JSON.parse(ua); const B = JSON.parse(ub)
            for (let i = 0; i < Math.max(A.length, B.length); i++) if (JSON.stringify(A[i]) !== JSON.stringify(B[i])) { console.log(id, i, JSON.stringify(A[i]), JSON.stringify(B[i])); break }
          }
          r.units_sha256 = sha(Buffer.from(ub))
          const readDs = u => { const d = new UDec(decoding.l1(u)); Y.readClientsStructRefs(d, new Map(), new Y.Doc()); return Y.readDeleteSet(d) }
          // the lazy diff keeps the input's delete set (P-ref-2 for a single input); the reference's Doc
          // additionally marks what integration deletes (children of deleted types, overwritten map entries:
          // Item.js:403-517), so its set must contain the engine's
          r.ds_coverage = coverage(readDs(out))
          r.pref_diff_ds = r.ds_coverage === coverage(readDs(inputs[0]))
          r.pref_diff_ds_in_ref = covSubset(JSON.parse(r.ds_coverage), JSON.parse(coverage(readDs(ref))))
          r.applicable = pending(doc) === 0
          if (!r.applicable) r.reason = 'the update leaves pending structs or delete ranges in the reference (gaps)'
        } else {
          const doc = new Y.Doc({ gc: false })
          apply(doc, inputs[0])
          const want = Y.decodeStateVector(Y.encodeStateVector(doc))
          const got = Y.decodeStateVector(out)
          const eq = want.size === got.size && [...want].every(([k, v]) => got.get(k) === v)
          r.pref_sv = eq
          r.applicable = pending(doc) === 0
          if (!r.applicable) r.reason = 'the update leaves pending structs in the reference (gaps)'
        }
      } catch (e) {
        r.applicable = false
        r.reason = 'reference throws: ' + e.constructor.name + ': ' + e.message
      }
      const key = `${g}/${c.op}/${r.applicable ? 'applicable' : 'not applicable'}`
      stats[key] = (stats[key] || 0) + 1
      const ok = r.applicable && (c.op === 'merge' ? r.pref1 && r.pref2 && r.pref3 : c.op === 'diff' ? r.pref_diff && r.pref_diff_ds && r.pref_diff_ds_in_ref : r.pref_sv)
      if (r.applicable && !ok) stats[`${g}/${c.op}/FAILED`] = (stats[`${g}/${c.op}/FAILED`] || 0) + 1
      cases.push(r)
    }
  }
  fs.mkdirSync(OUT, { recursive: true })
  fs.writeFileSync(path.join(OUT, 'pref.json'), JSON.stringify({
    generator: 'oracle/gen/make_pref_fixtures.cjs',
    reference: 'gaberogan/yjs@v0 (yjs 13.4.9, /root/reference/src) under Node 12 ESM with a lib0 shim over the bundled lib0 0.2.42 (oracle/gen/ref_yjs.cjs)',
    stats,
    cases
  }, null, 0))
  console.log(JSON.stringify(stats, null, 1))
})().catch(e => { console.error(e); process.exit(1) })
