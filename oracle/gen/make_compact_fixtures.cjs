// Doc round-trip compaction fixtures (SURVEY.md §8(f) row 1), test infrastructure, container-only: the
// reference's own compaction -- gaberogan/yjs@v0 (yjs 13.4.9, /root/reference/src via ref_yjs.cjs):
// every update applied to a default Doc (gc: true, Doc.js:40) in order, one transaction each
// (applyUpdate[V2], encoding.js:462-473: resumeStructIntegration :225-321 -> Item.integrate Item.js:403-517,
// readAndApplyDeleteSet DeleteSet.js:270-323; cleanupTransactions Transaction.js:244-367: tryGcDeleteSet,
// tryMergeDeleteSet, tryToMergeWithLeft), then encodeStateAsUpdate[V2] (encoding.js:490-526).
// Inputs: every golden merge case, per workload template set (C1-C5) the first documents' update lists,
// randomized formatted-text histories, and gapped histories (updates dropped: the reference keeps what
// they would have enabled in pendingStack / pendingClientsStructRefs / pendingDeleteReaders and
// encodeStateAsUpdate writes only the integrated store, encoding.js:490-493).  Output:
// tests/golden/compact.json {cases: [{id, group, fmt, inputs (b64), expect (b64) | src {ymb, doc, drop?},
// expect_sha256, expect_len | error {name, message}; pending [structRefs, stack, deleteReaders];
// single_tx_same, sv (encodeStateVector(doc))}]}.  A case whose applyUpdate / encodeStateAsUpdate throws records the exception's class
// and message instead of bytes.  single_tx_same records whether applying mergeUpdates(inputs) in one
// transaction gives the same bytes.
'use strict'
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const { loadReference } = require('./ref_yjs.cjs')
const { Y: Y13 } = require('./yjs_bundle.cjs')

const GOLDEN = path.join(__dirname, '../../tests/golden')
const u8 = b64 => new Uint8Array(Buffer.from(b64, 'base64'))
const b64 = u => Buffer.from(u).toString('base64')

function loadYmb (name) {
  const b = zlib.gunzipSync(fs.readFileSync(path.join(__dirname, '../../bench_data', name + '.ymb.gz')))
  const nd = b.readUInt32LE(4); const nu = b.readUInt32LE(8)
  let o = 12
  const docUpd = []; for (let i = 0; i <= nd; i++) { docUpd.push(b.readUInt32LE(o)); o += 4 }
  const off = []; for (let i = 0; i <= nu; i++) { off.push(Number(b.readBigUInt64LE(o))); o += 8 }
  const arena = b.subarray(o)
  const docs = []
  for (let d = 0; d < nd; d++) {
    const ups = []
    for (let u = docUpd[d]; u < docUpd[d + 1]; u++) ups.push(new Uint8Array(arena.subarray(off[u], off[u + 1])))
    docs.push(ups)
  }
  return docs
}

;(async () => {
  const Y = await loadReference()
  const pending = doc => [doc.store.pendingClientsStructRefs.size, doc.store.pendingStack.length, doc.store.pendingDeleteReaders.length]
  const cases = []
  const stats = {}
  const add = (id, group, fmt, inputs, src) => {
    const v2 = +fmt === 2
    const apply = v2 ? Y.applyUpdateV2 : Y.applyUpdate
    const encode = v2 ? Y.encodeStateAsUpdateV2 : Y.encodeStateAsUpdate
    const r = src ? { id, group, fmt: v2 ? 2 : 1, src } : { id, group, fmt: v2 ? 2 : 1, inputs: inputs.map(b64) }
    try {
      const doc = new Y.Doc()
      for (const u of inputs) apply(doc, u)
      const pend = pending(doc)
      const out = encode(doc)
      if (pend[0] + pend[1] + pend[2] !== 0) {
        r.pending = pend
        stats[group + '/pending'] = (stats[group + '/pending'] || 0) + 1
      }
      let same = null
      if (!r.pending) {
        try {
          const one = new Y.Doc()
          apply(one, inputs.length === 1 ? inputs[0] : (v2 ? Y13.mergeUpdatesV2 : Y13.mergeUpdates)(inputs))
          same = Buffer.compare(Buffer.from(encode(one)), Buffer.from(out)) === 0
        } catch (e) { same = null }
      }
      // workload documents name their bench_data source instead of repeating its bytes
      // (and, being large, carry the SHA-256 and length of the expected bytes)
      if (src) { r.expect_sha256 = require('crypto').createHash('sha256').update(out).digest('hex'); r.expect_len = out.length } else r.expect = b64(out)
      // the Doc's own state vector (encoding.js:572-611: clients in StructStore insertion order)
      r.sv = b64(Y.encodeStateVector(doc))
      r.single_tx_same = same
    } catch (e) {
      // the reference's exception (applyUpdate's transaction still runs its cleanup in `finally`)
      r.error = { name: e.constructor.name, message: e.message }
      stats[group + '/throws'] = (stats[group + '/throws'] || 0) + 1
    }
    cases.push(r)
    stats[group] = (stats[group] || 0) + 1
    if (r.single_tx_same === false) stats[group + '/single_tx_differs'] = (stats[group + '/single_tx_differs'] || 0) + 1
  }
  for (const f of fs.readdirSync(GOLDEN).filter(f => f.endsWith('.json') && f !== 'compact.json').sort()) {
    const g = path.basename(f, '.json')
    if (g === 'ties') continue  // inconsistent histories (a GC and an Item for one ID): order-dependent by design
    for (const c of JSON.parse(fs.readFileSync(path.join(GOLDEN, f))).cases) {
      if (c.op !== 'merge' || !c.expect || !c.inputs || c.inputs.length === 0) continue
      add(`${g}/${c.name}/v${c.fmt}`, g, c.fmt, c.inputs.map(u8))
    }
  }
  for (const [wl, n] of [['c1_v1', 1], ['c1_v2', 1], ['c2_v1', 24], ['c2_v2', 24], ['c4_v1', 12], ['c4_v2', 12]]) {
    const docs = loadYmb(wl)
    for (let d = 0; d < n && d < docs.length; d++) add(`wl_${wl}/doc${d}`, 'wl_' + wl.slice(0, 2), wl.endsWith('v2') ? 2 : 1, docs[d], { ymb: wl, doc: d })
  }
  // the workloads with formatted text (C5: nested Y.XmlText) and their bigger documents (C3)
  for (const [wl, n] of [['c3_v1', 3], ['c3_v2', 3], ['c5_v1', 4], ['c5_v2', 4]]) {
    const docs = loadYmb(wl)
    for (let d = 0; d < n && d < docs.length; d++) add(`wl_${wl}/doc${d}`, 'wl_' + wl.slice(0, 2), wl.endsWith('v2') ? 2 : 1, docs[d], { ymb: wl, doc: d })
  }
  // gapped histories: every 5th update of the workload documents dropped (the lost messages of a provider);
  // what depends on them stays pending in the reference's store
  for (const [wl, n] of [['c2_v1', 24], ['c2_v2', 24], ['c4_v1', 8], ['c4_v2', 8], ['c5_v1', 2], ['c5_v2', 2]]) {
    const docs = loadYmb(wl)
    for (let d = 0; d < n && d < docs.length; d++) add(`gap_${wl}/doc${d}`, 'gap_' + wl.slice(0, 2), wl.endsWith('v2') ? 2 : 1, docs[d].filter((u, i) => i % 5 !== 4), { ymb: wl, doc: d, drop: 5 })
  }
  const histories = []
  // randomized concurrent histories over nested Y.Text / Y.XmlText with formatting, deletes of whole nested
  // types, map overwrites and embeds, produced by yjs 13.5.16 peers; every peer's update events are applied to
  // the compacting Doc in a shuffled order that keeps each peer's own order (the YText observer's remote
  // formatting cleanup, ContentType.gc and the nested cleanup transaction all run)
  let seed = 0x5eed
  const rnd = () => { seed = (seed + 0x6D2B79F5) | 0; let t = seed; t = Math.imul(t ^ (t >>> 15), t | 1); t ^= t + Math.imul(t ^ (t >>> 7), t | 61); return ((t ^ (t >>> 14)) >>> 0) / 4294967296 }
  const ri = (a, b) => a + Math.floor(rnd() * (b - a + 1))
  const pick = a => a[Math.floor(rnd() * a.length)]
  const words = ['a', 'bc', 'def', 'gh ', 'ij\n', 'klmno', '\u00e9t\u00e9', '\ud83d\ude00x']
  const attrsOf = () => pick([{}, { bold: true }, { italic: true }, { bold: null }, { bold: true, italic: true }, { color: 'red' }, { color: '#00f' }, { bold: false }, { size: 0 }, { link: { href: 'x' } }])
  for (let h = 0; h < 160; h++) {
    const npeers = ri(2, 4)
    const peers = []
    const msgs = []
    for (let p = 0; p < npeers; p++) {
      const doc = new Y13.Doc({ gc: rnd() < 0.7 })
      doc.clientID = 1000 + h * 8 + p
      const log = []
      const log2 = []
      doc.on('update', u => log.push(u))
      doc.on('updateV2', u => log2.push(u))
      peers.push({ doc, log, log2 })
    }
    const root = d => d.getMap('root')
    // peer 0 creates the structure
    peers[0].doc.transact(() => {
      const m = root(peers[0].doc)
      const t = new Y13.Text(); m.set('text', t); t.insert(0, 'hello world', { bold: true })
      const frag = new Y13.XmlFragment(); m.set('frag', frag)
      const el = new Y13.XmlElement('p'); frag.insert(0, [el])
      const xt = new Y13.XmlText(); el.insert(0, [xt]); xt.insert(0, 'xml text', { italic: true })
      const arr = new Y13.Array(); m.set('arr', arr)
      const t2 = new Y13.Text(); arr.insert(0, [t2, 'plain']); t2.insert(0, 'inner')
    })
    const sync = (a, b) => Y13.applyUpdate(b.doc, Y13.encodeStateAsUpdate(a.doc, Y13.encodeStateVector(b.doc)))
    for (let p = 1; p < npeers; p++) sync(peers[0], peers[p])
    const texts = d => {
      const m = root(d)
      const out = []
      for (const k of ['text']) if (m.get(k) instanceof Y13.Text) out.push(m.get(k))
      const frag = m.get('frag')
      if (frag instanceof Y13.XmlFragment) frag.toArray().forEach(el => { if (el instanceof Y13.XmlElement) el.toArray().forEach(x => { if (x instanceof Y13.XmlText) out.push(x) }) })
      const arr = m.get('arr')
      if (arr instanceof Y13.Array) arr.toArray().forEach(x => { if (x instanceof Y13.Text) out.push(x) })
      return out
    }
    const rounds = ri(2, 6)
    for (let r = 0; r < rounds; r++) {
      for (const pe of peers) {
        const ops = ri(1, 6)
        for (let o = 0; o < ops; o++) {
          const ts = texts(pe.doc)
          const op = rnd()
          if (ts.length > 0 && op < 0.75) {
            const t = pick(ts)
            const len = t.length
            const k = rnd()
            if (k < 0.35) t.insert(ri(0, len), pick(words), attrsOf())
            else if (k < 0.6 && len > 0) { const i = ri(0, len - 1); t.format(i, ri(1, len - i), attrsOf()) }
            else if (k < 0.8 && len > 0) { const i = ri(0, len - 1); t.delete(i, ri(1, Math.min(4, len - i))) }
            else if (k < 0.9) t.insertEmbed(ri(0, len), { img: pick(['a', 'b']) }, attrsOf())
            else t.insert(ri(0, len), pick(words))
          } else if (op < 0.85) {
            root(pe.doc).set(pick(['k1', 'k2']), pick([1, 'v', null, [1, 2], { a: 1 }]))
          } else if (op < 0.93) {
            const m = root(pe.doc)
            const frag = m.get('frag')
            if (frag instanceof Y13.XmlFragment && rnd() < 0.5) {
              const el = new Y13.XmlElement(pick(['p', 'h1'])); frag.insert(ri(0, frag.length), [el])
              const xt = new Y13.XmlText(); el.insert(0, [xt]); xt.insert(0, pick(words), attrsOf())
            } else if (frag instanceof Y13.XmlFragment && frag.length > 0) frag.delete(ri(0, frag.length - 1), 1)
          } else if (op < 0.97) {
            const arr = root(pe.doc).get('arr')
            if (arr instanceof Y13.Array && arr.length > 0 && rnd() < 0.5) arr.delete(ri(0, arr.length - 1), 1)
            else if (arr instanceof Y13.Array) { const t2 = new Y13.Text(); arr.insert(ri(0, arr.length), [t2]); t2.insert(0, pick(words), attrsOf()) }
          } else {
            const t = new Y13.Text(); root(pe.doc).set('text', t); t.insert(0, pick(words), attrsOf())
          }
        }
      }
      // partial sync: some pairs exchange their states
      for (let q = 0; q < npeers; q++) if (rnd() < 0.6) { const a = pick(peers), b = pick(peers); if (a !== b) sync(a, b) }
    }
    // every peer's own update events, interleaved in a random order that keeps each peer's order; drop the
    // updates that only relay what another peer produced (they come from syncs) -- keep them all: a relayed
    // update is exactly what a provider would hand the compacting Doc
    const v2 = h % 2 === 1
    const queues = peers.map(p => (v2 ? p.log2 : p.log).slice())
    while (queues.some(q => q.length > 0)) {
      const live = queues.filter(q => q.length > 0)
      const q = pick(live)
      const take = ri(1, Math.min(3, q.length))
      for (let i = 0; i < take; i++) msgs.push(q.shift())
    }
    add(`fuzz_fmt/h${h}/v${v2 ? 2 : 1}`, 'fuzz_fmt', v2 ? 2 : 1, msgs)
    histories.push([v2, msgs])
  }
  // the same histories with messages lost (each dropped with p = 0.15) and some delivered twice or late:
  // pending structs wait on the stack, deletes of unknown clocks wait as pending delete readers, and a
  // late message resumes them
  seed = 0x9a7
  for (let h = 0; h < histories.length; h++) {
    const [v2, msgs] = histories[h]
    const out = []
    const late = []
    for (const m of msgs) {
      const x = rnd()
      if (x < 0.15) continue
      if (x < 0.25) { late.push(m); continue }
      out.push(m)
      if (x > 0.95) out.push(m)
    }
    for (const m of late) if (rnd() < 0.5) out.push(m)
    add(`fuzz_gap/h${h}/v${v2 ? 2 : 1}`, 'fuzz_gap', v2 ? 2 : 1, out)
  }
  // V1 delete sets with zero-length ranges (readDsLen is a plain varuint in V1): one past the client's state
  // goes to the unapplied set, whose writeDeleteSet(DSEncoderV2) throws at it (UpdateEncoder.js:255-258); one
  // below the state only splits the item there; an error while reading a later client comes first
  {
    const vu = v => { const o = []; while (v > 127) { o.push(0x80 | (v & 127)); v = Math.floor(v / 128) } o.push(v); return o }
    const dsOnly = clients => { const o = [0, ...vu(clients.length)]; for (const [c, rs] of clients) { o.push(...vu(c), ...vu(rs.length)); for (const [k, l] of rs) o.push(...vu(k), ...vu(l)) } return new Uint8Array(o) }
    const src = new Y13.Doc()
    src.clientID = 1
    const log = []
    src.on('update', u => log.push(u))
    src.getText('t').insert(0, 'abcd')
    src.getText('t').insert(4, 'ef')
    const cs = [
      ['past_state', [...log, dsOnly([[1, [[9, 0]]]])]],
      ['unknown_client', [dsOnly([[77, [[0, 0]]]])]],
      ['below_state', [...log, dsOnly([[1, [[2, 0]]]])]],
      ['below_then_past', [...log, dsOnly([[1, [[1, 0], [7, 0]]]])]],
      ['mixed_ranges', [...log, dsOnly([[1, [[1, 2], [8, 0], [10, 3]]]])]],
      ['two_clients', [...log, dsOnly([[2, [[0, 0]]], [1, [[0, 2]]]])]],
      ['then_truncated', [...log, new Uint8Array([0, 2, 1, 1, 9, 0, 2, 1])]],
      ['pending_then_zero', [log[1], log[0], dsOnly([[1, [[3, 0]]]])]],
      ['zero_after_resume', [dsOnly([[1, [[5, 1]]]]), ...log, dsOnly([[1, [[1, 0]]]])]]
    ]
    for (const [name, inputs] of cs) add(`ds_zero/${name}/v1`, 'ds_zero', 1, inputs)
  }
  fs.writeFileSync(path.join(GOLDEN, 'compact.json'), JSON.stringify({
    generator: 'oracle/gen/make_compact_fixtures.cjs',
    reference: 'gaberogan/yjs@v0 (yjs 13.4.9, /root/reference/src) under Node 12 ESM with a lib0 shim over the bundled lib0 0.2.42 (oracle/gen/ref_yjs.cjs): new Doc() (gc: true), applyUpdate[V2] per input, encodeStateAsUpdate[V2]',
    stats,
    cases
  }))
  console.log(JSON.stringify(stats, null, 1), cases.length)
})().catch(e => { console.error(e); process.exit(1) })
