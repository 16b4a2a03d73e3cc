// Benchmark workload templates (container-only recipe; the outputs are data committed under bench_data/).
//
// Builds the BASELINE.json configs with yjs 13.5.16's own Doc API, per SURVEY.md §8(d):
//   C1  1 doc, client 7, Y.Text, 10,000 ops in 1,000 transactions of 10 (60% insert [a-z]{1,5},
//       40% delete 1-3), seed 12345.  mergeUpdates of all 1,000 updates.
//   C2  docs of 4 clients x 100 transactions (60% insert word, 20% of them {bold:true}; 40% delete
//       1-3; 30% one-way sync after each tx), seed = doc+1; local updates only.  TEMPLATES docs are
//       generated and bench.py replicates them to 10,000 docs (doc i = template i % TEMPLATES).
//   C3  B4-like single-client trace (259,778 single-char ops: 2% random jump, 29.7% backspace, else
//       type), final state V1/V2; bench replicates it with random state vectors.
//   C4  Y.Map docs, 64 clients, 128 broadcast transactions, keys k0..k7, delete p=0.6 when present;
//       4,096 templates (SURVEY.md §8(d)).
//   C5  Y.XmlFragment docs, 1,024 clients x 16 transactions each (V1 and V2), see genXml.
//   C2R the C2 shape (50 transactions: documents of ~2 KB, inside the LDS fast path's budget) with rich content (Quill-style): formats {bold: true}, {header: 1..3} (a number),
//       {link: {href}} (an object), {color: '#rrggbb'}, and image embeds {image: url} (genTextRich).
//   C4R the C4 shape (96 transactions) whose map values are objects {x, y: [..], tag} and arrays [word, n] (genMapRich).
// File format (.ymb, little endian): "YMB1" u32 n_docs u32 n_upd | u32 doc_upd[n_docs+1] |
// u64 upd_off[n_upd+1] | arena bytes; gzip-compressed.
'use strict'
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const { Y } = require('./yjs_bundle.cjs')

const OUT = process.argv[2] || path.join(__dirname, '../../bench_data')
const which = (process.argv[3] || 'c1,c2,c3,c4').split(',')

function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return {
    u32: next,
    int: (lo, hi) => lo + (next() % (hi - lo + 1)),
    real: () => next() / 4294967296,
    word: (lo, hi) => { const n = lo + (next() % (hi - lo + 1)); let w = ''; for (let i = 0; i < n; i++) w += String.fromCharCode(97 + next() % 26); return w }
  }
}

function writeYmb (file, docs) {
  const nDocs = docs.length
  let nUpd = 0; let bytes = 0
  for (const d of docs) { nUpd += d.length; for (const u of d) bytes += u.length }
  const head = Buffer.alloc(12 + 4 * (nDocs + 1) + 8 * (nUpd + 1))
  head.write('YMB1', 0, 'latin1')
  head.writeUInt32LE(nDocs, 4); head.writeUInt32LE(nUpd, 8)
  let o = 12; let u = 0
  for (let i = 0; i <= nDocs; i++) { head.writeUInt32LE(u, o); o += 4; if (i < nDocs) u += docs[i].length }
  let off = 0
  head.writeBigUInt64LE(BigInt(0), o); o += 8
  const arena = Buffer.alloc(bytes)
  for (const d of docs) for (const x of d) { arena.set(x, off); off += x.length; head.writeBigUInt64LE(BigInt(off), o); o += 8 }
  fs.writeFileSync(file, zlib.gzipSync(Buffer.concat([head, arena]), { level: 9 }))
  console.log(file, nDocs, 'docs', nUpd, 'updates', bytes, 'bytes')
}

function genText (seed, nClients, nTx, opsPerTx, bold, syncP, ids) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = ids[c]
    d.on('update', (u, origin) => { if (origin !== 'remote') v1.push(u) })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') v2.push(u) })
    docs.push(d)
  }
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const text = d.getText('text')
    d.transact(() => {
      for (let o = 0; o < opsPerTx; o++) {
        const len = text.length
        if (len === 0 || r.real() < 0.6) {
          const pos = r.int(0, len); const w = r.word(1, 5)
          if (bold && r.real() < 0.2) text.insert(pos, w, { bold: true }); else text.insert(pos, w)
        } else {
          const pos = r.int(0, len - 1)
          text.delete(pos, Math.min(r.int(1, 3), len - pos))
        }
      }
    })
    if (nClients > 1 && r.real() < syncP) {
      const a = docs[r.u32() % docs.length]; const b = docs[r.u32() % docs.length]
      if (a !== b) Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)), 'remote')
    }
  }
  return { v1, v2 }
}

function genMap (seed, nClients, nTx, nKeys) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) { const d = new Y.Doc(); d.clientID = 500 + 31 * c; docs.push(d) }
  for (const d of docs) {
    d.on('update', (u, origin) => { if (origin === 'remote') return; v1.push(u); for (const o of docs) if (o !== d) Y.applyUpdate(o, u, 'remote') })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') v2.push(u) })
  }
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const m = d.getMap('map')
    const key = 'k' + (r.u32() % nKeys)
    if (m.has(key) && r.real() < 0.6) m.delete(key)
    else m.set(key, r.real() < 0.5 ? r.int(0, 1000000) : r.word(1, 6))
  }
  return { v1, v2 }
}

// genMap with the 64 always-synced peers folded into one Doc: every transaction is followed by a broadcast
// to all peers, so every peer holds the same state and a transaction of peer c is that state edited under
// clientID c.  One Doc whose clientID is switched per transaction emits the very same update bytes (same
// origins, clocks and delete sets; checked against genMap by `node make_bench_data.cjs <dir> c4check`) at
// 1/64 of the cost.
function genMapShared (seed, nClients, nTx, nKeys) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const ids = []
  for (let c = 0; c < nClients; c++) ids.push(500 + 31 * c)
  const d = new Y.Doc(); d.clientID = ids[0]
  d.on('update', u => v1.push(u))
  d.on('updateV2', u => v2.push(u))
  for (let t = 0; t < nTx; t++) {
    d.clientID = ids[r.u32() % nClients]
    const m = d.getMap('map')
    const key = 'k' + (r.u32() % nKeys)
    if (m.has(key) && r.real() < 0.6) m.delete(key)
    else m.set(key, r.real() < 0.5 ? r.int(0, 1000000) : r.word(1, 6))
  }
  return { v1, v2 }
}

// C5: Y.XmlFragment('xml'), nClients clients x nTx transactions (16 per client), 30% one-way sync
// between random peers after each transaction; local updates only (SURVEY.md §8(d) C5).  40% insert an
// XmlElement('p'|'h1') with a `class` attribute and a formatted XmlText; 35% formatted text insert
// into an existing element; 25% delete an element.
function genXml (seed, nClients, nTx) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = 3000 + 17 * c
    d.on('update', (u, origin) => { if (origin !== 'remote') v1.push(u) })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') v2.push(u) })
    docs.push(d)
  }
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const frag = d.getXmlFragment('xml')
    const p = r.real()
    d.transact(() => {
    if (p < 0.4 || frag.length === 0) {
      const el = new Y.XmlElement(r.u32() % 2 ? 'p' : 'h1')
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
    } else {
      frag.delete(r.int(0, frag.length - 1), 1)
    }
    })
    if (r.real() < 0.3) {
      const a = docs[r.u32() % docs.length]; const b = docs[r.u32() % docs.length]
      if (a !== b) Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)), 'remote')
    }
  }
  return { v1, v2 }
}

// C2R: genText with Quill-style rich content
function genTextRich (seed, nClients, nTx, syncP, ids) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = ids[c]
    d.on('update', (u, origin) => { if (origin !== 'remote') v1.push(u) })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') v2.push(u) })
    docs.push(d)
  }
  const fmt = () => {
    const p = r.real()
    if (p < 0.25) return { bold: true }
    if (p < 0.45) return { header: r.int(1, 3) }
    if (p < 0.6) return { link: { href: 'https://e.x/' + r.word(2, 6) } }
    if (p < 0.75) return { color: '#' + (r.u32() & 0xffffff).toString(16).padStart(6, '0') }
    return {}
  }
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const text = d.getText('text')
    d.transact(() => {
      const len = text.length
      const p = r.real()
      if (len === 0 || p < 0.5) text.insert(r.int(0, len), r.word(1, 5), fmt())
      else if (p < 0.6) text.insertEmbed(r.int(0, len), { image: 'https://e.x/i' + r.int(0, 999) + '.png' })
      else if (p < 0.7) { const pos = r.int(0, len - 1); text.format(pos, Math.min(r.int(1, 4), len - pos), fmt()) }
      else { const pos = r.int(0, len - 1); text.delete(pos, Math.min(r.int(1, 3), len - pos)) }
    })
    if (nClients > 1 && r.real() < syncP) {
      const a = docs[r.u32() % docs.length]; const b = docs[r.u32() % docs.length]
      if (a !== b) Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)), 'remote')
    }
  }
  return { v1, v2 }
}
// C4R: genMapShared whose values are objects and arrays
function genMapRich (seed, nClients, nTx, nKeys) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const ids = []
  for (let c = 0; c < nClients; c++) ids.push(500 + 31 * c)
  const d = new Y.Doc(); d.clientID = ids[0]
  d.on('update', u => v1.push(u))
  d.on('updateV2', u => v2.push(u))
  for (let t = 0; t < nTx; t++) {
    d.clientID = ids[r.u32() % nClients]
    const m = d.getMap('map')
    const key = 'k' + (r.u32() % nKeys)
    if (m.has(key) && r.real() < 0.6) m.delete(key)
    else if (r.real() < 0.6) m.set(key, { x: r.int(0, 1000000), y: [r.int(0, 99), r.int(0, 99)], tag: r.word(1, 6) })
    else m.set(key, [r.word(1, 6), r.int(0, 1000), r.real() < 0.5])
  }
  return { v1, v2 }
}

// C2U: the C2 shape (50 transactions, as C2R: documents of ~2 KB) with realistic text: ~30% of the short
// inserts are CJK words, emoji (surrogate pairs) or accented Latin, 10% of the inserts are pastes of 20-200
// characters of mixed text; 20% bold.  Inserts and deletes never fall inside a surrogate pair (an editor
// moves by code points).
function genTextUnicode (seed, nClients, nTx, syncP, ids) {
  const r = rng(seed)
  const v1 = []; const v2 = []
  const docs = []
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = ids[c]
    d.on('update', (u, origin) => { if (origin !== 'remote') v1.push(u) })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') v2.push(u) })
    docs.push(d)
  }
  const cjk = n => { let w = ''; for (let i = 0; i < n; i++) w += String.fromCodePoint(0x4e00 + r.u32() % 0x51a0); return w }
  const emoji = n => { let w = ''; for (let i = 0; i < n; i++) w += String.fromCodePoint(0x1f600 + r.u32() % 0x50); return w }
  const accent = n => { const a = 'éèêëàâäôöûüçñß'; let w = ''; for (let i = 0; i < n; i++) w += r.real() < 0.4 ? a[r.u32() % a.length] : String.fromCharCode(97 + r.u32() % 26); return w }
  const word = () => {
    const p = r.real()
    if (p < 0.7) return r.word(1, 5)
    if (p < 0.82) return cjk(r.int(1, 4))
    if (p < 0.91) return emoji(r.int(1, 3))
    return accent(r.int(2, 7))
  }
  const paste = () => {
    const n = r.int(20, 200); let s = ''
    while ([...s].length < n) s += (s ? ' ' : '') + word()
    return [...s].slice(0, n).join('')
  }
  // a UTF-16 position at a code point boundary of s (pos <= s.length)
  const cpPos = (s, pos) => (pos > 0 && pos < s.length && s.charCodeAt(pos) >= 0xdc00 && s.charCodeAt(pos) <= 0xdfff) ? pos - 1 : pos
  for (let t = 0; t < nTx; t++) {
    const d = docs[r.u32() % docs.length]
    const text = d.getText('text')
    d.transact(() => {
      const s = text.toString()
      const len = s.length
      if (len === 0 || r.real() < 0.6) {
        const pos = cpPos(s, r.int(0, len)); const w = r.real() < 0.1 ? paste() : word()
        if (r.real() < 0.2) text.insert(pos, w, { bold: true }); else text.insert(pos, w)
      } else {
        const pos = cpPos(s, r.int(0, len - 1))
        const end = cpPos(s, Math.min(pos + r.int(1, 3), len))
        if (end > pos) text.delete(pos, end - pos)
      }
    })
    if (nClients > 1 && r.real() < syncP) {
      const a = docs[r.u32() % docs.length]; const b = docs[r.u32() % docs.length]
      if (a !== b) Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)), 'remote')
    }
  }
  return { v1, v2 }
}

fs.mkdirSync(OUT, { recursive: true })
if (which.includes('c2u')) {
  const T = Number(process.env.C2_TEMPLATES || 1024)
  const d1 = []; const d2 = []
  for (let doc = 0; doc < T; doc++) {
    const { v1, v2 } = genTextUnicode(doc + 11001, 4, 50, 0.3, [1000, 8919, 16838, 24757])
    d1.push(v1); d2.push(v2)
  }
  writeYmb(path.join(OUT, 'c2u_v1.ymb.gz'), d1)
  writeYmb(path.join(OUT, 'c2u_v2.ymb.gz'), d2)
}
if (which.includes('c2r')) {
  const T = Number(process.env.C2_TEMPLATES || 1024)
  const d1 = []; const d2 = []
  for (let doc = 0; doc < T; doc++) {
    const { v1, v2 } = genTextRich(doc + 7001, 4, 50, 0.3, [1000, 8919, 16838, 24757])
    d1.push(v1); d2.push(v2)
  }
  writeYmb(path.join(OUT, 'c2r_v1.ymb.gz'), d1)
  writeYmb(path.join(OUT, 'c2r_v2.ymb.gz'), d2)
}
if (which.includes('c4r')) {
  const T = Number(process.env.C4_TEMPLATES || 1024)
  const d1 = []; const d2 = []
  for (let doc = 0; doc < T; doc++) {
    const { v1, v2 } = genMapRich(doc + 9001, 64, 96, 8)
    d1.push(v1); d2.push(v2)
  }
  writeYmb(path.join(OUT, 'c4r_v1.ymb.gz'), d1)
  writeYmb(path.join(OUT, 'c4r_v2.ymb.gz'), d2)
}
if (which.includes('c1')) {
  const { v1, v2 } = genText(12345, 1, 1000, 10, false, 0, [7])
  writeYmb(path.join(OUT, 'c1_v1.ymb.gz'), [v1])
  writeYmb(path.join(OUT, 'c1_v2.ymb.gz'), [v2])
}
if (which.includes('c2')) {
  const T = Number(process.env.C2_TEMPLATES || 1024)
  const d1 = []; const d2 = []
  for (let doc = 0; doc < T; doc++) {
    const { v1, v2 } = genText(doc + 1, 4, 100, 1, true, 0.3, [1000, 8919, 16838, 24757])
    d1.push(v1); d2.push(v2)
  }
  writeYmb(path.join(OUT, 'c2_v1.ymb.gz'), d1)
  writeYmb(path.join(OUT, 'c2_v2.ymb.gz'), d2)
}
if (which.includes('c3')) {
  const r = rng(4242)
  const d = new Y.Doc(); d.clientID = 1
  const text = d.getText('text')
  let cursor = 0
  for (let i = 0; i < 259778; i++) {
    if (r.real() < 0.02) cursor = r.int(0, text.length)
    if (cursor > 0 && r.real() < 0.297) { text.delete(cursor - 1, 1); cursor-- } else { text.insert(cursor, String.fromCharCode(97 + r.u32() % 26)); cursor++ }
  }
  writeYmb(path.join(OUT, 'c3_v1.ymb.gz'), [[Y.encodeStateAsUpdate(d)]])
  writeYmb(path.join(OUT, 'c3_v2.ymb.gz'), [[Y.encodeStateAsUpdateV2(d)]])
}
if (which.includes('c4check')) {  // genMapShared == genMap, byte for byte
  for (let doc = 0; doc < 16; doc++) {
    const a = genMap(doc + 1, 64, 128, 8); const b = genMapShared(doc + 1, 64, 128, 8)
    const same = (x, y) => x.length === y.length && x.every((u, i) => Buffer.compare(Buffer.from(u), Buffer.from(y[i])) === 0)
    if (!same(a.v1, b.v1) || !same(a.v2, b.v2)) throw new Error('genMapShared differs from genMap for template ' + doc)
  }
  console.log('genMapShared == genMap on 16 templates')
} else if (which.includes('c4')) {
  const T = Number(process.env.C4_TEMPLATES || 4096)
  const d1 = []; const d2 = []
  for (let doc = 0; doc < T; doc++) {
    const { v1, v2 } = genMapShared(doc + 1, 64, 128, 8)
    d1.push(v1); d2.push(v2)
  }
  writeYmb(path.join(OUT, 'c4_v1.ymb.gz'), d1)
  writeYmb(path.join(OUT, 'c4_v2.ymb.gz'), d2)
}
if (which.includes('c5')) {
  const T = Number(process.env.C5_TEMPLATES || 8)
  const NC = Number(process.env.C5_CLIENTS || 1024)
  const d1 = []; const d2 = []
  for (let doc = 0; doc < T; doc++) {
    const { v1, v2 } = genXml(doc + 101, NC, 16 * NC)
    d1.push(v1); d2.push(v2)
  }
  writeYmb(path.join(OUT, 'c5_v1.ymb.gz'), d1)
  writeYmb(path.join(OUT, 'c5_v2.ymb.gz'), d2)
}
