// Golden vectors for the snapshot codec (test infrastructure, container-only).
//
// ym_snapshot re-encodes encoded snapshots: encodeSnapshot[V2](decodeSnapshot[V2](buf))
// (gaberogan/yjs@v0 src/utils/Snapshot.js:84-124).  This script builds inputs -- real snapshots of
// yjs-edited documents (Y.snapshot of Docs with text / map / array edits by several clients, deletes,
// syncs) in both encodings, plus hand-built corner cases: a client whose delete entries come in several
// runs (readDeleteSet appends them to its first appearance), runs with no entries (not added), repeated
// state-vector clients (Map.set: first position, last clock), out-of-order entries (negative V2 deltas
// through lib0 writeVarUint), zero lengths (DSEncoderV2.writeDsLen throws), clocks summing past 2^32 in V2,
// truncations and trailing bytes -- and records yjs 13.5.16's result for the V1 and the V2 output encoding
// (op snap_to_v1 / snap_to_v2, fmt = the input encoding) in tests/golden/snapshot.json.  Every case is
// also evaluated by the reference itself (oracle/gen/ref_yjs.cjs); the script fails if the two disagree.
// Usage: node make_snapshot_fixtures.cjs [golden dir]
'use strict'
const fs = require('fs')
const path = require('path')
const { Y, load } = require('./yjs_bundle.cjs')
const { loadReference } = require('./ref_yjs.cjs')
const enc = load(29194)
const E = { create: enc.Mf, toU8: enc._f, vu: enc.uE }
const DIR = process.argv[2] || path.join(__dirname, '../../tests/golden')

function rng (seed) {
  let s = (seed >>> 0) || 1
  const next = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s }
  return { int: (lo, hi) => lo + (next() % (hi - lo + 1)), chance: p => next() / 4294967296 < p, u32: next }
}
const b64 = u8 => Buffer.from(u8).toString('base64')

// a document edited by a few clients; the snapshot of one of them
function docSnapshot (seed) {
  const r = rng(seed)
  const n = r.int(1, 4)
  const docs = []
  for (let i = 0; i < n; i++) { const d = new Y.Doc({ gc: r.chance(0.5) }); d.clientID = 10 + 1000 * i + r.int(0, 99); docs.push(d) }
  const steps = r.int(1, 60)
  for (let t = 0; t < steps; t++) {
    const d = docs[r.int(0, n - 1)]
    const k = r.int(0, 5)
    d.transact(() => {
      if (k <= 2) {
        const text = d.getText('t')
        if (text.length > 0 && r.chance(0.4)) { const p = r.int(0, text.length - 1); text.delete(p, Math.min(r.int(1, 4), text.length - p)) } else text.insert(r.int(0, text.length), 'abcdefgh'.slice(0, r.int(1, 8)))
      } else if (k === 3) {
        const m = d.getMap('m')
        const key = 'k' + r.int(0, 4)
        if (m.has(key) && r.chance(0.5)) m.delete(key); else m.set(key, r.int(0, 1000))
      } else {
        const a = d.getArray('a')
        if (a.length > 0 && r.chance(0.4)) a.delete(r.int(0, a.length - 1), 1); else a.insert(r.int(0, a.length), [r.int(0, 9)])
      }
    })
    if (n > 1 && r.chance(0.4)) {
      const x = docs[r.int(0, n - 1)]; const y = docs[r.int(0, n - 1)]
      if (x !== y) Y.applyUpdate(y, Y.encodeStateAsUpdate(x, Y.encodeStateVector(y)))
    }
  }
  return Y.snapshot(docs[r.int(0, n - 1)])
}

// hand-built encoded snapshots: runs = [[client, [[clock, len], ...]], ...], sv = [[client, clock], ...]
function rawSnapshot (runs, sv, v2) {
  const e = E.create()
  E.vu(e, runs.length)
  for (const [client, items] of runs) {
    E.vu(e, client); E.vu(e, items.length)
    let cur = 0
    for (const [clock, len] of items) {
      if (v2) { E.vu(e, clock - cur); E.vu(e, len - 1); cur = clock + len } else { E.vu(e, clock); E.vu(e, len) }
    }
  }
  E.vu(e, sv.length)
  for (const [client, clock] of sv) { E.vu(e, client); E.vu(e, clock) }
  return E.toU8(e)
}

;(async () => {
  const R = await loadReference()
  const run = (lib, buf, fmt, to) => {
    const s = fmt === 2 ? lib.decodeSnapshotV2(buf) : lib.decodeSnapshot(buf)
    return to === 2 ? lib.encodeSnapshotV2(s) : lib.encodeSnapshot(s)
  }
  const cases = []
  let disagree = 0
  function add (name, buf, fmt) {
    for (const to of [1, 2]) {
      const c = { name, op: to === 2 ? 'snap_to_v2' : 'snap_to_v1', fmt, inputs: [b64(buf)] }
      let want, wantRef
      try { want = b64(run(Y, buf, fmt, to)); c.expect = want } catch (e) { c.error = e.constructor.name; c.message = String(e.message); want = 'ERR:' + c.error + ':' + c.message }
      try { wantRef = b64(run(R, buf, fmt, to)) } catch (e) { wantRef = 'ERR:' + e.constructor.name + ':' + String(e.message) }
      if (want !== wantRef) { disagree++; console.error('reference disagrees', name, to, want, wantRef) }
      cases.push(c)
    }
  }
  const N = +(process.env.SNAP_DOCS || 120)
  for (let d = 0; d < N; d++) {
    const s = docSnapshot(500 + d)
    add(`doc${d}/v1`, Y.encodeSnapshot(s), 1)
    add(`doc${d}/v2`, Y.encodeSnapshotV2(s), 2)
  }
  add('empty/v1', Y.encodeSnapshot(Y.emptySnapshot), 1)
  add('empty/v2', Y.encodeSnapshotV2(Y.emptySnapshot), 2)
  for (const v2 of [false, true]) {
    const f = v2 ? 2 : 1
    const tag = v2 ? 'v2' : 'v1'
    add(`repeated_client_runs/${tag}`, rawSnapshot([[5, [[0, 2], [10, 1]]], [9, [[3, 3]]], [5, [[20, 4]]]], [[5, 30], [9, 7]], v2), f)
    add(`zero_entry_run/${tag}`, rawSnapshot([[5, []], [9, [[1, 1]]], [5, [[2, 2]]]], [[9, 3]], v2), f)
    add(`repeated_sv_client/${tag}`, rawSnapshot([], [[3, 10], [4, 2], [3, 99], [4, 7], [3, 1]], v2), f)
    add(`large_clients/${tag}`, rawSnapshot([[4294967295, [[7, 1]]], [2 ** 31, [[0, 5]]]], [[4294967295, 8], [2 ** 31, 5]], v2), f)
    add(`trailing_bytes/${tag}`, Uint8Array.from([...rawSnapshot([[1, [[0, 1]]]], [[1, 1]], v2), 7, 7, 7]), f)
    const small = rawSnapshot([[5, [[0, 2], [4, 1]]], [300, [[1, 9]]]], [[5, 5], [300, 10]], v2)
    for (let cut = 0; cut < small.length; cut++) add(`truncated_${cut}/${tag}`, small.slice(0, cut), f)
  }
  // V1 inputs only: out-of-order entries (negative V2 deltas), zero lengths, clocks near 2^32
  add('unsorted_entries/v1', rawSnapshot([[5, [[10, 2], [3, 1], [7, 1]]]], [[5, 12]], false), 1)
  add('zero_len/v1', rawSnapshot([[5, [[1, 0]]]], [[5, 2]], false), 1)
  add('huge_clocks/v1', rawSnapshot([[5, [[4294967290, 5], [3, 4294967295]]]], [[5, 4294967295]], false), 1)
  // V2 inputs whose running clock passes 2^32 (JS numbers): the V1 output writes them through writeVarUint
  {
    const e = E.create()
    E.vu(e, 1); E.vu(e, 5); E.vu(e, 3)
    E.vu(e, 4294967290); E.vu(e, 9); E.vu(e, 4294967295); E.vu(e, 0); E.vu(e, 100); E.vu(e, 4294967295)
    E.vu(e, 1); E.vu(e, 5); E.vu(e, 1)
    add('clock_past_2p32/v2', E.toU8(e), 2)
  }
  fs.writeFileSync(path.join(DIR, 'snapshot.json'), JSON.stringify({
    generator: 'oracle/gen/make_snapshot_fixtures.cjs',
    oracle: 'yjs 13.5.16 (JupyterLab bundle) encodeSnapshot[V2](decodeSnapshot[V2](buf)); every case agrees with gaberogan/yjs@v0 (13.4.9, ref_yjs.cjs)',
    cases
  }))
  console.log('snapshot.json', cases.length, 'cases', cases.filter(c => c.error).length, 'errors', disagree, 'disagreements with the reference')
  if (disagree) process.exit(1)
})().catch(e => { console.error(e); process.exit(1) })
