// A batched sync round through the Node drop-in (js/sync.js) over the golden C2 documents: the client's
// SyncStep1 is answered with SyncStep2, applying it makes the peers' state vectors equal.
'use strict'
const fs = require('fs')
const path = require('path')
const Y = require('..')
const S = require('../sync.js')
const cases = JSON.parse(fs.readFileSync(path.join(__dirname, '..', '..', 'tests', 'golden', 'c2_text.json'))).cases
  .filter(c => c.op === 'merge' && c.fmt === 1 && c.inputs.length > 4).slice(0, 16)
const u8 = b => new Uint8Array(Buffer.from(b, 'base64'))
const server = cases.map(c => Y.mergeUpdates(c.inputs.map(u8)))
const client = cases.map(c => { const x = c.inputs.map(u8); return Y.mergeUpdates(x.slice(0, x.length >> 1)) })
const msgs = client.map(c => S.writeSyncStep1(c))
const r1 = S.readSyncMessagesBatch(msgs, server)
const r2 = S.readSyncMessagesBatch(r1.replies, client)
let ok = 0
r2.stored.forEach((c, i) => {
  if (Buffer.compare(Buffer.from(Y.encodeStateVectorFromUpdate(c)), Buffer.from(Y.encodeStateVectorFromUpdate(server[i]))) === 0) ok++
})
console.log(JSON.stringify({ docs: server.length, converged: ok }))
process.exit(ok === server.length ? 0 : 1)
