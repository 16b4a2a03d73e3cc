// ym_compact.h -- Doc round-trip compaction on the device.
//
// Per document: a fresh gc=true Doc of the reference (gaberogan/yjs@v0 = yjs 13.4.9), applyUpdate[V2] of
// every input in order, then encodeStateAsUpdate[V2] of the result -- the reference's own compaction, which
// merges runs of structs and replaces deleted content by ContentDeleted / GC.  One GPU thread owns one
// document (the integration of a struct depends on every struct integrated before it); all state lives in
// the document's HBM workspace.  Restated from the reference's sources:
//   readUpdateV2 / readStructs / mergeReadStructsIntoPendingReads / resumeStructIntegration
//                                        src/utils/encoding.js:127-321
//   Item.integrate / getMissing / splitItem / gc / delete      src/structs/Item.js:85-125, 325-560
//   readAndApplyDeleteSet                src/utils/DeleteSet.js:270-323; createDeleteSetFromStructStore :185-210
//   cleanupTransactions / tryGcDeleteSet / tryMergeDeleteSet / tryToMergeWithLeft
//                                        src/utils/Transaction.js:165-367
//   YText._callObserver's remote formatting cleanup     src/types/YText.js:348-437, 803-856
//   iterateStructs / findIndexCleanStart src/utils/StructStore.js:173-273
//   writeClientsStructs / writeDeleteSet src/utils/encoding.js:71-116, DeleteSet.js:219-232
// (the test oracle's restatement of the same code is oracle/ymerge_oracle.c compact_impl).
//
// Content is never decoded into values: a ContentString is a list of pieces of its inputs' UTF-8 bytes
// (ContentString.splice's U+FFFD rule recorded as flags at the cut), ContentAny / ContentJSON a list of
// element ranges, the other contents point at their source bytes; they are re-encoded by ym_core.h's
// writers (payloads copied when canonical, re-encoded through ym_canon.h otherwise).
#pragma once
#include "ym_core.h"

namespace ym {
// small routines called per struct / per write: inlined into the kernel (an out-of-line call saves and
// restores the caller's live registers through scratch, which dominated the kernel's time)
#ifdef __HIP_DEVICE_COMPILE__
#define YM_HOT YM_HD inline __attribute__((always_inline))
#else
#define YM_HOT YM_HD inline
#endif
namespace cpt {

constexpr int32_t NIL = -1;

// ---- workspace: fixed pools (stable indices) + a bump region for growable vectors -------------------
struct Arena { uint8_t *base; uint64_t cap, used; };
YM_INL void *aalloc(Ctx &c, Arena &a, uint64_t n) {
  const uint64_t p = (a.used + 15) & ~15ull;
  if (c.err || p + n > a.cap) { seterr(c, ST_RETRY); return nullptr; }
  a.used = p + n;
  return a.base + p;
}
template <class T> struct Vec { T *p; uint32_t n, cap; };
template <class T> YM_INL bool vgrow(Ctx &c, Arena &a, Vec<T> &v, uint32_t need) {
  if (need <= v.cap) return true;
  uint32_t nc = v.cap ? 2 * v.cap : 8;
  while (nc < need) nc *= 2;
  // the arena's last allocation grows in place (a vector pushed to in a loop no longer leaves its
  // outgrown copies behind)
  if (v.p && (uint8_t *)(v.p + v.cap) == a.base + a.used && a.used + (uint64_t)(nc - v.cap) * sizeof(T) <= a.cap) {
    a.used += (uint64_t)(nc - v.cap) * sizeof(T);
    v.cap = nc;
    return true;
  }
  T *np = (T *)aalloc(c, a, (uint64_t)nc * sizeof(T));
  if (!np) return false;
  for (uint32_t i = 0; i < v.n; i++) np[i] = v.p[i];
  v.p = np;
  v.cap = nc;
  return true;
}
template <class T> YM_INL bool vpush(Ctx &c, Arena &a, Vec<T> &v, T x) {
  if (!vgrow(c, a, v, v.n + 1)) return false;
  v.p[v.n++] = x;
  return true;
}
template <class T> YM_INL void vinsert(Ctx &c, Arena &a, Vec<T> &v, uint32_t at, T x) {
  if (!vgrow(c, a, v, v.n + 1)) return;
  for (uint32_t i = v.n; i > at; i--) v.p[i] = v.p[i - 1];
  v.p[at] = x;
  v.n++;
}
template <class T> YM_INL void vremove(Vec<T> &v, uint32_t at) {
  for (uint32_t i = at; i + 1 < v.n; i++) v.p[i] = v.p[i + 1];
  v.n--;
}

// ---- content ---------------------------------------------------------------------------------------
// A piece of a ContentString: [U+FFFD] [the lone low half of the 4-byte character ending at off] the UTF-8
// bytes [off, off + n) [the lone high half of the 4-byte character at off + n] [U+FFFD]; n16 UTF-16 units.
// A piece of a ContentAny / ContentJSON: elements [off, off + n) of the element pool (n16 = n).
struct Piece { uint64_t off; uint32_t n, n16; uint8_t fffd, lo, hi, tfffd; int32_t next; };
// an Any value / JSON text of the inputs (V1: the varString body; V2 JSON: a slice of the string column)
struct Elem { uint64_t off; uint32_t n, n16; uint8_t nc, undef, pad0, pad1; };
// a single-valued content (Binary, Embed, Format, Type, Doc) as read
struct Src;

struct Item {
  int64_t client, clock, len;
  int64_t oc, ok, rc, rk;  // origin / rightOrigin
  int64_t pc, pk;          // parent ID as read (pkind 2)
  Span pkey, psub;
  int32_t left, right;     // left / right (the list neighbours)
  int32_t parent, type;    // resolved parent type; ContentType: its type
  int32_t chead, ctail;    // ContentString / Any / JSON pieces
  int32_t src;             // single-valued content
  uint32_t gen_before, gen_conf;  // Item.integrate's itemsBeforeOrigin / conflictingItems sets
  uint8_t gc, has_origin, has_right, pkind, has_psub, deleted, ref, pad;
};
struct Type {
  int32_t start, item, tref;  // _start, _item, typeRef (-1: a root type)
  Span key;                   // a root type's key
  Vec<Span> mk;               // _map, insertion order
  Vec<int32_t> mv;
};
struct Cl { int64_t client; Vec<int32_t> a; };
struct Pend { int64_t client; int32_t *refs; uint32_t n, i; uint8_t live; };
struct DIt { int64_t clock, len; };
struct DCl { int64_t client; Vec<DIt> it; };
struct DSet { Vec<DCl> cl; Arena *ar; };  // ar: the arena its vectors grow in (nullptr: the document's)
struct Wt { int64_t thresh; uint32_t pos; };  // pending delete reader `pos` waits for state(client) > thresh
struct WL { int64_t client; Vec<Wt> w; };
struct Tx {
  DSet ds;
  Vec<int32_t> ms;   // _mergeStructs
  int64_t *bc;       // beforeState, by store client index
  uint32_t nbc;
  Vec<int32_t> chg;  // changed types, Map insertion order
  uint8_t local;
};
// a format value for YText's cleanup (ContentFormat.value compared with ===): V1 its canonical JSON text,
// V2 its any encoding; objects / arrays by identity (the source)
enum : uint8_t { FV_UNDEF = 0, FV_NULL, FV_BOOL, FV_NUM, FV_STR, FV_BIG, FV_OBJ };
struct FVal { const uint8_t *p; uint32_t n; int32_t ident; double num; uint8_t t, truthy, pad0, pad1; };
struct AttrE { Span key; FVal v; };
// a single-valued content (Binary, Embed, Format, Type, Doc) as read; a format's value once computed
struct Src { Span a, b; int64_t cnt; FVal fv; uint8_t nca, ncb, keyundef, ref, fv_done; };

struct Doc {
  Ctx *c;
  Arena *a;   // persistent: the store's vectors, pending structs / deletes, types
  Arena *ta;  // transient: one update's reader and transaction (released after each update)
  uint32_t v2;
  uint32_t nogc;       // Doc({ gc: false }): deleted content is kept (no tryGcDeleteSet), Doc.js:40-43
  Item *it; uint32_t nit, capit;
  Piece *pc; uint32_t npc, cappc;
  Elem *el; uint32_t nel, capel;
  Src *src; uint32_t nsrc, capsrc;
  Type *ty; uint32_t nty, capty;
  Vec<Cl> cl;
  int64_t *hk; uint32_t *hv; uint32_t hcap;  // client -> store index + 1 (open addressing)
  Vec<Pend> pend;      // store.pendingClientsStructRefs, sorted by client (cd_pend)
  Vec<int32_t> stack;  // store.pendingStack
  // store.pendingDeleteReaders, append-only: a re-read reader's remainder takes its place, a reader applied in
  // full leaves a hole (cl.n == 0), so positions keep the reference's order.  tryResumePendingDeleteReaders
  // re-reads every reader on every update, but a reader none of whose ranges starts below its client's state
  // leaves the store as it was: only the readers some client's state has passed since (`awake`, found by the
  // per-client watch lists add_struct consults) are re-read (pdel_watch / pdel_wake).
  Vec<DSet> pdel;
  int64_t *wk; uint32_t *wv; uint32_t wcap;  // client -> watch list index + 1 (open addressing)
  Vec<WL> wl;
  Vec<uint32_t> awake;
  Vec<int32_t> roots;  // doc.share
  uint32_t gen;
  Tx *tx;
  uint32_t *ord;       // output order of the store's clients (descending)
  int64_t *svst;       // target state vector: per client the first clock written, -1: none (doc_write)
};

YM_INL Item &IT(Doc &d, int32_t i) { return d.it[i]; }
YM_INL Type &TY(Doc &d, int32_t i) { return d.ty[i]; }
YM_INL int32_t new_item(Doc &d) {
  if (d.nit >= d.capit) { seterr(*d.c, ST_RETRY); return NIL; }
  Item &x = d.it[d.nit];
  __builtin_memset(&x, 0, sizeof(Item));
  x.left = x.right = x.parent = x.type = x.chead = x.ctail = x.src = NIL;
  return (int32_t)d.nit++;
}
YM_INL int32_t new_piece(Doc &d) {
  if (d.npc >= d.cappc) { seterr(*d.c, ST_RETRY); return NIL; }
  Piece &p = d.pc[d.npc];
  __builtin_memset(&p, 0, sizeof(Piece));
  p.next = NIL;
  return (int32_t)d.npc++;
}
YM_INL int32_t new_type(Doc &d) {
  if (d.nty >= d.capty) { seterr(*d.c, ST_RETRY); return NIL; }
  Type &t = d.ty[d.nty];
  __builtin_memset(&t, 0, sizeof(Type));
  t.start = t.item = NIL;
  t.tref = -1;
  return (int32_t)d.nty++;
}

// string equality of two read strings (keys, parentSubs): same UTF-16 units
YM_INL bool str_eq(const Ctx &c, const Span &x, const Span &y) {
  if (x.n != y.n || x.fffd != y.fffd || x.lo != y.lo || x.hi != y.hi) return false;
  for (uint32_t i = 0; i < x.n; i++)
    if (c.A[x.off + i] != c.A[y.off + i]) return false;
  if (x.lo && sur_lo(c, x.off - 4) != sur_lo(c, y.off - 4)) return false;
  if (x.hi && sur_hi(c, x.off + x.n) != sur_hi(c, y.off + y.n)) return false;
  return true;
}

// ---- struct store -------------------------------------------------------------------------------------
YM_INL uint32_t cl_hslot(const Doc &d, int64_t client) {
  uint32_t h = (uint32_t)(((uint64_t)client * 0x9E3779B97F4A7C15ull) >> 40) & (d.hcap - 1);
  while (d.hv[h] != 0 && d.hk[h] != client) h = (h + 1) & (d.hcap - 1);
  return h;
}
YM_INL int32_t cd_client(Doc &d, int64_t client) {
  if (d.hcap == 0) return NIL;
  const uint32_t h = cl_hslot(d, client);
  return d.hv[h] ? (int32_t)(d.hv[h] - 1) : NIL;
}
YM_HOT void cl_hput(Doc &d, int64_t client, uint32_t idx) {
  Ctx &c = *d.c;
  if (2 * (d.cl.n + 1) > d.hcap) {
    const uint32_t nc = d.hcap ? 2 * d.hcap : 64;
    int64_t *ok = d.hk;
    uint32_t *ov = d.hv, oc = d.hcap;
    d.hk = (int64_t *)aalloc(c, *d.a, 8ull * nc);
    d.hv = (uint32_t *)aalloc(c, *d.a, 4ull * nc);
    if (c.err) return;
    for (uint32_t i = 0; i < nc; i++) d.hv[i] = 0;
    d.hcap = nc;
    for (uint32_t i = 0; i < oc; i++)
      if (ov[i]) { const uint32_t h = cl_hslot(d, ok[i]); d.hk[h] = ok[i]; d.hv[h] = ov[i]; }
  }
  const uint32_t h = cl_hslot(d, client);
  d.hk[h] = client;
  d.hv[h] = idx + 1;
}
YM_INL int64_t cl_state(Doc &d, int32_t s) {
  if (s == NIL || d.cl.p[s].a.n == 0) return 0;
  const Item &l = d.it[d.cl.p[s].a.p[d.cl.p[s].a.n - 1]];
  return l.clock + l.len;
}
YM_INL int64_t cd_state(Doc &d, int64_t client) { return cl_state(d, cd_client(d, client)); }  // getState
// ---- watch lists of the pending delete readers (Doc.pdel) ----
YM_INL uint32_t wl_hslot(const Doc &d, int64_t client) {
  uint32_t h = (uint32_t)(((uint64_t)client * 0x9E3779B97F4A7C15ull) >> 40) & (d.wcap - 1);
  while (d.wv[h] != 0 && d.wk[h] != client) h = (h + 1) & (d.wcap - 1);
  return h;
}
// the watch list of `client` (created when `add`), or NIL
YM_HOT int32_t wl_get(Doc &d, int64_t client, bool add) {
  Ctx &c = *d.c;
  if (d.wcap) {
    const uint32_t h = wl_hslot(d, client);
    if (d.wv[h]) return (int32_t)(d.wv[h] - 1);
  }
  if (!add) return NIL;
  if (2 * (d.wl.n + 1) > d.wcap) {
    const uint32_t nc = d.wcap ? 2 * d.wcap : 64;
    int64_t *ok = d.wk;
    uint32_t *ov = d.wv, oc = d.wcap;
    d.wk = (int64_t *)aalloc(c, *d.a, 8ull * nc);
    d.wv = (uint32_t *)aalloc(c, *d.a, 4ull * nc);
    if (c.err) return NIL;
    for (uint32_t i = 0; i < nc; i++) d.wv[i] = 0;
    d.wcap = nc;
    for (uint32_t i = 0; i < oc; i++)
      if (ov[i]) { const uint32_t h = wl_hslot(d, ok[i]); d.wk[h] = ok[i]; d.wv[h] = ov[i]; }
  }
  WL z;
  __builtin_memset(&z, 0, sizeof(WL));
  z.client = client;
  if (!vpush(c, *d.a, d.wl, z)) return NIL;
  const uint32_t h = wl_hslot(d, client);
  d.wk[h] = client;
  d.wv[h] = d.wl.n;
  return (int32_t)(d.wl.n - 1);
}
// reader d.pdel[pos] (just written): per client, woken once that client's state passes its first clock; a
// reader one of whose ranges already starts below the state (possible after writeDeleteSet's round trip of an
// unsorted or empty range) is awake at once
YM_HOT void pdel_watch(Doc &d, uint32_t pos) {
  Ctx &c = *d.c;
  const DSet &ds = d.pdel.p[pos];
  bool now = false;
  for (uint32_t ci = 0; ci < ds.cl.n && !c.err; ci++) {
    const DCl &z = ds.cl.p[ci];
    if (z.it.n == 0) continue;
    int64_t th = z.it.p[0].clock;
    for (uint32_t k = 1; k < z.it.n; k++) th = z.it.p[k].clock < th ? z.it.p[k].clock : th;
    if (th < cd_state(d, z.client)) { now = true; continue; }
    const int32_t w = wl_get(d, z.client, true);
    if (w == NIL) return;
    const Wt e = {th, pos};
    vpush(c, *d.a, d.wl.p[w].w, e);
  }
  if (now) vpush(c, *d.a, d.awake, pos);
}
// client's state is now `state` (add_struct): the readers waiting on it are awake (a watcher of a reader since
// replaced wakes its position for nothing: the re-read finds no range to apply)
YM_HOT void pdel_wake(Doc &d, int64_t client, int64_t state) {
  if (d.wcap == 0) return;
  const int32_t w = wl_get(d, client, false);
  if (w == NIL) return;
  Vec<Wt> &v = d.wl.p[w].w;
  for (uint32_t k = 0; k < v.n;) {
    if (v.p[k].thresh < state) {
      if (!vpush(*d.c, *d.a, d.awake, v.p[k].pos)) return;
      v.p[k] = v.p[--v.n];
    } else {
      k++;
    }
  }
}
// findIndexSS (StructStore.js:123-151); an absent clock is an unexpected case (returns 0)
YM_INL uint32_t find_index(Doc &d, int32_t s, int64_t clock) {
  if (s == NIL || d.cl.p[s].a.n == 0) { seterr(*d.c, ST_UNEXPECTED); return 0; }
  const Vec<int32_t> &a = d.cl.p[s].a;
  uint32_t lo = 0, hi = a.n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    const Item &m = d.it[a.p[mid]];
    if (m.clock <= clock) {
      if (clock < m.clock + m.len) return mid;
      lo = mid + 1;
    } else {
      hi = mid;
    }
  }
  seterr(*d.c, ST_UNEXPECTED);
  return 0;
}
YM_INL int32_t cd_get(Doc &d, int64_t client, int64_t clock) {  // getItem
  const int32_t s = cd_client(d, client);
  const uint32_t i = find_index(d, s, clock);
  return d.c->err ? NIL : d.cl.p[s].a.p[i];
}
YM_HOT void add_struct(Doc &d, int32_t i) {  // addStruct (StructStore.js:92-104)
  Ctx &c = *d.c;
  const Item &x = d.it[i];
  int32_t s = cd_client(d, x.client);
  if (s == NIL) {
    Cl z;
    __builtin_memset(&z, 0, sizeof(Cl));
    z.client = x.client;
    cl_hput(d, x.client, d.cl.n);
    if (!vpush(c, *d.a, d.cl, z)) return;
    s = (int32_t)(d.cl.n - 1);
  } else {
    const Item &l = d.it[d.cl.p[s].a.p[d.cl.p[s].a.n - 1]];
    if (l.clock + l.len != x.clock) { seterr(c, ST_UNEXPECTED); return; }
  }
  if (vpush(c, *d.a, d.cl.p[s].a, i)) pdel_wake(d, x.client, x.clock + x.len);
}
YM_INL int32_t cd_root(Doc &d, const Span &key) {  // doc.get(key): created on first use
  for (uint32_t i = 0; i < d.roots.n; i++)
    if (str_eq(*d.c, d.ty[d.roots.p[i]].key, key)) return d.roots.p[i];
  const int32_t t = new_type(d);
  if (t == NIL) return NIL;
  d.ty[t].key = key;
  vpush(*d.c, *d.a, d.roots, t);
  return t;
}
YM_INL int32_t map_get(Doc &d, int32_t t, const Span &k) {
  Type &T = d.ty[t];
  for (uint32_t i = 0; i < T.mk.n; i++)
    if (str_eq(*d.c, T.mk.p[i], k)) return T.mv.p[i];
  return NIL;
}
YM_INL void map_set(Doc &d, int32_t t, const Span &k, int32_t v) {
  Type &T = d.ty[t];
  for (uint32_t i = 0; i < T.mk.n; i++)
    if (str_eq(*d.c, T.mk.p[i], k)) { T.mv.p[i] = v; return; }
  if (vpush(*d.c, *d.a, T.mk, k)) vpush(*d.c, *d.a, T.mv, v);
}

// ---- delete sets ---------------------------------------------------------------------------------------
YM_INL int32_t ds_get_or_add(Doc &d, DSet &ds, int64_t client) {
  for (uint32_t i = 0; i < ds.cl.n; i++)
    if (ds.cl.p[i].client == client) return (int32_t)i;
  DCl z;
  __builtin_memset(&z, 0, sizeof(DCl));
  z.client = client;
  if (!vpush(*d.c, ds.ar ? *ds.ar : *d.a, ds.cl, z)) return NIL;
  return (int32_t)(ds.cl.n - 1);
}
YM_INL void tds_add(Doc &d, DSet &ds, int64_t client, int64_t clock, int64_t len) {  // addToDeleteSet
  const int32_t k = ds_get_or_add(d, ds, client);
  if (k == NIL) return;
  DIt e = {clock, len};
  vpush(*d.c, ds.ar ? *ds.ar : *d.a, ds.cl.p[k].it, e);
}
// sortAndMergeDeleteSet, the reference's own (DeleteSet.js:113-135): stable sort by clock, exactly
// adjacent ranges coalesce
YM_HOT void ds_sort_merge(DSet &ds) {
  for (uint32_t ci = 0; ci < ds.cl.n; ci++) {
    Vec<DIt> &v = ds.cl.p[ci].it;
    for (uint32_t i = 1; i < v.n; i++) {  // insertion sort: stable
      const DIt x = v.p[i];
      uint32_t j = i;
      while (j > 0 && v.p[j - 1].clock > x.clock) { v.p[j] = v.p[j - 1]; j--; }
      v.p[j] = x;
    }
    uint32_t i, j;
    for (i = 1, j = 1; i < v.n; i++) {
      DIt &l = v.p[j - 1];
      const DIt r = v.p[i];
      if (l.clock + l.len == r.clock) l.len += r.len;
      else { if (j < i) v.p[j] = r; j++; }
    }
    if (v.n > 0) v.n = j;
  }
}

// ---- content splice / merge ------------------------------------------------------------------------
// units of a string piece's UTF-8 body
YM_INL uint32_t body16(const Piece &p) { return p.n16 - p.fffd - p.lo - p.hi - p.tfffd; }
// the two parts of string piece P split at unit k (0 < k < n16): str.slice(0, k) and str.slice(k) of the
// piece's units, a surrogate pair cut in two leaving a lone high half in L and a lone low half in R
YM_INL void piece_split_str(const Ctx &c, const Piece &P, uint32_t k, Piece &L, Piece &R) {
  L = P;
  R = P;
  L.tfffd = 0; L.hi = 0;
  R.fffd = 0; R.lo = 0;
  uint32_t u = k;
  bool done = false;
  if (P.fffd) {  // k >= 1: the leading U+FFFD stays left
    u--;
    if (u == 0) { L.lo = 0; L.n = 0; L.n16 = 1; R.lo = P.lo; R.n16 = P.n16 - 1; done = true; }
  }
  if (!done && P.lo) {
    if (u == 0) {  // (only without a leading U+FFFD: k >= 1)
      L.lo = 0; L.n = 0; L.n16 = k; R.lo = 1; R.n16 = P.n16 - k; done = true;
    } else {
      u--;
      if (u == 0) { L.n = 0; L.n16 = k; R.n16 = P.n16 - k; done = true; }
    }
  }
  if (!done) {
    const uint32_t nb = body16(P);
    if (u <= nb) {
      int split = 0;
      const uint64_t b = utf8_unit_offset(c, P.off, P.n, u, &split);
      L.n = (uint32_t)b;
      L.hi = split ? 1 : 0;
      L.n16 = k;
      R.off = P.off + b + (split ? 4 : 0);
      R.n = P.n - (uint32_t)b - (split ? 4 : 0);
      R.lo = split ? 1 : 0;
      R.n16 = P.n16 - k;
    } else {  // past the body: in the trailing high half / U+FFFD
      u -= nb;
      L.n16 = k;
      R.off = P.off + P.n;
      R.n = 0;
      R.n16 = P.n16 - k;
      if (P.hi && u >= 1) { L.hi = 1; u--; R.hi = 0; } else { R.hi = P.hi; }
      R.tfffd = P.tfffd;
      (void)u;
    }
  }
}
// splits piece q at unit k (0 < k < n16): q keeps [0, k), the new piece (returned, linked after q) [k, n16)
YM_HOT int32_t piece_cut_str(Doc &d, int32_t q, uint32_t k) {
  const int32_t r = new_piece(d);
  if (r == NIL) return NIL;
  Piece L, R;
  piece_split_str(*d.c, d.pc[q], k, L, R);
  R.next = d.pc[q].next;
  L.next = r;
  d.pc[q] = L;
  d.pc[r] = R;
  return r;
}
YM_INL int32_t piece_cut_arr(Doc &d, int32_t q, uint32_t k) {
  const int32_t r = new_piece(d);
  if (r == NIL) return NIL;
  Piece &P = d.pc[q];
  Piece &R = d.pc[r];
  R = P;
  R.off = P.off + k;
  R.n = R.n16 = P.n - k;
  P.n = P.n16 = k;
  P.next = r;
  return r;
}
// drops the first unit of string piece q
YM_INL void piece_drop_first(Doc &d, int32_t q) {
  Piece &p = d.pc[q];
  if (p.fffd) p.fffd = 0;
  else if (p.lo) p.lo = 0;
  else if (p.n > 0) {
    const uint8_t b = d.c->A[p.off];
    const uint32_t L = b < 0x80 ? 1 : (b & 0xE0) == 0xC0 ? 2 : (b & 0xF0) == 0xE0 ? 3 : 4;
    if (L == 4) { p.lo = 1; }  // the high half goes: the low half stays, as a lone unit
    p.off += L;
    p.n -= L;
  } else if (p.hi) p.hi = 0;
  else if (p.tfffd) p.tfffd = 0;
  p.n16--;
}
// content.splice(diff) of item l into the new item r (ContentString.js:51-66, ContentAny / ContentJSON
// slicing, ContentDeleted length); other contents cannot be split
YM_HOT void content_split(Doc &d, int32_t l, int32_t r, int64_t diff) {
  Item &L = d.it[l];
  const uint8_t ref = L.ref;
  if (ref == 1) return;
  if (ref != 2 && ref != 4 && ref != 8) { seterr(*d.c, ST_METHOD); return; }
  // find the piece holding unit diff - 1 (the last unit of the left part)
  int32_t q = L.chead;
  int64_t before = 0;
  while (q != NIL && before + d.pc[q].n16 < diff) { before += d.pc[q].n16; q = d.pc[q].next; }
  if (q == NIL) { seterr(*d.c, ST_UNEXPECTED); return; }
  const uint32_t k = (uint32_t)(diff - before);
  int32_t rh;
  if (k < d.pc[q].n16) rh = ref == 4 ? piece_cut_str(d, q, k) : piece_cut_arr(d, q, k);
  else rh = d.pc[q].next;
  if (d.c->err) return;
  Item &L2 = d.it[l];
  Item &R = d.it[r];
  R.chead = rh;
  R.ctail = (rh == NIL) ? NIL : (q == L2.ctail ? rh : L2.ctail);
  L2.ctail = q;
  d.pc[q].next = NIL;
  if (ref == 4 && rh != NIL) {  // the left part ends with a high surrogate: both halves become U+FFFD
    Piece &P = d.pc[q];
    if (P.hi && !P.tfffd) {
      P.hi = 0;
      P.tfffd = 1;
      piece_drop_first(d, rh);
      d.pc[rh].fffd = 1;
      d.pc[rh].n16++;
    }
  }
}

// ---- items -------------------------------------------------------------------------------------------
YM_INL void ms_push(Doc &d, int32_t i) { vpush(*d.c, *d.ta, d.tx->ms, i); }
YM_INL int64_t tx_before_at(const Tx &t, uint32_t idx) { return idx < t.nbc ? t.bc[idx] : 0; }
YM_INL int64_t tx_before(Doc &d, const Tx &t, int64_t client) {
  const int32_t s = cd_client(d, client);
  return s != NIL ? tx_before_at(t, (uint32_t)s) : 0;
}
YM_INL void changed_add(Doc &d, int32_t t) {  // addChangedTypeToTransaction (Transaction.js:154-159)
  if (t == NIL) return;
  Tx &x = *d.tx;
  const int32_t ti = d.ty[t].item;
  if (ti != NIL && !(d.it[ti].clock < tx_before(d, x, d.it[ti].client) && !d.it[ti].deleted)) return;
  for (uint32_t i = 0; i < x.chg.n; i++)
    if (x.chg.p[i] == t) return;
  vpush(*d.c, *d.ta, x.chg, t);
}
YM_INL void changed_del(Doc &d, int32_t t) {
  Tx &x = *d.tx;
  for (uint32_t i = 0; i < x.chg.n; i++)
    if (x.chg.p[i] == t) { vremove(x.chg, i); return; }
}
// splitItem (Item.js:85-125)
YM_HOT int32_t split_item(Doc &d, int32_t l, int64_t diff) {
  const int32_t r = new_item(d);
  if (r == NIL) return NIL;
  Item &L = d.it[l];
  Item &R = d.it[r];
  R = L;
  R.clock = L.clock + diff;
  R.left = l;
  R.has_origin = 1;
  R.oc = L.client;
  R.ok = L.clock + diff - 1;
  R.right = L.right;
  R.len = L.len - diff;
  R.gen_before = R.gen_conf = 0;
  R.type = NIL;
  R.chead = R.ctail = NIL;
  content_split(d, l, r, diff);
  if (d.c->err) return NIL;
  Item &L2 = d.it[l];
  Item &R2 = d.it[r];
  L2.right = r;
  if (R2.right != NIL) d.it[R2.right].left = r;
  ms_push(d, r);
  if (R2.has_psub && R2.right == NIL) map_set(d, R2.parent, R2.psub, r);
  L2.len = diff;
  return r;
}
YM_INL int32_t get_clean_start(Doc &d, int64_t client, int64_t clock) {  // getItemCleanStart
  const int32_t s = cd_client(d, client);
  const uint32_t idx = find_index(d, s, clock);
  if (d.c->err) return NIL;
  const int32_t st = d.cl.p[s].a.p[idx];
  if (d.it[st].clock < clock && !d.it[st].gc) {
    const int32_t r = split_item(d, st, clock - d.it[st].clock);
    if (r == NIL) return NIL;
    vinsert(*d.c, *d.a, d.cl.p[s].a, idx + 1, r);
    return r;
  }
  return st;
}
YM_INL int32_t get_clean_end(Doc &d, int64_t client, int64_t clock) {  // getItemCleanEnd
  const int32_t s = cd_client(d, client);
  const uint32_t idx = find_index(d, s, clock);
  if (d.c->err) return NIL;
  const int32_t st = d.cl.p[s].a.p[idx];
  if (clock != d.it[st].clock + d.it[st].len - 1 && !d.it[st].gc) {
    const int32_t r = split_item(d, st, clock - d.it[st].clock + 1);
    if (r == NIL) return NIL;
    vinsert(*d.c, *d.a, d.cl.p[s].a, idx + 1, r);
  }
  return st;
}
YM_INL void mark_deleted(Doc &d, int32_t i) {
  Item &x = d.it[i];
  x.deleted = 1;
  tds_add(d, d.tx->ds, x.client, x.clock, x.len);
  changed_add(d, d.it[i].parent);
}
// Item.delete (Item.js) with ContentType.delete's walk over the type's children (ContentType.js:101-125),
// depth-first in the reference's order on an explicit stack
struct DelFrame { int32_t t, cur; uint32_t mi; uint32_t phase; };
YM_HOT void it_delete(Doc &d, int32_t root) {
  Ctx &c = *d.c;
  if (d.it[root].deleted) return;
  mark_deleted(d, root);
  if (!(d.it[root].ref == 7 && d.it[root].type != NIL)) return;
  Vec<DelFrame> st = {nullptr, 0, 0};
  DelFrame f0 = {d.it[root].type, d.ty[d.it[root].type].start, 0, 0};
  if (!vpush(c, *d.a, st, f0)) return;
  while (st.n > 0 && !c.err) {
    DelFrame &f = st.p[st.n - 1];
    int32_t y = NIL;
    if (f.phase == 0) {
      if (f.cur != NIL) { y = f.cur; f.cur = d.it[y].right; }
      else f.phase = 1;
    }
    if (y == NIL && f.phase == 1) {
      const Type &T = d.ty[f.t];
      if (f.mi < T.mv.n) y = T.mv.p[f.mi++];
      else { changed_del(d, f.t); st.n--; continue; }
    }
    if (d.it[y].deleted) { ms_push(d, y); continue; }
    mark_deleted(d, y);
    if (d.it[y].ref == 7 && d.it[y].type != NIL) {
      DelFrame g = {d.it[y].type, d.ty[d.it[y].type].start, 0, 0};
      vpush(c, *d.a, st, g);
    }
  }
}
YM_INL void cd_replace(Doc &d, int32_t old, int32_t nw) {  // replaceStruct
  const int32_t s = cd_client(d, d.it[old].client);
  const uint32_t i = find_index(d, s, d.it[old].clock);
  if (!d.c->err) d.cl.p[s].a.p[i] = nw;
}
YM_INL int32_t new_gc(Doc &d, int64_t client, int64_t clock, int64_t len) {
  const int32_t g = new_item(d);
  if (g == NIL) return NIL;
  Item &x = d.it[g];
  x.gc = 1; x.client = client; x.clock = clock; x.len = len; x.deleted = 1;
  return g;
}
// Item.gc (Item.js) with ContentType.gc (ContentType.js:127-141): the type's children are replaced by GC
// structs (parentGCd); the item itself becomes ContentDeleted, or a GC when its parent was GC'd
YM_BIG void it_gc(Doc &d, int32_t root) {
  Ctx &c = *d.c;
  struct G { int32_t i; int32_t pgcd; };
  Vec<G> st = {nullptr, 0, 0};
  G g0 = {root, 0};
  if (!vpush(c, *d.a, st, g0)) return;
  while (st.n > 0 && !c.err) {
    const G g = st.p[--st.n];
    if (!d.it[g.i].deleted) { seterr(c, ST_UNEXPECTED); return; }
    if (d.it[g.i].ref == 7 && d.it[g.i].type != NIL) {
      const int32_t t = d.it[g.i].type;
      for (int32_t x = d.ty[t].start; x != NIL && !c.err; x = d.it[x].right) { G h = {x, 1}; vpush(c, *d.a, st, h); }
      d.ty[t].start = NIL;
      for (uint32_t k = 0; k < d.ty[t].mv.n && !c.err; k++)
        for (int32_t x = d.ty[t].mv.p[k]; x != NIL && !c.err; x = d.it[x].left) { G h = {x, 1}; vpush(c, *d.a, st, h); }
      d.ty[t].mk.n = d.ty[t].mv.n = 0;
    }
    if (g.pgcd) {
      if (d.it[g.i].gc) continue;
      const int32_t n = new_gc(d, d.it[g.i].client, d.it[g.i].clock, d.it[g.i].len);
      if (n != NIL) cd_replace(d, g.i, n);
    } else {
      Item &x = d.it[g.i];
      x.ref = 1;  // ContentDeleted(length)
      x.chead = x.ctail = NIL;
      x.src = NIL;
    }
  }
}

// Item.getMissing: the client of a missing dependency, or -1 (and left / right / parent resolved)
YM_HOT int64_t it_missing(Doc &d, int32_t i) {
  Item &x = d.it[i];
  if (x.gc) return -1;
  if (x.has_origin && x.oc != x.client && x.ok >= cd_state(d, x.oc)) return x.oc;
  if (x.has_right && x.rc != x.client && x.rk >= cd_state(d, x.rc)) return x.rc;
  if (x.pkind == 2 && x.client != x.pc && x.pk >= cd_state(d, x.pc)) return x.pc;
  if (x.has_origin) {
    const int32_t l = get_clean_end(d, x.oc, x.ok);
    if (l == NIL) return -1;
    Item &y = d.it[i];
    y.left = l;
    y.oc = d.it[l].client;
    y.ok = d.it[l].clock + d.it[l].len - 1;
  }
  if (d.it[i].has_right) {
    const int32_t r = get_clean_start(d, d.it[i].rc, d.it[i].rk);
    if (r == NIL) return -1;
    Item &y = d.it[i];
    y.right = r;
    y.rc = d.it[r].client;
    y.rk = d.it[r].clock;
  }
  Item &y = d.it[i];
  bool par_set = y.pkind != 0;  // `this.parent` truthy before the neighbour rules
  if ((y.left != NIL && d.it[y.left].gc) || (y.right != NIL && d.it[y.right].gc)) { par_set = false; y.parent = NIL; y.pkind = 0; }
  if (!par_set) {
    if (y.left != NIL && !d.it[y.left].gc) { const Item &l = d.it[y.left]; y.parent = l.parent; y.has_psub = l.has_psub; y.psub = l.psub; }
    if (y.right != NIL && !d.it[y.right].gc) { const Item &r = d.it[y.right]; y.parent = r.parent; y.has_psub = r.has_psub; y.psub = r.psub; }
  } else if (y.pkind == 2) {
    const int32_t p = cd_get(d, y.pc, y.pk);
    if (p == NIL) return -1;
    d.it[i].parent = (!d.it[p].gc && d.it[p].ref == 7) ? d.it[p].type : NIL;  // a GC'd parent, or no type: GC
  }
  return -1;
}
YM_INL bool id_eq(uint8_t ha, int64_t ac, int64_t ak, uint8_t hb, int64_t bc, int64_t bk) {
  return ha == hb && (!ha || (ac == bc && ak == bk));
}
// Item.integrate (Item.js:403-517) / GC.integrate
YM_HOT void it_integrate(Doc &d, int32_t i, int64_t off) {
  Ctx &c = *d.c;
  if (d.it[i].gc) {
    if (off > 0) { d.it[i].clock += off; d.it[i].len -= off; }
    add_struct(d, i);
    return;
  }
  if (off > 0) {
    d.it[i].clock += off;
    const int32_t l = get_clean_end(d, d.it[i].client, d.it[i].clock - 1);
    if (l == NIL) return;
    Item &x = d.it[i];
    x.left = l;
    x.oc = d.it[l].client;
    x.ok = d.it[l].clock + d.it[l].len - 1;
    x.has_origin = 1;
    // content.splice(offset): the item keeps the right part
    const int32_t tmp = new_item(d);
    if (tmp == NIL) return;
    d.it[tmp].ref = d.it[i].ref;
    d.it[tmp].chead = d.it[i].chead;
    d.it[tmp].ctail = d.it[i].ctail;
    d.it[tmp].len = d.it[i].len;
    content_split(d, tmp, i, off);
    if (c.err) return;
    if (d.it[i].ref == 1) { d.it[i].chead = d.it[i].ctail = NIL; }
    d.it[i].len -= off;
  }
  if (d.it[i].parent == NIL) {  // parent is not defined: integrate a GC struct instead
    const int32_t g = new_gc(d, d.it[i].client, d.it[i].clock, d.it[i].len);
    if (g != NIL) add_struct(d, g);
    return;
  }
  const int32_t P = d.it[i].parent;
  // 13.4.9 with a GC on the left (getClean* on a GC id; a parent from the right neighbour, Item.js:375-387,
  // or the own-client predecessor of an offset): a GC has no `right`, undefined !== this.right, so the
  // conflict scan starts at o = undefined and reads o.origin (Item.js:413, 425, 450)
  if (d.it[i].left != NIL && d.it[d.it[i].left].gc) { seterr(c, st_d(ST_TYPE, D_ORIGIN_UNDEF)); return; }
  {
    Item &x = d.it[i];
    if ((x.left == NIL && (x.right == NIL || d.it[x.right].left != NIL)) || (x.left != NIL && d.it[x.left].right != x.right)) {
      int32_t left = x.left, o;
      if (left != NIL) o = d.it[left].right;
      else if (x.has_psub) {
        o = map_get(d, P, x.psub);
        while (o != NIL && d.it[o].left != NIL) o = d.it[o].left;
      } else {
        o = d.ty[P].start;
      }
      const uint32_t gb = ++d.gen;
      uint32_t gcf = ++d.gen;
      while (o != NIL && o != d.it[i].right && !c.err) {
        Item &ob = d.it[o];
        ob.gen_before = gb;
        ob.gen_conf = gcf;
        const Item &xi = d.it[i];
        if (id_eq(xi.has_origin, xi.oc, xi.ok, ob.has_origin, ob.oc, ob.ok)) {
          if (ob.client < xi.client) { left = o; gcf = ++d.gen; }
          else if (id_eq(xi.has_right, xi.rc, xi.rk, ob.has_right, ob.rc, ob.rk)) break;
        } else if (ob.has_origin) {
          const int32_t oo = cd_get(d, ob.oc, ob.ok);
          if (oo == NIL) { seterr(c, ST_UNEXPECTED); return; }  // (unreachable: an integrated origin is stored)
          if (d.it[oo].gen_before == gb) {
            if (d.it[oo].gen_conf != gcf) { left = o; gcf = ++d.gen; }
          } else {
            break;
          }
        } else {
          break;
        }
        o = d.it[o].right;
      }
      d.it[i].left = left;
    }
  }
  Item &x = d.it[i];
  if (x.left != NIL) {
    x.right = d.it[x.left].right;
    d.it[x.left].right = i;
  } else {
    int32_t r;
    if (x.has_psub) {
      r = map_get(d, P, x.psub);
      while (r != NIL && d.it[r].left != NIL) r = d.it[r].left;
    } else {
      r = d.ty[P].start;
      d.ty[P].start = i;
    }
    x.right = r;
  }
  if (d.it[i].right != NIL) {
    d.it[d.it[i].right].left = i;
  } else if (d.it[i].has_psub) {
    map_set(d, P, d.it[i].psub, i);
    if (d.it[i].left != NIL) it_delete(d, d.it[i].left);
  }
  add_struct(d, i);
  if (c.err) return;
  if (d.it[i].ref == 7) {  // type._integrate
    const int32_t t = new_type(d);
    if (t == NIL) return;
    d.it[i].type = t;
    d.ty[t].item = i;
    d.ty[t].tref = (int32_t)d.src[d.it[i].src].cnt;
  }
  if (d.it[i].ref == 1) {  // ContentDeleted.integrate
    tds_add(d, d.tx->ds, d.it[i].client, d.it[i].clock, d.it[i].len);
    d.it[i].deleted = 1;
  }
  changed_add(d, P);
  const int32_t pi = d.ty[P].item;
  if ((pi != NIL && d.it[pi].deleted) || (d.it[i].has_psub && d.it[i].right != NIL)) it_delete(d, i);
}

// ---- pending structs ---------------------------------------------------------------------------------
// d.pend is kept sorted by client (one entry per client): the reference's Map is only ever read in that
// order (resumeStructIntegration sorts its keys), so lookups are a binary search and the sort is free
YM_INL uint32_t pend_lb(const Doc &d, int64_t client) {
  uint32_t lo = 0, hi = d.pend.n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    if (d.pend.p[mid].client < client) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
YM_INL int32_t cd_pend(Doc &d, int64_t client) {
  const uint32_t i = pend_lb(d, client);
  return i < d.pend.n && d.pend.p[i].live && d.pend.p[i].client == client ? (int32_t)i : NIL;
}
YM_INL void refs_sort(Doc &d, int32_t *a, uint32_t n) {  // stable sort by clock (V8's sort is stable)
  for (uint32_t i = 1; i < n; i++) {
    const int32_t v = a[i];
    uint32_t j = i;
    while (j > 0 && d.it[a[j - 1]].clock > d.it[v].clock) { a[j] = a[j - 1]; j--; }
    a[j] = v;
  }
}
// resumeStructIntegration (encoding.js:225-321)
YM_HOT void resume_integration(Doc &d) {
  Ctx &c = *d.c;
  Arena &A = *d.a;
  Arena &T = *d.ta;  // the state cache lives for this call only
  // the pending clients in ascending order are d.pend itself (sorted by client, every entry live, not
  // reordered here): the target is the last entry not yet exhausted
  uint32_t nids = d.pend.n;
  if (nids == 0) return;
  int32_t cur = NIL;
  auto next_target = [&]() {
    cur = (int32_t)(nids - 1);
    while (cur != NIL && d.pend.p[cur].n == d.pend.p[cur].i) {
      nids--;
      if (nids > 0) cur = (int32_t)(nids - 1);
      else { d.pend.n = 0; cur = NIL; break; }
    }
  };
  next_target();
  if (cur == NIL && d.stack.n == 0) return;
  int32_t head;
  if (d.stack.n > 0) head = d.stack.p[--d.stack.n];
  else head = d.pend.p[cur].refs[d.pend.p[cur].i++];
  Vec<int64_t> scc = {nullptr, 0, 0}, sck = {nullptr, 0, 0};  // state cache: client, clock
  while (!c.err) {
    const int64_t hc = d.it[head].client;
    int64_t local = -1;
    for (uint32_t i = 0; i < scc.n; i++)
      if (scc.p[i] == hc) { local = sck.p[i]; break; }
    if (local < 0) {
      local = cd_state(d, hc);
      vpush(c, T, scc, hc);
      vpush(c, T, sck, local);
    }
    const int64_t off = d.it[head].clock < local ? local - d.it[head].clock : 0;
    if (d.it[head].clock + off != local) {
      const int32_t sr = cd_pend(d, hc);
      if (sr != NIL && d.pend.p[sr].n != d.pend.p[sr].i) {
        Pend &P = d.pend.p[sr];
        const int32_t r = P.refs[P.i];
        if (d.it[r].clock < d.it[head].clock) {
          P.refs[P.i] = head;
          head = r;
          const uint32_t rn = P.n - P.i;
          int32_t *na = (int32_t *)aalloc(c, A, 4ull * (rn + 1));
          if (!na) return;
          Pend &P2 = d.pend.p[sr];
          for (uint32_t k = 0; k < rn; k++) na[k] = P2.refs[P2.i + k];
          refs_sort(d, na, rn);
          P2.refs = na; P2.n = rn; P2.i = 0;
          continue;
        }
      }
      vpush(c, A, d.stack, head);
      return;
    }
    const int64_t missing = it_missing(d, head);
    if (c.err) return;
    if (missing < 0) {
      if (off == 0 || off < d.it[head].len) {
        it_integrate(d, head, off);
        if (c.err) return;
        for (uint32_t i = 0; i < scc.n; i++)
          if (scc.p[i] == d.it[head].client) sck.p[i] = d.it[head].clock + d.it[head].len;
      }
      if (d.stack.n > 0) head = d.stack.p[--d.stack.n];
      else if (cur != NIL && d.pend.p[cur].i < d.pend.p[cur].n) head = d.pend.p[cur].refs[d.pend.p[cur].i++];
      else {
        next_target();
        if (cur == NIL) break;
        head = d.pend.p[cur].refs[d.pend.p[cur].i++];
      }
    } else {
      const int32_t sr = cd_pend(d, missing);
      if (sr == NIL || d.pend.p[sr].n == d.pend.p[sr].i) {
        vpush(c, A, d.stack, head);
        return;
      }
      vpush(c, A, d.stack, head);
      head = d.pend.p[sr].refs[d.pend.p[sr].i++];
    }
  }
  d.pend.n = 0;
}

// readAndApplyDeleteSet over decoded ranges (DeleteSet.js:270-323); unapplied ranges become a pending
// delete reader, appended to d.pdel, or written at `slot` (the re-read reader's own position, a hole before).
// A pending reader none of whose ranges starts below its client's state would come back range for range (its
// ranges have made writeDeleteSet's round trip once already), so the caller re-reads only readers with such a
// range (tryResumePendingDeleteReaders, cd_transact).  An unapplied range of length 0 (a V1 delete set may hold
// one) sets *zero: the reference's writeDeleteSet of the unapplied set throws at it (DSEncoderV2.writeDsLen,
// UpdateEncoder.js:255-258), after every client of the update's delete set has been read and applied.
YM_HOT void apply_ds(Doc &d, const DSet &ds, bool *zero = nullptr, uint32_t slot = 0xffffffffu) {
  Ctx &c = *d.c;
  DSet un = {{nullptr, 0, 0}, d.ta};
  for (uint32_t ci = 0; ci < ds.cl.n && !c.err; ci++) {
    const int64_t client = ds.cl.p[ci].client;
    const int32_t s = cd_client(d, client);
    const int64_t state = cd_state(d, client);
    for (uint32_t k = 0; k < ds.cl.p[ci].it.n && !c.err; k++) {
      const int64_t clock = ds.cl.p[ci].it.p[k].clock, end = clock + ds.cl.p[ci].it.p[k].len;
      if (clock < state) {
        if (state < end) tds_add(d, un, client, state, end - state);
        uint32_t idx = find_index(d, s, clock);
        if (c.err) return;
        int32_t st = d.cl.p[s].a.p[idx];
        if (!d.it[st].deleted && d.it[st].clock < clock) {
          const int32_t r = split_item(d, st, clock - d.it[st].clock);
          if (r == NIL) return;
          vinsert(c, *d.a, d.cl.p[s].a, idx + 1, r);
          idx++;
        }
        while (idx < d.cl.p[s].a.n && !c.err) {
          st = d.cl.p[s].a.p[idx++];
          if (d.it[st].clock < end) {
            if (!d.it[st].deleted) {
              if (end < d.it[st].clock + d.it[st].len) {
                const int32_t r = split_item(d, st, end - d.it[st].clock);
                if (r == NIL) return;
                vinsert(c, *d.a, d.cl.p[s].a, idx, r);
              }
              it_delete(d, st);
            }
          } else {
            break;
          }
        }
      } else {
        tds_add(d, un, client, clock, end - clock);
      }
    }
  }
  if (c.err || un.cl.n == 0) return;
  // the reader pushed is a DSDecoderV2 over writeDeleteSet(DSEncoderV2, unappliedDS) (DeleteSet.js:317-321):
  // per client the clock is written as a delta to the previous range's end and the length as len - 1, both
  // by writeVarUint, which writes a negative value as its low 7 bits.  Ranges sorted, disjoint and non-empty
  // (what yjs writes) come back unchanged; the others come back as that round trip makes them.  The
  // transient reader moves to the persistent arena.
  DSet keep = {{nullptr, 0, 0}, nullptr};
  if (!vgrow(c, *d.a, keep.cl, un.cl.n)) return;
  for (uint32_t k = 0; k < un.cl.n; k++) {
    DCl z = {un.cl.p[k].client, {nullptr, 0, 0}};
    if (!vgrow(c, *d.a, z.it, un.cl.p[k].it.n)) return;
    int64_t enc = 0, dec = 0;
    for (uint32_t q = 0; q < un.cl.p[k].it.n; q++) {
      const DIt r = un.cl.p[k].it.p[q];
      if (r.len == 0 && zero) *zero = true;
      const int64_t dc = r.clock - enc, dl = r.len - 1;
      enc = r.clock + r.len;
      dec += dc > 127 ? dc : (dc & 127);
      const int64_t len = (dl > 127 ? dl : (dl & 127)) + 1;
      z.it.p[q] = {dec, len};
      dec += len;
    }
    z.it.n = un.cl.p[k].it.n;
    keep.cl.p[keep.cl.n++] = z;
  }
  if (slot == 0xffffffffu) {
    slot = d.pdel.n;
    if (!vpush(c, *d.a, d.pdel, keep)) return;
  } else {
    d.pdel.p[slot] = keep;
  }
  pdel_watch(d, slot);
}

// ---- reading -----------------------------------------------------------------------------------------
// one struct's content into item i (readItemContent, Item.js:665-683): strings as a piece, Any / JSON as
// element ranges, the single-valued contents as a source record
YM_HOT void read_item_content(Doc &d, Reader &r, int32_t i, int info) {
  Ctx &c = *d.c;
  SStruct s;
  __builtin_memset(&s, 0, sizeof(SStruct));
  read_content(c, r, s, info);
  if (c.err) return;
  Item &x = d.it[i];
  x.ref = s.ref;
  x.len = s.len;
  switch (s.ref) {
    case 1: break;
    case 4: {
      const int32_t q = new_piece(d);
      if (q == NIL) return;
      Piece &p = d.pc[q];
      p.off = s.a.off; p.n = s.a.n; p.n16 = s.a.n16; p.fffd = s.a.fffd; p.lo = s.a.lo; p.hi = s.a.hi;
      d.it[i].chead = d.it[i].ctail = q;
      break;
    }
    case 2: case 8: {
      const uint32_t e0 = d.nel;
      if (d.nel + (uint64_t)s.cnt > d.capel) { seterr(c, ST_RETRY); return; }
      uint64_t p = s.a.off;
      UOptCol ls = s.lsnap;
      for (int64_t k = 0; k < s.cnt && !c.err; k++) {
        Elem &e = d.el[d.nel++];
        __builtin_memset(&e, 0, sizeof(Elem));
        if (s.ref == 8) {
          Rd rd = {p, s.a.off + s.a.n - p, 0};
          int nc = 0;
          any_skip(c, rd, &nc);
          e.off = p; e.n = (uint32_t)rd.pos; e.nc = s.nca && nc;
          p += rd.pos;
        } else {
          if (s.lsb) {  // V2: lengths from the string-length column snapshot
            const uint32_t L = uopt_read(c, ls);
            int split = 0;
            e.off = p;
            e.n = (uint32_t)utf8_unit_offset(c, p, s.a.off + s.a.n - p, L, &split);
            e.n16 = L;
          } else {
            Rd rd = {p, s.a.off + s.a.n - p, 0};
            const uint32_t L = rd_vu(c, rd);
            e.off = p + rd.pos;
            e.n = L;
            uint32_t n16 = 0;
            utf8_check(c, e.off, e.n, &n16);
            e.n16 = n16;
          }
          e.undef = e.n == 9 && c.A[e.off] == 'u' && c.A[e.off + 1] == 'n' && c.A[e.off + 2] == 'd' &&
                    c.A[e.off + 3] == 'e' && c.A[e.off + 4] == 'f' && c.A[e.off + 5] == 'i' &&
                    c.A[e.off + 6] == 'n' && c.A[e.off + 7] == 'e' && c.A[e.off + 8] == 'd';
          if (s.nca && !e.undef) {
            int nc = 0;
            json_check(c, e.off, e.n, &nc);
            e.nc = nc != 0;
          }
          p = e.off + e.n;
        }
      }
      if (s.cnt > 0) {
        const int32_t q = new_piece(d);
        if (q == NIL) return;
        d.pc[q].off = e0;
        d.pc[q].n = d.pc[q].n16 = (uint32_t)s.cnt;
        d.it[i].chead = d.it[i].ctail = q;
      }
      break;
    }
    default: {
      if (d.nsrc >= d.capsrc) { seterr(c, ST_RETRY); return; }
      Src &z = d.src[d.nsrc];
      z.a = s.a; z.b = s.b; z.cnt = s.cnt; z.nca = s.nca; z.ncb = s.ncb; z.keyundef = s.keyundef; z.ref = s.ref;
      z.fv_done = 0;
      d.it[i].src = (int32_t)d.nsrc++;
      break;
    }
  }
}
// readClientsStructRefs (encoding.js:127-198): per section a ref list; a repeated client replaces the
// earlier list (Map.set); info & 31 == 0 is a GC
YM_HOT void read_refs(Doc &d, Reader &r, Vec<Pend> &out) {
  Ctx &c = *d.c;
  const uint32_t nsec = rd_vu(c, r.rest);
  for (uint32_t si = 0; si < nsec && !c.err; si++) {
    const uint32_t ns = rd_vu(c, r.rest);
    const int64_t client = r.v2 ? (int64_t)uopt_read(c, r.cl) : (int64_t)rd_vu(c, r.rest);
    int64_t clock = rd_vu(c, r.rest);
    if (c.err) return;
    int32_t *refs = (int32_t *)aalloc(c, *d.ta, 4ull * (ns + 1));  // (what stays pending moves to *d.a)
    if (!refs) return;
    for (uint32_t k = 0; k < ns && !c.err; k++) {
      const int info = r.v2 ? rle_read(c, r.in) : rbyte(c, r.rest);
      const int32_t i = new_item(d);
      if (i == NIL) return;
      d.it[i].client = client;
      d.it[i].clock = clock;
      if ((info & 31) != 0) {
        const bool cant_copy = (info & 0xC0) == 0;
        if (info & 0x80) { d.it[i].has_origin = 1; rd_left(c, r, d.it[i].oc, d.it[i].ok); }
        if (info & 0x40) { d.it[i].has_right = 1; rd_right(c, r, d.it[i].rc, d.it[i].rk); }
        if (cant_copy) {
          const bool ykey = r.v2 ? rle_read(c, r.pi) == 1 : rd_vu(c, r.rest) == 1;
          if (ykey) {
            d.it[i].pkind = 1;
            d.it[i].pkey = rd_string(c, r);
            if (c.err) return;
            d.it[i].parent = cd_root(d, d.it[i].pkey);
          } else {
            d.it[i].pkind = 2;
            rd_left(c, r, d.it[i].pc, d.it[i].pk);
          }
          if (info & 0x20) { d.it[i].has_psub = 1; d.it[i].psub = rd_string(c, r); }
        }
        if (c.err) return;
        if ((info & 31) == 10) { seterr(c, st_d(ST_TYPE, D_CONTENT_REF)); return; }  // contentRefs[10]: undefined (13.4.9)
        read_item_content(d, r, i, info);
      } else {
        d.it[i].gc = 1;
        d.it[i].deleted = 1;
        d.it[i].len = rd_len(c, r);
      }
      refs[k] = i;
      clock += d.it[i].len;
    }
    uint32_t at = out.n;
    for (uint32_t q = 0; q < out.n; q++)
      if (out.p[q].client == client) at = q;
    Pend p = {client, refs, ns, 0, 1};
    if (at == out.n) vpush(c, *d.ta, out, p);
    else out.p[at] = p;
  }
}

// ---- transactions ------------------------------------------------------------------------------------
YM_INL Tx *tx_new(Doc &d, uint8_t local) {  // new Transaction: beforeState = getStateVector(store)
  Ctx &c = *d.c;
  Tx *t = (Tx *)aalloc(c, *d.ta, sizeof(Tx));
  if (!t) return nullptr;
  __builtin_memset(t, 0, sizeof(Tx));
  t->ds.ar = d.ta;
  t->local = local;
  t->nbc = d.cl.n;
  t->bc = (int64_t *)aalloc(c, *d.ta, 8ull * (d.cl.n + 1));
  if (!t->bc) return nullptr;
  for (uint32_t i = 0; i < d.cl.n; i++) t->bc[i] = cl_state(d, (int32_t)i);
  return t;
}
// tryToMergeWithLeft (Transaction.js:165-176) with Item.mergeWith / AbstractContent.mergeWith
YM_HOT void try_merge_left(Doc &d, int32_t s, uint32_t pos) {
  const int32_t l = d.cl.p[s].a.p[pos - 1], r = d.cl.p[s].a.p[pos];
  Item &L = d.it[l];
  const Item &R = d.it[r];
  if (L.deleted != R.deleted || L.gc != R.gc) return;
  bool ok;
  if (L.gc) {
    L.len += R.len;
    ok = true;
  } else {
    ok = id_eq(R.has_origin, R.oc, R.ok, 1, L.client, L.clock + L.len - 1) && L.right == r &&
         id_eq(L.has_right, L.rc, L.rk, R.has_right, R.rc, R.rk) && L.client == R.client && L.clock + L.len == R.clock &&
         L.deleted == R.deleted && L.ref == R.ref && (L.ref == 1 || L.ref == 2 || L.ref == 4 || L.ref == 8);
    if (ok) {
      if (L.ref != 1) {  // concatenation of the piece lists
        if (L.ctail != NIL) d.pc[L.ctail].next = R.chead;
        else L.chead = R.chead;
        if (R.ctail != NIL) L.ctail = R.ctail;
      }
      L.right = R.right;
      if (L.right != NIL) d.it[L.right].left = l;
      L.len += R.len;
    }
  }
  if (ok) {
    vremove(d.cl.p[s].a, pos);
    const Item &R2 = d.it[r];
    if (!R2.gc && R2.has_psub && R2.parent != NIL && map_get(d, R2.parent, R2.psub) == r) map_set(d, R2.parent, R2.psub, l);
  }
}

// ---- YText's remote formatting cleanup (YText.js:348-437, 803-856) ---------------------------------------
// the value of format item i (ContentFormat.value): V1 JSON.parse of its text (compared through the
// canonical text), V2 readAny; objects by identity
YM_BIG FVal fval_compute(Doc &d, int32_t i) {
  Ctx &c = *d.c;
  FVal v;
  __builtin_memset(&v, 0, sizeof(FVal));
  const Src &z = d.src[d.it[i].src];
  v.ident = d.it[i].src;
  if (!d.v2) {
    const uint8_t *p = c.A + z.b.off;
    uint32_t n = z.b.n;
    if (z.ncb) {  // the canonical text, into the workspace
      const uint64_t q = js_ws(c.A, z.b.off, z.b.off + z.b.n);
      const SinkLen L = canon_len(c, c.A, q, z.b.off + z.b.n, G_JSON, T_JSON);
      uint8_t *buf = (uint8_t *)aalloc(c, *d.a, L.bytes + 1);
      if (!buf) return v;
      Out o = {buf, 0};
      canon_out(c, o, c.A, q, z.b.off + z.b.n, G_JSON, T_JSON);
      p = buf;
      n = (uint32_t)o.n;
    }
    v.p = p;
    v.n = n;
    const uint8_t f = n ? p[0] : 'n';
    if (f == 'n') { v.t = FV_NULL; v.truthy = 0; }
    else if (f == 't' || f == 'f') { v.t = FV_BOOL; v.truthy = f == 't'; }
    else if (f == '"') { v.t = FV_STR; v.truthy = n > 2; }
    else if (f == '{' || f == '[') { v.t = FV_OBJ; v.truthy = 1; }
    else { v.t = FV_NUM; v.truthy = !(n == 1 && p[0] == '0'); }
    return v;
  }
  const uint8_t *p = c.A + z.b.off;
  v.p = p;
  v.n = z.b.n;
  switch (p[0]) {
    case 127: v.t = FV_UNDEF; break;
    case 126: v.t = FV_NULL; break;
    case 121: v.t = FV_BOOL; v.truthy = 0; break;
    case 120: v.t = FV_BOOL; v.truthy = 1; break;
    case 125: {  // varInt
      Rd r = {z.b.off + 1, z.b.n - 1, 0};
      const VI x = rd_vi(c, r);
      v.t = FV_NUM;
      v.num = x.neg ? -(double)x.mag : (double)x.mag;
      v.truthy = x.mag != 0;
      break;
    }
    case 124: {
      const uint32_t b = ((uint32_t)p[1] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 8) | p[4];
      float f;
      __builtin_memcpy(&f, &b, 4);
      v.t = FV_NUM;
      v.num = (double)f;
      v.truthy = !(v.num == 0 || v.num != v.num);
      break;
    }
    case 123: {
      uint64_t b = 0;
      for (int k = 1; k <= 8; k++) b = (b << 8) | p[k];
      double f;
      __builtin_memcpy(&f, &b, 8);
      v.t = FV_NUM;
      v.num = f;
      v.truthy = !(f == 0 || f != f);
      break;
    }
    case 122: {
      v.t = FV_BIG;
      v.p = p + 1;
      v.n = 8;
      for (int k = 1; k <= 8; k++) v.truthy |= p[k] != 0;
      break;
    }
    case 119: {  // string: its UTF-8 bytes
      Rd r = {z.b.off + 1, z.b.n - 1, 0};
      const uint32_t L = rd_vu(c, r);
      v.t = FV_STR;
      v.p = c.A + z.b.off + 1 + r.pos;
      v.n = L;
      v.truthy = L != 0;
      break;
    }
    default: v.t = FV_OBJ; v.truthy = 1; break;
  }
  return v;
}
YM_INL FVal fval_of(Doc &d, int32_t i) {
  Src &z = d.src[d.it[i].src];
  if (!z.fv_done) { z.fv = fval_compute(d, i); z.fv_done = 1; }
  return z.fv;
}
// (x || null) === v: x an attribute value (nullptr: absent), v a ContentFormat's value
YM_INL bool or_null_eq(const FVal *x, const FVal &v, uint32_t v2) {
  if (x == nullptr || !x->truthy) return v.t == FV_NULL;
  if (x->t != v.t) return false;
  if (x->t == FV_OBJ) return x->ident == v.ident;
  if (v2 && x->t == FV_NUM) return x->num == v.num;
  if (v2 && x->t == FV_BOOL) return x->truthy == v.truthy;
  if (x->n != v.n) return false;
  for (uint32_t k = 0; k < x->n; k++)
    if (x->p[k] != v.p[k]) return false;
  return true;
}
YM_INL FVal *am_get(Doc &d, Vec<AttrE> &m, const Span &k) {
  for (uint32_t i = 0; i < m.n; i++)
    if (str_eq(*d.c, m.p[i].key, k)) return &m.p[i].v;
  return nullptr;
}
YM_INL void am_set(Doc &d, Vec<AttrE> &m, const Span &k, const FVal &v) {
  FVal *x = am_get(d, m, k);
  if (x) { *x = v; return; }
  AttrE e = {k, v};
  vpush(*d.c, *d.a, m, e);
}
YM_INL void am_del(Doc &d, Vec<AttrE> &m, const Span &k) {
  for (uint32_t i = 0; i < m.n; i++)
    if (str_eq(*d.c, m.p[i].key, k)) { m.p[i] = m.p[m.n - 1]; m.n--; return; }
}
YM_INL void am_copy(Doc &d, Vec<AttrE> &dst, const Vec<AttrE> &src) {
  dst.n = 0;
  if (!vgrow(*d.c, *d.a, dst, src.n)) return;
  for (uint32_t i = 0; i < src.n; i++) dst.p[i] = src.p[i];
  dst.n = src.n;
}
YM_INL void am_update(Doc &d, Vec<AttrE> &m, int32_t f) {  // updateCurrentAttributes (YText.js:182-189)
  const FVal v = fval_of(d, f);
  const Span &k = d.src[d.it[f].src].a;
  if (v.t == FV_NULL) am_del(d, m, k);
  else am_set(d, m, k, v);
}
YM_INL bool is_text(const Doc &d, int32_t i) { return d.it[i].ref == 4 || d.it[i].ref == 5; }
// cleanupFormattingGap (YText.js:348-374)
YM_BIG void cleanup_gap(Doc &d, int32_t start, int32_t end, Vec<AttrE> &sa, Vec<AttrE> &ea) {
  while (end != NIL && !is_text(d, end) && !d.c->err) {
    if (!d.it[end].deleted && d.it[end].ref == 6) am_update(d, ea, end);
    end = d.it[end].right;
  }
  while (start != end && start != NIL && !d.c->err) {
    if (!d.it[start].deleted && d.it[start].ref == 6) {
      const FVal v = fval_of(d, start);
      const Span &k = d.src[d.it[start].src].a;
      if (!or_null_eq(am_get(d, ea, k), v, d.v2) || or_null_eq(am_get(d, sa, k), v, d.v2)) it_delete(d, start);
    }
    start = d.it[start].right;
  }
}
YM_BIG void cleanup_ytext(Doc &d, int32_t t) {  // cleanupYTextFormatting (YText.js:412-437)
  int32_t start = d.ty[t].start, end = d.ty[t].start;
  Vec<AttrE> sa = {nullptr, 0, 0}, cur = {nullptr, 0, 0};
  while (end != NIL && !d.c->err) {
    if (!d.it[end].deleted) {
      if (d.it[end].ref == 6) am_update(d, cur, end);
      else if (is_text(d, end)) {
        cleanup_gap(d, start, end, sa, cur);
        am_copy(d, sa, cur);
        start = end;
      }
    }
    end = d.it[end].right;
  }
}
YM_BIG void cleanup_contextless(Doc &d, int32_t it) {  // cleanupContextlessFormattingGap (YText.js:380-398)
  while (it != NIL && d.it[it].right != NIL && (d.it[d.it[it].right].deleted || !is_text(d, d.it[it].right))) it = d.it[it].right;
  Vec<AttrE> seen = {nullptr, 0, 0};
  while (it != NIL && (d.it[it].deleted || !is_text(d, it)) && !d.c->err) {
    if (!d.it[it].deleted && d.it[it].ref == 6) {
      const Span &k = d.src[d.it[it].src].a;
      if (am_get(d, seen, k)) it_delete(d, it);
      else { FVal z; __builtin_memset(&z, 0, sizeof(FVal)); am_set(d, seen, k, z); }
    }
    it = d.it[it].left;
  }
}
struct ObsCb { int kind, found; int32_t t; };
YM_INL void obs_visit(Doc &d, ObsCb &cb, int32_t st) {
  const Item &x = d.it[st];
  switch (cb.kind) {
    case 0: if (!x.deleted && x.ref == 6) cb.found = 1; break;  // a new non-deleted format item
    case 1: if (!x.gc && !cb.found && x.parent == cb.t && x.ref == 6) cb.found = 1; break;
    case 2: if (!x.gc && x.parent == cb.t) cleanup_contextless(d, st); break;
  }
}
YM_INL uint32_t find_clean_start(Doc &d, int32_t s, int64_t clock) {  // findIndexCleanStart
  const uint32_t idx = find_index(d, s, clock);
  if (d.c->err) return 0;
  const int32_t st = d.cl.p[s].a.p[idx];
  if (d.it[st].clock < clock && !d.it[st].gc) {
    const int32_t r = split_item(d, st, clock - d.it[st].clock);
    if (r == NIL) return 0;
    vinsert(*d.c, *d.a, d.cl.p[s].a, idx + 1, r);
    return idx + 1;
  }
  return idx;
}
// iterateStructs (StructStore.js:259-273), splitting at both ends under d.tx
YM_HOT void iterate_structs(Doc &d, int32_t s, int64_t clock, int64_t len, ObsCb &cb) {
  if (len == 0 || s == NIL) return;
  const int64_t end = clock + len;
  uint32_t idx = find_clean_start(d, s, clock);
  do {
    if (d.c->err) return;
    const int32_t st = d.cl.p[s].a.p[idx++];
    if (end < d.it[st].clock + d.it[st].len) find_clean_start(d, s, end);
    obs_visit(d, cb, st);
  } while (idx < d.cl.p[s].a.n && d.it[d.cl.p[s].a.p[idx]].clock < end);
}
// iterateDeletedStructs (DeleteSet.js:58-65): the loops see entries appended while they run
YM_BIG void iterate_deleted(Doc &d, DSet &ds, ObsCb &cb) {
  for (uint32_t ci = 0; ci < ds.cl.n && !d.c->err; ci++)
    for (uint32_t k = 0; k < ds.cl.p[ci].it.n && !d.c->err; k++) {
      const DIt di = ds.cl.p[ci].it.p[k];
      iterate_structs(d, cd_client(d, ds.cl.p[ci].client), di.clock, di.len, cb);
    }
}
YM_BIG void ytext_observer(Doc &d, Tx *x, int32_t t, Tx **nested) {
  ObsCb cb = {0, 0, t};
  d.tx = x;
  for (uint32_t ci = 0; ci < d.cl.n && !cb.found && !d.c->err; ci++) {  // afterState, store order
    const int64_t before = tx_before_at(*x, ci), after = cl_state(d, (int32_t)ci);
    if (after == before) continue;
    iterate_structs(d, (int32_t)ci, before, after, cb);  // (len = afterClock, as the reference passes it)
  }
  if (!cb.found) { cb.kind = 1; iterate_deleted(d, x->ds, cb); }
  // transact(doc, ...): the first observer opens a local transaction; later observers join it
  if (!*nested) *nested = tx_new(d, 1);
  if (!*nested) return;
  d.tx = *nested;
  if (cb.found) cleanup_ytext(d, t);
  else { ObsCb c2 = {2, 0, t}; iterate_deleted(d, (*nested)->ds, c2); }
  d.tx = x;
}
// cleanupTransactions (Transaction.js:244-367) for one transaction; returns the one its observers opened
YM_HOT Tx *tx_cleanup(Doc &d, Tx *x) {
  Ctx &c = *d.c;
  d.tx = x;
  ds_sort_merge(x->ds);
  Tx *nested = nullptr;
  if (!x->local) {  // observers of the changed types, in Map order: only Y.Text / Y.XmlText act
    const uint32_t nchg = x->chg.n;
    int32_t *chg = (int32_t *)aalloc(c, *d.ta, 4ull * (nchg + 1));
    if (!chg) return nullptr;
    for (uint32_t i = 0; i < nchg; i++) chg[i] = x->chg.p[i];
    for (uint32_t i = 0; i < nchg && !c.err; i++) {
      const int32_t t = chg[i];
      const int32_t ti = d.ty[t].item;
      if (ti != NIL && d.it[ti].deleted) continue;
      if (d.ty[t].tref == 2 || d.ty[t].tref == 6) ytext_observer(d, x, t, &nested);
    }
  }
  d.tx = x;
  for (uint32_t ci = 0; ci < x->ds.cl.n && !c.err && !d.nogc; ci++) {  // tryGcDeleteSet (doc.gc, Transaction.js:302-304)
    const int32_t s = cd_client(d, x->ds.cl.p[ci].client);
    for (uint32_t k = x->ds.cl.p[ci].it.n; k-- > 0 && !c.err;) {
      const int64_t clock = x->ds.cl.p[ci].it.p[k].clock, end = clock + x->ds.cl.p[ci].it.p[k].len;
      for (uint32_t si = find_index(d, s, clock); !c.err && si < d.cl.p[s].a.n && d.it[d.cl.p[s].a.p[si]].clock < end; si++) {
        const int32_t st = d.cl.p[s].a.p[si];
        if (!d.it[st].gc && d.it[st].deleted) it_gc(d, st);
      }
    }
  }
  for (uint32_t ci = 0; ci < x->ds.cl.n && !c.err; ci++) {  // tryMergeDeleteSet
    const int32_t s = cd_client(d, x->ds.cl.p[ci].client);
    for (uint32_t k = x->ds.cl.p[ci].it.n; k-- > 0 && !c.err;) {
      const int64_t clock = x->ds.cl.p[ci].it.p[k].clock, len = x->ds.cl.p[ci].it.p[k].len;
      uint32_t mr = find_index(d, s, clock + len - 1) + 1;
      if (c.err) break;
      if (mr > d.cl.p[s].a.n - 1) mr = d.cl.p[s].a.n - 1;
      for (uint32_t si = mr; si > 0 && d.it[d.cl.p[s].a.p[si]].clock >= clock; si--) try_merge_left(d, s, si);
    }
  }
  for (uint32_t ci = 0; ci < d.cl.n && !c.err; ci++) {  // the clients whose state changed (afterState)
    const int64_t before = tx_before_at(*x, ci);
    if (before == cl_state(d, (int32_t)ci)) continue;
    uint32_t first = find_index(d, (int32_t)ci, before);
    if (c.err) break;
    if (first < 1) first = 1;
    for (uint32_t i = d.cl.p[ci].a.n - 1; i >= first && i > 0; i--) try_merge_left(d, (int32_t)ci, i);
  }
  for (uint32_t q = 0; q < x->ms.n && !c.err; q++) {  // _mergeStructs
    const int32_t m = x->ms.p[q];
    const int32_t s = cd_client(d, d.it[m].client);
    const uint32_t pos = find_index(d, s, d.it[m].clock);
    if (c.err) break;
    if (pos + 1 < d.cl.p[s].a.n) try_merge_left(d, s, pos + 1);
    if (pos > 0) try_merge_left(d, s, pos);
  }
  return nested;
}
// transact(readUpdateV2, local = false) + cleanupTransactions (encoding.js readUpdateV2)
YM_HOT void cd_transact(Doc &d, Reader &r) {
  Ctx &c = *d.c;
  Tx *x = tx_new(d, 0);
  if (!x) return;
  d.tx = x;
  Vec<Pend> refs = {nullptr, 0, 0};
  read_refs(d, r, refs);  // readStructs
  for (uint32_t q = 0; q < refs.n && !c.err; q++) {  // mergeReadStructsIntoPendingReads
    const int32_t p = cd_pend(d, refs.p[q].client);
    if (p == NIL) {
      vinsert(c, *d.a, d.pend, pend_lb(d, refs.p[q].client), refs.p[q]);
    } else {
      const uint32_t rn = d.pend.p[p].n - d.pend.p[p].i, m = refs.p[q].n;
      int32_t *na = (int32_t *)aalloc(c, *d.a, 4ull * (rn + m + 1));
      if (!na) return;
      for (uint32_t k = 0; k < rn; k++) na[k] = d.pend.p[p].refs[d.pend.p[p].i + k];
      for (uint32_t k = 0; k < m; k++) na[rn + k] = refs.p[q].refs[k];
      refs_sort(d, na, rn + m);
      d.pend.p[p].refs = na; d.pend.p[p].n = rn + m; d.pend.p[p].i = 0;
    }
  }
  if (c.err) return;
  resume_integration(d);
  {  // cleanupPendingStructs: the finished entries leave the Map; the rest keep their order
    uint32_t w = 0;
    for (uint32_t q = 0; q < d.pend.n; q++) {
      Pend p = d.pend.p[q];
      if (!p.live || p.i == p.n) continue;
      p.refs += p.i; p.n -= p.i; p.i = 0;
      if ((const uint8_t *)p.refs >= d.ta->base && (const uint8_t *)p.refs < d.ta->base + d.ta->cap) {
        int32_t *na = (int32_t *)aalloc(c, *d.a, 4ull * (p.n + 1));  // this update's refs outlive it
        if (!na) return;
        for (uint32_t k = 0; k < p.n; k++) na[k] = p.refs[k];
        p.refs = na;
      }
      d.pend.p[w++] = p;
    }
    d.pend.n = w;
  }
  if (d.awake.n) {  // tryResumePendingDeleteReaders: the awake readers re-read in order, each remainder in its
                    // reader's place (what a reader pushes now is re-read on the next update, as in the reference)
    const uint32_t n = d.awake.n;
    uint32_t *aw = (uint32_t *)aalloc(c, *d.ta, 4ull * n);
    if (!aw) return;
    for (uint32_t k = 0; k < n; k++) {  // insertion sort (a few positions per update)
      const uint32_t v = d.awake.p[k];
      uint32_t j = k;
      while (j > 0 && aw[j - 1] > v) { aw[j] = aw[j - 1]; j--; }
      aw[j] = v;
    }
    d.awake.n = 0;
    for (uint32_t k = 0; k < n && !c.err; k++) {
      const uint32_t q = aw[k];
      if (k > 0 && aw[k - 1] == q) continue;
      const DSet one = d.pdel.p[q];
      bool any = false;
      for (uint32_t ci = 0; ci < one.cl.n && !any; ci++) {
        const int64_t state = cd_state(d, one.cl.p[ci].client);
        for (uint32_t i = 0; i < one.cl.p[ci].it.n && !any; i++) any = one.cl.p[ci].it.p[i].clock < state;
      }
      if (!any) continue;  // (a hole, or a watcher of a replaced reader: nothing to apply)
      d.pdel.p[q].cl.n = 0;
      apply_ds(d, one, nullptr, q);
    }
  }
  {  // readAndApplyDeleteSet: each client's ranges are applied as read (the clients are independent)
    const uint32_t n = rd_vu(c, r.rest);
    bool zero = false;
    for (uint32_t i = 0; i < n && !c.err; i++) {
      r.dsCurr = 0;
      const int64_t client = rd_vu(c, r.rest);
      const uint32_t m = rd_vu(c, r.rest);
      DSet one = {{nullptr, 0, 0}, d.ta};  // read, applied, dropped
      const int32_t k = ds_get_or_add(d, one, client);
      if (k == NIL) return;
      for (uint32_t j = 0; j < m && !c.err; j++) {
        int64_t clock, len;
        if (r.v2) {  // DSDecoderV2: clock delta-coded, length - 1
          r.dsCurr += rd_vu(c, r.rest);
          clock = r.dsCurr;
          len = (int64_t)rd_vu(c, r.rest) + 1;
          r.dsCurr += len;
        } else {
          clock = rd_vu(c, r.rest);
          len = rd_vu(c, r.rest);
        }
        DIt e = {clock, len};
        vpush(c, *d.ta, one.cl.p[k].it, e);
      }
      if (!c.err) apply_ds(d, one, &zero);
    }
    if (zero && !c.err) seterr(c, ST_UNEXPECTED);
  }
  if (c.err) return;
  // cleanupTransactions: this one, then the one its observers opened (local: its observers do nothing)
  Tx *nested = tx_cleanup(d, x);
  if (nested && !c.err) tx_cleanup(d, nested);
  d.tx = nullptr;
}

// ---- writing -----------------------------------------------------------------------------------------
// ContentString.write of a piece list: V2 through the column's StringEncoder (lone halves pair up across
// strings), V1 writeVarString (a lone surrogate throws URIError)
// (first: the chain's first piece, possibly a local one linked into the document's list; nullptr: empty)
YM_INL const Piece *pnext(const Doc &d, const Piece *p) { return p->next == NIL ? nullptr : &d.pc[p->next]; }
YM_HOT void write_str(Ctx &c, Enc &e, const Doc &d, const Piece *first) {
  if (e.v2) {
    uint32_t n16 = 0;
    for (const Piece *pp = first; pp && !c.err; pp = pnext(d, pp)) {
      const Piece &p = *pp;
      const Span s = {p.off, p.n, 0, p.fffd, p.lo, p.hi, 0};
      e_str_bytes(e, c, s);
      if (p.tfffd) {
        if (e.pend_hi) { seterr(c, ST_URI); return; }
        o8(e.sb, 0xEF); o8(e.sb, 0xBF); o8(e.sb, 0xBD);
      }
      n16 += p.n16;
    }
    uopt_w(e.sl, e.sl_s, e.sl_n, n16);
    return;
  }
  uint64_t bytes = 0;
  bool pend = false;
  for (const Piece *pp = first; pp; pp = pnext(d, pp)) {
    const Piece &p = *pp;
    if (p.fffd) { if (pend) { seterr(c, ST_URI); return; } bytes += 3; }
    if (p.lo) { if (!pend) { seterr(c, ST_URI); return; } bytes += 4; pend = false; }
    if (pend && (p.n || p.hi || p.tfffd)) { seterr(c, ST_URI); return; }
    bytes += p.n;
    if (p.hi) pend = true;
    if (p.tfffd) { if (pend) { seterr(c, ST_URI); return; } bytes += 3; }
  }
  if (pend) { seterr(c, ST_URI); return; }
  ovu(e.rest, (int64_t)bytes);
  uint32_t hi = 0;
  for (const Piece *pp = first; pp; pp = pnext(d, pp)) {
    const Piece &p = *pp;
    if (p.fffd) { o8(e.rest, 0xEF); o8(e.rest, 0xBF); o8(e.rest, 0xBD); }
    if (p.lo) {
      const uint32_t cp = 0x10000 + ((hi - 0xD800) << 10) + (sur_lo(c, p.off - 4) - 0xDC00);
      o8(e.rest, 0xF0 | (cp >> 18)); o8(e.rest, 0x80 | ((cp >> 12) & 63)); o8(e.rest, 0x80 | ((cp >> 6) & 63)); o8(e.rest, 0x80 | (cp & 63));
    }
    ocopy(e.rest, c, p.off, p.n);
    if (p.hi) hi = sur_hi(c, p.off + p.n);
    if (p.tfffd) { o8(e.rest, 0xEF); o8(e.rest, 0xBF); o8(e.rest, 0xBD); }
  }
}
// Item.write / GC.write (Item.js:625-658, GC.js:45-48).  off > 0 (the first struct of a client written from
// a target state vector's clock, encoding.js:71-84): the origin becomes (client, clock + off - 1) and the
// content is written from unit off (ContentString str.slice(off), ContentAny / ContentJSON elements
// from off, ContentDeleted / GC len - off; other contents have length 1, so off is 0)
YM_HOT void item_write(Ctx &c, Enc &e, const Doc &d, int32_t i, int64_t off = 0) {
  const Item &x = d.it[i];
  if (x.gc) { e_info(e, 0); e_len(e, x.len - off); return; }
  const bool org = x.has_origin || off > 0;
  const int info = (x.ref & 31) | (org ? 0x80 : 0) | (x.has_right ? 0x40 : 0) | (x.has_psub ? 0x20 : 0);
  e_info(e, info);
  if (off > 0) e_left(e, x.client, x.clock + off - 1);
  else if (x.has_origin) e_left(e, x.oc, x.ok);
  if (x.has_right) e_right(e, x.rc, x.rk);
  if (!org && !x.has_right) {
    if (x.parent == NIL) { seterr(c, ST_UNEXPECTED); return; }
    const Type &P = d.ty[x.parent];
    if (P.item == NIL) { e_parent_info(e, 1); e_string(e, c, P.key); }
    else { e_parent_info(e, 0); e_left(e, d.it[P.item].client, d.it[P.item].clock); }
    if (x.has_psub) e_string(e, c, x.psub);
  }
  switch (x.ref) {
    case 1: e_len(e, x.len - off); break;
    case 4: {
      const Piece *first = x.chead == NIL ? nullptr : &d.pc[x.chead];
      Piece L, R;
      if (off > 0) {  // the piece holding unit off, cut there (the document's pieces stay as they are)
        uint32_t skip = (uint32_t)off;
        while (first && skip >= first->n16) { skip -= first->n16; first = pnext(d, first); }
        if (first && skip > 0) {
          piece_split_str(c, *first, skip, L, R);
          R.next = first->next;
          first = &R;
        }
      }
      write_str(c, e, d, first);
      break;
    }
    case 2: case 8: {
      e_len(e, x.len - off);
      uint64_t g = 0;  // element index within the content
      for (int32_t q = x.chead; q != NIL && !c.err; q = d.pc[q].next)
        for (uint32_t k = 0; k < d.pc[q].n && !c.err; k++, g++) {
          if ((int64_t)g < off) continue;
          const Elem &el = d.el[d.pc[q].off + k];
          if (x.ref == 8) {
            if (el.nc) canon_out(c, e.rest, c.A, el.off, el.off + el.n, G_ANY, T_ANY);
            else ocopy(e.rest, c, el.off, el.n);
          } else if (el.nc) {
            e_json_string(c, e, el.off, el.n);
          } else {
            const Span t = {el.off, el.n, el.n16, 0, 0, 0, 0};
            e_string(e, c, t);
          }
        }
      break;
    }
    default: {  // Binary, Embed, Format, Type, Doc: their source as read
      const Src &z = d.src[x.src];
      SStruct s;
      __builtin_memset(&s, 0, sizeof(SStruct));
      s.ref = z.ref; s.a = z.a; s.b = z.b; s.cnt = z.cnt; s.nca = z.nca; s.ncb = z.ncb; s.keyundef = z.keyundef;
      content_write(c, e, s, 0);
      break;
    }
  }
}
// encodeStateAsUpdate[V2](doc, targetStateVector): writeClientsStructs (encoding.js:94-116: clients
// descending, each from its clock in the target state vector -- 0 when absent; a client the target already
// has up to its state is left out) then writeDeleteSet(createDeleteSetFromStructStore(store)) (store
// order, adjacent deleted structs joined; the whole delete set, whatever the target).  d.svst: per client
// the first clock to write, -1 to leave the client out (nullptr: every client from 0)
YM_BIG void doc_write(Ctx &c, Enc &e, Doc &d, uint32_t *ord) {
  uint32_t nw = d.cl.n;
  if (d.svst) {
    nw = 0;
    for (uint32_t ci = 0; ci < d.cl.n; ci++) nw += d.svst[ci] >= 0;
  }
  ovu(e.rest, (int64_t)nw);
  for (uint32_t oi = 0; oi < d.cl.n && !c.err; oi++) {
    const Cl &s = d.cl.p[ord[oi]];
    const int64_t clock = d.svst ? d.svst[ord[oi]] : 0;
    if (clock < 0) continue;
    if (s.a.n == 0) { ovu(e.rest, 0); e_client(e, s.client); ovu(e.rest, 0); continue; }
    const uint32_t i0 = clock == 0 ? 0 : find_index(d, (int32_t)ord[oi], clock);  // writeStructs, :71-84
    if (c.err) return;
    ovu(e.rest, (int64_t)(s.a.n - i0));
    e_client(e, s.client);
    ovu(e.rest, clock);
    item_write(c, e, d, s.a.p[i0], clock - d.it[s.a.p[i0]].clock);
    for (uint32_t i = i0 + 1; i < s.a.n && !c.err; i++) item_write(c, e, d, s.a.p[i]);
  }
  uint32_t ndc = 0;
  for (uint32_t ci = 0; ci < d.cl.n; ci++) {
    const Vec<int32_t> &a = d.cl.p[ci].a;
    for (uint32_t i = 0; i < a.n; i++)
      if (d.it[a.p[i]].deleted) { ndc++; break; }
  }
  ovu(e.rest, (int64_t)ndc);
  for (uint32_t ci = 0; ci < d.cl.n; ci++) {
    const Vec<int32_t> &a = d.cl.p[ci].a;
    uint32_t m = 0;
    for (uint32_t i = 0; i < a.n; i++) {
      if (!d.it[a.p[i]].deleted) continue;
      int64_t end = d.it[a.p[i]].clock + d.it[a.p[i]].len;
      while (i + 1 < a.n && d.it[a.p[i + 1]].clock == end && d.it[a.p[i + 1]].deleted) { end += d.it[a.p[i + 1]].len; i++; }
      m++;
    }
    if (m == 0) continue;
    ovu(e.rest, d.cl.p[ci].client);
    ovu(e.rest, (int64_t)m);
    int64_t cur = 0;  // DSEncoderV2: clocks delta-coded within a client, lengths minus one
    for (uint32_t i = 0; i < a.n; i++) {
      if (!d.it[a.p[i]].deleted) continue;
      const int64_t clock = d.it[a.p[i]].clock;
      int64_t end = clock + d.it[a.p[i]].len;
      while (i + 1 < a.n && d.it[a.p[i + 1]].clock == end && d.it[a.p[i + 1]].deleted) { end += d.it[a.p[i + 1]].len; i++; }
      if (e.v2) { ovu(e.rest, clock - cur); ovu(e.rest, end - clock - 1); cur = end; }
      else { ovu(e.rest, clock); ovu(e.rest, end - clock); }
    }
  }
  e_flush_columns(c, e);
}

#ifdef YM_CPT_DEBUG
inline void cpt_debug_check(Doc &d, uint32_t u) {
  for (uint32_t ci = 0; ci < d.cl.n; ci++)
    for (uint32_t i = 0; i < d.cl.p[ci].a.n; i++) {
      const int32_t x = d.cl.p[ci].a.p[i];
      const Item &it = d.it[x];
      if (it.gc || (it.ref != 2 && it.ref != 4 && it.ref != 8)) continue;
      int64_t n = 0;
      for (int32_t q = it.chead; q != NIL; q = d.pc[q].next) { n += d.pc[q].n16; if (d.pc[q].next == NIL && q != it.ctail) fprintf(stderr, "tail mismatch after %u item %d ref %d len %lld head %d tail %d last %d del %d\n", u, x, it.ref, (long long)it.len, it.chead, it.ctail, q, it.deleted); }
      if (n != it.len) fprintf(stderr, "after update %u: item %d (%lld:%lld) len %lld pieces %lld deleted %d\n", u, x, (long long)it.client, (long long)it.clock, (long long)it.len, (long long)n, it.deleted);
    }
}
#endif
// ---- one document ------------------------------------------------------------------------------------
// workspace of a document of `bytes` input bytes in k updates; mul grows it on ST_RETRY
struct WsSize { uint64_t it, pc, el, src, ty, gen, gent, total; };
YM_INL WsSize ws_size(uint32_t k, uint64_t bytes, uint32_t mul) {
  WsSize z;
  const uint64_t base = bytes + 16ull * k + 64;
  z.it = (base / 4 + 64) * mul;
  z.pc = (base / 4 + 64) * mul;
  z.el = (base / 2 + 16) * mul;
  z.src = (base / 8 + 16) * mul;
  z.ty = (base / 16 + 16) * mul;
  z.gen = (16 * base + 16384) * mul;
  z.gent = (4 * base + 4096) * mul;
  z.total = al16(z.it * sizeof(Item)) + al16(z.pc * sizeof(Piece)) + al16(z.el * sizeof(Elem)) +
            al16(z.src * sizeof(Src)) + al16(z.ty * sizeof(Type)) + al16(z.gen) + z.gent + al16(sizeof(Doc)) +
            2 * al16(sizeof(Arena)) + 64;
  return z;
}
// Applies the k updates of a document (offsets upd_off[u0 .. u0 + k]) to a fresh Doc and sizes / writes
// its encodeStateAsUpdate[V2].  out == nullptr: sizing only (L.total); else the bytes are written there.
// The engine state stays in the workspace between the two calls of one document (pass 2 only writes).
struct Result { uint64_t col[C_N]; uint64_t rest, total, sv; };
// encodeStateVector(doc) (encoding.js:572-611: writeStateVector over getStateVector, StructStore.js:49-56):
// vu(#clients) | (client, state)* with the clients in StructStore insertion order (d.cl: add_struct appends),
// state = the last struct's clock + length; the same bytes through DSEncoderV1 and DSEncoderV2
YM_INL uint64_t doc_sv(const Doc &d, uint8_t *out) {
  Out o = {out, 0};  // out == nullptr: size only
  ovu(o, (int64_t)d.cl.n);
  for (uint32_t ci = 0; ci < d.cl.n; ci++) {
    const Cl &s = d.cl.p[ci];
    const Item &l = d.it[s.a.p[s.a.n - 1]];
    ovu(o, s.client);
    ovu(o, l.clock + l.len);
  }
  return o.n;
}
// flags: bit 0 V2, bit 1 Doc({ gc: false }), bit 2 the Doc's encodeStateVector written first (YM_SV_FIRST).  svp / svlen: the encoded target state vector of
// encodeStateAsUpdate[V2](doc, sv) (svp == nullptr: none, every struct is written)
YM_BIG void compact_doc(Ctx &c, uint8_t *ws, const WsSize &z, uint32_t flags, const uint64_t *upd_off, uint32_t u0, uint32_t k,
                        const uint8_t *svp, uint64_t svlen, Result &R, uint8_t *out) {
  const uint32_t v2 = flags & 1;
  Doc *dp = (Doc *)ws;  // the document's state heads its workspace
  Arena *ap = (Arena *)(ws + al16(sizeof(Doc)));
  Arena *tp = (Arena *)(ws + al16(sizeof(Doc)) + al16(sizeof(Arena)));
  uint8_t *p = ws + al16(sizeof(Doc)) + 2 * al16(sizeof(Arena));
  Doc &d = *dp;
  if (!out) {
    __builtin_memset(&d, 0, sizeof(Doc));
    d.c = &c;
    d.a = ap;
    d.ta = tp;
    d.v2 = v2;
    d.nogc = (flags >> 1) & 1;
    d.it = (Item *)p; d.capit = (uint32_t)z.it; p += al16(z.it * sizeof(Item));
    d.pc = (Piece *)p; d.cappc = (uint32_t)z.pc; p += al16(z.pc * sizeof(Piece));
    d.el = (Elem *)p; d.capel = (uint32_t)z.el; p += al16(z.el * sizeof(Elem));
    d.src = (Src *)p; d.capsrc = (uint32_t)z.src; p += al16(z.src * sizeof(Src));
    d.ty = (Type *)p; d.capty = (uint32_t)z.ty; p += al16(z.ty * sizeof(Type));
    ap->base = p;
    ap->cap = z.gen;
    ap->used = 0;
    tp->base = p + al16(z.gen);
    tp->cap = z.gent;
    tp->used = 0;
    for (uint32_t u = 0; u < k && !c.err; u++) {
      Reader r;
      reader_open(c, r, upd_off[u0 + u], upd_off[u0 + u + 1] - upd_off[u0 + u], v2);
      if (c.err) return;
      if (v2) {
        r.keys_cap = (uint32_t)(upd_off[u0 + u + 1] - upd_off[u0 + u]) + 16;
        r.keys = (Span *)aalloc(c, *tp, sizeof(Span) * (uint64_t)r.keys_cap);
        if (c.err) return;
      }
      cd_transact(d, r);
      tp->used = 0;  // the update's reader and transactions are gone
#ifdef YM_CPT_DEBUG
      cpt_debug_check(d, u);
#endif
    }
    if (c.err) return;
    // structs still waiting for a missing dependency (pending refs, the pending stack) and deletes of
    // clocks not yet seen (pending delete readers) stay out of the output: encodeStateAsUpdate writes the
    // integrated store and its delete set only (encoding.js:490-493)
  }
  d.c = &c;
  if (!out) {
    d.ord = (uint32_t *)aalloc(c, *ap, 4ull * (d.cl.n + 1));
    if (c.err) return;
    uint32_t *ord = d.ord;
    for (uint32_t i = 0; i < d.cl.n; i++) ord[i] = i;
    for (uint32_t i = 1; i < d.cl.n; i++) {  // clients descending
      const uint32_t v = ord[i];
      uint32_t j = i;
      while (j > 0 && d.cl.p[ord[j - 1]].client < d.cl.p[v].client) { ord[j] = ord[j - 1]; j--; }
      ord[j] = v;
    }
    d.svst = nullptr;
    if (svp) {  // decodeStateVector (encoding.js:536-565, DSDecoderV1 for both formats; later entries win)
      int64_t *st = (int64_t *)aalloc(c, *ap, 8ull * (d.cl.n + 1));
      if (c.err) return;
      for (uint32_t i = 0; i < d.cl.n; i++) st[i] = 0;  // absent from the target: from clock 0
      Ctx cs = {0, svp};
      Rd sd = {0, svlen, 0};
      const uint32_t ns = rd_vu(cs, sd);
      for (uint32_t i = 0; i < ns && !cs.err; i++) {
        const int64_t client = rd_vu(cs, sd);
        const int64_t clock = rd_vu(cs, sd);
        if (cs.err) break;
        const int32_t ci = cd_client(d, client);
        // a client the target has up to (or past) its state is left out (encoding.js:97-102)
        if (ci != NIL) st[ci] = cl_state(d, ci) > clock ? clock : -1;
      }
      if (cs.err) { seterr(c, cs.err); return; }
      d.svst = st;
    }
  }
  uint32_t *ord = d.ord;
  Enc e;
  enc_init(e, v2);
  if (!out) {  // sizing: every stream counts
    doc_write(c, e, d, ord);
    Out *cols[C_N] = {&e.kc, &e.cl, &e.lc, &e.rc, &e.in, &e.sb, &e.sl, &e.pi, &e.tr, &e.ln};
    for (int i = 0; i < C_N; i++) R.col[i] = cols[i]->n;
    R.rest = e.rest.n;
    uint64_t h = 0;
    if (v2) {
      h = 1;
      for (int i = 0; i < C_N; i++) {
        if (i == C_SB || i == C_SL) continue;
        h += vu_size(R.col[i]) + R.col[i];
      }
      const uint64_t sc = vu_size(R.col[C_SB]) + R.col[C_SB] + R.col[C_SL];
      h += vu_size(sc) + sc;
    }
    R.total = h + R.rest;
    R.sv = (flags & 4) ? doc_sv(d, nullptr) : 0;
    R.total += R.sv;
    return;
  }
  if (R.sv) {  // encodeStateVector(doc), then the update after it
    doc_sv(d, out);
    out += R.sv;
  }
  // writing: every stream at its final place (UpdateEncoderV2.toUint8Array layout, ym_core.h Layout)
  Out hdr = {out, 0};
  if (v2) {
    o8(hdr, 0);
    Out *cols[C_N] = {&e.kc, &e.cl, &e.lc, &e.rc, &e.in, &e.sb, &e.sl, &e.pi, &e.tr, &e.ln};
    for (int i = 0; i < C_N; i++) {
      if (i == C_SL) continue;
      if (i == C_SB) {
        const uint64_t sc = vu_size(R.col[C_SB]) + R.col[C_SB] + R.col[C_SL];
        ovu(hdr, (int64_t)sc);
        ovu(hdr, (int64_t)R.col[C_SB]);
        e.sb.p = out; e.sb.n = hdr.n;
        hdr.n += R.col[C_SB];
        e.sl.p = out; e.sl.n = hdr.n;
        hdr.n += R.col[C_SL];
        continue;
      }
      ovu(hdr, (int64_t)R.col[i]);
      cols[i]->p = out;
      cols[i]->n = hdr.n;
      hdr.n += R.col[i];
    }
  }
  e.rest.p = out;
  e.rest.n = hdr.n;
  doc_write(c, e, d, ord);
}

}  // namespace cpt
}  // namespace ym
