// ym_fast.hip -- LDS fast path: one 64-lane wave per document, the whole document staged in LDS.
//
// Takes mergeUpdates (V1) documents whose inputs are "simple": every update's structs increase in
// (client desc, clock asc), no two structs overlap, no GC/Skip structs, canonical encodings.  For such
// documents yjs 13.5.16's k-way merge (bundle ds@39007) reduces to: all structs sorted by
// (client desc, clock asc), a Skip inserted before every clock gap, consecutive same-client structs
// grouped into one part (SURVEY.md App. B "Consequences for the GPU design").  Everything else is
// declined (status ST_PENDING) and handled exactly by the general path.
//
// Per document: coalesced copy of the update bytes into LDS -> lanes walk updates in parallel (count
// pass, scan, emit pass) -> bitonic sort of (client, clock) keys -> parallel sizes + wave scans ->
// delete-set union -> output staged in LDS -> one atomicAdd for the output slot -> coalesced store.
#include <hip/hip_runtime.h>

#include "ym_core.h"
#include "ym_kernels.h"

namespace ymk {
using namespace ym;

constexpr int F_IN = 6144;   // input bytes per document
constexpr int F_UPD = 256;   // updates per document
constexpr int F_REC = 256;   // structs per document (power of two for the bitonic sort)
constexpr int F_DS = 256;    // delete-set entries per document (power of two)
constexpr int F_OUT = 7168;  // output bytes per document

struct FastLds {
  uint64_t rkey[F_REC];   // sort key: (~client << 32) | clock
  uint64_t dkey[F_DS];    // (client << 32) | clock
  uint32_t uoff[F_UPD + 1];
  uint32_t rlen[F_REC];
  uint32_t dlen[F_DS];
  uint32_t rpos[F_REC];   // output offset of each sorted record
  uint16_t ridx[F_REC];   // sort payload
  uint16_t rstart[F_REC]; // struct start (info byte) in `in`
  uint16_t rblen[F_REC];  // struct byte length incl. info byte
  uint16_t rupd[F_REC];
  uint16_t didx[F_DS];
  uint16_t ubase[F_UPD + 1];  // record prefix per update
  uint16_t dbase[F_UPD + 1];  // ds prefix per update
  uint8_t rinfo[F_REC];
  uint8_t in[F_IN];
  uint8_t out[F_OUT];
  uint32_t nrec, nds, decline, total, struct_bytes, ds_bytes, nparts;
  uint64_t out_off;
};

// wave-wide exclusive scan of one value per lane (64 lanes)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
  uint32_t lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

__device__ __forceinline__ bool json_simple_canonical(const Ctx &c, uint64_t off, uint32_t n) {
  // fast accept of the texts yjs itself writes for formats/embeds: true/false/null, small ints,
  // plain strings without escapes; anything else goes through the full checker
  if (n == 4 && c.A[off] == 't' && c.A[off + 1] == 'r' && c.A[off + 2] == 'u' && c.A[off + 3] == 'e') return true;
  if (n == 4 && c.A[off] == 'n' && c.A[off + 1] == 'u' && c.A[off + 2] == 'l' && c.A[off + 3] == 'l') return true;
  if (n == 5 && c.A[off] == 'f' && c.A[off + 1] == 'a' && c.A[off + 2] == 'l' && c.A[off + 3] == 's' && c.A[off + 4] == 'e') return true;
  if (n >= 2 && c.A[off] == '"' && c.A[off + n - 1] == '"') {
    for (uint32_t i = 1; i + 1 < n; i++) {
      uint8_t ch = c.A[off + i];
      if (ch < 0x20 || ch == '"' || ch == '\\') return false;
    }
    return true;
  }
  return false;
}

// lib0 readVarUint that also flags non-canonical (overlong / >32-bit) encodings
__device__ __forceinline__ uint32_t fvu(Ctx &c, Rd &d, bool &nc) {
  uint64_t p0 = d.pos;
  uint32_t v = rd_vu(c, d);
  uint64_t n = d.pos - p0;
  if (n > 1) {
    uint8_t last = (d.pos - 1) < d.len ? c.A[d.start + d.pos - 1] : 0;
    if (last == 0 || n > 5 || (n == 5 && (last & 0x70))) nc = true;
  }
  return v;
}
__device__ __forceinline__ Span fvstr(Ctx &c, Rd &d, bool &nc) {
  uint64_t p0 = d.pos;
  Rd t = d;
  fvu(c, t, nc);  // length prefix canonical?
  (void)p0;
  return rd_vstr(c, d);
}

// Walks one V1 update held in LDS.  EMIT=false: counts structs / DS entries and checks fast-path
// eligibility; EMIT=true: writes the records.  Returns false when the document must be declined.
template <bool EMIT>
__device__ __attribute__((noinline)) bool walk_v1(FastLds &S, uint32_t u, uint32_t &nrec, uint32_t &nds) {
  Ctx c = {0, S.in};
  Rd r = {S.uoff[u], S.uoff[u + 1] - S.uoff[u], 0};
  bool nc = false;
  uint32_t ri = EMIT ? S.ubase[u] : 0, di = EMIT ? S.dbase[u] : 0;
  nrec = 0;
  nds = 0;
  uint32_t nclients = fvu(c, r, nc);
  uint64_t prev_key = 0;
  bool have_prev = false;
  for (uint32_t ci = 0; ci < nclients && !c.err; ci++) {
    uint32_t nstructs = fvu(c, r, nc);
    uint32_t client = fvu(c, r, nc);
    uint64_t clock = fvu(c, r, nc);
    for (uint32_t si = 0; si < nstructs && !c.err; si++) {
      uint32_t s0 = (uint32_t)(r.start + r.pos);
      int info = rbyte(c, r);
      if (info < 0 || info == 10 || (info & 31) == 0) return false;  // truncated / Skip / GC
      if (info & 0x80) { fvu(c, r, nc); fvu(c, r, nc); }
      if (info & 0x40) { fvu(c, r, nc); fvu(c, r, nc); }
      if ((info & 0xC0) == 0) {
        uint32_t pi = fvu(c, r, nc);
        if (pi > 1) return false;  // parentInfo re-encodes as 0
        if (pi == 1) fvstr(c, r, nc);
        else { fvu(c, r, nc); fvu(c, r, nc); }
        if (info & 0x20) fvstr(c, r, nc);
      }
      uint64_t len = 1;
      switch (info & 31) {
        case 1: len = fvu(c, r, nc); break;
        case 3: { Rd t = r; fvu(c, t, nc); rd_vbytes(c, r); break; }
        case 4: { Span s = fvstr(c, r, nc); len = s.n16; break; }
        case 5: {
          Span s = fvstr(c, r, nc);
          if (!c.err && !json_simple_canonical(c, s.off, s.n)) { int q = 0; if (json_check(c, s.off, s.n, &q) || q) return false; }
          break;
        }
        case 6: {
          fvstr(c, r, nc);
          Span s = fvstr(c, r, nc);
          if (!c.err && !json_simple_canonical(c, s.off, s.n)) { int q = 0; if (json_check(c, s.off, s.n, &q) || q) return false; }
          break;
        }
        case 7: {
          uint32_t t = fvu(c, r, nc);
          if (t > 6) return false;
          if (t == 3 || t == 5) fvstr(c, r, nc);
          break;
        }
        case 8: {
          len = fvu(c, r, nc);
          for (uint64_t i = 0; i < len && !c.err; i++) {
            int q = 0;
            any_skip(c, r, &q);
            if (q) return false;
          }
          break;
        }
        default: return false;  // ContentJSON / ContentDoc / invalid refs: general path
      }
      if (c.err || len == 0) return false;
      uint64_t end = clock + len;
      if (end > 0xffffffffull) return false;
      uint64_t key = ((uint64_t)(~client) << 32) | clock;
      if (have_prev && key <= prev_key) return false;  // reader must be increasing
      prev_key = key + len - 1;
      have_prev = true;
      if (EMIT) {
        uint32_t k = ri + nrec;
        S.rkey[k] = key;
        S.rlen[k] = (uint32_t)len;
        S.rstart[k] = (uint16_t)s0;
        S.rblen[k] = (uint16_t)(r.start + r.pos - s0);
        S.rinfo[k] = (uint8_t)info;
        S.rupd[k] = (uint16_t)u;
        S.ridx[k] = (uint16_t)k;
      }
      nrec++;
      clock = end;
    }
  }
  if (c.err || nc) return false;
  // delete set (DeleteSet.js:241-256)
  uint32_t ndc = fvu(c, r, nc);
  for (uint32_t i = 0; i < ndc && !c.err; i++) {
    uint32_t client = fvu(c, r, nc);
    uint32_t m = fvu(c, r, nc);
    for (uint32_t q = 0; q < m && !c.err; q++) {
      uint32_t clock = fvu(c, r, nc);
      uint32_t len = fvu(c, r, nc);
      if (EMIT) {
        uint32_t k = di + nds;
        S.dkey[k] = ((uint64_t)client << 32) | clock;
        S.dlen[k] = len;
        S.didx[k] = (uint16_t)k;
      }
      nds++;
    }
  }
  return !c.err && !nc;
}

template <class K>
__device__ __forceinline__ void bitonic_sort(K *key, uint16_t *idx, uint32_t n_pow2) {
  uint32_t lane = threadIdx.x;
  for (uint32_t size = 2; size <= n_pow2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (uint32_t t = lane; t < n_pow2 / 2; t += 64) {
        uint32_t i = 2 * t - (t & (stride - 1));
        uint32_t jx = i + stride;
        bool up = ((i & size) == 0);
        K a = key[i], b = key[jx];
        if ((a > b) == up) {
          key[i] = b; key[jx] = a;
          uint16_t x = idx[i]; idx[i] = idx[jx]; idx[jx] = x;
        }
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t vu_sz(uint64_t v) { return ym::vu_size(v); }
__device__ __forceinline__ uint32_t put_vu(uint8_t *o, uint64_t v) {
  uint32_t n = 0;
  while (v > 127) { o[n++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; }
  o[n++] = (uint8_t)v;
  return n;
}

__global__ void __launch_bounds__(64) k_fast_merge_v1(GeneralJob j) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  FastLds &S = *reinterpret_cast<FastLds *>(smem);
  const uint32_t lane = threadIdx.x;
  for (uint32_t d = blockIdx.x; d < j.n; d += gridDim.x) {
    const uint32_t u0 = j.doc_upd[d], k = j.doc_upd[d + 1] - u0;
    const uint64_t b0 = j.upd_off[u0], bytes = j.upd_off[u0 + k] - b0;
    if (k == 1 || k > F_UPD || bytes > F_IN || k == 0) {
      if (lane == 0) j.status[d] = ST_PENDING;
      continue;
    }
    // 1. stage the document and its update offsets in LDS
    for (uint64_t i = lane; i < bytes; i += 64) S.in[i] = j.A[b0 + i];
    for (uint32_t i = lane; i <= k; i += 64) S.uoff[i] = (uint32_t)(j.upd_off[u0 + i] - b0);
    if (lane == 0) S.decline = 0;
    __syncthreads();
    // 2. count pass (one lane per update)
    uint32_t myrec = 0, myds = 0;
    uint32_t cnt_r[F_UPD / 64], cnt_d[F_UPD / 64];
    bool ok = true;
#pragma unroll
    for (int q = 0; q < F_UPD / 64; q++) {
      uint32_t u = lane + 64 * q;
      cnt_r[q] = cnt_d[q] = 0;
      if (u < k) ok &= walk_v1<false>(S, u, cnt_r[q], cnt_d[q]);
    }
    if (!ok) S.decline = 1;
    __syncthreads();
    if (S.decline) { if (lane == 0) j.status[d] = ST_PENDING; __syncthreads(); continue; }
    // prefix over updates in update order: update u = lane + 64q -> rounds q outer, lanes inner
    uint32_t base_r = 0, base_d = 0;
#pragma unroll
    for (int q = 0; q < F_UPD / 64; q++) {
      uint32_t tr, td;
      uint32_t er = wave_excl_scan(cnt_r[q], &tr);
      uint32_t ed = wave_excl_scan(cnt_d[q], &td);
      uint32_t u = lane + 64 * q;
      if (u < k) { S.ubase[u] = (uint16_t)(base_r + er); S.dbase[u] = (uint16_t)(base_d + ed); }
      base_r += tr;
      base_d += td;
    }
    myrec = base_r;
    myds = base_d;
    if (myrec > F_REC || myds > F_DS || myrec == 0) {
      if (lane == 0) j.status[d] = ST_PENDING;
      __syncthreads();
      continue;
    }
    __syncthreads();
    // 3. emit pass
#pragma unroll
    for (int q = 0; q < F_UPD / 64; q++) {
      uint32_t u = lane + 64 * q, a, b;
      if (u < k) walk_v1<true>(S, u, a, b);
    }
    const uint32_t nrec = myrec, nds = myds;
    uint32_t np2 = 64;
    while (np2 < nrec) np2 <<= 1;
    for (uint32_t i = nrec + lane; i < np2; i += 64) { S.rkey[i] = ~0ull; S.ridx[i] = 0; }
    uint32_t dp2 = 64;
    while (dp2 < nds) dp2 <<= 1;
    for (uint32_t i = nds + lane; i < dp2; i += 64) { S.dkey[i] = ~0ull; S.didx[i] = 0; }
    // 4. sort structs by (client desc, clock asc) and DS entries by (client, clock)
    bitonic_sort(S.rkey, S.ridx, np2);
    if (nds > 1) bitonic_sort(S.dkey, S.didx, dp2);
    // 5. simplicity check + per-record output sizes (record i in sorted order)
    //    size = [part header] + [skip before] + 1 + body
    const uint32_t per = (nrec + 63) / 64;
    uint32_t lo = lane * per, hi = lo + per < nrec ? lo + per : nrec;
    bool bad = false;
    uint32_t local = 0, units = 0;
    for (uint32_t i = lo; i < hi; i++) {
      uint32_t id = S.ridx[i];
      uint64_t key = S.rkey[i];
      uint32_t sz = S.rblen[id];
      uint32_t un = 1;
      if (i > 0) {
        uint64_t pk = S.rkey[i - 1];
        uint32_t pid = S.ridx[i - 1];
        if ((pk >> 32) == (key >> 32)) {
          uint64_t pend = (pk & 0xffffffffull) + S.rlen[pid];
          uint64_t cl = key & 0xffffffffull;
          if (pend > cl) bad = true;
          else if (pend < cl) { sz += 1 + vu_sz(cl - pend); un++; }
        }
      }
      local += sz;
      units += un;
    }
    if (__any(bad)) {
      if (lane == 0) j.status[d] = ST_PENDING;
      __syncthreads();
      continue;
    }
    // part headers need the number of output structs per client run: prefix of units
    uint32_t tot_units;
    uint32_t u_excl = wave_excl_scan(units, &tot_units);
    (void)tot_units;
    // record-level prefixes (units, and later byte offsets) kept in rpos temporarily as units
    {
      uint32_t acc = u_excl;
      for (uint32_t i = lo; i < hi; i++) {
        uint32_t id = S.ridx[i];
        uint32_t un = 1;
        if (i > 0 && (S.rkey[i - 1] >> 32) == (S.rkey[i] >> 32)) {
          uint64_t pend = (S.rkey[i - 1] & 0xffffffffull) + S.rlen[S.ridx[i - 1]];
          if (pend < (S.rkey[i] & 0xffffffffull)) un++;
        }
        (void)id;
        acc += un;
        S.rpos[i] = acc;  // inclusive unit prefix
      }
    }
    __syncthreads();
    // header bytes for run starts: vu(units in run) vu(client) vu(clock)
    uint32_t nparts_local = 0;
    for (uint32_t i = lo; i < hi; i++) {
      bool start = i == 0 || (S.rkey[i - 1] >> 32) != (S.rkey[i] >> 32);
      if (!start) continue;
      nparts_local++;
      uint32_t e = i + 1;
      while (e < nrec && (S.rkey[e] >> 32) == (S.rkey[i] >> 32)) e++;
      uint32_t run_units = S.rpos[e - 1] - (i ? S.rpos[i - 1] : 0);
      uint32_t client = ~(uint32_t)(S.rkey[i] >> 32);
      local += vu_sz(run_units) + vu_sz(client) + vu_sz(S.rkey[i] & 0xffffffffull);
    }
    __syncthreads();
    uint32_t tot_bytes, nparts;
    uint32_t b_excl = wave_excl_scan(local, &tot_bytes);
    wave_excl_scan(nparts_local, &nparts);
    // 6. delete set: union per client (sorted), clients ordered by first appearance (lane 0)
    if (lane == 0) {
      // group boundaries over dkey (sorted by client, clock); first appearance = min original index
      uint32_t ng = 0;
      uint32_t gstart[64], gfirst[64], gcnt[64];
      bool overflow = false;
      for (uint32_t i = 0; i < nds;) {
        uint32_t cl = (uint32_t)(S.dkey[i] >> 32);
        uint32_t e = i, first = 0xffffffffu;
        while (e < nds && (uint32_t)(S.dkey[e] >> 32) == cl) { if (S.didx[e] < first) first = S.didx[e]; e++; }
        // union in place (>= touching merge, max end)
        uint32_t w = i + 1;
        for (uint32_t q = i + 1; q < e; q++) {
          uint64_t lc = S.dkey[w - 1] & 0xffffffffull;
          uint64_t lend = lc + S.dlen[S.didx[w - 1]];
          uint64_t rc = S.dkey[q] & 0xffffffffull;
          uint64_t rend = rc + S.dlen[S.didx[q]];
          if (lend >= rc) {
            if (rend > lend) S.dlen[S.didx[w - 1]] = (uint32_t)(rend - lc);
          } else {
            S.dkey[w] = S.dkey[q];
            S.didx[w] = S.didx[q];
            w++;
          }
        }
        if (ng < 64) { gstart[ng] = i; gfirst[ng] = first; gcnt[ng] = w - i; } else overflow = true;
        ng++;
        i = e;
      }
      // order groups by first appearance (insertion sort, few clients)
      for (uint32_t a = 1; a < ng && a < 64; a++) {
        uint32_t fs = gfirst[a], st = gstart[a], cn = gcnt[a];
        int b = (int)a - 1;
        while (b >= 0 && gfirst[b] > fs) { gfirst[b + 1] = gfirst[b]; gstart[b + 1] = gstart[b]; gcnt[b + 1] = gcnt[b]; b--; }
        gfirst[b + 1] = fs; gstart[b + 1] = st; gcnt[b + 1] = cn;
      }
      uint32_t hdr = vu_sz(nparts);
      uint32_t total = hdr + tot_bytes;
      // DS bytes written straight into the staging buffer after the struct section
      uint32_t p = total;
      bool fits = !overflow;
      if (fits) {
        if (p + 5 > F_OUT) fits = false;
        else p += put_vu(S.out + p, ng);
        for (uint32_t g = 0; g < ng && fits; g++) {
          uint32_t st = gstart[g];
          if (p + 10 > F_OUT) { fits = false; break; }
          p += put_vu(S.out + p, (uint32_t)(S.dkey[st] >> 32));
          p += put_vu(S.out + p, gcnt[g]);
          for (uint32_t q = 0; q < gcnt[g]; q++) {
            if (p + 10 > F_OUT) { fits = false; break; }
            p += put_vu(S.out + p, S.dkey[st + q] & 0xffffffffull);
            p += put_vu(S.out + p, S.dlen[S.didx[st + q]]);
          }
        }
      }
      if (!fits || total > F_OUT) S.decline = 1;
      else {
        put_vu(S.out, nparts);
        S.total = p;
        S.struct_bytes = hdr;  // struct section begins after vu(nparts)
        S.out_off = atomicAdd((unsigned long long *)j.used, (unsigned long long)p);
      }
    }
    __syncthreads();
    if (S.decline) { if (lane == 0) j.status[d] = ST_PENDING; __syncthreads(); continue; }
    // 7. write the struct section into LDS staging (each lane its slice of sorted records)
    {
      uint32_t p = S.struct_bytes + b_excl;
      for (uint32_t i = lo; i < hi; i++) {
        uint32_t id = S.ridx[i];
        uint64_t key = S.rkey[i];
        uint32_t client = ~(uint32_t)(key >> 32);
        uint64_t clock = key & 0xffffffffull;
        bool start = i == 0 || (S.rkey[i - 1] >> 32) != (key >> 32);
        if (start) {
          uint32_t e = i + 1;
          while (e < nrec && (S.rkey[e] >> 32) == (key >> 32)) e++;
          uint32_t run_units = S.rpos[e - 1] - (i ? S.rpos[i - 1] : 0);
          p += put_vu(S.out + p, run_units);
          p += put_vu(S.out + p, client);
          p += put_vu(S.out + p, clock);
        } else {
          uint64_t pend = (S.rkey[i - 1] & 0xffffffffull) + S.rlen[S.ridx[i - 1]];
          if (pend < clock) {  // Skip(len = gap): info 10 + varuint
            S.out[p++] = 10;
            p += put_vu(S.out + p, clock - pend);
          }
        }
        uint32_t info = S.rinfo[id];
        if (info & 0xC0) info &= ~0x20u;  // parentSub is only read (and re-written) without origins
        S.out[p++] = (uint8_t)info;
        uint32_t s0 = S.rstart[id] + 1, n = S.rblen[id] - 1;
        for (uint32_t b = 0; b < n; b++) S.out[p + b] = S.in[s0 + b];
        p += n;
      }
    }
    __syncthreads();
    // 8. coalesced store of the document's output
    const uint32_t total = S.total;
    const uint64_t oo = S.out_off;
    if (oo + total <= j.cap) {
      for (uint32_t i = lane; i < total; i += 64) j.out[oo + i] = S.out[i];
    }
    if (lane == 0) {
      j.out_off[d] = oo;
      j.out_len[d] = total;
      j.status[d] = oo + total <= j.cap ? ST_OK : ST_CAPACITY;
    }
    __syncthreads();
  }
}

int fast_launch(uint32_t op, const GeneralJob &j, hipStream_t st) {
  if (op != OP_MERGE || j.v2) return 0;  // fast path: V1 merges (the C2/C4 headline configs)
  uint32_t grid = j.n < 65536 ? j.n : 65536;
  size_t lds = sizeof(FastLds);
  k_fast_merge_v1<<<grid, 64, lds, st>>>(j);
  return 1;
}

}  // namespace ymk
