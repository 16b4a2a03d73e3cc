// TEST-ONLY host build of yjs_amd/csrc/ym_core.h: the general path's per-document entry (general_doc,
// the function k_general runs on the MI355X, one thread per document) compiled for the CPU, so the
// device core can be unit-tested in the GPU-less container and run under ASan / UBSan.
// It is not part of the product: libymerge.so only runs this code as HIP kernels.
//
// Usage: core_host <batch.in> <result.out>
//   batch.in : u32 op, u32 fmt, u32 n_docs, u32 n_upd, u64 arena_len, u64 sv_len,
//              u32 doc_upd[n_docs+1], u64 upd_off[n_upd+1], u8 arena[arena_len],
//              u64 sv_off[n_docs+1], u8 sv[sv_len]
//   result.out: per document: i32 status, u64 len, u8 bytes[len]
#define YM_HD
#include "../../yjs_amd/csrc/ym_core.h"
#include "../../yjs_amd/csrc/ym_compact.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

using namespace ym;

template <class T> static void rd(FILE *f, T *p, size_t n) {
  if (n && fread(p, sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
}

int main(int argc, char **argv) {
  if (argc != 3) { fprintf(stderr, "usage: core_host in out\n"); return 2; }
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint32_t hdr[4];
  uint64_t lens[2];
  rd(f, hdr, 4);
  rd(f, lens, 2);
  const uint32_t op = hdr[0], fmt = hdr[1], nd = hdr[2], nu = hdr[3];
  std::vector<uint32_t> doc_upd(nd + 1);
  std::vector<uint64_t> upd_off(nu + 1), sv_off(nd + 1);
  // +64: the lib0 readers may look one word past a short update (bounds are checked, loads are not)
  std::vector<uint8_t> arena(lens[0] + 64), sv(lens[1] + 64);
  rd(f, doc_upd.data(), nd + 1);
  rd(f, upd_off.data(), nu + 1);
  rd(f, arena.data(), lens[0]);
  rd(f, sv_off.data(), nd + 1);
  rd(f, sv.data(), lens[1]);
  fclose(f);
  FILE *o = fopen(argv[2], "wb");
  if (!o) return 2;
  const uint32_t v2 = (fmt & 0xff) == 2;
  // v2f bit 8: YM_DS_REF (ym_ds_merge); bit 9: V2 output (ym_snapshot: YM_OUT_V2, or a V2 input without YM_OUT_V1)
  const uint32_t v2out = op == OP_SNAP && ((fmt & 0x2000) || (v2 && !(fmt & 0x1000)));
  const uint32_t v2f = v2 | (op == OP_DSMERGE && (fmt & 0x100) ? 0x100u : 0u) | (v2out ? 0x200u : 0u);
  for (uint32_t d = 0; d < nd; d++) {
    const uint32_t u0 = doc_upd[d], k = doc_upd[d + 1] - u0;
    const uint64_t bytes = upd_off[doc_upd[d + 1]] - upd_off[u0];
    const uint64_t svlen = op == OP_DIFF ? sv_off[d + 1] - sv_off[d] : 0;
    const uint8_t *svp = op == OP_DIFF ? sv.data() + sv_off[d] : nullptr;
    int st = ST_RETRY;
    std::vector<uint8_t> out;
    if (op == 7) {  // Doc round-trip compaction (ym_compact.h compact_doc), same retry policy as the kernel
      // fmt bit 15 (test-only): the batch carries target state vectors (ym_batch.sv_arena != NULL)
      const uint8_t *tsv = (fmt & 0x8000) ? sv.data() + sv_off[d] : nullptr;
      const uint64_t tsvlen = (fmt & 0x8000) ? sv_off[d + 1] - sv_off[d] : 0;
      for (uint32_t mul = 1, round = 0; st == ST_RETRY && round < 5; mul *= 4, round++) {
        const cpt::WsSize z = cpt::ws_size(k, bytes, mul);
        std::vector<uint8_t> ws(z.total + 16);
        Ctx c = {0, arena.data()};
        cpt::Result R;
        memset(&R, 0, sizeof(R));
        const uint32_t cflags = v2 | ((fmt & 0x4000) ? 2u : 0u) | ((fmt & 0x10000) ? 4u : 0u);
        cpt::compact_doc(c, ws.data(), z, cflags, upd_off.data(), u0, k, tsv, tsvlen, R, nullptr);
        st = c.err;
        if (st) continue;
        if (getenv("YM_CPT_STATS")) {  // workspace use (sizing experiments): used / reserved per region
          const cpt::Doc *dp = (const cpt::Doc *)ws.data();
          const cpt::Arena *ap = (const cpt::Arena *)(ws.data() + ym::al16(sizeof(cpt::Doc)));
          fprintf(stderr, "CPT %u %llu it %u %u pc %u %u el %u %u src %u %u ty %u %u gen %llu %llu total %llu szit %zu szpc %zu szel %zu szsrc %zu szty %zu\n", k,
                  (unsigned long long)bytes, dp->nit, dp->capit, dp->npc, dp->cappc, dp->nel, dp->capel, dp->nsrc, dp->capsrc, dp->nty,
                  dp->capty, (unsigned long long)ap->used, (unsigned long long)ap->cap, (unsigned long long)z.total, sizeof(cpt::Item),
                  sizeof(cpt::Piece), sizeof(cpt::Elem), sizeof(cpt::Src), sizeof(cpt::Type));
        }
        out.assign(R.total + 1, 0);
        Ctx c2 = {0, arena.data()};
        cpt::compact_doc(c2, ws.data(), z, cflags, upd_off.data(), u0, k, tsv, tsvlen, R, out.data());
        st = c2.err ? (c2.err == ST_RETRY ? ST_UNEXPECTED : c2.err) : 0;
        out.resize(R.total);
      }
      const int32_t s32 = st;
      const uint64_t n = st ? 0 : out.size();
      fwrite(&s32, 4, 1, o);
      fwrite(&n, 8, 1, o);
      if (n) fwrite(out.data(), 1, n, o);
      continue;
    }
    for (uint32_t mul = 1, round = 0; st == ST_RETRY && round < 7; mul *= 8, round++) {
      const GeneralWsSize z = general_ws_size(k, bytes, mul, general_sv_bytes(op, svlen, bytes), v2);
      std::vector<uint8_t> ws(z.total + 16);
      DocWS w;
      general_carve(ws.data(), z, w);
      Layout L;
      memset(&L, 0, sizeof(L));
      Ctx c = {0, arena.data()};
      general_doc(c, w, op, v2f, upd_off.data(), u0, k, svp, svlen, 1, L, nullptr);
      st = c.err;
      if (st) continue;
      // pass 2 over the same workspace (the part table recorded by pass 1 is read back)
      out.assign(L.total + 1, 0);
      Ctx c2 = {0, arena.data()};
      general_doc(c2, w, op, v2f, upd_off.data(), u0, k, svp, svlen, 2, L, out.data());
      st = c2.err ? (c2.err == ST_RETRY ? ST_UNEXPECTED : c2.err) : 0;
      out.resize(L.total);
    }
    const int32_t s32 = st;
    const uint64_t n = st ? 0 : out.size();
    fwrite(&s32, 4, 1, o);
    fwrite(&n, 8, 1, o);
    if (n) fwrite(out.data(), 1, n, o);
  }
  fclose(o);
  return 0;
}
