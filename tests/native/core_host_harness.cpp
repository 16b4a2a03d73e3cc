// TEST-ONLY host build of yjs_amd/csrc/ym_core.h: runs the device core's per-document functions on
// the CPU so the GPU logic can be unit-tested in a GPU-less container.  Not part of the product
// library; the product (libymerge.so) only runs this code as HIP kernels on the MI355X.
#define YM_HD
#include "../../yjs_amd/csrc/ym_core.h"
#include <stdlib.h>
#include <string.h>
#include <vector>

using namespace ym;

struct WS {
  std::vector<Reader> rs;
  std::vector<uint32_t> arr, tmp;
  std::vector<PartRec> parts;
  std::vector<DSE> ds;
  std::vector<DSG> dsg;
  std::vector<int64_t> sv;
  DocWS view(uint32_t k, uint64_t bytes, uint32_t parts_cap, uint32_t sv_cap) {
    rs.assign(k ? k : 1, Reader());
    arr.assign(k + 1, 0);
    tmp.assign(k + 1, 0);
    parts.assign(parts_cap, PartRec());
    ds.assign(bytes / 2 + 2, DSE());
    dsg.assign(bytes / 2 + 2, DSG());
    sv.assign(2 * sv_cap + 2, 0);
    DocWS w;
    w.rs = rs.data(); w.arr = arr.data(); w.tmp = tmp.data();
    w.parts = parts.data(); w.parts_cap = parts_cap;
    w.ds = ds.data(); w.dsg = dsg.data(); w.ds_cap = bytes / 2 + 2;
    w.sv = sv.data(); w.sv_cap = sv_cap;
    return w;
  }
};

// op 0 merge, 1 diff, 2 sv.  Inputs concatenated in `arena` with offsets (k+1); returns status, output malloc'd
extern "C" int ymh_run(int op, int fmt, const uint8_t *arena, const uint64_t *upd_off, uint32_t k,
                       const uint8_t *sv, uint64_t svlen, uint8_t **out, uint64_t *out_len) {
  *out = nullptr;
  *out_len = 0;
  uint64_t total = upd_off[k];
  // arena + sv in one buffer (all spans are absolute)
  std::vector<uint8_t> A(total + svlen + 1);
  memcpy(A.data(), arena, total);
  if (svlen) memcpy(A.data() + total, sv, svlen);
  if (op == 0 && k == 1) {  // identity
    *out = (uint8_t *)malloc(total + 1);
    memcpy(*out, arena, total);
    *out_len = total;
    return 0;
  }
  uint32_t parts_cap = 8;
  for (int attempt = 0; attempt < 12; attempt++) {
    WS ws;
    DocWS w = ws.view(k, total, parts_cap, 1 << 16);
    Ctx c = {0, A.data()};
    Layout L;
    memset(&L, 0, sizeof(L));
    uint32_t v2 = fmt == 2;
    if (op == 0) merge_doc(c, w, upd_off, 0, k, v2, 1, L, nullptr);
    else if (op == 1) diff_doc(c, w, 0, upd_off[1], A.data() + total, svlen, v2, 1, L, nullptr);
    else sv_doc(c, w, 0, upd_off[1], v2, 1, L, nullptr);
    if (c.err == ST_RETRY) { parts_cap *= 4; continue; }
    if (c.err) return c.err;
    uint8_t *o = (uint8_t *)malloc(L.total + 1);
    Ctx c2 = {0, A.data()};
    std::vector<PartRec> saved(ws.parts);
    DocWS w2 = ws.view(k, total, parts_cap, 1 << 16);
    memcpy(w2.parts, saved.data(), sizeof(PartRec) * parts_cap);
    if (op == 0) merge_doc(c2, w2, upd_off, 0, k, v2, 2, L, o);
    else if (op == 1) diff_doc(c2, w2, 0, upd_off[1], A.data() + total, svlen, v2, 2, L, o);
    else sv_doc(c2, w2, 0, upd_off[1], v2, 2, L, o);
    if (c2.err) { free(o); return 1000 + c2.err; }
    *out = o;
    *out_len = L.total;
    return 0;
  }
  return ST_RETRY;
}
extern "C" void ymh_free(void *p) { free(p); }
