"""TEMP: stitch path counters on the bench's C3 V1 sv / diff cases (4 docs)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from yjs_amd import Engine, pack_docs
from yjs_amd.workloads import load_ymb, random_state_vectors
e = Engine(0, path=os.path.join(ROOT, 'yjs_amd', 'libymerge_prof.so'))
a, o, d = load_ymb("c3_v1")
upd = a.tobytes()
a2, o2, d2 = pack_docs([[upd] for _ in range(4)])
buf = (ctypes.c_ulonglong * 8)()
e.lib.ym__pw_prof(buf, 1)
sa, so_, sl, st = e.run_host("sv", 1, a2, o2, d2)
e.lib.ym__pw_prof(buf, 1)
print("sv  whole,found-not-whole,not-in-first8,batches,repairs,cheapfail,fast,slow:", list(buf), e.stats)
full = sa[int(so_[0]):int(so_[0]) + int(sl[0])].tobytes()
svs = random_state_vectors(full, 4, seed=7)
sva, svo, _ = pack_docs([[x] for x in svs])
e.run_host("diff", 1, a2, o2, d2, sva, svo)
e.lib.ym__pw_prof(buf, 1)
print("diff whole,found-not-whole,not-in-first8,batches,repairs,cheapfail,fast,slow:", list(buf), e.stats)
