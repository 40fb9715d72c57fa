"""Config-4 ingest diagnostic at world 1 (no exchange): the device generator's
source-0 stream straight into one store; per-kernel times and a check of
sampled owners against the C oracle.  python tools/diag_c4.py OWNERS [P] [G]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evolu_amd import _lib as L  # noqa: E402
from evolu_amd import synth  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402
from oracle import c_oracle as CO  # noqa: E402

O = int(sys.argv[1])
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
G = int(sys.argv[3]) if len(sys.argv) > 3 else 1
SEED = 0xE7010004
eng = Engine(0)
dev = torch.device("cuda", 0)
gen = synth.DeviceSynth()
parts = [gen.source(SEED, O, P, G, s, dev) for s in range(G)]
ts = torch.cat([p[0] for p in parts])
owner = torch.cat([p[1] for p in parts])
n = ts.shape[0]
print("n", n, flush=True)
for rep in range(2):
    st = eng.store_new(O)
    eng.prof_enable(True)
    eng.prof_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f, status = st.ingest(ts, owner, 0, raise_on_error=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = eng.prof_report()
    eng.prof_enable(False)
    print("rep %d status %d %.2f ms, stats %s" % (rep, status, dt * 1e3, eng.stats()), flush=True)
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:12]:
        print("   %-32s %8.3f ms %d" % (k, v[0], v[1]))
    fl = f.cpu().numpy()
    print("   INS count", int(((fl & L.MSG_INS) != 0).sum()), "of", n, flush=True)
    if rep == 0:
        st.free()
# oracle check of sampled owners
own_np = owner.cpu().numpy().view(np.uint32)
ts_np = ts.cpu().numpy()
sample = np.unique(np.linspace(0, O - 1, 50).astype(np.int64))
m = np.isin(own_np, sample)
srv = CO.Server(O, int(m.sum()) + 1)
stc, fw = srv.ingest(ts_np[m], own_np[m])
print("oracle status", stc, "flags equal", np.array_equal(fl[m], fw), flush=True)
tree = st.tree()
bad = [int(o) for o in sample if tree.to_json(int(o)) != srv.tree_json(int(o))]
print("tree mismatches", len(bad), bad[:5], flush=True)
