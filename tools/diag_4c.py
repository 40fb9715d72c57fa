"""Which client path do config4c's per-owner batches take? (diagnostic)"""
import numpy as np
import torch

from evolu_amd import synth
from evolu_amd.engine import Dist, Engine, dist_unique_id

eng = Engine(0)
ts_np, cell_np = synth.config2(1_250_000, 1000, seed_config=40000)
ts, cell = eng.dev(ts_np), eng.dev(cell_np)
empty = eng.tree_new(1)
flags = torch.empty(len(ts_np), dtype=torch.uint8, device="cuda")
win = torch.empty(1000, dtype=torch.int32, device="cuda")


def run(tag, t, c):
    eng.prof_enable(True)
    eng.prof_reset()
    s0 = eng.stats()
    _, _, tree, st = eng.apply_batch(empty, t, c, 1000, flags=flags[: t.shape[0]], winner=win)
    torch.cuda.synchronize()
    s1 = eng.stats()
    rep = eng.prof_report()
    eng.prof_enable(False)
    print(tag, "status", st, {k: s1[k] - s0[k] for k in ("tc_batches", "tc_redos")},
          sorted(((k, round(v[0], 3), v[1]) for k, v in rep.items()), key=lambda x: -x[1])[:8], flush=True)
    tree.free()


run("direct", ts, cell)
d = Dist(eng, dist_unique_id(), 0, 1)
own = eng.dev(np.zeros(len(ts_np), dtype=np.uint32))
d.route(ts, own, aux=cell)
t2, o2, c2, _, g = d.take(group=8)
print("group_off", g)
run("routed", t2, c2)
print("same rows", bool(torch.equal(t2, ts)), bool(torch.equal(c2, cell.view(torch.int32))))
# 8 owners: each a slice of one config2 stream (as bench client_routed at world 1)
M = 10_000_000
rng = np.random.default_rng(4000)
owner_np = rng.integers(0, 8, M).astype(np.uint32)
cnt = np.bincount(owner_np, minlength=8)
big = np.empty((M, 48), dtype=np.uint8)
bc = np.empty(M, dtype=np.uint32)
for gg in range(8):
    t_g, c_g = synth.config2(int(cnt[gg]), 1000, seed_config=40_000 + 64 * gg)
    at = np.nonzero(owner_np == gg)[0]
    big[at] = t_g
    bc[at] = c_g
    mins = np.unique(t_g[:, :16].copy().view("S16"))
    print("owner", gg, "n", cnt[gg], "minutes", mins[0], mins[-1])
d.route(eng.dev(big), eng.dev(owner_np), aux=eng.dev(bc))
t2, o2, c2, _, g = d.take(group=8)
for gg in range(3):
    run("owner%d" % gg, t2[g[gg]:g[gg + 1]].contiguous(), c2[g[gg]:g[gg + 1]].contiguous())
d.free()
