"""Segment path vs sort path: first mismatching flags (diagnostic)."""
import numpy as np

from evolu_amd import _lib as L
from evolu_amd import synth
from evolu_amd.engine import Engine

eng = Engine(0)
ts_np, owner_np, _ = synth.config5(200, 600_000, seed_config=61)
cut = len(ts_np) * 3 // 5
cnt = np.bincount(owner_np, minlength=200)
print("owners >1024:", int((cnt > 1024).sum()), "max", cnt.max())
res = {}
for path in (0, 2):
    eng.set_option(L.OPT_SERVER_PATH, path)
    store = eng.store_new(200)
    fl = []
    for a, b in ((0, cut), (cut, len(ts_np))):
        f, st = store.ingest(eng.dev(ts_np[a:b]), eng.dev(owner_np[a:b]), a)
        fl.append(f.cpu().numpy().copy())
        print("path", path, "ingest", a, b, "status", st, "inserted", int((fl[-1] == 4).sum()), flush=True)
    res[path] = np.concatenate(fl)
    store.free()
bad = np.nonzero(res[0] != res[2])[0]
print("mismatches", len(bad), "first", bad[:10])
for i in bad[:10]:
    t = bytes(ts_np[i, :46]).decode()
    same = np.nonzero((ts_np[:, :46] == ts_np[i, :46]).all(1) & (owner_np == owner_np[i]))[0]
    print(i, "owner", owner_np[i], "cnt", cnt[owner_np[i]], t, "seg", res[0][i], "sort", res[2][i], "copies", same)
