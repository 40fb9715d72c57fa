"""Config-3 rounds through the native sync server (evm_sync_round) on
bench.py's bodies: device-resident rounds and host-bodies rounds (pinned H2D
-> round -> pinned D2H), two of each on fresh servers, timed by part.
`python tools/e2e_host.py` (E2E_OWNERS to shrink, E2E_HOST=0: device rounds only)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from evolu_amd import synth  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402
from evolu_amd.server import SyncServer  # noqa: E402

owners, per = int(os.environ.get("E2E_OWNERS", 100_000)), 1000
ts_np, owner_np, millis = synth.config3(owners, per, seed_config=3, request=per)
eng = Engine(0)
dev = torch.device("cuda", 0)
ts_r = eng.dev(ts_np)
lown = torch.from_numpy(owner_np.astype(np.int32)).to(dev)
o64 = owner_np.astype(np.int64)
order = np.lexsort((millis, o64))
rank = np.empty(len(order), dtype=np.int64)
cnt = np.bincount(o64, minlength=owners)
rank[order] = np.arange(len(order)) - (np.cumsum(cnt) - cnt)[o64[order]]
keep = torch.from_numpy(rank < (0.9 * cnt[o64]).astype(np.int64)).to(dev)
client = eng.merkle_insert(eng.tree_new(owners), ts_r[keep].contiguous(), lown[keep].contiguous())
arena, off = bench.e2e_bodies(eng, ts_np, owner_np, client)
del ts_r, lown, keep
client.free()
print("bodies ready: %d bytes" % int(off[-1]), flush=True)
a_d = torch.from_numpy(arena).to(dev)
pick = np.linspace(0, len(off) - 2, 8).round().astype(np.int64)
ref = None
for rep in range(3):
    srv = SyncServer(eng, owners)
    if rep == 2:  # (a profiled round: the kernels' times)
        eng.prof_enable(True)
        eng.prof_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = srv.sync_device(a_d, off)
    torch.cuda.synchronize()
    if rep == 2:
        prof = eng.prof_report()
        eng.prof_enable(False)
        print("kernels ms", {k: round(v[0], 3) for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:14]})
    else:
        print("device round %.1f ms" % ((time.perf_counter() - t0) * 1e3),
              {k: round(v * 1e3, 2) for k, v in srv.timing.items()}, flush=True)
    ref = [res.get(int(k)) for k in pick]
    srv.close()
del a_d
torch.cuda.empty_cache()
for rep in range(int(os.environ.get("E2E_HOST", 2))):
    srv = SyncServer(eng, owners)
    t0 = time.perf_counter()
    out = srv.sync_arena(arena, off)
    wall = time.perf_counter() - t0
    same = all(bytes(out[int(k)]) == r for k, r in zip(pick, ref))
    print("host round %.1f ms (responses %d bytes, sample same as device: %s)"
          % (wall * 1e3, sum(len(x) for x in out if isinstance(x, memoryview)), same),
          {k: round(v * 1e3, 2) for k, v in srv.timing.items()}, flush=True)
    del out
    srv.close()
