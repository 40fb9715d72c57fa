"""One config-3 device round (SyncServer.sync_device) on bench.py's bodies, for
profiling its kernels alone: `rocprofv3 ... -- python tools/e2e_once.py`."""
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
a_d = torch.from_numpy(arena).to(dev)
print("bodies ready", flush=True)
srv = SyncServer(eng, owners)
torch.cuda.synchronize()
t0 = time.perf_counter()
res = srv.sync_device(a_d, off)
torch.cuda.synchronize()
print("round %.1f ms" % ((time.perf_counter() - t0) * 1e3), {k: round(v * 1e3, 2) for k, v in srv.timing.items()},
      flush=True)
srv.close()
