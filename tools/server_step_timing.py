"""Wall time of each call of one server bench step (diagnostic)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from evolu_amd import synth  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402

owners, per = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 100_000, 1000
ts_np, owner_np, millis = synth.config3(owners, per, seed_config=3)
eng = Engine(0)
ts = eng.dev(ts_np)
own = torch.from_numpy(owner_np.astype(np.int32)).cuda()
node = torch.from_numpy(np.frombuffer(b"0123456789abcdef" * owners, dtype=np.uint8).copy()).cuda()
client = eng.tree_new(owners)
flags = torch.empty(len(ts_np), dtype=torch.uint8, device="cuda")
if "--prof" in sys.argv:
    eng.prof_enable(True)
for it in range(4):
    t = [time.perf_counter()]
    store = eng.store_new(owners)
    torch.cuda.synchronize(); t.append(time.perf_counter())
    store.ingest(ts, own, 0, flags=flags)
    torch.cuda.synchronize(); t.append(time.perf_counter())
    diff, off, ids = store.select(client, node)
    torch.cuda.synchronize(); t.append(time.perf_counter())
    r, p = store.tree().roots()
    t.append(time.perf_counter())
    store.free()
    torch.cuda.synchronize(); t.append(time.perf_counter())
    d = np.diff(t) * 1e3
    print("store_new %.2f ingest %.2f select %.2f roots %.2f free %.2f ms" % tuple(d), flush=True)
