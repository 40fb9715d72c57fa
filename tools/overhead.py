"""Host-overhead probe: wall time of evm_apply_batch on tiny batches (the
per-call floor) on the default stream and on a dedicated stream."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np
import torch

from evolu_amd import synth
from evolu_amd.engine import Engine

eng = Engine(0)
for n in (64, 100_000, 1_000_000):
    ts_np, cell_np = synth.config2(n, 1000)
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    empty = eng.tree_new(1)
    for label in ("default", "own"):
        if label == "own":
            s = torch.cuda.Stream()
            eng.bind_stream(s)
        for _ in range(3):
            eng.apply_batch(empty, ts, cell, 1000)[2].free()
        torch.cuda.synchronize()
        t = time.perf_counter()
        k = 20
        for _ in range(k):
            tr = eng.apply_batch(empty, ts, cell, 1000)[2]
            tr.free()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / k
        print("n=%8d %-8s %8.1f us/call" % (n, label, dt * 1e6), flush=True)
    eng.bind_stream(torch.cuda.current_stream())
