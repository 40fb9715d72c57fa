"""Fixed cost of one evm_apply_batch call (host launches + syncs + Python
wrapper), from tiny batches where the kernels take ~nothing.

    python tools/call_overhead.py
"""
import time

import torch

from evolu_amd import synth
from evolu_amd.engine import Engine


def main():
    eng = Engine(0)
    for n in (1024, 65536, 1 << 20):
        ts_np, cell_np = synth.config2(n, 1000, seed_config=2)
        ts, cell = eng.dev(ts_np), eng.dev(cell_np)
        flags = torch.empty(n, dtype=torch.uint8, device=ts.device)
        winner = torch.empty(1000, dtype=torch.int32, device=ts.device)
        empty = eng.tree_new(1)
        for _ in range(20):
            eng.apply_batch(empty, ts, cell, 1000, flags=flags, winner=winner)[2].free()
        torch.cuda.synchronize()
        reps = 200
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.apply_batch(empty, ts, cell, 1000, flags=flags, winner=winner)[2].free()
        torch.cuda.synchronize()
        print("n=%8d  %.1f us/call" % (n, (time.perf_counter() - t0) / reps * 1e6), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
