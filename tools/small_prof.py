"""Per-kernel times of the small-batch client path (EVM_OPT_CLIENT_PATH 4)
and wall time per call at the config-1 sizes a client applies -- where the
latency of one applyMessages batch goes.  python tools/small_prof.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from evolu_amd import synth  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402


def main():
    eng = Engine(0)
    ts_np, cell_np, _, _ = synth.config1(100_000)
    empty = eng.tree_new(1)
    out = {}
    for path in (4, 0):
        eng.set_option(1, path)
        for k in (100, 1000, 10_000, 100_000):
            used, cid = np.unique(cell_np[:k], return_inverse=True)
            ts, cell = eng.dev(ts_np[:k]), eng.dev(cid.astype(np.uint32))
            fl = torch.empty(k, dtype=torch.uint8, device=ts.device)
            wn = torch.empty(len(used), dtype=torch.int32, device=ts.device)

            def one():
                eng.apply_batch(empty, ts, cell, len(used), flags=fl, winner=wn)[2].free()

            for _ in range(5):
                one()
            eng.prof_enable(True)
            eng.prof_reset()
            for _ in range(20):
                one()
            prof = eng.prof_report()
            eng.prof_enable(False)
            xs = []
            for _ in range(40):
                t0 = time.perf_counter()
                one()
                xs.append((time.perf_counter() - t0) * 1e3)
            xs.sort()
            out["path%d_%d" % (path, k)] = {
                "p50_ms": xs[len(xs) // 2],
                "kernels_us": {kk: round(v[0] / 20 * 1e3, 1) for kk, v in sorted(prof.items(), key=lambda kv: -kv[1][0])},
                "stats": eng.stats(),
            }
    eng.set_option(1, 0)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
