"""k_diff at config-3 scale (100k owners x 1,000 messages, client trees ~90 %):
duration per EVM_OPT_DIFF_GRID setting (workgroups per CU), from the engine's
HIP events.  Usage: python tools/diff_sweep.py [grid ...]  (one JSON line)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from evolu_amd import synth  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402


def main():
    grids = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3, 4, 6, 8]
    O, P = 100_000, 1000
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    gen = synth.DeviceSynth()
    ts, own, keep = gen.source(0xE7010004, O, P, 1, 0, dev, keep=True)
    store = eng.store_new(O)
    store.ingest(ts, own, 0)
    kb = keep.bool()
    client = eng.merkle_insert(eng.tree_new(O), ts[kb].contiguous(), own[kb].contiguous())
    tree = store.tree()
    out = {}
    ref = None
    for g in grids:
        try:
            eng.set_option(6, g)
        except Exception:  # (an older build without the knob: its default grid only)
            if g:
                continue
        for _ in range(3):
            d = eng.merkle_diff(tree, client)
        if ref is None:
            ref = d.clone()
        assert torch.equal(d, ref), g
        eng.prof_enable(True)
        eng.prof_reset()
        for _ in range(10):
            eng.merkle_diff(tree, client)
        torch.cuda.synchronize()
        rep = eng.prof_report()
        eng.prof_enable(False)
        ms, n = rep["k_diff"]
        out[str(g)] = ms / n
    print(json.dumps({"k_diff_ms_by_grid": out, "owners": O, "server_leaves": tree.n_leaves,
                      "client_leaves": client.n_leaves, "some": int((ref >= 0).sum())}))


if __name__ == "__main__":
    main()
