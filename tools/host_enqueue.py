"""Host cost of enqueuing one config-2 applyMessages batch (evm_apply_batch_async):
wall time of the call itself, the GPU time of a batch, and what a pipelined loop
achieves (diagnostic for the bench's host-bound gaps)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from evolu_amd import synth  # noqa: E402
from evolu_amd.engine import Engine  # noqa: E402

n, C = 10_000_000, 1000
ts_np, cell_np = synth.config2(n, C, seed_config=2)
eng = Engine(0)
ts, cell = eng.dev(ts_np), eng.dev(cell_np)
empty = eng.tree_new(1)
outs = [(torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(C, dtype=torch.int32, device="cuda"))
        for _ in range(4)]
for _ in range(3):
    eng.apply_batch_async(empty, ts, cell, C, *outs[0]).wait()[2].free()
torch.cuda.synchronize()
enq = []
pend = []
for k in range(4):
    t0 = time.perf_counter()
    pend.append(eng.apply_batch_async(empty, ts, cell, C, *outs[k]))
    enq.append((time.perf_counter() - t0) * 1e6)
w0 = time.perf_counter()
for p in pend:
    p.wait()[2].free()
torch.cuda.synchronize()
print("enqueue us per batch:", [round(x, 1) for x in enq])
print("4 batches drained in %.1f us after the enqueues" % ((time.perf_counter() - w0) * 1e6))
# a raw empty launch through torch for scale
x = torch.zeros(1, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100):
    x.add_(1)
t1 = time.perf_counter()
torch.cuda.synchronize()
print("torch tiny launch: %.1f us each (host)" % ((t1 - t0) / 100 * 1e6))
