"""Seeded small workloads with the edge cases the parity tests need."""
from __future__ import annotations

import random

from oracle import evolu_oracle as O

T0 = 1704067200000


def node_id(rng: random.Random, upper: bool = False) -> str:
    s = "".join(rng.choice("0123456789abcdef") for _ in range(16))
    if upper:
        s = "".join(c.upper() if c.isalpha() and rng.random() < 0.5 else c for c in s)
    return s


def hlc_timestamps(rng: random.Random, count: int, nodes, t0=T0, span=3600_000, tie_frac=0.3):
    """Timestamps from per-node HLC sends (timestamp.ts:97-123), many equal millis."""
    state = {n: (t0, 0) for n in nodes}
    out = []
    shared_now = t0
    for _ in range(count):
        n = rng.choice(nodes)
        if rng.random() >= tie_frac:
            shared_now += rng.randrange(0, span // max(1, count) * 2 + 2)
        m, c = state[n]
        now = shared_now
        if now > m:
            m, c = now, 0
        else:
            c += 1
        state[n] = (m, c)
        out.append(O.timestamp_to_string(m, c, n))
    return out


def client_batch(seed: int, n: int = 400, n_cells: int = 12, n_nodes: int = 4, upper: bool = True,
                 redeliver: float = 0.15, t0=T0):
    """A CrdtMessage batch over a few cells with ties, redeliveries (some stale)."""
    rng = random.Random(seed)
    nodes = [node_id(rng, upper and i % 2 == 1) for i in range(n_nodes)]
    if upper and n_nodes >= 2:
        # same hex, different case: exercises the case-rank order
        nodes[-1] = nodes[0].upper() if nodes[0].upper() != nodes[0] else nodes[-1]
    cells = [("todo", "row%02d" % (i // 3), ["title", "isCompleted", "categoryId"][i % 3]) for i in range(n_cells)]
    tss = hlc_timestamps(rng, n, nodes, t0=t0)
    msgs = []
    for i, ts in enumerate(tss):
        c = cells[rng.randrange(n_cells)]
        msgs.append({"timestamp": ts, "table": c[0], "row": c[1], "column": c[2], "value": "v%d" % i})
    # redeliveries: exact copies re-appended (same cell), some after newer writes
    extra = []
    for _ in range(int(n * redeliver)):
        m = dict(rng.choice(msgs))
        extra.append(m)
    for m in extra:
        msgs.insert(rng.randrange(len(msgs) + 1), m)
    return msgs, cells
