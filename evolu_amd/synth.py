"""Seeded synthetic message streams for the BASELINE configs (numpy, vectorised).

Generator spec: SURVEY.md section 8(d).  Every timestamp is canonical and is
produced by per-node HLC sends (timestamp.ts:97-123 rules: millis = max(last,
now); counter increments when millis repeats), so (millis, counter, node)
triples are unique per node.  seed = 0xE7010000 + config number.
"""
from __future__ import annotations

import numpy as np

BENCH_T0 = 1704067200000  # 2024-01-01T00:00:00.000Z
DAY_MS = 86400000
HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
HEXU = np.frombuffer(b"0123456789ABCDEF", dtype=np.uint8)


def rng_for(config: int) -> np.random.Generator:
    return np.random.default_rng(0xE7010000 + config)


def civil_from_days(z: np.ndarray):
    z = z + 719468
    era = np.floor_divide(z, 146097)
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = np.where(mp < 10, mp + 3, mp - 9)
    return y + (m <= 2), m, d


def format_timestamps(millis: np.ndarray, counter: np.ndarray, node_bytes: np.ndarray, stride: int = 48) -> np.ndarray:
    """(n,) millis, (n,) counter, (n,16) uint8 node -> (n, stride) uint8 arena of
    timestamp.ts:43-48 strings (4-digit years only)."""
    n = millis.shape[0]
    millis = millis.astype(np.int64)
    days = millis // DAY_MS
    ms = millis - days * DAY_MS
    y, mo, d = civil_from_days(days)
    if n and (y.min() < 0 or y.max() > 9999):
        raise ValueError("year outside 0000-9999")
    hh = ms // 3600000
    mi = (ms // 60000) % 60
    ss = (ms // 1000) % 60
    sss = ms % 1000
    out = np.zeros((n, stride), dtype=np.uint8)

    def put(col, val, width):
        v = val.astype(np.int64)
        for k in range(width - 1, -1, -1):
            out[:, col + k] = 48 + (v % 10)
            v = v // 10

    put(0, y, 4)
    out[:, 4] = ord("-")
    put(5, mo, 2)
    out[:, 7] = ord("-")
    put(8, d, 2)
    out[:, 10] = ord("T")
    put(11, hh, 2)
    out[:, 13] = ord(":")
    put(14, mi, 2)
    out[:, 16] = ord(":")
    put(17, ss, 2)
    out[:, 19] = ord(".")
    put(20, sss, 3)
    out[:, 23] = ord("Z")
    out[:, 24] = ord("-")
    c = counter.astype(np.int64)
    for k in range(3, -1, -1):
        out[:, 25 + k] = HEXU[c % 16]
        c = c // 16
    out[:, 29] = ord("-")
    out[:, 30:46] = node_bytes
    return out


def random_nodes(rng, count: int, upper_frac: float = 0.0) -> np.ndarray:
    nodes = HEX[rng.integers(0, 16, size=(count, 16))]
    if upper_frac > 0:
        up = (rng.random(count) < upper_frac)[:, None] & (nodes >= ord("a"))
        nodes = np.where(up, nodes - 32, nodes).astype(np.uint8)
    return nodes


def hlc_stream(rng, n_per_node: np.ndarray, t0: int, span_ms: int, zero_gap_frac: float = 0.05):
    """Per-node HLC sends.  Returns (millis, counter, node_index) in node-major order."""
    total = int(n_per_node.sum())
    node_idx = np.repeat(np.arange(len(n_per_node)), n_per_node)
    mean_gap = max(1, span_ms // max(1, int(n_per_node.max())))
    gaps = rng.integers(1, 2 * mean_gap + 1, size=total)
    gaps[rng.random(total) < zero_gap_frac] = 0
    starts = np.concatenate([[0], np.cumsum(n_per_node)[:-1]])
    gaps[starts] = rng.integers(0, mean_gap + 1, size=len(n_per_node))
    cs = np.cumsum(gaps)
    millis = t0 + cs - np.repeat(cs[starts], n_per_node) + np.repeat(gaps[starts], n_per_node)
    # counter: position inside each run of equal millis of one node
    new_run = np.ones(total, dtype=bool)
    new_run[1:] = (millis[1:] != millis[:-1]) | (node_idx[1:] != node_idx[:-1])
    run_start = np.maximum.accumulate(np.where(new_run, np.arange(total), 0))
    counter = np.arange(total) - run_start
    if counter.max(initial=0) > 65535:
        raise ValueError("counter overflow in synthetic stream")
    return millis, counter, node_idx


def config2(n: int = 10_000_000, n_cells: int = 1000, n_nodes: int = 64, stride: int = 48, seed_config: int = 2):
    """1 owner, n messages over n_cells cells (10x10x10), n_nodes nodes, shuffled."""
    rng = rng_for(seed_config)
    per = np.full(n_nodes, n // n_nodes, dtype=np.int64)
    per[: n - per.sum()] += 1
    millis, counter, nidx = hlc_stream(rng, per, BENCH_T0, 30 * DAY_MS)
    nodes = random_nodes(rng, n_nodes)
    perm = rng.permutation(n)
    ts = format_timestamps(millis[perm], counter[perm], nodes[nidx[perm]], stride)
    cell = rng.integers(0, n_cells, size=n, dtype=np.uint32)
    return ts, cell


def config3(n_owners: int = 100_000, per_owner: int = 1000, nodes_per_owner: int = 4, stride: int = 48,
            seed_config: int = 3, request: int = 100):
    """Server ingest: n_owners x per_owner messages, as the server receives
    them: SyncRequests of one owner each (index.ts:224-248), `request`
    messages per request (an owner's messages in random order, cut into
    requests), requests of all owners in random order; request=1 shuffles
    single messages (no request structure).  Returns (ts arena, owner ids,
    millis), in batch order."""
    rng = rng_for(seed_config)
    n = n_owners * per_owner
    per = np.full(n_owners * nodes_per_owner, per_owner // nodes_per_owner, dtype=np.int64)
    per[:: nodes_per_owner] += per_owner - per.reshape(n_owners, nodes_per_owner).sum(1)
    millis, counter, nidx = hlc_stream(rng, per, BENCH_T0, 30 * DAY_MS)
    nodes = random_nodes(rng, n_owners * nodes_per_owner)
    owner = (nidx // nodes_per_owner).astype(np.uint32)
    if request <= 1:
        perm = rng.permutation(n)
    else:
        # messages are owner-major here; shuffle inside each owner, cut into requests, shuffle requests
        key = owner.astype(np.float64) + rng.random(n)  # random order inside each owner
        inner = np.argsort(key, kind="stable")
        rank = np.empty(n, dtype=np.int64)
        rank[inner] = np.arange(n)
        start = np.searchsorted(owner[inner], np.arange(n_owners))
        pos_in_owner = rank - start[owner]
        req_id = owner.astype(np.int64) * ((per_owner + request - 1) // request) + pos_in_owner // request
        n_req = n_owners * ((per_owner + request - 1) // request)
        req_order = rng.permutation(n_req)
        order_key = req_order[req_id] * (request + 1) + pos_in_owner % request
        perm = np.argsort(order_key, kind="stable")
    ts = format_timestamps(millis[perm], counter[perm], nodes[nidx[perm]], stride)
    return ts, owner[perm], millis[perm]


def config5(n_owners: int, n: int, zipf_s: float = 1.2, cells_per_owner: int = 50, nodes_per_owner: int = 4,
            stride: int = 48, seed_config: int = 5, redelivery: float = 0.10, upper_frac: float = 0.01,
            with_millis: bool = False):
    """Adversarial stream (BASELINE config 5): owner sizes Zipf(s); per owner
    its nodes send on a coarse shared time grid, so many messages share millis
    across nodes (ties broken by counter, then by node bytes) and nodes repeat
    millis (counter increments); ~1 % of nodes carry upper-case hex; a
    `redelivery` fraction of messages is re-sent later in the batch (same
    owner, same cell: half of them after a newer write to that cell -> the
    stale-redelivery XOR toggle of applyMessages).  Returns (ts arena, owner
    u32, cell u32 global ids = owner * cells_per_owner + local cell), batch
    order; with_millis adds each message's millis (int64) as a fourth."""
    rng = rng_for(seed_config)
    w = 1.0 / np.arange(1, n_owners + 1, dtype=np.float64) ** zipf_s
    base = int(n * (1 - redelivery))
    counts = rng.multinomial(base, w / w.sum())
    owner = np.repeat(np.arange(n_owners, dtype=np.int64), counts)
    node_local = rng.integers(0, nodes_per_owner, size=base)
    gnode = owner * nodes_per_owner + node_local
    # coarse grid: ~4 messages per slot per owner -> frequent equal millis
    slots = np.maximum(1, counts // 4)
    millis = BENCH_T0 + (rng.random(base) * slots[owner]).astype(np.int64) * 1000
    # per (node, millis): counter = rank of the message among that node's equal-millis sends
    order = np.lexsort((np.arange(base), millis, gnode))
    g_s, m_s = gnode[order], millis[order]
    new_run = np.ones(base, dtype=bool)
    new_run[1:] = (g_s[1:] != g_s[:-1]) | (m_s[1:] != m_s[:-1])
    run_start = np.maximum.accumulate(np.where(new_run, np.arange(base), 0))
    counter = np.empty(base, dtype=np.int64)
    counter[order] = np.arange(base) - run_start
    nodes = random_nodes(rng, n_owners * nodes_per_owner, upper_frac=upper_frac)
    cell = owner * cells_per_owner + rng.integers(0, cells_per_owner, size=base)
    perm = rng.permutation(base)
    ts = format_timestamps(millis[perm], counter[perm], nodes[gnode[perm]], stride)
    owner, cell, ms = owner[perm], cell[perm], millis[perm]
    # redeliveries: copies of earlier messages appended later in the batch
    k = n - base
    src = rng.integers(0, base, size=k)
    ts = np.concatenate([ts, ts[src]])
    owner = np.concatenate([owner, owner[src]])
    cell = np.concatenate([cell, cell[src]])
    ms = np.concatenate([ms, ms[src]])
    mix = rng.permutation(n - base) + base  # interleave the copies among the tail
    tail = np.arange(base, n)
    ts[tail], owner[tail], cell[tail], ms[tail] = ts[mix], owner[mix], cell[mix], ms[mix]
    if with_millis:
        return ts, owner.astype(np.uint32), cell.astype(np.uint32), ms
    return ts, owner.astype(np.uint32), cell.astype(np.uint32)


# ---------------------------------------------------------------------------
# Config 4 (1B messages over 1M owners, sharded by murmur3(userId) mod G):
# generated on the device by libevmsynth.so (evolu_amd/csrc/evm_synth.hip);
# this is its numpy twin (same bytes), for tests and small cases.
# ---------------------------------------------------------------------------
C4_SPAN = 30 * DAY_MS
C4_PERM_A = 1000003
_U = np.uint64


def _sm(x):
    with np.errstate(over="ignore"):
        z = x + _U(0x9E3779B97F4A7C15)
        z = (z ^ (z >> _U(30))) * _U(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U(27))) * _U(0x94D049BB133111EB)
        return z ^ (z >> _U(31))


def _H(seed, t, x, y):
    x = np.asarray(x).astype(np.uint64)
    y = np.asarray(y).astype(np.uint64)
    s = _sm(np.full(1, seed, dtype=np.uint64) ^ _U(t))
    return _sm(_sm(s ^ x) ^ y)


def config4_shape(P: int):
    slots = max(1, ((P + 3) // 4 + 1) // 2)
    return slots, C4_SPAN // slots, slots * 9 // 10


def _hex16(v: np.ndarray) -> np.ndarray:
    sh = np.arange(60, -1, -4, dtype=np.uint64)
    return HEX[((v[:, None] >> sh[None, :]) & _U(15)).astype(np.int64)]


def config4_owner_ids(seed: int, n: int) -> np.ndarray:
    """userId strings of owners 0..n-1: (n, 21) uint8, lower-case hex."""
    o = np.arange(n, dtype=np.uint64)
    a = _H(seed, 1, o, 0)
    b = _H(seed, 1, o, 1) >> _U(44)
    tail = HEX[((b[:, None] >> np.arange(16, -1, -4, dtype=np.uint64)[None, :]) & _U(15)).astype(np.int64)]
    return np.concatenate([_hex16(a), tail], 1)


def config4_messages(seed: int, P: int, o: np.ndarray, j: np.ndarray):
    """Message j of owner o -> (ts rows (n, 48), keep bool)."""
    slots, gap, keep_slots = config4_shape(P)
    o = np.asarray(o, dtype=np.int64)
    j = np.asarray(j, dtype=np.int64)
    q, k = j & 3, j >> 2
    slot, ctr = k >> 1, k & 1
    h = _H(seed, 3, o, (q << 16) | slot)
    millis = BENCH_T0 + slot * gap + (h % _U(gap)).astype(np.int64)
    node = _hex16(_H(seed, 2, o, q))
    return format_timestamps(millis, ctr, node, 48), slot < keep_slots


def config4_source(seed: int, O: int, P: int, G: int, s: int):
    """Source rank s of G: (ts, owner u32, keep) -- twin of evs_config4_source."""
    m = (P - s + G - 1) // G
    r = np.arange(O * m, dtype=np.int64)
    p, t = r // m, r % m
    o = (p * C4_PERM_A + seed % O) % O
    ts, keep = config4_messages(seed, P, o, s + t * G)
    return ts, o.astype(np.uint32), keep


def config4_owners(seed: int, P: int, G: int, owners: np.ndarray):
    """All P messages of each owner, source-major for G sources (the order a
    rank receives them): (ts, list index u32, keep) -- twin of evs_config4_owners."""
    owners = np.asarray(owners, dtype=np.int64)
    js = np.concatenate([np.arange(s, P, G) for s in range(G)])
    o = np.repeat(owners, P)
    j = np.tile(js, len(owners))
    ts, keep = config4_messages(seed, P, o, j)
    return ts, np.repeat(np.arange(len(owners), dtype=np.uint32), P), keep


def config5_cdf(O: int, zipf_s: float = 1.2) -> np.ndarray:
    """Cumulative Zipf(s) owner probabilities (float64[O]) -- the config-5
    shape generator's input (the device and the twin search the same array)."""
    w = 1.0 / np.arange(1, O + 1, dtype=np.float64) ** zipf_s
    return np.cumsum(w / w.sum())


def config5_shape(seed: int, O: int, n: int, cdf: np.ndarray = None):
    """Twin of evs_config5_shape (evm_synth.hip): (ts (n, 48), owner u32, keep
    bool) -- Zipf owners, 4 nodes per owner (1 % upper-case), a 1-second
    grid of ~4 messages per slot per owner, shuffled, the last n / 10 rows
    exact redeliveries of earlier ones."""
    cdf = config5_cdf(O) if cdf is None else cdf
    base = n - n // 10 or n
    r = np.arange(n, dtype=np.uint64)
    src = np.where(r < _U(base), r, _H(seed, 9, r, 0) % _U(base)).astype(np.uint64)
    u = (_H(seed, 4, src, 0) >> _U(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    o = np.minimum(np.searchsorted(cdf, u, side="right"), O - 1).astype(np.int64)
    q = (_H(seed, 5, src, 0) & _U(3)).astype(np.int64)
    node = _hex16(_H(seed, 2, o, q))
    upper = (_H(seed, 6, o, q) % _U(100)) == 0
    node = np.where(upper[:, None] & (node >= ord("a")), node - 32, node).astype(np.uint8)
    p = cdf[o] - np.where(o > 0, cdf[np.maximum(o - 1, 0)], 0.0)
    slots = np.maximum(1, (np.float64(base) * p).astype(np.uint64) // _U(4)).astype(np.uint64)
    millis = BENCH_T0 + ((_H(seed, 7, src, 0) % slots).astype(np.int64)) * 1000
    ctr = (_H(seed, 8, src, 0) % _U(1024)).astype(np.int64)
    keep = (_H(seed, 10, src, 0) % _U(10)) != 0
    return format_timestamps(millis, ctr, node, 48), o.astype(np.uint32), keep


class DeviceSynth:
    """libevmsynth.so: the config-4 generator on the device (torch tensors)."""

    def __init__(self):
        import ctypes as C
        import os

        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libevmsynth.so")
        if not os.path.exists(path):
            raise RuntimeError("libevmsynth.so not built (%s)" % path)
        import torch  # noqa: F401  (one HIP runtime in the process)

        self.C = C
        L = C.CDLL(path)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        L.evs_config4_source.argtypes = [vp, u64, u32, u32, u32, u32, vp, vp, vp]
        L.evs_config4_owners.argtypes = [vp, u64, u32, u32, u32, vp, u32, vp, vp, vp]
        L.evs_owner_ids.argtypes = [vp, u64, u32, C.c_size_t, vp]
        L.evs_config5_shape.argtypes = [vp, u64, u32, u64, vp, vp, vp, vp]
        self.L = L

    @staticmethod
    def _p(t):
        import ctypes as C

        return None if t is None else C.c_void_p(t.data_ptr())

    def _stream(self, dev):
        import torch

        return self.C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def source(self, seed: int, O: int, P: int, G: int, s: int, dev, keep: bool = False):
        import torch

        m = (P - s + G - 1) // G
        n = O * m
        ts = torch.empty((n, 48), dtype=torch.uint8, device=dev)
        owner = torch.empty(n, dtype=torch.int32, device=dev)
        kp = torch.empty(n, dtype=torch.uint8, device=dev) if keep else None
        if self.L.evs_config4_source(self._stream(dev), seed, O, P, G, s, self._p(ts), self._p(owner), self._p(kp)):
            raise ValueError("evs_config4_source: bad arguments")
        return ts, owner, kp

    def owners(self, seed: int, O: int, P: int, G: int, owners, dev):
        import torch

        lst = owners.to(device=dev, dtype=torch.int32).contiguous()
        n = lst.numel() * P
        ts = torch.empty((max(n, 1), 48), dtype=torch.uint8, device=dev)
        li = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        kp = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        if self.L.evs_config4_owners(self._stream(dev), seed, O, P, G, self._p(lst), lst.numel(), self._p(ts),
                                     self._p(li), self._p(kp)):
            raise ValueError("evs_config4_owners: bad arguments")
        return ts[:n], li[:n], kp[:n]

    def owner_ids(self, seed: int, n: int, dev, stride: int = 24):
        import torch

        out = torch.empty((max(n, 1), stride), dtype=torch.uint8, device=dev)
        if self.L.evs_owner_ids(self._stream(dev), seed, n, stride, self._p(out)):
            raise ValueError("evs_owner_ids: bad arguments")
        return out[:n]


def client_adversarial(n: int = 10_000_000, n_cells: int = 1000, n_nodes: int = 64, stride: int = 48,
                       seed_config: int = 5):
    """BASELINE config 5 on the client side: ONE owner's applyMessages batch
    with config 5's adversarial structure (config5 above with one owner):
    millis on a coarse shared grid (equal-millis bursts across nodes: counter
    and node tie-breaks), 10 % redeliveries (half after a newer write to the
    cell: the stale XOR toggle; the rest exact copies of the cell max: ties),
    ~1 % upper-case nodes.  Returns (ts arena, cell u32)."""
    ts, _, cell = config5(1, n, cells_per_owner=n_cells, nodes_per_owner=n_nodes, stride=stride,
                          seed_config=seed_config)
    return ts, cell


NANOID = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_-", dtype=np.uint8)

# examples/nextjs/pages/index.tsx:23-34 + the common columns (types.ts:194-201)
TODO_COLUMNS = ("title", "isCompleted", "categoryId", "isDeleted")
CATEGORY_COLUMNS = ("name", "isDeleted")


def config1(n: int = 100_000, n_nodes: int = 3, stride: int = 48, seed_config: int = 1):
    """BASELINE config 1: one owner's todo app (examples/nextjs schema) as n
    CrdtMessages, the batch a client merges with applyMessages.

    Mutations (db.ts:268-300 createNewCrdtMessages: an insert appends
    createdAt + createdBy, an update appends updatedAt), mix 20 % todo insert
    (title, isCompleted, categoryId), 5 % category insert (name), 75 % update
    of one column of a random existing row (todo: title / isCompleted /
    categoryId / isDeleted; category: name / isDeleted).  Each mutation comes
    from one of n_nodes nodes at `now` += U[0, 20) ms, its messages stamped by
    that node's sendTimestamp (timestamp.ts:97-123: millis = max(last, now),
    counter + 1 on a repeat).  Row ids: 21-char nanoid alphabet.  Batch order =
    send order (the server returns ORDER BY timestamp per sender).
    Returns (ts arena, cell u32, cells [(table, row, column)], values list)."""
    rng = rng_for(seed_config)
    nodes = random_nodes(rng, n_nodes)
    owner_id = bytes(HEX[rng.integers(0, 16, size=21)]).decode()  # initDbModel.ts:21-22: 21 hex chars
    node_state = [(0, 0)] * n_nodes
    todos, cats = [], []
    cid = {}
    cells = []
    millis, counter, nidx, cell, values = [], [], [], [], []
    now = BENCH_T0

    def rid():
        return bytes(NANOID[rng.integers(0, 64, size=21)]).decode()

    def iso(ms):
        return format_timestamps(np.array([ms]), np.array([0]), np.zeros((1, 16), np.uint8) + 48)[0, :24].tobytes().decode()

    while len(millis) < n:
        now += int(rng.integers(0, 20))
        node = int(rng.integers(0, n_nodes))
        u = rng.random()
        if u < 0.20 or not todos:
            row = rid()
            todos.append(row)
            cat = cats[int(rng.integers(0, len(cats)))] if cats and rng.random() < 0.5 else None
            msgs = [("todo", row, "title", "todo %d" % len(todos)), ("todo", row, "isCompleted", 0),
                    ("todo", row, "categoryId", cat), ("todo", row, "createdAt", iso(now)),
                    ("todo", row, "createdBy", owner_id)]
        elif u < 0.25:
            row = rid()
            cats.append(row)
            msgs = [("todoCategory", row, "name", "category %d" % len(cats)), ("todoCategory", row, "createdAt", iso(now)),
                    ("todoCategory", row, "createdBy", owner_id)]
        else:
            if cats and rng.random() < 0.2:
                row, table = cats[int(rng.integers(0, len(cats)))], "todoCategory"
                col = CATEGORY_COLUMNS[int(rng.integers(0, 2))]
                val = 1 if col == "isDeleted" else "renamed %d" % len(millis)
            else:
                row, table = todos[int(rng.integers(0, len(todos)))], "todo"
                col = TODO_COLUMNS[int(rng.integers(0, 4))]
                val = {"title": "edited %d" % len(millis), "isCompleted": int(rng.integers(0, 2)),
                       "categoryId": cats[int(rng.integers(0, len(cats)))] if cats else None, "isDeleted": 1}[col]
            msgs = [(table, row, col, val), (table, row, "updatedAt", iso(now))]
        m, c = node_state[node]
        for table, row, col, val in msgs:
            if len(millis) == n:
                break
            if now > m:  # sendTimestamp
                m, c = now, 0
            else:
                c += 1
            key = (table, row, col)
            k = cid.get(key)
            if k is None:
                k = cid[key] = len(cells)
                cells.append(key)
            millis.append(m)
            counter.append(c)
            nidx.append(node)
            cell.append(k)
            values.append(val)
        node_state[node] = (m, c)
    ts = format_timestamps(np.array(millis, dtype=np.int64), np.array(counter, dtype=np.int64), nodes[np.array(nidx)],
                           stride)
    return ts, np.array(cell, dtype=np.uint32), cells, values


def device_config5_shape(gen: "DeviceSynth", seed: int, O: int, n: int, dev, zipf_s: float = 1.2):
    """evs_config5_shape on the device -> (ts (n, 48) uint8, owner int32, keep uint8) tensors."""
    import torch

    cdf = torch.from_numpy(config5_cdf(O, zipf_s)).to(dev)
    ts = torch.empty((max(n, 1), 48), dtype=torch.uint8, device=dev)
    owner = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    keep = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    if gen.L.evs_config5_shape(gen._stream(dev), seed, O, n, gen._p(cdf), gen._p(ts), gen._p(owner), gen._p(keep)):
        raise ValueError("evs_config5_shape: bad arguments")
    torch.cuda.current_stream(dev).synchronize()  # (cdf is freed on return)
    return ts[:n], owner[:n], keep[:n]
