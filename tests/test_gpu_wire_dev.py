"""The server round on bodies resident in device memory (SyncServer.sync_device:
evm_pb_scan_dev / split_dev, evm_tree_from_json_dev,
evm_pb_encode_responses_dev) against the host codecs and the host path on the
same bodies, and against the oracle's ServerDb.sync (index.ts:204-251):
byte-identical responses, the same errors, the same store."""
import ctypes as C
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import evolu_oracle as O
from tests import workloads as W
from tests.test_gpu_wire import _expected, _requests
from tests.test_wire import REQ

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


def _arena(bodies):
    off = np.zeros(len(bodies) + 1, dtype=np.uint64)
    np.cumsum([len(b) for b in bodies], out=off[1:])
    return np.frombuffer(b"".join(bodies) or b"\0", dtype=np.uint8).copy(), off


def _P(x):
    return C.c_void_p(x.data_ptr())


def test_scan_and_split_equal_the_host_codec(eng):
    from evolu_amd import _lib as L

    lib = L.load()
    bodies = _requests(4, n_users=8, n_req=60)
    bodies.insert(3, b"\x0a\x05ab")                      # truncated
    bodies.insert(9, b"\x08\x01" + bodies[9])            # an unknown varint field first: skipped
    bodies.insert(12, b"\x0b")                           # a group: rejected
    bodies.insert(15, b"")                               # empty: all defaults
    bodies.insert(18, REQ(messages=[dict(timestamp="short", content=b"x")], userId="u", nodeId="0123456789abcdef",
                          merkleTree="{}").SerializeToString())  # a timestamp that is not 46 bytes
    arena, off = _arena(bodies)
    n = len(bodies)
    from evolu_amd import wire

    hinfo = (wire._Sync * n)()
    hst = np.zeros(n, dtype=np.int32)
    L.check(lib.evm_pb_scan_batch(L.PB_SYNC_REQUEST, C.c_void_p(arena.ctypes.data), C.c_void_p(off.ctypes.data), n,
                                  hinfo, C.c_void_p(hst.ctypes.data)), "scan")
    hi = np.ctypeslib.as_array(hinfo).view(np.uint64).reshape(n, 9)
    a_d, off_d = eng.dev(arena), eng.dev(off.view(np.int64))
    info_d = torch.empty((n, 9), dtype=torch.int64, device=a_d.device)
    st_d = torch.empty(n, dtype=torch.int32, device=a_d.device)
    L.check(lib.evm_pb_scan_dev(eng.h, L.PB_SYNC_REQUEST, _P(a_d), _P(off_d), n, _P(info_d), _P(st_d)), "scan_dev")
    assert (st_d.cpu().numpy() == hst).all()
    assert (info_d.cpu().numpy().view(np.uint64) == hi).all()
    assert hst[3] != 0 and hst[12] != 0 and hst[15] == 0 and hi[18, 8] == 1
    # split
    mb = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(hi[:, 0], out=mb[1:])
    cb = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(hi[:, 1], out=cb[1:])
    N, CB = int(mb[-1]), int(cb[-1])
    hts = np.zeros((max(N, 1), 48), dtype=np.uint8)
    hco = np.zeros(N + 1, dtype=np.uint64)
    hc = np.zeros(max(CB, 1), dtype=np.uint8)
    p = lambda x: C.c_void_p(x.ctypes.data)  # noqa: E731
    L.check(lib.evm_pb_split_batch(L.PB_SYNC_REQUEST, p(arena), p(off), n, p(hst), p(mb), p(cb), p(hts), 48, None, None,
                                   p(hco), p(hc)), "split")
    dts = torch.zeros((max(N, 1), 48), dtype=torch.uint8, device=a_d.device)
    dco = torch.zeros(N + 1, dtype=torch.int64, device=a_d.device)
    dco[N] = CB
    dc = torch.zeros(max(CB, 1), dtype=torch.uint8, device=a_d.device)
    own_of = torch.arange(n, dtype=torch.int32, device=a_d.device) + 7
    down = torch.zeros(max(N, 1), dtype=torch.int32, device=a_d.device)
    mb_d, cb_d = eng.dev(mb.view(np.int64)), eng.dev(cb.view(np.int64))
    L.check(lib.evm_pb_split_dev(eng.h, L.PB_SYNC_REQUEST, _P(a_d), _P(off_d), n, _P(st_d), _P(mb_d), _P(cb_d),
                                 _P(own_of), _P(dts), 48, _P(dco), _P(dc), _P(down)), "split_dev")
    assert (dts.cpu().numpy()[:N] == hts[:N]).all()
    assert (dco.cpu().numpy().view(np.uint64) == hco).all()
    assert (dc.cpu().numpy()[:CB] == hc[:CB]).all()
    assert (down.cpu().numpy()[:N] == np.repeat(np.arange(n) + 7, hi[:, 0].astype(np.int64))).all()
    # the indexed pair: the scan records each message's place, the split reads it
    # (bodies whose timestamps are all 46 bytes; body 18's is not: left out here)
    slots = torch.full((int(off[-1]) // 50 + 1,), -1, dtype=torch.int64, device=a_d.device)
    info2 = torch.empty_like(info_d)
    st2 = torch.empty_like(st_d)
    L.check(lib.evm_pb_scan_index_dev(eng.h, L.PB_SYNC_REQUEST, _P(a_d), _P(off_d), n, _P(info2), _P(st2), _P(slots)),
            "scan_index_dev")
    assert (st2.cpu().numpy() == hst).all() and (info2.cpu().numpy().view(np.uint64) == hi).all()
    sl = slots.cpu().numpy()
    for k in np.flatnonzero((hst == 0) & (hi[:, 8] == 0)):
        at = sl[int(off[k]) // 50: int(off[k]) // 50 + int(hi[k, 0])]
        assert (at >= int(off[k])).all() and (at < int(off[k + 1])).all() and (np.diff(at) > 0).all()
        assert (arena[at] == 0x0A).all()  # (field 1, length-delimited)
    hx = hst.copy()
    hx[18] = 1
    ix = hi.copy()
    ix[18] = 0
    mb = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(ix[:, 0], out=mb[1:])
    cb = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(ix[:, 1], out=cb[1:])
    N, CB = int(mb[-1]), int(cb[-1])
    hts = np.zeros((max(N, 1), 48), dtype=np.uint8)
    hco = np.zeros(N + 1, dtype=np.uint64)
    hc = np.zeros(max(CB, 1), dtype=np.uint8)
    L.check(lib.evm_pb_split_batch(L.PB_SYNC_REQUEST, p(arena), p(off), n, p(hx), p(mb), p(cb), p(hts), 48, None, None,
                                   p(hco), p(hc)), "split")
    dts = torch.zeros((max(N, 1), 64), dtype=torch.uint8, device=a_d.device)
    dco = torch.zeros(N + 1, dtype=torch.int64, device=a_d.device)
    dc = torch.zeros(max(CB, 1), dtype=torch.uint8, device=a_d.device)
    down = torch.zeros(max(N, 1), dtype=torch.int32, device=a_d.device)
    hx_d = eng.dev(hx)
    mb_d, cb_d = eng.dev(mb.view(np.int64)), eng.dev(cb.view(np.int64))
    L.check(lib.evm_pb_split_index_dev(eng.h, L.PB_SYNC_REQUEST, _P(a_d), _P(off_d), n, _P(hx_d), _P(mb_d), _P(cb_d),
                                       _P(own_of), _P(dts), 64, _P(dco), _P(dc), _P(down), _P(slots)), "split_index_dev")
    assert (dts.cpu().numpy()[:N, :48] == hts[:N]).all() and not dts.cpu().numpy()[:N, 48:].any()
    assert (dco.cpu().numpy().view(np.uint64) == hco).all()
    assert (dc.cpu().numpy()[:CB] == hc[:CB]).all()
    assert (down.cpu().numpy()[:N] == np.repeat(np.arange(n) + 7, ix[:, 0].astype(np.int64))).all()
    # a body whose messages do not fit its slots (the shorter timestamp, body 18 kept): refused
    if hi[18, 0] > (int(off[19]) // 50 - int(off[18]) // 50):
        mbf = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(hi[:, 0], out=mbf[1:])
        mbf_d = eng.dev(mbf.view(np.int64))
        dts = torch.zeros((int(mbf[-1]), 64), dtype=torch.uint8, device=a_d.device)
        dco = torch.zeros(int(mbf[-1]) + 1, dtype=torch.int64, device=a_d.device)
        dc = torch.zeros(int(hi[:, 1].sum()) + 1, dtype=torch.uint8, device=a_d.device)
        with pytest.raises(L.EngineError):
            L.check(lib.evm_pb_split_index_dev(eng.h, L.PB_SYNC_REQUEST, _P(a_d), _P(off_d), n, _P(st_d), _P(mbf_d),
                                               _P(cb_d), None, _P(dts), 64, _P(dco), _P(dc), None, _P(slots)), "split")


def _tree_texts():
    rng = random.Random(11)
    js = json.load(open(os.path.join(GOLD, "js_vectors.json")))
    good = [t["json"] for t in js["trees"]]
    # multi-length keys and hash-0 nodes (a node with children and a leaf of its own)
    nodes = [W.node_id(rng) for _ in range(3)]
    for base in (0, 5 * 60000, W.T0, 2582803260000 - 600000):
        t = {}
        for s in W.hlc_timestamps(rng, 80, nodes, t0=base, span=40 * 86_400_000):
            t = O.insert_into_merkle_tree(t, O.parse_canonical(s))
        good.append(O.merkle_tree_to_string(t))
    t = {}
    for s in W.hlc_timestamps(rng, 30, nodes, t0=0, span=3 * 86_400_000) + W.hlc_timestamps(rng, 30, nodes, t0=W.T0):
        t = O.insert_into_merkle_tree(t, O.parse_canonical(s))
    good.append(O.merkle_tree_to_string(t))
    spaced = good[-1].replace(",", ", ").replace(":", " : ")
    bad = ['{"hash":', '{"hash":0}', '{"0":{"hash":1}}', '{"0":{"hash":1},"hash":2}', '{"0":{"hash":-0},"hash":0}',
           '{"0":{"hash":2147483648},"hash":0}', '{"0":{"hash":01},"hash":1}', '{"3":{"hash":1},"hash":1}',
           '{"0":{"hash":1},"0":{"hash":1},"hash":0}', '{"0":{"hash":1.5},"hash":0}', '{} ', ' {}x', '[]',
           '{"0":{"hash":1,"hash":1},"hash":1}', '{"0":{},"hash":0}', '{"hash":0,"0":{"hash":0}}x']
    deep = '{"0":' * 21 + '{"hash":1}' + '}' * 21
    unsorted = '{"1":{"hash":3},"0":{"hash":5},"hash":6}'
    # trees of many steps of k_json_wave (1 KB each): one key length, then keys of many lengths
    for n, t0, span in ((1500, W.T0, 40 * 86_400_000), (400, 0, 10 ** 12)):
        t = {}
        for s in W.hlc_timestamps(rng, n, nodes, t0=t0, span=span):
            t = O.insert_into_merkle_tree(t, O.parse_canonical(s))
        good.append(O.merkle_tree_to_string(t))
    return good + [spaced, unsorted, deep, "{}", ""] + bad


def _mutants(texts, n, seed):
    """n texts of one to three random edits (a byte replaced, deleted, inserted,
    a span duplicated) of the short good trees: mostly malformed, some still
    trees (another hash, another key) -- device and host must decide alike."""
    rng = random.Random(seed)
    alpha = b'{}":,0123456789-h '
    src = [t.encode() for t in texts if 20 < len(t) < 4000 and " " not in t]
    out = []
    for _ in range(n):
        b = bytearray(rng.choice(src))
        for _ in range(rng.randint(1, 3)):
            op, p = rng.random(), rng.randrange(len(b) + 1)
            if op < 0.4 and p < len(b):
                b[p] = rng.choice(alpha)
            elif op < 0.7 and p < len(b):
                del b[p]
            elif op < 0.85:
                b[p:p] = bytes([rng.choice(alpha)])
            else:
                q = rng.randrange(len(b) + 1)
                b[p:p] = b[q:q + rng.randint(1, 20)]
        out.append(b.decode("latin-1"))
    return out


def test_tree_parse_equals_the_host_parser(eng):
    from evolu_amd import _lib as L

    lib = L.load()
    texts = _tree_texts()
    n_base = len(texts)
    texts += _mutants(texts, 400, 17)
    raw = [t.encode("latin-1") for t in texts]
    arena, off = _arena(raw)
    a_d = eng.dev(arena)
    n = len(raw)
    at_d = eng.dev(off[:-1].view(np.int64))
    ln_d = eng.dev(np.diff(off).astype(np.int64))
    st_d = torch.empty(n, dtype=torch.int32, device=a_d.device)
    h = C.c_void_p()
    L.check(lib.evm_tree_from_json_dev(eng.h, n, _P(a_d), _P(at_d), _P(ln_d), _P(st_d), C.byref(h)), "from_json_dev")
    from evolu_amd.engine import Trees

    dt = Trees(eng, h)
    st = st_d.cpu().numpy()
    doff, dck, dxr = dt.leaves()
    for k, t in enumerate(texts):
        try:
            ht = eng.tree_from_json([t or "{}"])
        except (L.EngineError, UnicodeError):
            ht = None
        if t == '{"1":{"hash":3},"0":{"hash":5},"hash":6}':
            assert st[k] == L.TREE_UNSORTED and ht is not None
        if st[k] == L.TREE_UNSORTED:  # (keys out of order: left to the host parser, which decides)
            if ht is not None:
                ht.free()
            continue
        if ht is None:
            assert st[k] == L.EVM_ETREE, (k, t)
            continue
        assert st[k] == 0, (k, t)
        ho, hck, hxr = ht.leaves()
        a, b = int(doff[k]), int(doff[k + 1])
        assert b - a == int(ho[1]), (k, t)
        dk, dx = dck[a:b] & ((1 << 40) - 1), dxr[a:b]
        bad = np.flatnonzero((dk != hck[: b - a]) | (dx != hxr[: b - a]))
        assert not len(bad), (k, t[:300], b - a, bad[:8].tolist(), [hex(int(x)) for x in dk[bad[:4]]],
                              [hex(int(x)) for x in hck[bad[:4]]], dx[bad[:4]].tolist(), hxr[bad[:4]].tolist())
        assert dt.to_json(k) == ht.to_json(0)
        if k < n_base and t and " " not in t:
            assert ht.to_json(0) == t
        ht.free()
    dt.free()


def _e2e(eng, owners, per, seed):
    import bench
    from evolu_amd import synth

    ts_np, owner_np, millis = synth.config3(owners, per, seed_config=seed, request=per)
    o64 = owner_np.astype(np.int64)
    order = np.lexsort((millis, o64))
    rank = np.empty(len(order), dtype=np.int64)
    cnt = np.bincount(o64, minlength=owners)
    rank[order] = np.arange(len(order)) - (np.cumsum(cnt) - cnt)[o64[order]]
    keep = rank < (0.9 * cnt[o64]).astype(np.int64)
    client = eng.merkle_insert(eng.tree_new(owners), eng.dev(np.ascontiguousarray(ts_np[keep])),
                               eng.dev(np.ascontiguousarray(owner_np[keep])))
    arena, off = bench.e2e_bodies(eng, ts_np, owner_np, client)
    client.free()
    return arena, off


def test_sync_device_equals_sync_and_the_reference(eng):
    from evolu_amd.server import SyncServer

    arena, off = _e2e(eng, 24, 60, 31)
    bodies = [arena[int(off[k]):int(off[k + 1])].tobytes() for k in range(len(off) - 1)]
    want = _expected(bodies)
    a, b = SyncServer(eng, 24), SyncServer(eng, 24)
    res = a.sync_device(eng.dev(arena), off)
    assert all(r is True for r in res.result)
    got = res.to_host()
    assert got == want == b.sync(bodies)
    assert set(a.timing) >= {"decode", "users", "ingest", "trees", "select", "encode"}
    # a second round of the same users: new messages, the client trees of round one
    arena2, off2 = _e2e(eng, 24, 40, 57)
    bodies2 = [arena2[int(off2[k]):int(off2[k + 1])].tobytes() for k in range(len(off2) - 1)]
    want2 = _expected(bodies + bodies2)[len(bodies):]
    got2 = a.sync_device(eng.dev(arena2), off2).to_host()
    assert got2 == want2 == b.sync(bodies2)
    assert a.store.n_messages == b.store.n_messages
    a.close()
    b.close()


def _same(x, y):
    assert len(x) == len(y)
    for p, q in zip(x, y):
        assert type(p) is type(q) and (not isinstance(p, bytes) or p == q), (p, q)


def test_sync_device_mixed_with_host_calls_and_per_request_cases(eng):
    """Host and device calls on one server (log segments on both sides), an
    invalid date (its owner rejected by the ingest: the per-request round's
    500), a client tree that does not parse (that request's 500 only), keys
    out of order (the host parser), RangeError of the diff -- and the calls
    the device does not model at all (a truncated body, a userId twice, a
    nodeId that is not hex) through sync(): every result equals sync()'s."""
    from evolu_amd.server import RangeError, SyncServer

    rng = random.Random(3)
    bodies = _requests(8, n_users=12, n_req=12)
    users = [REQ.FromString(b).userId for b in bodies]
    # one request per user per call (the device path's round)
    seen, first = set(), []
    for b, u in zip(bodies, users):
        if u not in seen:
            seen.add(u)
            first.append(b)
    nodes = [W.node_id(rng) for _ in range(2)]
    extra = [
        REQ(messages=[dict(timestamp="2024-02-32T10:00:00.000Z-0000-" + nodes[1], content=b"z")], userId="bad-date",
            nodeId=nodes[1], merkleTree="{}").SerializeToString(),
        REQ(messages=REQ.FromString(first[0]).messages, userId="tree-bad", nodeId=nodes[0],
            merkleTree='{"hash":').SerializeToString(),
        REQ(messages=REQ.FromString(first[1]).messages, userId="tree-unsorted", nodeId=nodes[0],
            merkleTree='{"1":{"hash":3},"0":{"hash":5},"hash":6}').SerializeToString(),
    ]
    call1 = first[: len(first) // 2] + extra
    call2 = first[len(first) // 2:]
    a, b = SyncServer(eng, 40), SyncServer(eng, 40)
    _same(a.sync(call1), b.sync(call1))  # a host call first: its log segment reaches the device encoder later
    arena2, off2 = _arena(call2)
    ga2 = a.sync_device(eng.dev(arena2), off2)
    assert all(r is True for r in ga2.result)
    assert ga2.to_host() == b.sync(call2)
    # the per-request cases inside a device call (users new to this server)
    call3 = [REQ(messages=REQ.FromString(x).messages, userId=REQ.FromString(x).userId + "-3",
                 nodeId=REQ.FromString(x).nodeId, merkleTree=REQ.FromString(x).merkleTree).SerializeToString()
             for x in extra] + [REQ(messages=REQ.FromString(first[2]).messages, userId="rng",
                                    nodeId=nodes[0], merkleTree='{"0":{"hash":5},"hash":5}').SerializeToString()]
    arena3, off3 = _arena(call3)
    r3 = a.sync_device(eng.dev(arena3), off3)
    g3 = r3.to_host()
    _same(g3, b.sync(call3))
    assert isinstance(g3[0], RangeError)
    # an unparsable body and a nodeId that is not hex: answered inside the
    # device round; a userId twice: the call cut into rounds on the host
    for call, whole in (([b"\x0a\x05ab"] + call2[:2], False),
                        ([call2[0], call2[0]], True),
                        ([REQ(userId="nh", nodeId="xyz", merkleTree="{}").SerializeToString()] + call2[:1], False)):
        ar, of = _arena(call)
        _same(a.sync_device(eng.dev(ar), of).to_host(), b.sync(call))
        assert ("device_fallback" in a.timing) == whole
    assert a.store.n_messages == b.store.n_messages
    a.close()
    b.close()


def test_absent_or_empty_merkle_tree_is_a_500_on_both_paths(eng):
    """index.ts:187 JSON.parse(request.merkleTree): an empty or absent field
    (proto3 decodes it as "") throws -> that request answers 500 after its
    addMessages committed -- on the device round exactly as on the host
    path and the per-request path."""
    from evolu_amd import _lib as L
    from evolu_amd.server import SyncServer

    rng = random.Random(11)
    node = W.node_id(rng)
    ts = W.hlc_timestamps(rng, 12, [node])
    msgs = lambda a, b: [dict(timestamp=t, content=b"c") for t in ts[a:b]]  # noqa: E731
    call = [REQ(messages=msgs(0, 4), userId="empty", nodeId=node, merkleTree="").SerializeToString(),
            REQ(messages=msgs(4, 8), userId="absent", nodeId=node).SerializeToString(),
            REQ(messages=msgs(8, 12), userId="fine", nodeId=node, merkleTree="{}").SerializeToString()]
    a, b, c = SyncServer(eng, 8), SyncServer(eng, 8), SyncServer(eng, 8)
    ar, of = _arena(call)
    got = a.sync_device(eng.dev(ar), of).to_host()
    host = b.sync(call)
    per = c.sync_per_request(call)
    for g in (got, host, per):
        assert isinstance(g[0], L.EngineError) and isinstance(g[1], L.EngineError)
        assert isinstance(g[2], bytes)
    assert got[2] == host[2] == per[2]
    # the rows were committed all the same (addMessages ran before getMessages)
    assert a.store.n_messages == b.store.n_messages == c.store.n_messages == 12
    for s_ in (a, b, c):
        s_.close()


# ---- large bodies with bytes that look like message fields inside contents
# and tree texts, repeated and unknown fields, errors deep inside
def _vi(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(field, payload):  # a length-delimited field
    return _vi(field << 3 | 2) + _vi(len(payload)) + payload


FAKE = b"\x0a\x30\x0a\x2e"  # a message field's first bytes (tag, length, its timestamp's tag and length)


def _msg(rng, ts_len=46, clen=None, plant=True):
    ts = bytes(rng.choice(b"0123456789-:T.Z") for _ in range(ts_len))
    n = rng.choice([0, 5, 40, 120, 300]) if clen is None else clen
    c = bytearray(rng.getrandbits(8) for _ in range(n))
    if plant and n >= 8:  # false starts inside the content
        for _ in range(rng.randint(1, 3)):
            at = rng.randrange(0, n - 4)
            c[at:at + 4] = FAKE
    body = _ld(1, ts) + (_ld(2, bytes(c)) if n or rng.random() < 0.5 else b"")
    return _ld(1, body)


def _field_places(body):
    """The top-level message fields' offsets (a plain protobuf walk; None if it fails)."""
    p, out = 0, []
    while p < len(body):
        at, tag, sh = p, 0, 0
        while True:
            b = body[p]
            p += 1
            tag |= (b & 0x7F) << sh
            sh += 7
            if not b & 0x80:
                break
        f, wt = tag >> 3, tag & 7
        if wt == 2:
            ln, sh = 0, 0
            while True:
                b = body[p]
                p += 1
                ln |= (b & 0x7F) << sh
                sh += 7
                if not b & 0x80:
                    break
            if f == 1:
                out.append(at)
            p += ln
        elif wt == 0:
            while body[p] & 0x80:
                p += 1
            p += 1
        elif wt == 1:
            p += 8
        elif wt == 5:
            p += 4
        else:
            return None
    return out if p == len(body) else None


def _large_bodies(seed):
    rng = random.Random(seed)
    user, node = _ld(2, b"u" * 21), _ld(3, b"0123456789abcdef")
    tree_text = b'{"1":{"hash":5},' + FAKE * 4000 + b'"hash":5}'
    B = []
    B.append(b"".join(_msg(rng) for _ in range(2000)) + user + node + _ld(4, b'{"hash":1}'))  # the usual order
    B.append(_ld(4, tree_text) + b"".join(_msg(rng) for _ in range(600)) + user)  # a long text first
    mid = [_msg(rng) for _ in range(900)]
    B.append(b"".join(mid[:400]) + _ld(4, tree_text) + b"".join(mid[400:]) + _ld(4, b"{}") + node)  # repeated: the last wins
    B.append(b"".join(_msg(rng, clen=0, plant=False) for _ in range(5000)))  # 50-B messages: every slot used
    B.append(b"".join(_msg(rng, ts_len=45) for _ in range(700)))  # timestamps that are not 46 bytes
    x = b"".join(_msg(rng) for _ in range(800))
    B.append(x[:-3])  # truncated at the end
    B.append(x[:len(x) // 2] + b"\x00" + x[len(x) // 2:])  # (a field 0 mid-body, unless it lands inside a message)
    y = b"".join(_msg(rng) + (b"\x48\x07" if i % 7 == 0 else b"") + (b"\x51" + bytes(8) if i % 11 == 0 else b"")
                 + (b"\x5d" + bytes(4) if i % 13 == 0 else b"") for i in range(900))
    B.append(y)  # unknown varint / fixed64 / fixed32 fields among the messages
    B.append(y[:len(y) // 3] + b"\x0b" + y[len(y) // 3:])  # a group: rejected
    B.append(b"".join(_msg(rng, plant=False) for _ in range(80)))
    return B


def test_scan_of_large_adversarial_bodies_equals_the_host_codec(eng):
    from evolu_amd import _lib as L
    from evolu_amd import wire

    lib = L.load()
    bodies = _large_bodies(11)
    arena, off = _arena(bodies)
    n = len(bodies)
    hinfo = (wire._Sync * n)()
    hst = np.zeros(n, dtype=np.int32)
    L.check(lib.evm_pb_scan_batch(L.PB_SYNC_REQUEST, C.c_void_p(arena.ctypes.data), C.c_void_p(off.ctypes.data), n,
                                  hinfo, C.c_void_p(hst.ctypes.data)), "scan")
    hi = np.ctypeslib.as_array(hinfo).view(np.uint64).reshape(n, 9)
    assert hst[0] == 0 and hst[5] != 0 and hst[8] != 0 and hi[4, 8] == 700 and hi[2, 7] == 2  # (the fixture's cases)
    a_d, off_d = eng.dev(arena), eng.dev(off.view(np.int64))
    info_d = torch.empty((n, 9), dtype=torch.int64, device=a_d.device)
    st_d = torch.empty(n, dtype=torch.int32, device=a_d.device)
    slots = torch.full((int(off[-1]) // 50 + 1,), -1, dtype=torch.int64, device=a_d.device)
    L.check(lib.evm_pb_scan_index_dev(eng.h, L.PB_SYNC_REQUEST, _P(a_d), _P(off_d), n, _P(info_d), _P(st_d), _P(slots)),
            "scan_index_dev")
    assert (st_d.cpu().numpy() == hst).all()
    assert (info_d.cpu().numpy().view(np.uint64) == hi).all()
    sl = slots.cpu().numpy()
    for k in np.flatnonzero(hst == 0):
        want = _field_places(bodies[k])
        assert want is not None and len(want) == int(hi[k, 0])
        s0 = int(off[k]) // 50
        room = int(off[k + 1]) // 50 - s0
        got = sl[s0: s0 + min(len(want), room)] - int(off[k])
        assert (got == np.array(want[:room], dtype=np.int64)).all(), k
