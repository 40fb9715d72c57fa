"""The server's wire path end to end on the GPU:
SyncRequest bodies -> evm_pb_split -> evm_server_ingest -> evm_server_select
-> evm_pb_encode, against the oracle's ServerDb.sync (index.ts:204-216) with
the bodies built and the expected responses serialised by google.protobuf
from the same schema (protos/protobuf.proto).  Byte-identical responses."""
import random

import pytest

from oracle import evolu_oracle as O
from tests import workloads as W
from tests.test_wire import REQ, RESP

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


def _requests(seed, n_users=6, n_req=40):
    rng = random.Random(seed)
    users = ["%021x" % rng.getrandbits(84) for _ in range(n_users)]
    nodes = [W.node_id(rng) for _ in range(4)]
    pools = {u: W.hlc_timestamps(rng, 120, nodes) for u in users}
    sent = {u: [] for u in users}
    bodies = []
    for _ in range(n_req):
        u = rng.choice(users)
        k = rng.choice([0, 1, 3, 12, 30])
        msgs = []
        for _ in range(k):
            t = rng.choice(pools[u])
            # a redelivered timestamp may come with other bytes: the stored (first) content wins
            msgs.append(dict(timestamp=t, content=bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3, 40])))))
        sent[u] += [m["timestamp"] for m in msgs]
        # the requester's tree: a part of what the owner has sent so far
        have = sorted(set(sent[u]))
        tree = {}
        for t in have[: int(len(have) * rng.random())]:
            tree = O.insert_into_merkle_tree(tree, O.parse_canonical(t))
        node = rng.choice(nodes + [nodes[0].upper()])
        bodies.append(REQ(messages=msgs, userId=u, nodeId=node,
                          merkleTree=O.merkle_tree_to_string(tree)).SerializeToString())
    return bodies


def _expected(bodies):
    sdb = O.ServerDb()
    out = []
    for b in bodies:
        try:
            r = REQ()
            r.ParseFromString(b)
        except Exception:
            out.append("ParseBodyError")
            continue
        try:
            tree, _, rows = sdb.sync(r.userId, r.nodeId, r.merkleTree, [(m.timestamp, m.content) for m in r.messages])
        except (O.RangeErrorJS, ValueError):  # (ValueError: JSON.parse of the client's tree threw)
            out.append("500")  # index.ts:224-233: the request rolled back
            continue
        out.append(RESP(messages=[dict(timestamp=t, content=c) for t, c in rows],
                        merkleTree=O.merkle_tree_to_string(tree)).SerializeToString())
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sync_bodies_match_reference(eng, seed):
    from evolu_amd.server import ParseBodyError, SyncServer

    bodies = _requests(seed)
    if seed == 2:
        bodies.insert(7, b"\x0a\x05ab")  # truncated: SyncRequest.fromBinary throws -> 500
    want = _expected(bodies)
    srv = SyncServer(eng, 16)
    got = srv.sync(bodies)
    for i, (g, w) in enumerate(zip(got, want)):
        if w == "ParseBodyError":
            assert isinstance(g, ParseBodyError), i
        else:
            assert g == w, i
    # a second call continues the same store (the server's state persists)
    more = _requests(seed + 100)
    users = sorted({REQ.FromString(b).userId for b in bodies if b != b"\x0a\x05ab"})
    more = [REQ(messages=REQ.FromString(b).messages, userId=users[k % len(users)], nodeId=REQ.FromString(b).nodeId,
                merkleTree="{}").SerializeToString() for k, b in enumerate(more)]
    want2 = _expected(bodies + more)[len(bodies):]
    assert srv.sync(more) == want2
    srv.close()


def test_empty_requests_and_unknown_user(eng):
    from evolu_amd.server import SyncServer

    rng = random.Random(9)
    ts = W.hlc_timestamps(rng, 10, [W.node_id(rng)])
    bodies = [REQ(userId="a", nodeId="0123456789abcdef", merkleTree="{}").SerializeToString(),
              REQ(messages=[dict(timestamp=t, content=b"x") for t in ts], userId="b", nodeId="0123456789abcdef",
                  merkleTree="{}").SerializeToString(),
              REQ(userId="b", nodeId="0123456789abcdef", merkleTree="{}").SerializeToString()]
    srv = SyncServer(eng, 4)
    assert srv.sync(bodies) == _expected(bodies)
    srv.close()


def test_per_request_failure_and_lenient_timestamps(eng):
    """index.ts:147-169 / :224-233: a request with an invalid date fails alone
    (500, nothing of it stored) while the other requests of the round commit;
    a lenient but valid timestamp (V8 rolls 02-30 into March; a lower-case
    counter parses) is stored under its raw spelling and XORed in its
    canonical form -- the responses, including later requests of the same
    owners, are byte-identical to the reference's."""
    from evolu_amd.server import HandedOver, RangeError, SyncServer

    rng = random.Random(21)
    users = ["%021x" % rng.getrandbits(84) for _ in range(5)]
    nodes = [W.node_id(rng) for _ in range(3)]
    pools = {u: W.hlc_timestamps(rng, 40, nodes) for u in users}

    def req(u, ts, node=None, tree="{}"):
        return REQ(messages=[dict(timestamp=t, content=("c%d" % k).encode()) for k, t in enumerate(ts)], userId=u,
                   nodeId=node or nodes[0], merkleTree=tree).SerializeToString()

    bad_date = "2024-02-32T10:00:00.000Z-0000-" + nodes[1]
    lenient = ["2024-02-30T23:59:59.999Z-000a-" + nodes[1], "2023-04-31t12:00:00.000z-00FF-" + nodes[2].upper()]
    # a canonical row right next to a lenient one: raw-string order differs from canonical order
    near = "2024-03-01T23:59:59.999Z-0000-" + nodes[2]
    bodies = [
        req(users[0], pools[users[0]][:10]),
        req(users[1], pools[users[1]][:5] + [bad_date] + pools[users[1]][5:8]),  # -> 500
        req(users[2], pools[users[2]][:6] + lenient + [near]),
        req(users[3], pools[users[3]][:12], node=nodes[1]),
        # later requests of the same owners
        req(users[1], pools[users[1]][8:14]),  # the failed request stored nothing
        req(users[2], pools[users[2]][6:9] + [lenient[0]], node=nodes[2]),  # a redelivered lenient row
        req(users[2], [], node=nodes[0]),  # getMessages over rows kept under lenient spellings (raw order)
        req(users[0], pools[users[0]][10:12] + ["2024-13-01T00:00:00.000Z-0000-" + nodes[0]]),  # -> 500
        req(users[0], pools[users[0]][12:15]),
    ]
    want = _expected(bodies)
    assert want[1] == "500" and want[7] == "500"
    srv = SyncServer(eng, 8)
    got = srv.sync(bodies)
    for i, (g, w) in enumerate(zip(got, want)):
        if w == "500":
            assert isinstance(g, RangeError), i
        else:
            assert g == w, i
    assert not srv.detached
    # one timestamp under two spellings (lenient, then canonical): the reference
    # stores both; the device keeps one key -> that user is handed to the caller
    canon = "2024-03-01T23:59:59.999Z-000A-" + nodes[1]
    more = [req(users[2], [canon]), req(users[2], pools[users[2]][9:11]), req(users[4], pools[users[4]][:3])]
    got2 = srv.sync(more)
    want2 = _expected(bodies + more)[len(bodies):]
    # (the conflicting request was committed before the conflict showed: not None)
    assert isinstance(got2[0], HandedOver) and got2[0].applied
    assert got2[1] is None and users[2] in srv.detached
    assert got2[2] == want2[2]
    srv.close()


def test_node_id_not_hex_is_handed_over_unapplied(eng):
    """A nodeId the engine cannot use in NOT LIKE '%' || nodeId: the request is
    not applied (None) and the user's later requests are the caller's too."""
    from evolu_amd.server import SyncServer

    rng = random.Random(5)
    node = W.node_id(rng)
    ts = W.hlc_timestamps(rng, 10, [node])
    b = [REQ(messages=[dict(timestamp=t, content=b"x") for t in ts[:5]], userId="u", nodeId="not-a-node",
             merkleTree="{}").SerializeToString(),
         REQ(messages=[dict(timestamp=t, content=b"x") for t in ts[5:]], userId="u", nodeId=node,
             merkleTree="{}").SerializeToString(),
         REQ(messages=[dict(timestamp=t, content=b"y") for t in ts[:3]], userId="v", nodeId=node,
             merkleTree="{}").SerializeToString()]
    srv = SyncServer(eng, 4)
    got = srv.sync(b)
    assert got[0] is None and got[1] is None and "u" in srv.detached
    assert got[2] == _expected(b[2:])[0]
    assert srv.store.n_messages == 3  # nothing of "u" was stored
    srv.close()


def test_fast_path_equals_per_request_path(eng):
    """sync() runs a call as native rounds (evm_sync_round: the bodies
    staged to the device, decoded, ingested, their trees parsed, selected and
    encoded there); sync_per_request() runs every request through the
    per-request path.  Same bytes, same errors, over
    several rounds per user, a truncated body, a client tree that does not
    parse, a nodeId that is not 16 hex chars, an invalid date (500) and a
    lenient timestamp."""
    from evolu_amd.server import SyncServer

    rng = random.Random(77)
    bodies = _requests(5, n_users=20, n_req=160)
    nodes = [W.node_id(rng) for _ in range(2)]
    u0 = REQ.FromString(bodies[0]).userId
    bodies.insert(11, b"\x0a\x05ab")
    bodies.insert(20, REQ(messages=REQ.FromString(bodies[3]).messages, userId="tree-bad", nodeId=nodes[0],
                          merkleTree='{"hash":').SerializeToString())
    bodies.insert(30, REQ(messages=REQ.FromString(bodies[4]).messages, userId="node-bad", nodeId="xyz",
                          merkleTree="{}").SerializeToString())
    bodies.insert(40, REQ(messages=[dict(timestamp="2024-02-32T10:00:00.000Z-0000-" + nodes[1], content=b"z")],
                          userId=u0, nodeId=nodes[1], merkleTree="{}").SerializeToString())
    bodies.insert(50, REQ(messages=[dict(timestamp="2024-02-30T23:59:59.999Z-000a-" + nodes[1], content=b"l")],
                          userId="lenient", nodeId=nodes[1], merkleTree="{}").SerializeToString())
    bodies.append(REQ(messages=REQ.FromString(bodies[60]).messages, userId="lenient", nodeId=nodes[0],
                      merkleTree="{}").SerializeToString())
    a = SyncServer(eng, 32)
    b = SyncServer(eng, 32)
    ga, gb = a.sync(bodies), b.sync_per_request(bodies)
    assert set(a.timing) >= {"h2d", "decode", "users", "ingest", "trees", "select", "encode", "d2h", "per_request"}
    for i, (x, y) in enumerate(zip(ga, gb)):
        if isinstance(x, (bytes, type(None))):
            assert x == y, i
        else:
            assert type(x) is type(y), (i, x, y)
    want = _expected(bodies)
    for i, (x, w) in enumerate(zip(ga, want)):
        if isinstance(x, bytes):
            assert x == w, i
    assert sum(isinstance(x, bytes) for x in ga) > 150
    a.close()
    b.close()


def test_e2e_bodies_vs_oracle(eng):
    """The bench's config3_e2e round in miniature (bench.e2e_bodies: one
    SyncRequest per owner with its client tree's JSON from the device
    emitter): SyncServer.sync_arena's responses byte for byte against the
    oracle's ServerDb.sync (index.ts:204-216) of the same bodies."""
    import numpy as np

    import bench
    from evolu_amd import synth
    from evolu_amd.server import SyncServer

    owners, per = 24, 60
    ts_np, owner_np, millis = synth.config3(owners, per, seed_config=31, request=per)
    o64 = owner_np.astype(np.int64)
    order = np.lexsort((millis, o64))
    rank = np.empty(len(order), dtype=np.int64)
    cnt = np.bincount(o64, minlength=owners)
    rank[order] = np.arange(len(order)) - (np.cumsum(cnt) - cnt)[o64[order]]
    keep = rank < (0.9 * cnt[o64]).astype(np.int64)
    client = eng.merkle_insert(eng.tree_new(owners), eng.dev(np.ascontiguousarray(ts_np[keep])),
                               eng.dev(np.ascontiguousarray(owner_np[keep])))
    arena, off = bench.e2e_bodies(eng, ts_np, owner_np, client)
    bodies = [arena[int(off[k]):int(off[k + 1])].tobytes() for k in range(len(off) - 1)]
    want = _expected(bodies)
    srv = SyncServer(eng, owners)
    got = srv.sync_arena(arena, off)
    assert len(got) == len(want) == owners
    for g, w in zip(got, want):
        assert isinstance(g, memoryview) and bytes(g) == w
    srv.close()
    client.free()
