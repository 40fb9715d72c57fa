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
        tree, _, rows = sdb.sync(r.userId, r.nodeId, r.merkleTree, [(m.timestamp, m.content) for m in r.messages])
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
