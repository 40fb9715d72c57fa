"""evm_tree_to_json_batch: every requested owner's merkleTreeToString
(types.ts:80-84, JSON.stringify) in one device call must be byte-identical
to the host emitter (evm_tree_to_json, pinned by node's JSON.stringify of
persistent-spread tries in tests/golden/js_vectors.json) and to the
oracle's -- for the reference snapshots, node's trees, multi-owner trees with
short / 16 / 17-digit keys and hash-0 nodes, owner subsets in any order,
empty trees, gapped store trees and owners larger than the LDS stage."""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import evolu_oracle as O
from tests import workloads as W

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
JSV = json.load(open(os.path.join(GOLD, "js_vectors.json")))
MT = json.load(open(os.path.join(GOLD, "reference_snapshots.json")))["merkleTree.test.ts.snap"]


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


def _texts(trees, owners=None, count=None):
    buf, off = trees.to_json_batch(owners, count)
    b = buf.cpu().numpy().tobytes()
    o = off.cpu().numpy()
    return [b[o[k]:o[k + 1]].decode() for k in range(len(o) - 1)]


def test_reference_snapshots_and_node_trees(eng):
    n1 = "0000000000000001"
    ts1, ts2 = O.timestamp_to_string(0, 0, n1), O.timestamp_to_string(1656873738591, 0, n1)
    for strings, snap in (([ts1], "insertIntoMerkleTree 1"), ([ts2], "insertIntoMerkleTree 2"),
                          ([ts1, ts2], "insertIntoMerkleTree 3")):
        t = eng.merkle_insert(eng.tree_new(1), eng.timestamps(strings))
        (got,) = _texts(t)
        assert json.loads(got) == MT[snap] and got == t.to_json(0)
    assert _texts(eng.tree_new(3)) == ["{}", "{}", "{}"]
    # node's JSON.stringify of tries built by persistent spreads (merkleTree.ts:8-29)
    trees = [t for t in JSV["trees"]]
    tt = eng.tree_from_json([t["json"] for t in trees])
    assert _texts(tt) == [t["json"] for t in trees]


def test_multi_owner_keys_of_every_length(eng):
    rng = random.Random(7)
    n_owners = 61
    strings, owners = [], []
    for o in range(n_owners):
        nodes = [W.node_id(rng) for _ in range(3)]
        base = rng.choice([0, 5 * 60000, W.T0, 2582803260000 - 600000])  # short, 16 and 17-digit keys
        for s in W.hlc_timestamps(rng, rng.randrange(0, 300), nodes, t0=base,
                                  span=rng.choice([7200_000, 40 * 86_400_000])):
            strings.append(s)
            owners.append(o)
            if rng.random() < 0.2:  # a duplicate: XOR cancels, the nodes stay with hash 0
                strings.append(s)
                owners.append(o)
    trees = eng.merkle_insert(eng.tree_new(n_owners), eng.timestamps(strings),
                              eng.dev(np.array(owners, dtype=np.uint32)))
    want = [trees.to_json(o) for o in range(n_owners)]
    for o in range(n_owners):
        assert want[o] == O.merkle_tree_to_string(
            _oracle_tree([s for s, oo in zip(strings, owners) if oo == o]))
    assert _texts(trees) == want
    pick = [5, 0, 60, 5, 17]  # a subset, any order, repeats
    assert _texts(trees, eng.dev(np.array(pick, dtype=np.uint32))) == [want[k] for k in pick]
    assert _texts(trees, count=10) == want[:10]


def _oracle_tree(strings):
    t = {}
    for s in strings:
        t = O.insert_into_merkle_tree(t, O.parse_canonical(s))
    return t


def test_gapped_store_tree_and_large_owners(eng):
    """A config-3 store tree straight after ingest (gapped: each owner's leaves
    where K5 wrote them), and owners with more leaves than the emitter stages
    in LDS (read from global memory)."""
    from evolu_amd import synth
    from tests.test_gpu_server import _is_gapped

    ts, own, _ = synth.config3(300, 700, request=700, seed_config=55)
    store = eng.store_new(300)
    store.ingest(eng.dev(ts), eng.dev(own), 0)
    tree = store.tree()
    assert _is_gapped(eng, tree)
    got = _texts(tree)
    assert _is_gapped(eng, tree)  # (the emitter reads it as it lies)
    assert got == [tree.to_json(o) for o in range(300)]  # (to_json compacts)
    store.free()
    # one owner of ~5,000 leaves (> the 2,048 staged in LDS), beside small ones
    rng = random.Random(3)
    nodes = [W.node_id(rng) for _ in range(4)]
    big = W.hlc_timestamps(rng, 6000, nodes, t0=W.T0, span=20 * 86_400_000)
    small = W.hlc_timestamps(rng, 50, nodes, t0=W.T0)
    trees = eng.merkle_insert(eng.tree_new(3), eng.timestamps(big + small + small[:7]),
                              eng.dev(np.array([1] * len(big) + [2] * len(small) + [0] * 7, dtype=np.uint32)))
    assert trees.leaves()[0][2] - trees.leaves()[0][1] > 2048
    assert _texts(trees) == [trees.to_json(o) for o in range(3)]


def test_owner_out_of_range_is_refused(eng):
    from evolu_amd import _lib as L

    t = eng.tree_new(4)
    with pytest.raises(L.EngineError) as e:
        t.to_json_batch(eng.dev(np.array([1, 4], dtype=np.uint32)))
    assert e.value.status == L.EVM_EINVAL
    assert torch.cuda.is_available()


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def test_hashes_of_every_length_and_sign(eng):
    """The emitter writes a node's hash as its decimal digits in pieces of up
    to eight bytes: every length 1..10, both signs, 0 and -2**31, at every
    depth and in every position (first child, later child, the root)."""
    vals = [0, -1, 9, 10, -99, 12345678, -12345678, 99999999, 100000000, -100000000, 123456789,
            2147483647, -2147483648, 1000000000, -999999999, 7, 4096]
    rng = random.Random(5)
    texts = []
    for k in range(40):
        # a small trie: a few depth-1 children, each with leaves below
        def node(depth):
            if depth == 0 or rng.random() < 0.3:
                return rng.choice(vals), None
            kids = sorted(rng.sample("012", rng.randint(1, 3)))
            parts, x = [], 0
            for d in kids:
                h, body = node(depth - 1)
                x ^= h
                parts.append('"%s":%s' % (d, body if body else '{"hash":%d}' % h))
            return _i32(x), "{" + ",".join(parts) + ',"hash":%d}' % _i32(x)
        h, body = node(rng.randint(1, 4))
        texts.append(body if body else '{"0":{"hash":%d},"hash":%d}' % (h, h))
    tt = eng.tree_from_json(texts)
    assert _texts(tt) == texts
