"""evm_tree_merge: the union of two insert sets' trees, XOR-combined -- the
tree insertIntoMerkleTree gives for all inserts together in any order
(merkleTree.test.ts:30-42).  It combines the partial trees of an owner split
over GPUs (evm_dist_merge_trees, evolu_amd/sharded.py)."""
import random

import numpy as np
import pytest

from oracle import evolu_oracle as O
from tests import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from evolu_amd.engine import Engine

    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("seed", range(3))
def test_tree_merge_is_insert_union(eng, seed):
    rng = random.Random(seed)
    n_owners = 5
    nodes = [W.node_id(rng) for _ in range(4)]
    pool = W.hlc_timestamps(rng, 400, nodes, span=rng.choice([3_600_000, 5 * 86_400_000]))
    if seed == 2:
        pool += W.hlc_timestamps(rng, 50, nodes, t0=60_000 * 7)  # short keys: mixed key lengths
    a = [(rng.randrange(n_owners), rng.choice(pool)) for _ in range(300)]
    b = [(rng.randrange(n_owners), rng.choice(pool)) for _ in range(300)] + a[:40]  # shared inserts cancel

    def build(msgs):
        ts = eng.timestamps([t for _, t in msgs])
        own = eng.dev(np.array([o for o, _ in msgs], dtype=np.uint32))
        return eng.merkle_insert(eng.tree_new(n_owners), ts, own)

    merged = eng.tree_merge(build(a), build(b))
    want = build(a + b)
    for x, y in zip(merged.leaves(), want.leaves()):
        assert np.array_equal(x, y)
    for o in range(n_owners):
        tree = {}
        for oo, t in a + b:
            if oo == o:
                tree = O.insert_into_merkle_tree(tree, O.parse_canonical(t))
        assert merged.to_json(o) == O.merkle_tree_to_string(tree)
