"""receiveMessages (receive.ts:45-66) as a GPU scan vs the oracle's sequential
receiveTimestamp fold (timestamp.ts:125-165): final clock, or the first error."""
import random

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


def oracle_fold(local, strings, now, drift=60000):
    t = local
    for i, s in enumerate(strings):
        try:
            t = O.receive_timestamp(t, O.parse_canonical(s), now, drift)
        except O.TimestampError as e:
            return e.kind, {"index": i, "next": e.info.get("next", 0)}
    return "ok", t


def _case(rng, n, local_node, mode):
    now = W.T0 + rng.randrange(0, 10_000)
    nodes = [W.node_id(rng, upper=rng.random() < 0.3) for _ in range(3)]
    strings = []
    t = now - rng.randrange(0, 5000)
    for _ in range(n):
        r = rng.random()
        if r < 0.3:
            t += 0  # equal millis: counter max-merge
        elif r < 0.9:
            t += rng.randrange(0, 40)
        else:
            t -= rng.randrange(0, 100)
        c = rng.randrange(0, 5) if rng.random() < 0.95 else rng.randrange(60000, 65536)
        strings.append(O.timestamp_to_string(max(t, 0), c, rng.choice(nodes)))
    if mode == "dup":
        strings.insert(rng.randrange(len(strings)), O.timestamp_to_string(now, 0, local_node))
    if mode == "drift":
        strings.insert(rng.randrange(len(strings)), O.timestamp_to_string(now + 60001 + rng.randrange(5), 0, nodes[0]))
    if mode == "overflow":
        k = rng.randrange(len(strings))
        m = O.parse_canonical(strings[k])[0]
        strings.insert(k + 1, O.timestamp_to_string(m + 30000, 65535, nodes[1]))
        strings.insert(k + 2, O.timestamp_to_string(m + 30000, 7, nodes[2]))
    local = (now - rng.randrange(0, 3000), rng.randrange(0, 100), local_node)
    return local, strings, now


@pytest.mark.parametrize("mode", ["plain", "dup", "drift", "overflow"])
@pytest.mark.parametrize("seed", range(5))
def test_receive_fold_vs_oracle(eng, mode, seed):
    rng = random.Random(seed * 17 + len(mode))
    local_node = W.node_id(rng)
    local, strings, now = _case(rng, rng.choice([1, 7, 300, 5000]), local_node, mode)
    got = eng.receive_fold(eng.timestamps(strings), local, now)
    want = oracle_fold(local, strings, now)
    if want[0] == "ok":
        assert got == want
    else:
        assert got[0] == want[0] and got[1]["index"] == want[1]["index"]
        if want[0] == "TimestampDriftError":
            assert got[1]["next"] == want[1]["next"]


def test_receive_fold_snapshot_cases(eng):
    # timestamp.test.ts:94-152 as one-message folds
    n1, n2 = "0000000000000001", "0000000000000002"
    cases = [((0, 0, n1), (0, 0, n2), 1, ("ok", (1, 0, n1))),
             ((1, 0, n1), (1, 1, n2), 0, ("ok", (1, 2, n1))),
             ((1, 1, n1), (1, 0, n2), 0, ("ok", (1, 2, n1))),
             ((2, 0, n1), (1, 0, n2), 0, ("ok", (2, 1, n1))),
             ((1, 0, n1), (2, 0, n2), 0, ("ok", (2, 1, n1))),
             ((0, 0, n1), (0, 0, n1), 1, ("TimestampDuplicateNodeError", None)),
             ((60001, 0, "0000000000000000"), (0, 0, n2), 0, ("TimestampDriftError", 60001)),
             ((0, 0, n2), (60001, 0, "0000000000000000"), 0, ("TimestampDriftError", 60001))]
    for local, remote, now, want in cases:
        got = eng.receive_fold(eng.timestamps([O.timestamp_to_string(*remote)]), local, now)
        assert got[0] == want[0]
        if want[0] == "ok":
            assert got[1] == want[1]
        elif want[0] == "TimestampDriftError":
            assert got[1]["next"] == want[1]


def test_receive_fold_large(eng):
    rng = random.Random(99)
    local_node = W.node_id(rng)
    local, strings, now = _case(rng, 300_000, local_node, "plain")
    assert eng.receive_fold(eng.timestamps(strings), local, now) == oracle_fold(local, strings, now)
