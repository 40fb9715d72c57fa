"""Pins the CPU oracle against the reference's own snapshot values and
against real JavaScript semantics (node 12 + imurmurhash vectors)."""
import json
import os

import pytest

from oracle import evolu_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SNAP = json.load(open(os.path.join(GOLD, "reference_snapshots.json")))
TS = SNAP["timestamp.test.ts.snap"]
MT = SNAP["merkleTree.test.ts.snap"]
JSV = json.load(open(os.path.join(GOLD, "js_vectors.json")))

NODE1 = "0000000000000001"  # test/testUtils.ts:3-9
NODE2 = "0000000000000002"


def test_timestamp_to_string_snapshot():
    # timestamp.test.ts:37-39
    assert O.timestamp_to_string(*O.create_sync_timestamp()) == TS["timestampToString 1"]


def test_timestamp_roundtrip():
    # timestamp.test.ts:41-44
    t = O.create_sync_timestamp()
    assert O.timestamp_from_string(O.timestamp_to_string(*t)) == t


def test_timestamp_hash_snapshot():
    # timestamp.test.ts:46-48
    assert O.timestamp_to_hash(*O.create_sync_timestamp()) == TS["timestampToHash 1"] == 4179357717


def _either(fn):
    try:
        m, c, n = fn()
        return {"_tag": "Right", "right": {"counter": c, "millis": m, "node": n}}
    except O.TimestampError as e:
        return {"_tag": "Left", "left": dict(type=e.kind, **e.info)}


def test_send_timestamp_snapshots():
    # timestamp.test.ts:53-92
    s = O.create_sync_timestamp
    assert _either(lambda: O.send_timestamp(s(), 1)) == TS["sendTimestamp > should send monotonically with a monotonic clock 1"]
    assert _either(lambda: O.send_timestamp(s(), 0)) == TS["sendTimestamp > should send monotonically with a stuttering clock 1"]
    assert _either(lambda: O.send_timestamp(s(1), 0)) == TS["sendTimestamp > should send monotonically with a regressing clock 1"]
    assert _either(lambda: O.send_timestamp(s(60001), 0)) == TS["sendTimestamp > should fail with clock drift 1"]

    def overflow():
        t = s()
        for _ in range(65536):
            t = O.send_timestamp(t, 0)
        return t

    assert _either(overflow) == TS["sendTimestamp > should fail with counter overflow 1"]


def test_receive_timestamp_snapshots():
    # timestamp.test.ts:94-152
    n1 = lambda m=0, c=0: (m, c, NODE1)
    n2 = lambda m=0, c=0: (m, c, NODE2)
    pre = "receiveTimestamp > "
    assert _either(lambda: O.receive_timestamp(n1(), n2(0, 0), 1)) == TS[pre + "wall clock is later than both the local and remote timestamps 1"]
    k = pre + "wall clock is somehow behind > "
    assert _either(lambda: O.receive_timestamp(n1(1, 0), n2(1, 1), 0)) == TS[k + "for the same timestamps millis, we take the bigger counter 1"]
    assert _either(lambda: O.receive_timestamp(n1(1, 1), n2(1, 0), 0)) == TS[k + "for the same timestamps millis, we take the bigger counter 2"]
    assert _either(lambda: O.receive_timestamp(n1(2), n2(1), 0)) == TS[k + "local millis is later than remote 1"]
    assert _either(lambda: O.receive_timestamp(n1(1), n2(2), 0)) == TS[k + "remote millis is later than local 1"]
    assert _either(lambda: O.receive_timestamp(n1(), n1(), 1)) == TS[pre + "TimestampDuplicateNodeError 1"]
    sync = O.create_sync_timestamp(60001)
    assert _either(lambda: O.receive_timestamp(sync, n2(), 0)) == TS[pre + "should fail with clock drift 1"]
    assert _either(lambda: O.receive_timestamp(n2(), sync, 0)) == TS[pre + "should fail with clock drift 2"]


def test_merkle_insert_snapshots():
    # merkleTree.test.ts:12-43
    assert {} == MT["createInitialMerkleTree 1"]
    ts1 = (0, 0, NODE1)
    ts2 = (1656873738591, 0, NODE1)
    t1 = O.insert_into_merkle_tree({}, ts1)
    t2 = O.insert_into_merkle_tree({}, ts2)
    t12 = O.insert_into_merkle_tree(t1, ts2)
    t21 = O.insert_into_merkle_tree(t2, ts1)
    assert t1 == MT["insertIntoMerkleTree 1"]
    assert t2 == MT["insertIntoMerkleTree 2"]
    assert t12 == MT["insertIntoMerkleTree 3"]
    assert t12 == t21
    assert t12["hash"] == 1335454297
    # JSON text of the snapshot object == our JSON.stringify restatement
    assert json.loads(O.merkle_tree_to_string(t12)) == MT["insertIntoMerkleTree 3"]


def test_merkle_diff_snapshots():
    # merkleTree.test.ts:45-58
    assert O.diff_merkle_trees({}, {}) is None and MT["diffMerkleTrees 1"] == {"_tag": "None"}
    mt = O.insert_into_merkle_tree({}, (1656873738591, 0, NODE1))
    assert O.diff_merkle_trees({}, mt) == MT["diffMerkleTrees 2"]["value"] == 1656873720000
    assert O.diff_merkle_trees(mt, {}) == O.diff_merkle_trees({}, mt)


def test_murmur_and_iso_against_js():
    for v in JSV["timestamps"]:
        assert O.iso_string(v["millis"]) == v["s"][:24]
        assert O.timestamp_to_string(v["millis"], v["counter"], v["node"]) == v["s"]
        assert O.murmur3_32(v["s"].encode()) == v["hash"], v["s"]
        assert O.minute_key(v["millis"]) == v["key"]
        assert O.parse_canonical(v["s"]) == (v["millis"], v["counter"], v["node"])


def test_lenient_dates_are_flagged():
    for v in JSV["lenient"]:
        s = v["s"] + "-0000-0000000000000000"
        if v["parsed"] is not None and O.iso_string(v["parsed"]) == v["s"]:
            assert O.parse_canonical(s)[0] == v["parsed"]
        else:
            with pytest.raises(O.NonCanonical):
                O.parse_canonical(s)


def test_trie_json_against_js():
    for t in JSV["trees"]:
        tree = {}
        for m, c, n in t["ops"]:
            tree = O.insert_into_merkle_tree(tree, (m, c, n))
        assert O.merkle_tree_to_string(tree) == t["json"]
        assert O.merkle_tree_to_string(O.merkle_tree_from_string(t["json"])) == t["json"]


def test_key_to_timestamp_against_js():
    for v in JSV["keyMillis"]:
        assert O.key_to_timestamp(v["k"]) == v["millis"]
    with pytest.raises(O.RangeErrorJS):
        O.key_to_timestamp("1" * 17)
