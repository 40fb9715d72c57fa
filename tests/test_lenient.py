"""Lenient timestamp strings on the server path, pinned by node
(tests/golden/js_lenient.json from oracle/js/gen_lenient.js: the reference's
timestampToString(timestampFromString(raw)) or RangeError for 6,000 ISO-shaped
strings with fields at and past their limits).  Both the oracle's restatement
(oracle/evolu_oracle.py) and the host path's (evolu_amd/lenient.py) must agree
with V8 on every vector they model."""
import json
import os

from evolu_amd import lenient as LN
from oracle import evolu_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VEC = json.load(open(os.path.join(ROOT, "tests", "golden", "js_lenient.json")))["vectors"]


def test_vectors_cover_every_case():
    kinds = {"range": 0, "same": 0, "changed": 0}
    for v in VEC:
        kinds["range" if v["canonical"] == "RangeError" else ("same" if v["canonical"] == v["raw"] else "changed")] += 1
    assert min(kinds.values()) > 300, kinds


def test_oracle_timestamp_from_string_js_matches_v8():
    for v in VEC:
        millis, counter, node = O.timestamp_from_string_js(v["raw"])
        if v["canonical"] == "RangeError":
            assert millis is None, v
        else:
            assert O.timestamp_to_string(millis, counter, node) == v["canonical"], v


def test_host_classify_matches_v8():
    seen = {"ok": 0, "range_error": 0, "unsupported": 0}
    for v in VEC:
        kind, canon = LN.classify(v["raw"])
        seen[kind] += 1
        if kind == "range_error":
            assert v["canonical"] == "RangeError", v
        elif kind == "ok":
            assert canon == v["canonical"], v
            O.parse_canonical(canon)  # and it is canonical
        else:  # a valid date outside the engine's native domain (before 1970 / extended years)
            assert v["canonical"] != "RangeError", v
    assert seen["ok"] > 1000 and seen["range_error"] > 1000


def test_host_classify_rejects_unmodelled_shapes():
    for raw in ["2024-01-01T00:00:00Z-0000-0123456789abcdef",  # no millis
                "2024-01-01T00:00:00.000Z-00G0-0123456789abcdef",  # counter not hex
                "2024-01-01T00:00:00.000Z-0000-0123456789abcde",  # short node
                "2024-01-01T00:00:00.000Z-0000-0123456789abcdef-x"]:  # extra part
        assert LN.classify(raw)[0] == "unsupported", raw
    assert LN.classify("2024-02-30T00:00:00.000Z-000a-0123456789abcdef") == (
        "ok", "2024-03-01T00:00:00.000Z-000A-0123456789abcdef")
    assert LN.classify("2024-02-32T00:00:00.000Z-0000-0123456789abcdef") == ("range_error", None)


def test_oracle_server_stores_raw_and_hashes_canonical():
    """index.ts:151-159 on a lenient string: the raw string is the stored row
    (so two spellings of one timestamp are two rows, both XORed -- they cancel),
    the tree sees the canonical form; an invalid date fails the request."""
    db = O.ServerDb()
    raw = "2024-02-30T00:00:00.000Z-000a-0123456789abcdef"
    canon = "2024-03-01T00:00:00.000Z-000A-0123456789abcdef"
    t1 = db.add_messages({}, "u", [(raw, b"x")])
    t2 = O.insert_into_merkle_tree({}, O.parse_canonical(canon))
    assert t1 == t2
    t3 = db.add_messages(t1, "u", [(canon, b"y")])
    assert t3["hash"] == 0  # the same timestamp twice, under two spellings
    import pytest

    with pytest.raises(O.RangeErrorJS):
        db.add_messages(t3, "u", [(canon.replace("03-01", "03-02"), b"z"), ("2024-02-32T00:00:00.000Z-0000-0123456789abcdef", b"w")])
    # the failed request rolled back: its first message is not stored
    rows = db.conn.execute('SELECT "timestamp" FROM "message" WHERE "userId" = ? ORDER BY "timestamp"', ("u",)).fetchall()
    assert [r[0] for r in rows] == [raw, canon]
