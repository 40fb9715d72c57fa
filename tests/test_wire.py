"""SyncRequest / SyncResponse codec (protobuf.ts:60-171, protos/protobuf.proto)
against google.protobuf built from the same schema: byte-identical encoding
(proto3: defaults omitted, field-number order -- what protobuf-ts toBinary
writes) and identical decoding, incl. unknown fields, reordering and
truncation.  Host code only: runs without a GPU."""
import json
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

from evolu_amd import wire

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="evolu_protobuf.proto", syntax="proto3", package="t")

    def msg(name, fields):
        m = fdp.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("EncryptedCrdtMessage", [("timestamp", 1, F.TYPE_STRING, O, None), ("content", 2, F.TYPE_BYTES, O, None)])
    msg("SyncRequest", [("messages", 1, F.TYPE_MESSAGE, R, ".t.EncryptedCrdtMessage"),
                        ("userId", 2, F.TYPE_STRING, O, None), ("nodeId", 3, F.TYPE_STRING, O, None),
                        ("merkleTree", 4, F.TYPE_STRING, O, None)])
    msg("SyncResponse", [("messages", 1, F.TYPE_MESSAGE, R, ".t.EncryptedCrdtMessage"),
                         ("merkleTree", 2, F.TYPE_STRING, O, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName("t." + n))  # noqa: E731
    return get("SyncRequest"), get("SyncResponse")


REQ, RESP = _classes()


def _random_messages(rng, n):
    ts, contents = [], []
    for _ in range(n):
        r = rng.random()
        if r < 0.8:
            t = "2024-01-%02dT%02d:%02d:%02d.%03dZ-%04X-%016x" % (rng.randrange(1, 29), rng.randrange(24),
                                                                 rng.randrange(60), rng.randrange(60),
                                                                 rng.randrange(1000), rng.randrange(65536),
                                                                 rng.getrandbits(64))
        elif r < 0.9:
            t = ""
        else:
            t = "x" * rng.randrange(1, 300)
        ts.append(t)
        contents.append(bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 5, 130, 2000]))))
    return ts, contents


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("kind", [wire.REQUEST, wire.RESPONSE])
def test_encode_matches_protobuf(seed, kind):
    rng = random.Random(seed * 7 + kind)
    ts, contents = _random_messages(rng, rng.choice([0, 1, 3, 50, 400]))
    tree = rng.choice(["", "{}", '{"hash":1,"0":{"hash":1}}' * rng.randrange(1, 50)])
    cls = REQ if kind == wire.REQUEST else RESP
    ref = cls(messages=[dict(timestamp=t, content=c) for t, c in zip(ts, contents)], merkleTree=tree)
    kw = {}
    if kind == wire.REQUEST:
        kw = dict(user=rng.choice(["", "%021x" % rng.getrandbits(84)]), node=rng.choice(["", "0123456789abcdef"]))
        ref.userId, ref.nodeId = kw["user"], kw["node"]
    mine = wire.encode(kind, ts, contents, tree=tree, **kw)
    assert mine == ref.SerializeToString(deterministic=True)
    # and back
    d = wire.decode(kind, mine)
    assert d.contents() == contents and d.tree == tree
    assert list(d.ts_len) == [len(t.encode()) for t in ts] and d.raw == ts
    for i, t in enumerate(ts):
        if len(t) == 46:
            assert bytes(d.ts[i, :46]).decode() == t
        else:
            assert (d.ts[i, :46] == 0xFF).all()
    if kind == wire.REQUEST:
        assert (d.user, d.node) == (kw["user"], kw["node"])


def test_decode_unknown_fields_reordered_and_last_wins():
    rng = random.Random(5)
    ts, contents = _random_messages(rng, 20)
    ref = REQ(messages=[dict(timestamp=t, content=c) for t, c in zip(ts, contents)], userId="u1", nodeId="n1",
              merkleTree="{}")
    body = bytearray()
    # strings first, then messages interleaved with unknown fields of every wire type
    body += b"\x22\x02{}" + b"\x12\x02u0" + b"\x1a\x02n1"
    for k, m in enumerate(ref.messages):
        mb = m.SerializeToString()
        body += b"\x0a" + bytes([len(mb)]) if len(mb) < 128 else b""
        if len(mb) >= 128:
            body += b"\x0a" + _varint(len(mb))
        body += mb
        body += [b"\x28\x96\x01", b"\x31" + b"\0" * 8, b"\x3a\x03abc", b"\x45" + b"\0" * 4][k % 4]
    body += b"\x12\x02u1"  # last value wins
    d = wire.decode(wire.REQUEST, bytes(body))
    parsed = REQ()
    parsed.ParseFromString(bytes(body))
    assert d.user == parsed.userId == "u1" and d.node == parsed.nodeId and d.tree == parsed.merkleTree
    assert d.contents() == [m.content for m in parsed.messages]


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def test_decode_rejects_truncated_and_groups():
    """Every prefix of a valid body: we reject exactly the prefixes protobuf rejects."""
    from evolu_amd._lib import EngineError

    good = wire.encode(wire.RESPONSE, ["2024-01-01T00:00:00.000Z-0000-0123456789abcdef"] * 2, [b"abc", b""],
                       tree="{}")
    for cut in range(len(good) + 1):
        try:
            RESP().ParseFromString(good[:cut])
            ref_ok = True
        except Exception:
            ref_ok = False
        try:
            wire.decode(wire.RESPONSE, good[:cut])
            ok = True
        except EngineError:
            ok = False
        assert ok == ref_ok, cut
    for bad in (b"\x0b\x0c", b"\x08\x01", b"\x0a\x05ab"):  # group, wrong wire type, overrun
        with pytest.raises(EngineError):
            wire.decode(wire.RESPONSE, bad)


def test_empty_bodies():
    assert wire.encode(wire.RESPONSE, [], []) == b""
    d = wire.decode(wire.REQUEST, b"")
    assert len(d.ts_len) == 0 and d.user == "" and d.tree == ""


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "js", "evm_napi.node")) or shutil.which("node") is None,
                    reason="N-API addon / node not available")
def test_js_sync_codec_matches_protobuf(tmp_path):
    """The JS shim's SyncRequest/SyncResponse.fromBinary/toBinary (N-API) vs google.protobuf."""
    rng = random.Random(11)
    ts, contents = _random_messages(rng, 60)
    ts = [t if len(t) == 46 else "2024-02-02T00:00:00.000Z-0000-00000000000000%02x" % i for i, t in enumerate(ts)]
    req = REQ(messages=[dict(timestamp=t, content=c) for t, c in zip(ts, contents)], userId="owner-1",
              nodeId="0123456789abcdef", merkleTree='{"hash":7}')
    (tmp_path / "req.bin").write_bytes(req.SerializeToString())
    script = """
const fs = require('fs');
const { SyncRequest, SyncResponse } = require(%r);
const body = new Uint8Array(fs.readFileSync(%r));
const r = SyncRequest.fromBinary(body);
const again = SyncRequest.toBinary(r);
const resp = SyncResponse.toBinary({ messages: r.messages, merkleTree: r.merkleTree });
fs.writeFileSync(%r, Buffer.from(again));
fs.writeFileSync(%r, Buffer.from(resp));
console.log(JSON.stringify({ n: r.messages.length, userId: r.userId, nodeId: r.nodeId, tree: r.merkleTree,
  ts: r.messages.map((m) => m.timestamp), c: r.messages.map((m) => Buffer.from(m.content).toString('hex')) }));
""" % (os.path.join(ROOT, "js", "evolu_evm.js"), str(tmp_path / "req.bin"), str(tmp_path / "again.bin"),
       str(tmp_path / "resp.bin"))
    out = subprocess.run(["node", "-e", script], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout)
    assert got["n"] == 60 and got["ts"] == ts and got["c"] == [c.hex() for c in contents]
    assert (got["userId"], got["nodeId"], got["tree"]) == ("owner-1", "0123456789abcdef", '{"hash":7}')
    assert (tmp_path / "again.bin").read_bytes() == req.SerializeToString()
    resp = RESP(messages=req.messages, merkleTree=req.merkleTree)
    assert (tmp_path / "resp.bin").read_bytes() == resp.SerializeToString()
