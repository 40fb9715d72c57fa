"""Host-side pieces of SyncServer's device round (evolu_amd/server.py), no GPU:
the userId decode (the same strings the host path's per-body decode makes),
the message log's segments moving between host and device tensors, and the
DeviceResponses view."""
import numpy as np
import pytest
import torch

from evolu_amd import _lib as L

from evolu_amd.server import DeviceResponses, RangeError, _decode_spans, _Seg


def _spans(strs):
    b = [s if isinstance(s, bytes) else s.encode("utf-8") for s in strs]
    pk = np.frombuffer(b"".join(b) or b"\0", dtype=np.uint8)[: sum(len(x) for x in b)]
    off = np.zeros(len(b) + 1, dtype=np.uint64)
    np.cumsum([len(x) for x in b], out=off[1:])
    return b, pk, off, np.diff(off)


def test_decode_spans_matches_the_per_body_decode():
    cases = [
        ["%021x" % k for k in range(50)],                      # equal-length ASCII: the one-call path
        ["a", "bcd", "", "xyz0"],                               # ragged
        [b"ab\x00c", b"abcd"],                                  # a NUL byte: the per-span path
        [b"\xe9\xe9\xe9x", b"abcd"],                            # invalid UTF-8: replaced
        ["été", "abcde"],                             # multi-byte UTF-8
    ]
    for strs in cases:
        b, pk, off, ln = _spans(strs)
        assert _decode_spans(pk, off, ln) == [x.decode("utf-8", "replace") for x in b]


def test_log_segment_round_trip_between_host_and_device():
    rng = np.random.default_rng(1)
    ts = rng.integers(0, 256, size=(7, 48), dtype=np.uint8)
    coff = np.array([0, 3, 3, 10, 11, 11, 20, 24], dtype=np.uint64)
    content = rng.integers(0, 256, size=24, dtype=np.uint8)
    rowmap = np.array([6, 5, 4, 3, 2, 1, 0], dtype=np.uint64)
    s = _Seg(ts, coff, content, rowmap)
    d = s.dev(torch.device("cpu"))
    assert d[1].dtype == torch.int64 and (d[1].numpy().view(np.uint64) == coff).all()
    back = _Seg(*d)
    h = back.host()
    assert (h[0] == ts).all() and (h[1] == coff).all() and (h[2] == content).all() and (h[3] == rowmap).all()
    assert h[1].dtype == np.uint64 and h[3].dtype == np.uint64


def test_device_responses_view():
    buf = torch.from_numpy(np.frombuffer(b"AAABBBBCC", dtype=np.uint8).copy())
    off = np.array([0, 3, 3, 7, 9], dtype=np.uint64)
    err = RangeError("Invalid count value")
    r = DeviceResponses(buf, off, [True, None, True, True])
    assert r.to_host() == [b"AAA", None, b"BBBB", b"CC"]
    r2 = DeviceResponses(buf, off, [True, err, True, True])
    assert r2.to_host()[1] is err and len(r2) == 4


class _Srv:
    """SyncServer's user-directory state without an engine (the method and the
    property run on CPU tensors here)."""
    def __init__(self, capacity=100):
        from evolu_amd.server import SyncServer
        self._slot_d, self._dkeys, self._dlen, self._dhash, self._dslot, self._host_upto = {}, None, 0, None, None, 0
        self.capacity = capacity
        self.cls = SyncServer

    def slots(self, users):
        b = b"".join(u.encode() for u in users)
        packed = torch.from_numpy(np.frombuffer(b or b"\0", dtype=np.uint8).copy())
        ulen = np.array([len(u.encode()) for u in users], dtype=np.uint64)
        return self.cls._device_slots(self, packed, ulen, len(users))

    @property
    def slot(self):
        from evolu_amd.server import SyncServer
        return SyncServer.slot.fget(self)


def test_device_user_directory_assigns_the_dict_paths_slots():
    s = _Srv()
    r1 = ["%021x" % k for k in (5, 3, 9, 1)]
    assert s.slots(r1).tolist() == [0, 1, 2, 3]  # (a new server: request order)
    r2 = ["%021x" % k for k in (7, 9, 11, 5)]
    assert s.slots(r2).tolist() == [4, 2, 5, 0]  # (known users keep theirs; new ones in request order)
    assert s._host_upto == 0
    d = s.slot  # (the host dict, on demand)
    assert d == {u: i for i, u in enumerate(r1 + ["%021x" % 7, "%021x" % 11])} and s._host_upto == 6
    assert s.slots(["%021x" % 13]).tolist() == [6]
    assert s.slot["%021x" % 13] == 6
    # the host dict decides: a user twice, several lengths, non-ASCII, longer than 24 bytes
    assert s.slots(["%021x" % 20, "%021x" % 20]) is None
    assert s.slots(["%021x" % 21, "%020x" % 22]) is None
    assert s.slots(["é" * 10 + "a"]) is None
    assert _Srv().slots(["x" * 25]) is None
    # ids of another length than the directory's: the host dict decides
    assert s.slots(["%020x" % 23]) is None
    # capacity
    s2 = _Srv(capacity=2)
    assert s2.slots(["a" * 21, "b" * 21]).tolist() == [0, 1]
    with pytest.raises(L.EngineError):
        s2.slots(["c" * 21])
