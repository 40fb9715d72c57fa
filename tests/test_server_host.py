"""Host-side pieces of SyncServer's device round (evolu_amd/server.py), no GPU:
the userId decode (the same strings the host path's per-body decode makes),
the message log's segments moving between host and device tensors, and the
DeviceResponses view."""
import numpy as np
import torch

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
