"""Host-side pieces of SyncServer (evolu_amd/server.py), no GPU: how a call
is cut into rounds when a user sends several requests (the reference's
one-request-at-a-time order), the sub-arenas those rounds run on, and the
DeviceResponses view over a round's response arena."""
import numpy as np
import pytest

from evolu_amd.server import DeviceResponses, RangeError, _sub_arena, rounds_of


def test_rounds_of_puts_the_kth_request_of_a_user_in_round_k():
    users = [b"a", b"b", b"a", None, b"c", b"a", b"b"]
    assert rounds_of(users) == [[0, 1, 3, 4], [2, 6], [5]]
    assert rounds_of([]) == []
    assert rounds_of([b"x", b"y"]) == [[0, 1]]
    # every round has each user at most once, request order inside a round
    for rnd in rounds_of(users):
        us = [users[i] for i in rnd if users[i] is not None]
        assert len(us) == len(set(us)) and rnd == sorted(rnd)


def test_sub_arena_keeps_the_bodies_in_the_given_order():
    bodies = [b"aaa", b"", b"bbbb", b"cc"]
    off = np.zeros(len(bodies) + 1, dtype=np.uint64)
    np.cumsum([len(b) for b in bodies], out=off[1:])
    arena = np.frombuffer(b"".join(bodies), dtype=np.uint8)
    a, o = _sub_arena(arena, off, np.array([2, 0, 1], dtype=np.int64))
    assert o.tolist() == [0, 4, 7, 7]
    assert a[:7].tobytes() == b"bbbbaaa"


class _FakeSrv:
    """The two things DeviceResponses asks of its server."""

    def __init__(self, data: bytes):
        self._rounds = 1
        self.data = data

    def _fetch(self, nbytes):
        return np.frombuffer(self.data[:nbytes], dtype=np.uint8).copy()


def test_device_responses_view():
    srv = _FakeSrv(b"AAABBBBCC")
    off = np.array([0, 3, 3, 7, 9], dtype=np.uint64)
    err = RangeError("Invalid count value")
    r = DeviceResponses(srv, off, [True, None, True, True], 9)
    assert r.to_host() == [b"AAA", None, b"BBBB", b"CC"]
    r2 = DeviceResponses(srv, off, [True, err, True, True], 9)
    assert r2.to_host()[1] is err and len(r2) == 4
    # the server's next round reuses the arena: an old view refuses to read it
    srv._rounds += 1
    with pytest.raises(RuntimeError):
        r.to_host()
    # a call answered on the host path (no device arena)
    r3 = DeviceResponses(None, np.zeros(3, dtype=np.uint64), [b"x", None])
    assert r3.to_host() == [b"x", None]


def test_responses_sequence_views_and_overrides():
    """sync_arena(views=True)'s answer: memoryviews into one arena, made on
    access; a per-request result set on it overrides that entry."""
    from evolu_amd.server import Responses

    r = Responses(3)
    r.arena = memoryview(b"aabbbc")
    r.off = np.array([0, 2, 5, 6], dtype=np.uint64)
    assert [bytes(x) for x in r] == [b"aa", b"bbb", b"c"] and len(r) == 3
    assert isinstance(r[0], memoryview) and bytes(r[-1]) == b"c"
    err = RangeError("x")
    r[1] = err
    assert r[1] is err and bytes(r[2]) == b"c" and [bytes(x) for x in r[0:1]] == [b"aa"]
    with pytest.raises(IndexError):
        r[3]
