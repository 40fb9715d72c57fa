"""CPU checks of the config-4 stream (evolu_amd/synth.py, the numpy twin of
the device generator evm_synth.hip): every timestamp canonical, each owner's
(millis, counter, node) triples unique per node as sendTimestamp makes them,
the source slices partition every owner's messages exactly once, the
client's ~90 % and the userId strings -- and murmur3(userId) mod G, the rank
evm_dist_directory assigns, from the reference hash."""
import numpy as np

from evolu_amd import synth
from oracle import evolu_oracle as O

SEED = 0xE7010004


def test_owner_ids_are_21_lower_hex_and_distinct():
    ids = synth.config4_owner_ids(SEED, 5000)
    assert ids.shape == (5000, 21)
    assert np.isin(ids, np.frombuffer(b"0123456789abcdef", np.uint8)).all()
    assert len({bytes(r) for r in ids}) == 5000


def test_messages_canonical_and_hlc_unique():
    O_, P = 50, 1000
    ts, _, keep = synth.config4_owners(SEED, P, 1, np.arange(O_))
    strings = [bytes(r[:46]).decode() for r in ts]
    for s in strings[:: 97]:
        t = O.timestamp_from_string(s)
        assert O.timestamp_to_string(*t) == s  # canonical
    assert (ts[:, 46:] == 0).all()
    per_owner = [strings[o * P:(o + 1) * P] for o in range(O_)]
    for msgs in per_owner:
        assert len(set(msgs)) == P
        # per node: strictly increasing (millis, counter) in send order (j = q, q + 4, ...)
        for q in range(4):
            seq = msgs[q::4]
            assert all(a < b for a, b in zip(seq, seq[1:]))
            assert len({m[30:] for m in seq}) == 1  # one node
    frac = keep.mean()
    assert 0.85 < frac < 0.95
    assert ts[:, 0:4].tobytes()[:4] == b"2024"


def test_source_slices_partition_each_owner():
    O_, P, G = 97, 100, 3
    seen = []
    for s in range(G):
        ts, owner, _ = synth.config4_source(SEED, O_, P, G, s)
        assert len(ts) == O_ * ((P - s + G - 1) // G)
        # one request per owner: its rows contiguous
        change = np.flatnonzero(np.diff(owner.astype(np.int64)) != 0)
        assert len(change) == O_ - 1
        assert len(np.unique(owner)) == O_
        seen.append(set(zip(owner.tolist(), (bytes(r) for r in ts))))
    allrows = set().union(*seen)
    assert sum(len(x) for x in seen) == len(allrows) == O_ * P
    # the receive order of one owner (source-major) is what config4_owners gives
    t_list, _, _ = synth.config4_owners(SEED, P, G, np.array([5]))
    got = []
    for s in range(G):
        ts, owner, _ = synth.config4_source(SEED, O_, P, G, s)
        got.append(ts[owner == 5])
    assert np.array_equal(np.concatenate(got), t_list)


def test_directory_rank_is_reference_murmur3():
    """The rank of owner g is murmur3(userId_g) mod G (murmurhash@2.0.1, seed 0:
    the oracle's restatement, pinned by the reference's timestamp hash vectors)."""
    ids = synth.config4_owner_ids(SEED, 200)
    for G in (2, 3, 8):
        dest = np.array([O.murmur3_32(bytes(r)) % G for r in ids])
        assert set(dest.tolist()) == set(range(G))
