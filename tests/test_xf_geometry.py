"""Host checks of the fused cross-cell check + fold's integer arithmetic
(evm_client.hip XF section): the minute-bucket geometry and the multiply-high
divisions the kernels use instead of 64-bit divisions.  The constants are read
from the kernel source so a change there is checked here.  Pure numpy."""
import os
import re

import numpy as np

SRC = os.path.join(os.path.dirname(__file__), "..", "evolu_amd", "csrc", "evm_client.hip")


def _src():
    with open(SRC) as f:
        return f.read()


def test_minute_offset_magic_is_exact():
    """d = umulhi(rel >> 5, M) >> 10 == rel // 60000 for every rel < XF_SPAN32 * 60000."""
    s = _src()
    m = int(re.search(r"__umulhi\(\(u32\)\(\(\(tc >> 16\) - base_ms\) >> 5\), (\d+)u\) >> 10", s).group(1))
    span32 = int(re.search(r"XF_SPAN32 = (\d+);", s).group(1))
    assert span32 * 60000 < 2 ** 32 <= (span32 + 1) * 60000
    M = np.uint64(m)
    top = (span32 * 60000) >> 5
    for a in range(0, top + 1, 1 << 24):
        n = np.arange(a, min(a + (1 << 24), top + 1), dtype=np.uint64)
        assert np.array_equal(((n * M) >> np.uint64(32)) >> np.uint64(10), n // np.uint64(1875))


def _geom(span, kb):
    magic = ((1 << 32) + span - 1) // span if span > 1 else 0
    W = ((span + (1 << kb) - 1) >> kb) + 1
    return magic, W, (W - 1).bit_length()


def test_bucket_geometry():
    """Every (minute offset d, hash) maps to a bucket < 2^kb whose first
    minute + the pair's minute offset gives d back, the offset fits the
    pair's bits and the LDS histogram (XF_WMAX), and the multiply-high
    division is floor(N / span) exactly."""
    s = _src()
    assert re.search(r"XF_SPAN_MAX = FOLD_MAXWIN \* FOLD_WIN;", s)
    span_max = int(re.search(r"FOLD_WIN = (\d+);", s).group(1)) * int(re.search(r"FOLD_MAXWIN = (\d+);", s).group(1))
    min_kb = int(re.search(r"XF_MIN_KB = (\d+);", s).group(1))
    wmax = span_max // (1 << min_kb) + 2
    rng = np.random.default_rng(1)
    spans = list(range(1, 200)) + [int(x) for x in rng.integers(1, span_max + 1, 200)] + [span_max]
    for kb in range(min_kb, 12):
        for span in spans + [(1 << kb) - 1, 1 << kb, (1 << kb) + 1]:
            magic, W, mb = _geom(span, kb)
            assert W <= wmax
            d = np.concatenate([np.arange(span), rng.integers(0, span, 1000)]).astype(np.uint64)
            for h in (rng.integers(0, 1 << 32, len(d), dtype=np.uint64), np.full(len(d), (1 << 32) - 1, np.uint64)):
                N = (d << np.uint64(kb)) | (h >> np.uint64(32 - kb))
                if span > 1:
                    b = (N * np.uint64(magic)) >> np.uint64(32)
                    b = np.where(b * np.uint64(span) > N, b - np.uint64(1), b)
                else:
                    b = N
                assert np.array_equal(b, N // np.uint64(span))
                assert (b < (1 << kb)).all()
                m0 = (b * np.uint64(span)) >> np.uint64(kb)
                moff = d - m0
                assert (moff < W).all() and (moff < (1 << mb)).all()
                assert np.array_equal(m0 + moff, d)
