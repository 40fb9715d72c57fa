"""The JS restatement used as bench.py's CPU baseline (oracle/js/cpu_merge.js,
run by node) makes the same applyMessages decisions and builds the same
MerkleTree JSON as the verbatim-SQL Python oracle."""
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import evolu_oracle as O
from tests import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
@pytest.mark.parametrize("seed", range(3))
def test_js_cpu_merge_matches_oracle(seed):
    from evolu_amd.engine import encode_timestamps

    msgs, cells = W.client_batch(900 + seed, n=400, n_cells=6 + seed)
    cid = {c: i for i, c in enumerate(cells)}
    db = O.ClientDb()
    dec = []
    want_tree = O.apply_messages(db, {}, msgs, dec)
    with tempfile.TemporaryDirectory() as d:
        tsf, cf = os.path.join(d, "ts.bin"), os.path.join(d, "cell.bin")
        encode_timestamps([m["timestamp"] for m in msgs]).tofile(tsf)
        np.array([cid[(m["table"], m["row"], m["column"])] for m in msgs], dtype="<u4").tofile(cf)
        out = subprocess.run(["node", os.path.join(ROOT, "oracle", "js", "cpu_merge.js"), tsf, cf, str(len(msgs)), "60",
                              "--check"], check=True, capture_output=True, text=True).stdout
    got = json.loads(out)
    assert got["done"] == len(msgs)
    assert got["flags"] == [(1 if u else 0) | (2 if x else 0) for u, x, _ in dec]
    assert got["tree"] == O.merkle_tree_to_string(want_tree)
