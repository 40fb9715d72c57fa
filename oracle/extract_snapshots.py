"""Extract the reference's vitest snapshot values into a JSON fixture.

TEST INFRASTRUCTURE, run in the build container only (``/root/reference``
does not exist on the GPU box).  Reads
``packages/evolu/test/__snapshots__/{timestamp,merkleTree}.test.ts.snap``
and writes ``tests/golden/reference_snapshots.json``: a mapping from the
snapshot name to its value (pretty-format -> JSON by dropping trailing
commas).  The fixture holds data only -- expected outputs of the
reference's own tests -- never reference source text.

Usage: python oracle/extract_snapshots.py
"""
import json
import os
import re
import sys

REF = "/root/reference/packages/evolu/test/__snapshots__"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "reference_snapshots.json")


def parse_snap(path):
    text = open(path).read()
    out = {}
    for m in re.finditer(r"exports\[`(.*?)`\] = `(.*?)`;", text, re.S):
        name, body = m.group(1), m.group(2).strip()
        body = re.sub(r",(\s*[}\]])", r"\1", body)
        out[name] = json.loads(body)
    return out


def main():
    snaps = {}
    for f in ("timestamp.test.ts.snap", "merkleTree.test.ts.snap"):
        snaps[f] = parse_snap(os.path.join(REF, f))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as fh:
        json.dump(snaps, fh, indent=1, sort_keys=True)
    print("wrote", OUT, sum(len(v) for v in snaps.values()), "snapshots", file=sys.stderr)


if __name__ == "__main__":
    main()
