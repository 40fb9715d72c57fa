"""Step times and selected kernels of bench.py JSON lines (A/B runs):
python tools/ab_summary.py PATTERN FILE..."""
import json
import re
import sys

pat = re.compile(sys.argv[1])
for f in sys.argv[2:]:
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    pk = (d.get("pipeline") or {}).get("kernels_ms_per_step") or d.get("kernels_ms_per_step") or {}
    r = d.get("reingest") or {}
    out = {"step": round(d["ms_per_step"], 3), "k": {k: round(v, 3) for k, v in pk.items() if pat.search(k)}}
    if r:
        out["reingest"] = round(r["ms_per_ingest_median"], 3)
        out["rk"] = {k: round(v, 3) for k, v in (r.get("kernels_ms") or {}).items() if pat.search(k)}
    print(f.split("/")[-1], json.dumps(out))
