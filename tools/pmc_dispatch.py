"""Per-dispatch PMC counter values of the kernels whose name matches a pattern,
in dispatch order (e.g. to tell K5's empty-store launches from its reingest
launches in one bench run).  Usage: python tools/pmc_dispatch.py PATTERN DIR [DIR...]"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    pat = re.compile(sys.argv[1])
    rows = collections.defaultdict(dict)  # (dir, dispatch) -> counter -> value
    names = {}
    for d in sys.argv[2:]:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if not pat.search(r["Kernel_Name"]):
                    continue
                key = int(r["Dispatch_Id"])
                c = r["Counter_Name"]
                rows[key][c] = rows[key].get(c, 0.0) + float(r["Counter_Value"])
                names[key] = r["Kernel_Name"][:48]
    for key in sorted(rows):
        print(key, names[key], " ".join("%s=%.4g" % kv for kv in sorted(rows[key].items())))


if __name__ == "__main__":
    main()
