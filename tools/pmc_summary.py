"""Per-kernel mean of every PMC counter found under the given rocprofv3
output directories (csv).  Usage: python tools/pmc_summary.py DIR [DIR...]"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(p)):
                k = short(row["Kernel_Name"]) or row["Kernel_Name"][:40]
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(acc):
        vals = {c: sum(v) / len(v) for c, v in sorted(acc[k].items())}
        print(k, " ".join("%s=%.4g" % kv for kv in vals.items()))


if __name__ == "__main__":
    main()
