"""Per-kernel sums of rocprofv3 --pmc counters (any counters, one or more
passes): `python tools/pmc_sum.py <pass dir>...` prints, per kernel, each
counter's sum over its launches and the launch count, kernels ordered by the
first counter.  Names as tools/pmc_traffic.py shortens them."""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    order = []
    for d in sys.argv[1:]:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(p)):
                k = short(row["Kernel_Name"]) or row["Kernel_Name"][:40]
                c = row["Counter_Name"]
                if c not in order:
                    order.append(c)
                acc[k][c] += float(row["Counter_Value"])
                launches[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    for k in sorted(acc, key=lambda k: -acc[k].get(order[0], 0.0)):
        print("%-28s n=%-4d %s" % (k[:28], len(launches[k]), " ".join("%s=%.4g" % (c, acc[k][c]) for c in order if c in acc[k])))


if __name__ == "__main__":
    main()
