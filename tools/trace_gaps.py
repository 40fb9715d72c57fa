"""Per-step timeline from a rocprofv3 kernel trace (run_kernel_trace.csv):
for every step (a launch of the first kernel named on the command line, e.g.
k_cl_pack, starts one) the span from that launch to the next step's, the
time some kernel is running (union of intervals over all streams), the idle
rest, and the largest gaps with the kernels on either side.

    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv k_cl_pack [first_step last_step]

The optional step window (0-based, end exclusive) isolates one pass of the
bench, e.g. its timed pipelined region; "spans" prints every step's span.
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.split(r"[(<]", name)[0].replace("evm::", "")


def main(path, first, lo=None, hi=None, show=False):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] == first]
    if len(starts) < 3:
        print("fewer than 3 steps of", first)
        return
    if show:
        for j, (a, b) in enumerate(zip(starts[:-1], starts[1:])):
            print(j, "%.1f" % ((rows[b][0] - rows[a][0]) / 1e3))
        return
    if lo is not None:
        starts = starts[lo:hi + 1]
    spans, busys = [], []
    gaps_all = []
    # steps much longer than the median carry something else (the bench's
    # host-to-host pass, the CPU baseline): left out
    med = sorted(rows[b][0] - rows[a][0] for a, b in zip(starts[:-1], starts[1:]))[(len(starts) - 1) // 2]
    for a, b in zip(starts[:-1], starts[1:]):
        seg = rows[a:b]
        t0, t1 = seg[0][0], rows[b][0]
        if t1 - t0 > 1.5 * med:
            continue
        busy, cur_s, cur_e = 0, None, None
        for s, e, name in seg:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps_all.append((s - cur_e, prev_name, name))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev_name = name
        busy += min(cur_e, t1) - cur_s
        if t1 > cur_e:
            gaps_all.append((t1 - cur_e, prev_name, "(next step) " + first))
        spans.append(t1 - t0)
        busys.append(busy)
    k = len(spans)
    print("steps %d  mean span %.1f us  busy %.1f us  idle %.1f us" % (
        k, sum(spans) / k / 1e3, sum(busys) / k / 1e3, (sum(spans) - sum(busys)) / k / 1e3))
    agg = {}
    for g, p, n in gaps_all:
        key = (p, n)
        agg[key] = agg.get(key, 0) + g
    for (p, n), g in sorted(agg.items(), key=lambda kv: -kv[1])[:12]:
        print("  %8.1f us/step  %s -> %s" % (g / k / 1e3, p, n))


if __name__ == "__main__":
    args = sys.argv[1:]
    if len(args) > 2 and args[2] == "spans":
        main(args[0], args[1], show=True)
    elif len(args) > 3:
        main(args[0], args[1], int(args[2]), int(args[3]))
    else:
        main(args[0], args[1] if len(args) > 1 else "k_cl_pack")
