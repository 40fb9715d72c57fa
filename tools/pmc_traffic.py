"""HBM traffic per kernel launch from rocprofv3 PMC passes.

Run two separate counter passes (FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2:
they cannot share one), each with nothing but --pmc (MI355X_MICROARCH.md
§rocprofv3 PMC slots / §HBM):

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py ...

Corrections (MI355X_MICROARCH.md §HBM): both counters are in KiB; on gfx950
FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming
read, so it is doubled here (this kernel family's loads are 16-B-per-lane
streams); WRITE_SIZE reads exactly for 16-B streaming stores.  The Infinity
Cache is not excluded by these counters (bench inputs are 0.5 GB, > 256 MiB).

Usage: python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/traffic_<workload>.json
(one pair of passes per workload: a kernel's bytes per launch depend on the
workload's size, so bench.py reads the file of the leg it reports)
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d, counter):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = collections.defaultdict(list)
    for p in paths:
        for row in csv.DictReader(open(p)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            acc[name].append(float(row["Counter_Value"]))
    return acc


def short(name):
    """Kernel symbol -> the name bench.py's event profiler uses."""
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?(?:evm::)?([A-Za-z_0-9]+)(<[^>(]*>)?", name)
    if not m:
        return name
    base, targs = m.group(1), m.group(2) or ""
    if base in ("k_radix_scatter", "k_radix_hist", "k_scan_down", "k_scan_reduce", "k_scan_partials"):
        return None
    if base == "k_dist_scatter" and targs:
        return "(k_dist_scatter<%s>)" % ("SEND" if targs.strip("<>") == "0" else "RECV")
    if base == "k_dist_count" and targs:
        return "(k_dist_count<MODE>)"
    if base in ("k_svo_b", "k_tp_pack", "k_cl_fold_hist", "k_radix_onesweep", "k_radix_ghist") and targs:
        # KLAUNCH names a plain template launch by its text: "k_svo_b<true>"; the
        # parenthesised launches of the client/sort paths keep their own names
        t = targs.strip("<>").split(",")[0].strip()
        if base == "k_svo_b":
            return "k_svo_b<%s>" % t
        return base
    if base == "k_svo_a" and targs:
        # KLAUNCH names the template launch by its source text: "(k_svo_a<1024, true>)"
        # (template <CAP, SRC, THREADS = SVO_THREADS, LEAF = false>)
        args = [a.strip().rstrip("u") for a in targs[1:-1].split(",")]
        args = ["SVO_CAP" if a == "4096" else a for a in args]
        if len(args) >= 2:  # the source is an int template argument: 0 records, 1 rows, 2 received records
            args[1] = {"0": "false", "1": "true", "2": "SRC_WIRE"}.get(args[1], args[1])
        if len(args) == 4 and args[3] == "false":  # the default LEAF is not in the launch text
            args = args[:3]
        if len(args) == 4:  # the LEAF build names its workgroup size by the constant
            args[2] = "SVO_THREADS" if args[2] == "256" else args[2]
        if len(args) == 3 and args[2] == "256":  # the default workgroup size is not in the launch text
            args = args[:2]
        return "(k_svo_a<%s>)" % ", ".join(args)
    return base


def full_size(vals):
    """The launches of the leg's own size: a bench leg also launches its
    kernels on miniatures (warm-up shapes, self-checks on sampled owners), so
    the figure per launch is the mean over the launches within 2x of the
    largest -- never a miniature standing in for a full-size launch."""
    if not vals:
        return None, 0
    top = max(vals)
    big = [v for v in vals if v >= 0.5 * top]
    return sum(big) / len(big), len(big)


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    acc = {}
    for name in set(fetch) | set(write):
        k = short(name)
        if not k:
            continue
        f, w = acc.setdefault(k, ([], []))
        f.extend(fetch.get(name, []))
        w.extend(write.get(name, []))
    out = {}
    for k, (f, w) in acc.items():
        fm, fn = full_size(f)
        wm, wn = full_size(w)
        fb = 2.0 * 1024.0 * fm if fm is not None else None
        wb = 1024.0 * wm if wm is not None else None
        out[k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": (fb or 0.0) + (wb or 0.0),
                  "launches": max(fn, wn), "all_launches": max(len(f), len(w))}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
