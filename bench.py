"""Headline benchmark: CRDT messages merged/sec (LWW + Merkle) on MI355X.

Headline (BASELINE.json configs[1]): one
owner, 10M synthetic CrdtMessages over 1,000 cells (10 tables x 10 rows x 10
columns), 64 HLC nodes, shuffled batch order.  One step = one applyMessages
batch (evm_apply_batch: pack + canonical check + murmur3, cross-cell PK
check, LWW walks, Merkle fold) with the inputs already resident in HBM,
starting from an empty tree.

At N = 1 the same line carries the other BASELINE configs under extra keys:
  "client_adversarial": config 5 on the client side (equal-millis ties,
             exact and stale redeliveries, upper-case nodes), 10M messages,
             pipelined like the headline, its own roofline;
  "config1": the examples/nextjs todo-schema stream (100k messages, one
             owner, ~55k cells: the sort path), GPU time + CPU baseline;
  "config3": the sync server, 100k owners x 1,000 messages, one SyncRequest
             per owner (apps/server/src/index.ts:204-216: addMessages then
             getMessages against the client's tree), with its own roofline
             and CPU baseline (oracle/js/cpu_server.js, 1 and P threads);
  "config4": the N > 1 workload at world 1 (its weak-scaling base).

Multi-GPU (torchrun, one rank per GPU): BASELINE config 4 by default -- the
sync server over 125,000 owners x 1,000 messages per GPU (1B messages over
1M owners at 8 GPUs), owners sharded by murmur3(userId) mod N on the device,
every rank's slice routed over RCCL (evm_dist_route), roots all-gathered,
and an in-run self-check of sampled owners against an unsharded recompute
(`parity_checked`).  The elapsed time is the max over ranks.  `--workload
client` runs config 2 per rank, `--workload server` configs 3/5 standalone,
`--loopback N` rehearses config 4 with N ranks on one GPU.  Rank 0 prints one
JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CRDT messages merged/sec (LWW+Merkle) and % HBM roofline at 1/2/4/8 GPUs"
HBM_PEAK = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)

# Algorithmic (compulsory) bytes per message of each kernel on the client path,
# SURVEY.md section 8(d) accounting, restated per kernel in DESIGN.md.
ALG_BYTES_PER_MSG = {
    # streaming tc path (evm_client.hip TP1-TP3, the default)
    "k_tp_pack": 46 + 4 + 12,  # ts + cell in; packed (cell, tc) word 8 + hash 4 out (per-range cell maxima amortised)
    "k_tp_walk": 8 + 1,  # packed (cell, tc) word in, flag out
    "k_xf_scatter": 8 + 4 + 8,  # packed word + hash in, fingerprint pair out (minute buckets)
    "k_xf_dedup": 8,  # pair in (PK check + fold of the bucket's minutes in LDS)
    # exact walk path (a batch with a tie)
    "k_cl_pack": 46 + 28,  # ts in; order key 16 + rl 4 + hash 4 + minute 4 out
    "k_cl_scan1": 16 + 4 + 4,  # order key + rl + cell in (per-range aggregates amortised away)
    "k_cl_scan2": 16 + 4 + 4 + 1,  # order key + rl + cell in, flag out
    "k_xp_scatter": 4 + 8,  # hash in, (hash, index) out
    "k_xp_dedup": 8,  # (hash, index) in
    "k_cl_fold_hist": 9,  # flag + minute + hash in (per window)
    # sort path
    "k_pack": 46 + 4 + 32,  # ts string + cell in, 32-B record out
    "k_xcell": 24 + 8,  # key + hash read, one 8-B hash-set slot
    "(k_radix_scatter<K>)": 16,  # (cell, idx) in and out, per pass
    "(k_radix_hist<K>)": 4,
    "k_lww_reduce": 4 + 4 + 20,  # cell + idx + gathered key
    "k_lww_apply": 4 + 4 + 20 + 1,  # + flag out
    "k_fold_prep": 1 + 4 + 12 + 12,  # flag, pos, (minute, hash, aux) in; (ck, hash) out
}

# Server path (evm_server.hip), per message N and per new leaf L
SERVER_ALG = {
    "k_pack48": (46 + 4 + 32 + 4, 0),  # ts + owner in, 32-B record + minute out (only when records are needed)
    "k_minute48": (46 + 4 + 4, 0),  # ts + owner in, minute out (segment keys when K5 parses the rows)
    # per-owner ingest parsing the timestamp rows itself (requests of one owner, no owner above 1,024)
    "(k_svo_a<1024, true>)": (4 + 46 + 1 + 28, 8 + 4 + 1),  # perm + ts row in; flag + new row out; leaf code/xor/dup out
    # the same over packed records (interleaved owners / key-range segments)
    "(k_svo_a<1024, false>)": (4 + 32 + 1 + 28, 8 + 4 + 1),  # perm + record in; flag + new row out; leaf out
    # the same with 512-message capacity (first pass when the typical segment is small: Zipf tails)
    "(k_svo_a<512, true>)": (4 + 46 + 1 + 28, 8 + 4 + 1),
    "(k_svo_a<512, false>)": (4 + 32 + 1 + 28, 8 + 4 + 1),
    # the same over a route's received 24-B records, read where they arrived (evm_dist_ingest)
    # (into a store that has a tree: the new leaves' searches over the tree codes in LDS)
    "(k_svo_a<1024, true, SVO_THREADS, true>)": (4 + 46 + 1 + 28, 8 + 4 + 1),
    "(k_svo_a<1024, false, SVO_THREADS, true>)": (4 + 32 + 1 + 28, 8 + 4 + 1),
    "(k_svo_a<1024, SRC_WIRE>)": (4 + 24 + 1 + 28, 8 + 4 + 1),
    "(k_svo_a<512, SRC_WIRE>)": (4 + 24 + 1 + 28, 8 + 4 + 1),
    "k_wire_pack<false>": (24 + 4 + 4, 0),  # wire record + owner in, minute out (segment keys)
    "k_wire_pack<true>": (24 + 4 + 32 + 4, 0),  # wire record + owner in, 32-B record + minute out
    "k_svo_b": (28 + 32, 8 + 4 + 1 + 8 + 4),  # new rows in, store rows out; new leaves in, tree leaves out
    "k_svo_b<true>": (28 + 32, 8 + 4 + 1 + 8 + 4),  # (the merge into a non-empty store: LDS-staged keys)
    "k_svo_b<false>": (28 + 32, 8 + 4 + 1 + 8 + 4),  # (an empty store, a tree with leaves)
    "k_svo_copy": (28 + 32, 8 + 4 + 8 + 4 + 4),  # (an empty store and tree: rows unless K5 placed them, leaves + prefix XOR)
    "k_seg_key": (4 + 4 + 8, 0),  # owner + minute in, (segment, index) out
}
SERVER_PIPELINE_BYTES = 127  # the ideal server pipeline, one sort pass

# Kernels that run on the engine's second stream beside the walks (EVM_OPT_OVERLAP):
# their event durations include time spent sharing the chip, so they are not
# candidates for the roofline line while the overlap is on.
SIDE_KERNELS = {"k_xp_scatter", "k_xp_dedup", "k_xf_scatter", "k_xf_dedup"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--messages", type=int, default=10_000_000)
    ap.add_argument("--cells", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget per leg (0: skip)")
    ap.add_argument("--overlap", type=int, default=1, help="EVM_OPT_OVERLAP: independent checks on a second stream")
    ap.add_argument("--depth", type=int, default=4, help="config 2: batches in flight (evm_apply_batch_async)")
    ap.add_argument("--workload", choices=["auto", "client", "server", "config4", "adversarial", "config5",
                                           "config5c", "config5shape"], default="auto",
                    help="auto: client at N=1, config4 (+ the config5 and config5c legs) at N>1; "
                         "client: config 2 applyMessages (headline, + config 1, 3, 4 and 5-shape legs at N=1); "
                         "server: config 3 (or --zipf) ingest + diff + select alone, one GPU; "
                         "config4: the sharded sync server (1B msgs / 1M owners at 8 GPUs, weak scaling); "
                         "config5: the sharded sync server on config 5's stream (Zipf 1.2 owners, hot owners split "
                         "over every rank), self-checked; config5c: one owner's applyMessages batch split by cell, "
                         "self-checked; config5shape: the config-5 stream on one GPU, unsharded (profiling)")
    ap.add_argument("--radix", type=int, default=None,
                    help="EVM_OPT_RADIX for --workload config5shape (A/B of 10-bit digits)")
    ap.add_argument("--server-path", type=int, default=None,
                    help="EVM_OPT_SERVER_PATH for --workload config5shape (A/B; 4 = K5 on packed records)")
    ap.add_argument("--c5", type=int, default=1, help="N>1 default run: add the config5 and config5c legs")
    ap.add_argument("--c5-owners", type=int, default=125_000, help="config5: owners per GPU")
    ap.add_argument("--c5-messages", type=int, default=125_000_000, help="config5: messages per GPU")
    ap.add_argument("--c5-sample", type=int, default=200, help="config5: cold owners per rank in the self-check")
    ap.add_argument("--c5-share", type=float, default=0.1,
                    help="config5: an owner above this share of one rank's fair share of rows is split")
    ap.add_argument("--c5c-messages", type=int, default=10_000_000, help="config5c: messages per GPU")
    ap.add_argument("--c5c-cells", type=int, default=1000, help="config5c: cells per GPU")
    ap.add_argument("--c4-owners", type=int, default=125_000, help="config4: owners per GPU")
    ap.add_argument("--c4-per-owner", type=int, default=1000, help="config4: messages per owner")
    ap.add_argument("--c4-sample", type=int, default=1000, help="config4: owners per rank in the self-check")
    ap.add_argument("--c4-take", action="store_true",
                    help="config4 / config5: route + take + evm_server_ingest instead of evm_dist_ingest (A/B)")
    ap.add_argument("--loopback", type=int, default=0,
                    help="config4 (or --workload config5 / config5c) rehearsal: N loopback ranks (threads) sharing "
                         "GPU 0 through evm_dist_hub (not a multi-GPU measurement)")
    ap.add_argument("--extra", type=int, default=1, help="N=1 client run: add the config-1 and config-3 legs")
    ap.add_argument("--e2e", type=int, default=1, help="config 3 leg: add the end-to-end SyncServer round")
    ap.add_argument("--reingest", type=int, default=1, help="config 3 leg: add the reingest rounds (a growing store)")
    ap.add_argument("--shape", choices=["auto", "config2", "config4c"], default="auto",
                    help="client workload: config2 = one owner per GPU, no exchange; config4c = owners_per_rank "
                         "owners per GPU, every rank's batch holds messages of all the job's owners and routes them "
                         "to the owner's rank over RCCL (evm_dist_route); auto = config2 at N=1, config4c at N>1")
    ap.add_argument("--owners-per-rank", type=int, default=8, help="config4c: owners per GPU")
    ap.add_argument("--owners", type=int, default=100_000, help="server workload: owners per GPU")
    ap.add_argument("--per-owner", type=int, default=1000, help="server workload: messages per owner")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="server workload: owner sizes Zipf(s) (BASELINE config 5 skew, s = 1.2); owners x per-owner msgs in total")
    ap.add_argument("--request", type=int, default=1000,
                    help="server workload: messages per SyncRequest (one owner each, requests in random order); "
                         ">= per-owner: one request per owner (the reference's per-request sync exactly); "
                         "1 = every message shuffled on its own")
    ap.add_argument("--dom-events", type=int, default=1,
                    help="1: HIP events around the dominant kernel inside the timed region (the roofline's "
                         "duration); 0: none in the timed region, the duration from an identical pass after it")
    ap.add_argument("--traffic-dir", default=os.path.join(ROOT, "profiles", "r06"),
                    help="PMC-derived HBM bytes per launch per kernel, traffic_<workload>.json per workload "
                         "(written by tools/pmc_traffic.py from tools/gpu_prof.sh's passes)")
    return ap.parse_args()


def host_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    n = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except AttributeError:
        n_aff = n
    return {"nproc": n, "cpus_usable": n_aff, "cpu_model": model}


def node_bin():
    import shutil

    return shutil.which("node")


def cpu_baseline(ts_arena, cells, budget_s, what="config-2"):
    """The reference merge restated in JavaScript (oracle/js/cpu_merge.js:
    timestamp.ts / merkleTree.ts / applyMessages.ts decisions, SQLite
    replaced by Maps) under node on this host, one thread, over the first
    messages of the same stream; the Python oracle (verbatim SQL in sqlite3)
    when node is absent."""
    import subprocess
    import tempfile

    import numpy as np

    node = node_bin()
    if node is None:
        return cpu_baseline_python(ts_arena, cells, budget_s)
    k = min(len(cells), 2_000_000)
    with tempfile.TemporaryDirectory() as d:
        tsf, cf = os.path.join(d, "ts.bin"), os.path.join(d, "cell.bin")
        np.ascontiguousarray(ts_arena[:k, :48]).tofile(tsf)
        np.ascontiguousarray(cells[:k], dtype="<u4").tofile(cf)
        out = subprocess.run([node, os.path.join(ROOT, "oracle", "js", "cpu_merge.js"), tsf, cf, str(k),
                              str(budget_s)], check=True, capture_output=True, text=True, timeout=budget_s + 120).stdout
    r = json.loads(out)
    ver = subprocess.run([node, "--version"], capture_output=True, text=True).stdout.strip()
    return dict({
        "value": r["rate"],
        "unit": "msgs/s",
        "cores": 1,
        "kind": "port",
        "sample": "messages 0..%d of the %s stream applied by oracle/js/cpu_merge.js under node %s "
        "(applyMessages.ts decisions with the SQL as Maps, persistent-spread merkleTree.ts trie, murmur3), "
        "1 thread, %.1f s" % (r["done"], what, ver, r["seconds"]),
    }, **host_info())


def cpu_baseline_python(ts_arena, cells, budget_s):
    """The oracle (Python restatement, sqlite3 running the reference SQL) on
    the first S messages of the same workload, single-threaded."""
    from oracle import evolu_oracle as O

    def msgs(a, b):
        out = []
        for i in range(a, b):
            s = ts_arena[i, :46].tobytes().decode()
            c = int(cells[i])
            out.append({"timestamp": s, "table": "t%d" % (c // 100), "row": "r%d" % (c // 10 % 10),
                        "column": "c%d" % (c % 10), "value": i})
        return out

    pilot = msgs(0, 2000)
    db = O.ClientDb()
    t0 = time.perf_counter()
    tree = O.apply_messages(db, {}, pilot)
    rate = len(pilot) / (time.perf_counter() - t0)
    s = int(min(len(cells) - 2000, max(2000, rate * budget_s)))
    sample = msgs(2000, 2000 + s)
    t0 = time.perf_counter()
    O.apply_messages(db, tree, sample)
    dt = time.perf_counter() - t0
    return dict({
        "value": len(sample) / dt,
        "unit": "msgs/s",
        "cores": 1,
        "kind": "port",
        "sample": "messages 2000..%d of the stream applied by oracle/evolu_oracle.py "
        "(applyMessages.ts control flow, reference SQL verbatim in sqlite3, persistent-spread trie), "
        "1 thread, %.1f s" % (2000 + s, dt),
    }, **host_info())


def cpu_baseline_server(ts_np, owner_np, budget_s, what="config-3"):
    """apps/server/src/index.ts:121-216 restated in JavaScript
    (oracle/js/cpu_server.js: per SyncRequest getMerkleTree JSON.parse,
    INSERT OR IGNORE as a Set + persistent-spread inserts, the tree's
    JSON.stringify, diffMerkleTrees against the request's tree, the
    selection) under node: one thread (the reference's one server process)
    and P worker_threads over disjoint owners.  Sample: the first owners'
    requests of the same config-3 stream, in batch order."""
    import subprocess
    import tempfile

    import numpy as np

    node = node_bin()
    if node is None:
        return None
    hi = host_info()
    # P = the host's CPU share of ONE GPU (16 on this pool's boxes, OMP_NUM_THREADS): each
    # worker thread loads the whole sample, so P = nproc (256) would need P copies of it
    P = max(1, min(hi["cpus_usable"], CPU_SHARE_PER_GPU))
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for threads in sorted({1, P}):
            K = 500 * (threads + 1)  # owners in the sample: more than the budget gets through
            sel = owner_np < K
            tsf, of = os.path.join(d, "ts%d.bin" % threads), os.path.join(d, "o%d.bin" % threads)
            np.ascontiguousarray(ts_np[sel, :48]).tofile(tsf)
            np.ascontiguousarray(owner_np[sel], dtype="<u4").tofile(of)
            out = subprocess.run([node, os.path.join(ROOT, "oracle", "js", "cpu_server.js"), tsf, of,
                                  str(int(sel.sum())), str(budget_s), str(threads)], check=True, capture_output=True,
                                 text=True, timeout=4 * budget_s + 240).stdout
            res[threads] = json.loads(out)
    r1 = res[1]
    out = dict({
        "value": r1["rate"], "unit": "msgs/s", "cores": 1, "kind": "port",
        "sample": "the first %d SyncRequests (%d messages, one owner each) of the %s stream served by "
                  "oracle/js/cpu_server.js (index.ts getMerkleTree + addMessages + getMessages; SQL as Maps; "
                  "persistent-spread trie; murmur3), 1 thread, %.1f s" % (r1["requests"], r1["done"], what,
                                                                          r1["seconds"]),
    }, **hi)
    if P > 1:
        rp = res[P]
        out["threads_%d" % P] = {"value": rp["rate"], "cores": P, "requests": rp["requests"], "messages": rp["done"],
                                 "seconds": rp["seconds"], "sample": "worker_threads over disjoint owners (owner %% %d)" % P,
                                 "why_%d" % P: "the host's CPU share of one GPU on this pool (OMP_NUM_THREADS=16); "
                                               "P = nproc is not run: every worker loads the whole sample"}
    return out


CPU_SHARE_PER_GPU = 16


def cpu_baseline_server_n(world, budget_s, dev):
    """The CPU baseline of an N-GPU server line (rank 0, after the timed legs):
    cpu_server.js on a config-3-shaped stream (evs_config4_source with one
    source: every message of the first owners, one SyncRequest per owner),
    1 thread and the per-GPU CPU share; `per_node_share` states what N
    shares of it would do (linear in threads: owners are disjoint)."""
    from evolu_amd import synth

    gen = synth.DeviceSynth()
    K = 500 * (CPU_SHARE_PER_GPU + 1)
    ts, owner, _ = gen.source(C4_SEED, K, 1000, 1, 0, dev)
    out = cpu_baseline_server(ts.cpu().numpy(), owner.cpu().numpy().astype("uint32"), budget_s,
                              what="config-3-shaped (%d owners x 1,000, device generator)" % K)
    if out is not None:
        tk = "threads_%d" % CPU_SHARE_PER_GPU
        if tk in out:
            out["per_node_share"] = {"gpus": world, "threads": world * CPU_SHARE_PER_GPU,
                                     "value_extrapolated": world * out[tk]["value"],
                                     "how": "%d x the %d-thread rate (disjoint owners scale linearly)"
                                            % (world, CPU_SHARE_PER_GPU)}
    return out


def dominant(prof, alg_keys, exclude=()):
    known = {k: v for k, v in prof.items() if k in alg_keys and k not in exclude}
    return max(known, key=lambda k: known[k][0])


TRAFFIC_DIR = os.path.join(ROOT, "profiles")


def traffic_of(kernel, workload):
    """HBM bytes per launch of `kernel` in `workload` from the PMC passes
    (profiles/traffic_<workload>.json), or None."""
    path = os.path.join(TRAFFIC_DIR, "traffic_%s.json" % workload)
    if not os.path.exists(path):
        return None
    t = json.load(open(path)).get(kernel)
    if t is None:
        return None
    return t["bytes"] if isinstance(t, dict) else t  # HBM bytes per launch (PMC, corrected)


_STDOUT = None  # the real stdout: the one JSON line goes there, everything else to stderr


def quiet_stdout():
    """Libraries print banners on the C-level stdout (RCCL's version lines at
    communicator creation): route fd 1 to stderr for the whole run and keep
    the real stdout for the result line only."""
    global _STDOUT
    sys.stdout.flush()
    _STDOUT = os.dup(1)
    os.dup2(2, 1)


def _traffic_ratios(o):
    """Every roofline block with a PMC traffic figure also states it as a
    multiple of its algorithmic bytes (traffic well above 1x = re-reads)."""
    if isinstance(o, dict):
        t, a = o.get("traffic"), o.get("alg_bytes_per_launch")
        if "traffic" in o and "alg_bytes_per_launch" in o:
            o["traffic_ratio"] = (t / a) if t and a else None
            o["traffic_src"] = os.path.relpath(TRAFFIC_DIR, ROOT)
        for v in o.values():
            _traffic_ratios(v)
    elif isinstance(o, list):
        for v in o:
            _traffic_ratios(v)


def emit(obj):
    _traffic_ratios(obj)
    line = (json.dumps(obj) + "\n").encode()
    if _STDOUT is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_STDOUT, line)


def progress(what):
    """A line on stderr as each part of a long run starts (the JSON line comes at the end)."""
    print("bench: %s (%.0f s)" % (what, time.perf_counter() - T_START), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def main():
    global TRAFFIC_DIR
    quiet_stdout()
    a = parse()
    TRAFFIC_DIR = a.traffic_dir
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from evolu_amd import synth
    from evolu_amd.engine import Engine

    if a.loopback:
        if a.workload == "config5":
            emit(config5_loopback(a, a.loopback))
        elif a.workload == "config5c":
            emit(client_split_loopback(a, a.loopback))
        else:
            emit(config4_loopback(a, a.loopback))
        return
    workload = a.workload if a.workload != "auto" else ("client" if world == 1 else "config4")
    dev = torch.device("cuda", local)
    if workload in ("config4", "config5", "config5c"):
        comm = TorchComm(world, dev)

        def leg(fn, *args, **kw):
            eng = Engine(local)
            dd = make_dist(eng, rank, world)
            try:
                return fn(eng, dd, comm, *args, **kw)
            finally:
                dd.free()
                eng.close()
                torch.cuda.empty_cache()

        if workload == "config4":
            res = leg(config4_rank, a.c4_owners, a.c4_per_owner, a.steps, a.warmup, a.c4_sample,
                      dist_ingest=not getattr(a, "c4_take", False))
            data = "synthetic (seeded HLC streams generated on the device, SURVEY 8(d) config 4)"
        elif workload == "config5":
            res = leg(config5_rank, a.c5_owners, a.c5_messages, a.steps, a.warmup, a.c5_sample, a.c5_share,
                      dist_ingest=not getattr(a, "c4_take", False))
            data = "synthetic (device generator evs_config5_shape, SURVEY 8(d) config 5)"
        else:
            res = leg(client_split_rank, a.c5c_messages, a.c5c_cells, a.steps, a.warmup)
            data = "synthetic (synth.client_adversarial per slice, SURVEY 8(d) config 5, client side)"
        extra = {}
        if workload == "config4" and world > 1 and a.c5:
            # BASELINE config 5 at the same N: the server on the Zipf stream with hot owners
            # split, and one owner's client batch split by cell -- both self-checked
            c5 = leg(config5_rank, a.c5_owners, a.c5_messages, min(a.steps, 5), min(a.warmup, 1), a.c5_sample,
                     a.c5_share, dist_ingest=not getattr(a, "c4_take", False))
            c5c = leg(client_split_rank, a.c5c_messages, a.c5c_cells, min(a.steps, 5), min(a.warmup, 1))
            extra = {"config5": c5, "config5c": c5c}
        if rank == 0:
            out = {"metric": METRIC, "value": res.pop("value"), "unit": "msgs/s", "n_gpus": world,
                   "steps": a.steps, "warmup": a.warmup, "ms_per_step": res.pop("ms_per_step"),
                   "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
                   "data": data, "cpu_baseline": None}
            res.pop("steps"), res.pop("warmup", None)
            out.update(res)
            out.update(extra)
            if a.cpu_seconds > 0 and workload != "config5c":
                out["cpu_baseline"] = cpu_baseline_server_n(world, min(a.cpu_seconds, 10.0), dev)
            emit(out)
        if world > 1:
            dist.destroy_process_group()
        return
    if workload == "config5shape":  # the config-5 shape leg alone, one GPU (profiling)
        eng = Engine(local)
        if a.radix is not None:
            eng.set_option(4, a.radix)
        if a.server_path is not None:
            eng.set_option(2, a.server_path)
        emit(dict(config5_shape_leg(eng, a), metric=METRIC + " [server config 5 shape leg]"))
        eng.close()
        return
    if workload == "adversarial":  # the client_adversarial leg alone (profiling)
        eng = Engine(local)
        emit(dict(adversarial_leg(eng, a), metric=METRIC + " [client config 5 leg]"))
        eng.close()
        return
    if workload == "server":
        out = server_run(a, rank, world, local, a.owners, a.per_owner, a.zipf, a.request, cpu=rank == 0 and world == 1)
        if rank == 0:
            emit(out)
        if world > 1:
            dist.destroy_process_group()
        return
    shape = a.shape if a.shape != "auto" else ("config2" if world == 1 else "config4c")
    if shape == "config4c":
        out = client_routed(a, rank, world, local)
        if rank == 0:
            emit(out)
        if world > 1:
            dist.destroy_process_group()
        return
    # each rank: its own owner (seed per rank), same shape
    ts_np, cell_np = synth.config2(a.messages, a.cells, seed_config=2 + 1000 * rank)
    eng = Engine(local)
    eng.set_option(3, a.overlap)  # EVM_OPT_OVERLAP
    ts = eng.dev(ts_np)
    cell = eng.dev(cell_np)
    empty = eng.tree_new(1)
    # two output sets: batch k + 1 is enqueued (evm_apply_batch_async) before
    # batch k is waited, so the host's launches and status read overlap the GPU
    DEPTH = max(1, a.depth)  # batches enqueued ahead of the one being waited
    outs = [(torch.empty(a.messages, dtype=torch.uint8, device=ts.device),
             torch.empty(a.cells, dtype=torch.int32, device=ts.device)) for _ in range(DEPTH)]
    flags, winner = outs[0]

    def step():
        _, _, tree, _ = eng.apply_batch(empty, ts, cell, a.cells, flags=flags, winner=winner)
        return tree

    host_us = {"enqueue": [], "wait": []}

    def run_pipelined(k_steps):
        import collections

        q = collections.deque()
        for k in range(k_steps):
            if len(q) == DEPTH:
                w0 = time.perf_counter()
                q.popleft().wait()[2].free()
                host_us["wait"].append((time.perf_counter() - w0) * 1e6)
            e0 = time.perf_counter()
            q.append(eng.apply_batch_async(empty, ts, cell, a.cells, *outs[k % DEPTH]))
            host_us["enqueue"].append((time.perf_counter() - e0) * 1e6)
        while q:
            q.popleft().wait()[2].free()

    eng.prof_enable(True)  # warmup with events on: fills the engine's event pool
    for _ in range(a.warmup):
        step().free()
    run_pipelined(max(a.warmup, 2))
    torch.cuda.synchronize()
    # per-kernel breakdown (untimed, an event pair around every launch): picks
    # the dominant main-stream kernel
    eng.prof_reset()
    u0 = time.perf_counter()
    for _ in range(a.steps):
        step().free()
    torch.cuda.synchronize()
    ms_all_events = (time.perf_counter() - u0) / a.steps * 1e3
    prof = eng.prof_report()
    dom = dominant(prof, ALG_BYTES_PER_MSG, SIDE_KERNELS if a.overlap else ())
    # timed region: events only around the dominant kernel's launches
    eng.prof_only(dom)
    eng.prof_reset()
    eng.prof_enable(bool(a.dom_events))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    host_us["enqueue"].clear()
    host_us["wait"].clear()
    st0 = eng.stats()
    t0 = time.perf_counter()
    run_pipelined(a.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    st1 = eng.stats()
    # the path the timed batches took: every one on the tc streaming path, none redone
    path = {k: st1[k] - st0[k] for k in ("tc_batches", "tc_redos", "small_batches", "small_fallbacks")}
    path["batches"] = a.steps
    path["kernels"] = sorted(prof)
    if not a.dom_events:  # the dominant kernel's duration from an identical pass
        eng.prof_enable(True)
        run_pipelined(a.steps)
        torch.cuda.synchronize()
    eng.prof_enable(False)
    eng.prof_only(None)
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=ts.device)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    prof_dom = eng.prof_report()
    # host-to-host (never `value`): the batch in pinned host memory, H2D of
    # timestamps + cells, the step, D2H of flags + winners -- what a caller
    # that hands over host buffers (the N-API addon) sees
    ts_h = torch.from_numpy(ts_np).pin_memory()
    cell_h = torch.from_numpy(np.ascontiguousarray(cell_np).view(np.int32)).pin_memory()
    flags_h = torch.empty(a.messages, dtype=torch.uint8).pin_memory()
    win_h = torch.empty(a.cells, dtype=torch.int32).pin_memory()
    reps = max(1, min(a.steps, 5))
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(reps):
        ts.copy_(ts_h, non_blocking=True)
        cell.view(torch.int32).copy_(cell_h, non_blocking=True)
        step().free()
        flags_h.copy_(flags, non_blocking=True)
        win_h.copy_(winner, non_blocking=True)
    torch.cuda.synchronize()
    ms_h2h = (time.perf_counter() - h0) / reps * 1e3

    if rank == 0:
        ms_step = elapsed / a.steps * 1e3
        value = world * a.messages * a.steps / elapsed
        # dominant kernel and its roofline, from the timed region's events
        tot_ms, launches = prof_dom[dom]
        avg_s = tot_ms / launches / 1e3
        alg = ALG_BYTES_PER_MSG[dom] * a.messages
        achieved = alg / avg_s
        roof = {"bound": "hbm", "kernel": dom, "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": traffic_of(dom, "client"),
                "kernel_ms_avg": avg_s * 1e3, "alg_bytes_per_launch": alg,
                "kernel_share_of_step": tot_ms / (ms_step * a.steps)}
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "msgs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded HLC streams, SURVEY 8(d) config 2)",
            "config": {"workload": "config2: applyMessages, 1 owner per GPU, %d msgs, %d cells, 64 nodes, shuffled"
                       % (a.messages, a.cells), "messages_per_gpu": a.messages, "cells": a.cells,
                       "parallelism": "owner-sharded, %d rank(s)" % world},
            "roofline": roof,
            "path": path,
            "pipeline": {"alg_bytes_per_msg": 120, "ms_per_step_all_kernel_events": ms_all_events,
                         "batches_in_flight": DEPTH,
                         "host_enqueue_us_avg": sum(host_us["enqueue"]) / max(1, len(host_us["enqueue"])),
                         "host_wait_us_avg": sum(host_us["wait"]) / max(1, len(host_us["wait"])),
                         "host_to_host_ms_per_step": ms_h2h, "host_to_host_msgs_per_s": a.messages / ms_h2h * 1e3,
                         "pipeline_hbm_frac": 120 * a.messages / (elapsed / a.steps) / HBM_PEAK,
                         "kernels_ms_per_step": {k: v[0] / a.steps for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])}},
            "cpu_baseline": None,
        }
        if world == 1 and a.cpu_seconds > 0:
            progress("cpu baseline")
            out["cpu_baseline"] = cpu_baseline(ts_np, cell_np, a.cpu_seconds)
        del ts, cell, flags, ts_h, cell_h
        if world == 1 and a.extra:
            progress("leg client_adversarial")
            out["client_adversarial"] = adversarial_leg(eng, a)
            progress("leg config1")
            out["config1"] = config1_leg(eng, a)
            eng.close()
            torch.cuda.empty_cache()
            progress("leg config3")
            out["config3"] = server_run(a, 0, 1, local, 100_000, 1000, 0.0, 1000, cpu=a.cpu_seconds > 0, leg=True)
            # config 4 at world 1: the per-GPU work of the N-GPU line (its weak-scaling base)
            progress("leg config4")
            eng4 = Engine(local)
            dd4 = make_dist(eng4, 0, 1)
            out["config4"] = config4_rank(eng4, dd4, TorchComm(1, torch.device("cuda", local)), a.c4_owners,
                                          a.c4_per_owner, a.steps, a.warmup, a.c4_sample,
                                          dist_ingest=not getattr(a, "c4_take", False))
            dd4.free()
            eng4.close()
            torch.cuda.empty_cache()
            progress("leg config5_shape")
            eng5 = Engine(local)
            out["config5_shape"] = config5_shape_leg(eng5, a)
            eng5.close()
            torch.cuda.empty_cache()
        emit(out)
    if world > 1:
        dist.destroy_process_group()


XGMI_LINK = 153e9  # B/s per xGMI link (one link per peer in an 8-GPU node)
ROUTE_BYTES = 24  # wire record per routed message of a server route (evm_dist.hip narrow: tc, node, owner, case mask)
DIST_ALG = {  # (the server benches route 24-B records: no cell / source index travels)
    "(k_dist_count<MODE>)": 4,  # owner in (send side: caller's owner ids; take side: the records' owner field)
    "(k_dist_scatter<SEND>)": 48 + 4 + 24,  # ts row + owner in, wire record out
    "(k_dist_scatter<RECV>)": 24 + 48 + 4,  # wire record in; rebuilt ts row + owner out (evm_dist_take)
    "k_dist_owner": 24 + 4,  # wire record in (the owner field's sectors), local owner out (evm_dist_ingest)
}


def make_dist(eng, rank, world):
    """The RCCL communicator of evm_dist_*: rank 0's id broadcast over torch.distributed."""
    import torch
    import torch.distributed as dist

    from evolu_amd.engine import Dist, dist_unique_id

    uid = torch.zeros(128, dtype=torch.uint8, device=torch.device("cuda", eng.device))
    if rank == 0:
        uid.copy_(torch.frombuffer(bytearray(dist_unique_id()), dtype=torch.uint8))
    if world > 1:
        dist.broadcast(uid, 0)
    d = Dist(eng, bytes(uid.cpu().numpy()), rank, world)
    d.transport = "RCCL"
    return d


def client_routed(a, rank, world, local):
    """Config 4, client side (SURVEY 8(d) "4-C"): owners_per_rank owners per
    GPU, each with config-2 cell contention (a.cells cells, 64 HLC nodes per
    source rank).  Every rank's batch slice holds messages of ALL the job's
    owners in random order; one step = evm_dist_route (RCCL all-to-all by
    owner % world) + evm_dist_take grouped by local owner + one
    applyMessages batch per owner (enqueued together) + the owners' roots
    all-gathered (evm_dist_gather_roots).  Weak scaling: a.messages per GPU."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from evolu_amd import synth
    from evolu_amd.engine import Engine

    K = a.owners_per_rank
    G = K * world
    M = a.messages
    rng = np.random.default_rng(4000 + rank)
    owner_np = rng.integers(0, G, M).astype(np.uint32)
    cnt = np.bincount(owner_np, minlength=G)
    ts_np = np.empty((M, 48), dtype=np.uint8)
    cell_np = np.empty(M, dtype=np.uint32)
    for g in range(G):
        if cnt[g] == 0:
            continue
        t_g, c_g = synth.config2(int(max(cnt[g], 1000)), a.cells, seed_config=40_000 + 64 * g + rank)
        at = np.nonzero(owner_np == g)[0]
        ts_np[at] = t_g[: cnt[g]]
        cell_np[at] = c_g[: cnt[g]]
    eng = Engine(local)
    eng.set_option(3, a.overlap)
    dev = torch.device("cuda", local)
    dd = make_dist(eng, rank, world)
    ts, owner, cell = eng.dev(ts_np), eng.dev(owner_np), eng.dev(cell_np)
    del ts_np
    cap = int(M * 1.25) + 65536
    bufs = (torch.empty((cap, 48), dtype=torch.uint8, device=dev), torch.empty(cap, dtype=torch.int32, device=dev),
            torch.empty(cap, dtype=torch.int32, device=dev), None)
    flags = torch.empty(cap, dtype=torch.uint8, device=dev)
    winners = torch.empty((K, a.cells), dtype=torch.int32, device=dev)
    empty = eng.tree_new(1)
    route_ms = []

    def step():
        r0 = time.perf_counter()
        n_r = dd.route(ts, owner, aux=cell)
        t2, _, c2, _, goff = dd.take(group=K, src=False, out=bufs)
        route_ms.append((time.perf_counter() - r0) * 1e3)
        pend = [eng.apply_batch_async(empty, t2[goff[k]:goff[k + 1]], c2[goff[k]:goff[k + 1]], a.cells,
                                      flags[goff[k]:goff[k + 1]], winners[k]) for k in range(K)]
        trees = [p.wait()[2] for p in pend]
        # the rank's K owners' roots -> every owner's root on every rank
        root, present = dd.gather_roots(trees, G)
        for t in trees:
            t.free()
        return n_r, root

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    eng.prof_enable(True)
    eng.prof_reset()
    step()
    torch.cuda.synchronize()
    prof = eng.prof_report()
    alg_all = dict(ALG_BYTES_PER_MSG, **DIST_ALG)
    dom = dominant(prof, alg_all, SIDE_KERNELS if a.overlap else ())
    eng.prof_only(dom)
    eng.prof_reset()
    route_ms.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_recv = 0
    for _ in range(a.steps):
        n_recv, _ = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    prof_dom = eng.prof_report()
    eng.prof_enable(False)
    eng.prof_only(None)
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    route = torch.tensor([sum(route_ms) / max(1, len(route_ms))], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(route, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    route_ms_avg = float(route.item())
    ms = elapsed / a.steps * 1e3
    tot_ms, launches = prof_dom[dom]
    avg_s = tot_ms / launches / 1e3
    rows = n_recv if "RECV" in dom or dom in ALG_BYTES_PER_MSG else M
    alg = alg_all[dom] * rows / (K if dom in ALG_BYTES_PER_MSG else 1)  # client kernels run once per owner batch
    remote = M * (world - 1) / world  # rows leaving this rank (uniform owners)
    out = {
        "metric": METRIC, "value": world * M * a.steps / elapsed, "unit": "msgs/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (seeded HLC streams, SURVEY 8(d) config 4, client side)",
        "config": {"workload": "config4c: applyMessages, %d owners per GPU x %d cells each, %d msgs per GPU from all "
                               "%d owners of the job, routed by owner %% world over RCCL (evm_dist_route), one batch "
                               "per owner, roots all-gathered" % (K, a.cells, M, G),
                   "messages_per_gpu": M, "owners_per_gpu": K, "cells_per_owner": a.cells,
                   "parallelism": "owner-sharded, %d rank(s), RCCL all-to-all" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": alg / avg_s / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": alg / avg_s / HBM_PEAK, "traffic": traffic_of(dom, "config4c"),
                     "kernel_ms_avg": avg_s * 1e3, "alg_bytes_per_launch": alg,
                     "kernel_share_of_step": tot_ms / (ms * a.steps)},
        "route": {"ms_per_step": route_ms_avg, "bytes_per_msg": ROUTE_BYTES,
                  "remote_bytes_per_gpu": remote * ROUTE_BYTES,
                  "xgmi_frac": (remote * ROUTE_BYTES / (route_ms_avg / 1e3) / ((world - 1) * XGMI_LINK))
                  if world > 1 else None,
                  "xgmi_peak_GBps": (world - 1) * XGMI_LINK / 1e9 if world > 1 else None},
        "pipeline": {"alg_bytes_per_msg": 120,
                     "kernels_ms_per_step": {k: v[0] for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:14]}},
        "cpu_baseline": None,
    }
    dd.free()
    eng.close()
    return out


class TorchComm:
    """Rank coordination over torch.distributed (the bench's timing only)."""

    def __init__(self, world, dev):
        self.world, self.dev = world, dev

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist

            dist.barrier()

    def _reduce(self, x, dtype, op):
        import torch
        import torch.distributed as dist

        t = torch.tensor([x], dtype=dtype, device=self.dev)
        if self.world > 1:
            dist.all_reduce(t, op=op)
        return t.item()

    def max(self, x: float) -> float:
        import torch
        import torch.distributed as dist

        return float(self._reduce(x, torch.float64, dist.ReduceOp.MAX))

    def min(self, x: int) -> int:
        import torch
        import torch.distributed as dist

        return int(self._reduce(x, torch.int64, dist.ReduceOp.MIN))

    def sum_vec(self, v):
        """Element-wise sum over ranks of an int64 vector (numpy in, numpy out)."""
        import numpy as np
        import torch
        import torch.distributed as dist

        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.int64)).to(self.dev)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.cpu().numpy()

    def all_gather(self, t):
        """Every rank's tensor (same shape on every rank) -> list in rank order (device to device)."""
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return [t]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous())
        return out


class ThreadComm:
    """The same for loopback ranks (threads of one process, evm_dist_hub)."""

    def __init__(self, world):
        import threading

        self.world = world
        self.bar = threading.Barrier(world)
        self.vals = [None] * world

    def barrier(self):
        self.bar.wait()

    def _reduce(self, rank, x, f):
        self.bar.wait()
        self.vals[rank] = x
        self.bar.wait()
        r = f(self.vals)
        self.bar.wait()
        return r

    def bind(self, rank):
        comm = self

        class R:
            def barrier(self):
                comm.barrier()

            def max(self, x):
                return comm._reduce(rank, x, max)

            def min(self, x):
                return comm._reduce(rank, x, min)

            def sum_vec(self, v):
                import numpy as np

                return comm._reduce(rank, np.asarray(v, dtype=np.int64), lambda vs: np.sum(vs, axis=0))

            def all_gather(self, t):
                import torch

                torch.cuda.current_stream().synchronize()  # t is complete before a peer copies it

                def copies(vs):
                    out = [x.clone() for x in vs]
                    torch.cuda.current_stream().synchronize()  # (peers may free theirs after the barrier)
                    return out

                return comm._reduce(rank, t, copies)

        return R()


C4_SEED = 0xE7010004  # seed = 0xE7010000 + config number


def config4_rank(eng, dd, comm, owners_per_gpu=125_000, per_owner=1000, steps=10, warmup=2, sample=1000,
                 seed=C4_SEED, verbose=False, dist_ingest=True, src_wire_steps=3):
    """BASELINE config 4 on one rank: the sync server (index.ts:138-202,
    addMessages + getMessages) over owners_per_gpu x world owners of
    per_owner messages each, sharded by murmur3(userId) mod world.

    Every rank's input is its slice of the job's requests: for every owner of
    the job one SyncRequest with the messages j = rank, rank + world, ... of
    that owner, requests in a seeded owner order (evm_synth.hip).  One step
    = route (RCCL all-to-all of counts + 32-B packed records, evm_dist_route)
    + take with local owner ids + addMessages into an empty store
    (evm_server_ingest) + getMessages against each owner's client tree
    (the client knows ~90 % of the owner's messages; requester = the owner's
    node 0, excluded by the NOT LIKE filter) + every owner's root all-gathered
    (evm_dist_gather_roots).  Weak scaling: owners_per_gpu x per_owner
    messages per GPU (125M: 1B over 1M owners at 8 GPUs).

    After the timed steps every rank re-derives `sample` of its owners on its
    own -- their messages regenerated in receive order, one unsharded ingest
    + select on this GPU -- and compares inserted counts, roots (as
    all-gathered), diffs and the selected rows byte for byte; the result is
    agreed over the ranks (parity_checked)."""
    import numpy as np
    import torch

    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.sharded import ShardedServer

    rank, world = dd.rank, dd.world
    dev = torch.device("cuda", eng.device)
    O = owners_per_gpu * world
    P = per_owner
    gen = synth.DeviceSynth()
    t_setup = time.perf_counter()
    ids = gen.owner_ids(seed, O, dev)
    srv = ShardedServer(eng, dd, ids, 21)
    n_local = srv.n_local
    ts_in, owner_in, _ = gen.source(seed, O, P, world, rank, dev)
    # client trees (and requester nodes) of this rank's owners, in chunks
    client = eng.tree_new(n_local)
    node = torch.empty((max(n_local, 1), 16), dtype=torch.uint8, device=dev)
    chunk = max(1, 16_000_000 // P)
    for c0 in range(0, n_local, chunk):
        lst = srv.owners_here[c0:c0 + chunk]
        t_c, li_c, k_c = gen.owners(seed, O, P, 1, lst, dev)
        node[c0:c0 + lst.numel()] = t_c.view(lst.numel(), P, 48)[:, 0, 30:46]  # message 0 = node 0
        kb = k_c.bool()
        nxt = eng.merkle_insert(client, t_c[kb].contiguous(), (li_c[kb] + c0).contiguous())
        client.free()
        client = nxt
        del t_c, li_c, k_c, kb
    node = node.reshape(-1).contiguous()
    n_exp = n_local * P  # every message of every local owner arrives exactly once
    out = (torch.empty((max(n_exp, 1), 48), dtype=torch.uint8, device=dev),
           torch.empty(max(n_exp, 1), dtype=torch.int32, device=dev), None, None)
    flags = torch.empty(max(n_exp, 1), dtype=torch.uint8, device=dev)
    id_base = rank << 40
    torch.cuda.synchronize(dev)
    setup_s = time.perf_counter() - t_setup
    route_ms = []
    last = {}

    def step():
        r0 = time.perf_counter()
        if dist_ingest:
            # route + addMessages on the received records where they lie (evm_dist_ingest)
            n_r = srv.dd.route(ts_in, owner_in, need_src=False, keep_input=True)
            route_ms.append((time.perf_counter() - r0) * 1e3)
            srv.new_store()
            srv.dd.ingest(srv.store, id_base, flags)
        else:
            # route + take (48-B rows rebuilt) + evm_server_ingest
            t_r, o_r = srv.route(ts_in, owner_in, out=out)
            route_ms.append((time.perf_counter() - r0) * 1e3)
            n_r = t_r.shape[0]
            srv.new_store()
            srv.store.ingest(t_r, o_r, id_base, flags=flags)
        diff, off, sel = srv.select(client, node)
        root, present = srv.roots()
        last.update(n_r=n_r, diff=diff, off=off, sel=sel, root=root, present=present)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    # per-kernel breakdown (untimed): the dominant kernel
    eng.prof_enable(True)
    eng.prof_reset()
    step()
    torch.cuda.synchronize(dev)
    prof = eng.prof_report()
    alg_all = dict(DIST_ALG, **SERVER_ALG)
    dom = dominant(prof, alg_all)
    eng.prof_only(dom)
    eng.prof_reset()
    route_ms.clear()
    comm.barrier()
    torch.cuda.synchronize(dev)
    c0 = eng.stats()
    t0 = time.perf_counter()
    for k in range(steps):
        step()
        if verbose:
            print("rank %d step %d" % (rank, k), file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    c1 = eng.stats()
    allocs = {kk: c1[kk] - c0[kk] for kk in ("workspace_regrows", "scratch_pool_allocs", "block_allocs")}
    prof_dom = eng.prof_report()
    eng.prof_enable(False)
    eng.prof_only(None)
    elapsed = comm.max(t1 - t0)
    route_avg = comm.max(sum(route_ms) / max(1, len(route_ms)))

    # ---- self-check: `sample` owners re-derived unsharded on this GPU
    n_r = last["n_r"]
    if dist_ingest:
        srv.take_routed(out=out)  # the last round's rows (ids = receive index), for the byte compare
    k = min(sample, n_local)
    ok = n_r == n_exp
    detail = {"received": int(n_r), "expected": int(n_exp)}
    if k:
        li = torch.unique(torch.linspace(0, n_local - 1, k, device=dev).round().to(torch.int64))
        k = li.numel()
        glob = srv.owners_here[li]
        ts_s, own_s, _ = gen.owners(seed, O, P, world, glob, dev)
        ref = eng.store_new(k)
        f_s, _ = ref.ingest(ts_s, own_s, 0)
        t_c, li_c, k_c = gen.owners(seed, O, P, 1, glob, dev)
        kb = k_c.bool()
        client_s = eng.merkle_insert(eng.tree_new(k), t_c[kb].contiguous(), li_c[kb].contiguous())
        node_s = t_c.view(k, P, 48)[:, 0, 30:46].reshape(-1).contiguous()
        diff_s, off_s, sel_s = ref.select(client_s, node_s)
        r_s, p_s = ref.tree().roots()
        # inserted counts per owner
        ins_big = torch.bincount(out[1][:n_r][(flags[:n_r] & L.MSG_INS) != 0].to(torch.int64),
                                 minlength=n_local)[li]
        ins_ref = torch.bincount(own_s[(f_s & L.MSG_INS) != 0].to(torch.int64), minlength=k)
        ok_ins = bool(torch.equal(ins_big, ins_ref))
        # roots as all-gathered (any rank's view of these owners)
        g64 = glob.to(torch.int64)
        ok_root = (np.array_equal(last["root"][g64].cpu().numpy(), r_s) and
                   np.array_equal(last["present"][g64].cpu().numpy(), p_s))
        ok_diff = bool(torch.equal(last["diff"][li], diff_s))
        # selected rows, byte for byte, in order
        off, sel = last["off"], last["sel"]
        cnt_big = off[li + 1] - off[li]
        cnt_ref = off_s[1:] - off_s[:-1]
        ok_sel = bool(torch.equal(cnt_big, cnt_ref))
        n_sel = int(cnt_ref.sum().item())
        if ok_sel and n_sel:
            starts = torch.repeat_interleave(off[li], cnt_big)
            within = torch.arange(n_sel, device=dev) - torch.repeat_interleave(torch.cumsum(cnt_big, 0) - cnt_big,
                                                                               cnt_big)
            rows_big = out[0][(sel[starts + within] - id_base)]
            rows_ref = ts_s[sel_s]
            ok_sel = bool(torch.equal(rows_big[:, :46], rows_ref[:, :46]))
        ok = ok and ok_ins and ok_root and ok_diff and ok_sel
        detail.update(sample_owners=k, inserted=ok_ins, roots=ok_root, diffs=ok_diff, selections=ok_sel,
                      selected_rows=n_sel, inserted_rows=int(ins_ref.sum().item()))
        ref.free()
        client_s.free()
    parity = comm.min(1 if ok else 0) == 1
    # ---- the ingest kernel of the rows that crossed a link: at N > 1,
    # (N - 1) / N of every rank's rows arrive as 24-B records and K5 reads
    # them where they landed (k_svo_a<..., SRC_WIRE>); at world 1 the keep-input
    # route never moves a row, so these steps route WITHOUT keep-input (every
    # row a record) to time that kernel at the leg's full size
    src_wire = None
    if dist_ingest and src_wire_steps:
        wname = "(k_svo_a<1024, SRC_WIRE>)"
        ws_ms = []
        eng.prof_enable(True)
        eng.prof_only(wname)
        eng.prof_reset()
        comm.barrier()
        for _ in range(src_wire_steps + 1):
            torch.cuda.synchronize(dev)
            w0 = time.perf_counter()
            srv.dd.route(ts_in, owner_in, need_src=False, keep_input=False)
            srv.new_store()
            srv.dd.ingest(srv.store, id_base, flags)
            torch.cuda.synchronize(dev)
            ws_ms.append((time.perf_counter() - w0) * 1e3)
            if len(ws_ms) == 1:
                eng.prof_reset()  # (the first is a warm-up)
        pw = eng.prof_report()
        eng.prof_enable(False)
        eng.prof_only(None)
        if wname in pw:
            w_tot, w_n = pw[wname]
            w_avg = w_tot / w_n / 1e3
            per_msg, per_leaf = SERVER_ALG[wname]
            w_alg = per_msg * n_r + per_leaf * srv.store.tree().n_leaves
            src_wire = {"kernel": wname, "kernel_ms_avg": w_avg * 1e3, "alg_bytes_per_launch": w_alg,
                        "frac": w_alg / w_avg / HBM_PEAK, "rows": int(n_r),
                        "route_ingest_ms_per_step": sum(ws_ms[1:]) / max(1, len(ws_ms) - 1),
                        "traffic": traffic_of(wname, "config4"),
                        "note": "route without EVM_ROUTE_KEEP_INPUT: every row a 24-B record, as (N-1)/N of the "
                                "rows are at N GPUs; K5 reads them in place"}
    n = owners_per_gpu * P  # per GPU (weak scaling)
    ms = elapsed / steps * 1e3
    tot_ms, launches = prof_dom[dom]
    avg_s = tot_ms / launches / 1e3
    if dom in DIST_ALG:
        alg = DIST_ALG[dom] * n_r
    else:
        per_msg, per_leaf = SERVER_ALG[dom]
        alg = per_msg * n_r + per_leaf * srv.store.tree().n_leaves
    remote = n * (world - 1) / world
    res = {
        "value": world * n * steps / elapsed, "ms_per_step": ms, "steps": steps, "warmup": warmup,
        "config": {"workload": "config4: sync server (index.ts:138-202 addMessages + getMessages), %d owners x %d "
                               "msgs = %d msgs over %d GPU(s) (%d owners x %d msgs per GPU, weak scaling: 1B msgs over "
                               "1M owners at 8 GPUs), owners sharded by murmur3(userId) mod %d on the device "
                               "(evm_dist_directory), every rank's slice holds one request per owner of the job, "
                               "routed over %s (evm_dist_route, 24-B packed records), %s, "
                               "getMessages vs each owner's client tree (~90 %% known), roots all-gathered"
                               % (O, P, O * P, world, owners_per_gpu, P, world, dd.transport,
                                  "ingest of the received records in place into an empty store (evm_dist_ingest)"
                                  if dist_ingest else "take (rows rebuilt) + ingest into an empty store"),
                   "messages_per_gpu": n, "owners_total": O, "owners_per_gpu": owners_per_gpu,
                   "owners_this_rank": n_local, "parallelism": "owner-sharded (murmur3 mod %d), %s" % (world, dd.transport)},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": alg / avg_s / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": alg / avg_s / HBM_PEAK, "traffic": traffic_of(dom, "config4"),
                     "kernel_ms_avg": avg_s * 1e3, "alg_bytes_per_launch": alg,
                     "kernel_share_of_step": tot_ms / (ms * steps)},
        "pipeline": {"alg_bytes_per_msg": SERVER_PIPELINE_BYTES,
                     "pipeline_hbm_frac": SERVER_PIPELINE_BYTES * n / (elapsed / steps) / HBM_PEAK,
                     "kernels_ms_per_step": {kk: v[0] for kk, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:16]},
                     "all_kernels_ms_per_step": sum(v[0] for v in prof.values()),
                     "allocs_in_timed_steps": allocs},
        "route": {"ms_per_step": route_avg, "bytes_per_msg": ROUTE_BYTES, "remote_bytes_per_gpu": remote * ROUTE_BYTES,
                  "xgmi_frac": (remote * ROUTE_BYTES / (route_avg / 1e3) / ((world - 1) * XGMI_LINK))
                  if world > 1 else None},
        "parity_checked": parity, "self_check_rank%d" % rank: detail, "setup_s": setup_s, "src_wire": src_wire,
    }
    srv.close()
    client.free()
    del ts_in, owner_in, out, flags
    return res


def config4_loopback(a, world, device=0):
    """config4_rank on `world` loopback ranks: threads of this process on one
    GPU, evm_dist over an in-process hub (device-to-device copies instead of
    RCCL) -- the multi-rank partitions, exchange, directory and gathers run
    exactly as at N GPUs, at 1/world of the speed.  A correctness rehearsal,
    never a scaling number."""
    from evolu_amd.engine import run_loopback

    comm = ThreadComm(world)

    def fn(r, eng, dd):
        try:
            return config4_rank(eng, dd, comm.bind(r), a.c4_owners, a.c4_per_owner, a.steps, a.warmup, a.c4_sample,
                                dist_ingest=not getattr(a, "c4_take", False))
        except BaseException:
            comm.bar.abort()  # the other ranks may wait in a bench barrier, not a collective
            raise

    results = run_loopback(world, fn, device)
    res = results[0]
    for r in range(1, world):
        res.update({k: v for k, v in results[r].items() if k.startswith("self_check_rank")})
    out = {"metric": METRIC + " [loopback rehearsal, not a multi-GPU measurement]", "value": res.pop("value"),
           "unit": "msgs/s", "n_gpus": 1, "loopback_ranks": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": res.pop("ms_per_step"), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u64", "data": "synthetic (device generator, SURVEY 8(d) config 4)", "cpu_baseline": None}
    res.pop("steps"), res.pop("warmup")
    out.update(res)
    return out


C5_SEED = 0xE7010005  # seed = 0xE7010000 + config number


def c5_nodes(seed, glob):
    """Requester nodeId of every local slot (global owner ids, -1 unused):
    rank 0's node q = 0 of the owner in the config-5 generator (evm_synth.hip
    c5_message: H(seed, 2, owner, 0)), lower-case hex -- the same on every
    rank, so a split owner's shares are filtered alike (NOT LIKE is
    case-insensitive, index.ts:98-102).  -> uint8 [n, 16]."""
    import numpy as np

    from evolu_amd import synth

    g = np.maximum(np.asarray(glob, dtype=np.int64), 0).astype(np.uint64)
    return synth._hex16(synth._H(seed, 2, g, np.zeros_like(g))).astype(np.uint8)


def _leaves_equal(ta, a, tb, b, count=1):
    """Owners [a, a+count) of trees ta and [b, b+count) of tb hold identical leaf lists."""
    import torch

    oa, ca, xa = ta.slice_device(a, count)
    ob, cb, xb = tb.slice_device(b, count)
    return bool(torch.equal(oa, ob) and torch.equal(ca, cb) and torch.equal(xa, xb))


def config5_rank(eng, dd, comm, owners_per_gpu=125_000, n_per_gpu=125_000_000, steps=5, warmup=1, sample=200,
                 share=0.1, seed=C5_SEED, verbose=False, dist_ingest=True):
    """BASELINE config 5 on the server at N GPUs, through the C ABI the Node
    caller uses (evolu_amd/sharded.py ShardedServer):
    owners_per_gpu x world owners with Zipf(1.2) sizes, n_per_gpu messages
    per rank's slice (1B over 1M owners at 8 GPUs, weak scaling): equal-millis
    bursts on a 1-second grid, 1 % upper-case nodes, 10 % exact redeliveries,
    shuffled (evm_synth.hip evs_config5_shape, seed + rank per slice; the job's
    batch = the slices in rank order).

    Setup (untimed): the directory murmur3(userId) mod world
    (evm_dist_directory); the hot owners -- above `share` of one rank's fair
    share of the job's rows -- found over all ranks (evm_dist_hot_owners) and
    split over every rank by timestamp hash (evm_dist_split); one round routed
    and ingested to learn what each owner's client knows (keep flag, first
    copy); the client trees (a split owner's: every rank's part merged,
    evm_dist_merge_trees).  One step = route (evm_dist_route, 24-B records)
    + addMessages of the received records in place into an empty store
    (evm_dist_ingest; dist_ingest=False: take + evm_server_ingest) + getMessages
    (evm_server_select; split owners: full-tree diffs, each rank's share after
    the bound, shares merged in timestamp order by evm_dist_merge_select) +
    every owner's root all-gathered (evm_dist_gather_roots XORs the split
    owners' partial roots).

    Self-check (after the timed steps): every rank regenerates every slice,
    keeps the rows of a sample of its cold owners and of EVERY split owner, in
    global batch order, and recomputes them unsharded on one store of this
    GPU: inserted counts (a split owner's summed over ranks), roots (as
    all-gathered), diffs, the split owners' full trees, and the selected rows
    byte for byte (a split owner's merged list: each rank checks the entries
    that came from its own rows, every rank the count) -> parity_checked,
    agreed over the ranks."""
    import numpy as np
    import torch

    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.sharded import ShardedServer

    rank, world = dd.rank, dd.world
    dev = torch.device("cuda", eng.device)
    O = owners_per_gpu * world
    gen = synth.DeviceSynth()
    t_setup = time.perf_counter()
    ids = gen.owner_ids(seed, O, dev)
    srv = ShardedServer(eng, dd, ids, 21)
    del ids
    ts_in, owner_in, keep_in = synth.device_config5_shape(gen, seed + rank, O, n_per_gpu, dev)
    hot = srv.split_hot(owner_in, share=share)
    nh, base = int(hot.size), srv.hot_base
    n_local = srv.n_local
    # what each owner's client knows: its kept messages, each once (the first copy inserted)
    n_r = dd.route(ts_in, owner_in, aux=keep_in.to(torch.int32))
    t_r, o_r, k_r, _, _ = dd.take(src=False)
    first = eng.store_new(n_local)
    ins, _ = first.ingest(t_r, o_r, 0)
    first.free()
    known = (k_r != 0) & ((ins[:n_r] & L.MSG_INS) != 0)
    partial = eng.merkle_insert(eng.tree_new(n_local), t_r[known].contiguous(), o_r[known].contiguous())
    del t_r, o_r, k_r, ins, known, keep_in
    client = srv.client_trees(partial)
    if client is not partial:
        partial.free()
    glob = srv.local_owners().cpu().numpy()
    node = torch.from_numpy(c5_nodes(seed, glob).reshape(-1).copy()).to(dev)
    out = (torch.empty((max(n_r, 1), 48), dtype=torch.uint8, device=dev),
           torch.empty(max(n_r, 1), dtype=torch.int32, device=dev), None, None)
    flags = torch.empty(max(n_r, 1), dtype=torch.uint8, device=dev)
    id_base = rank << 40
    torch.cuda.synchronize(dev)
    setup_s = time.perf_counter() - t_setup
    route_ms = []
    last = {}

    def step():
        r0 = time.perf_counter()
        if dist_ingest:
            n_s = srv.dd.route(ts_in, owner_in, need_src=False, keep_input=True)
            route_ms.append((time.perf_counter() - r0) * 1e3)
            srv.new_store()
            srv.dd.ingest(srv.store, id_base, flags)
        else:
            t, o = srv.route(ts_in, owner_in, out=out)
            n_s = t.shape[0]
            route_ms.append((time.perf_counter() - r0) * 1e3)
            srv.new_store()
            srv.store.ingest(t, o, id_base, flags=flags)
        sel = srv.select(client, node)
        if nh:
            diff, (off, sid), (hoff, hid) = sel
        else:
            (diff, off, sid), hoff, hid = sel, None, None
        root, present = srv.roots()
        last.update(n=n_s, diff=diff, off=off, sid=sid, hoff=hoff, hid=hid, root=root, present=present)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.prof_enable(True)
    eng.prof_reset()
    step()
    torch.cuda.synchronize(dev)
    prof = eng.prof_report()
    alg_all = dict(DIST_ALG, **SERVER_ALG)
    dom = dominant(prof, alg_all)
    eng.prof_only(dom)
    eng.prof_reset()
    route_ms.clear()
    comm.barrier()
    torch.cuda.synchronize(dev)
    c0 = eng.stats()
    t0 = time.perf_counter()
    for k in range(steps):
        step()
        if verbose:
            print("rank %d config5 step %d" % (rank, k), file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    c1 = eng.stats()
    allocs = {kk: c1[kk] - c0[kk] for kk in ("workspace_regrows", "scratch_pool_allocs", "block_allocs")}
    prof_dom = eng.prof_report()
    eng.prof_enable(False)
    eng.prof_only(None)
    elapsed = comm.max(t1 - t0)
    route_avg = comm.max(sum(route_ms) / max(1, len(route_ms)))
    n_recv_max = int(comm.max(float(last["n"])))

    # ---- self-check: sampled cold owners + every split owner, unsharded on this GPU
    t_chk = time.perf_counter()
    n = last["n"]
    if dist_ingest:
        srv.take_routed(out=out)  # the last round's rows (ids = receive index), for the byte compare
    cold = np.flatnonzero(glob[:base] >= 0)
    pick = cold[np.unique(np.linspace(0, len(cold) - 1, min(sample, len(cold))).round().astype(np.int64))] \
        if len(cold) else np.zeros(0, dtype=np.int64)
    chk_local = np.concatenate([pick, base + np.arange(nh)]).astype(np.int64)
    chk_glob = glob[chk_local]
    order = np.argsort(chk_glob, kind="stable")
    k = len(order)
    loc_sorted = chk_local[order]  # local id of ref owner q (ref owners = the checked globals, sorted)
    g_sorted = torch.from_numpy(chk_glob[order].astype(np.int32)).to(dev)
    rows, own, kp = [], [], []
    for s_ in range(world):  # the job's batch: the slices in rank order
        t_s, o_s, k_s = synth.device_config5_shape(gen, seed + s_, O, n_per_gpu, dev)
        m = torch.isin(o_s, g_sorted)
        rows.append(t_s[m])
        own.append(o_s[m])
        kp.append(k_s[m])
        del t_s, o_s, k_s, m
    rows, own, kp = torch.cat(rows), torch.cat(own), torch.cat(kp)
    j = torch.searchsorted(g_sorted, own).to(torch.int32).contiguous()
    ref = eng.store_new(max(k, 1))
    f_ref, st_ref = ref.ingest(rows, j, 0)
    known = (kp != 0) & ((f_ref & L.MSG_INS) != 0)
    client_ref = eng.merkle_insert(eng.tree_new(max(k, 1)), rows[known].contiguous(), j[known].contiguous())
    node_ref = node.view(-1, 16)[torch.from_numpy(loc_sorted).to(dev)].reshape(-1).contiguous()
    diff_ref, off_ref, sel_ref = ref.select(client_ref, node_ref)
    r_ref, p_ref = ref.tree().roots()
    ins_ref = torch.bincount(j[(f_ref & L.MSG_INS) != 0].to(torch.int64), minlength=max(k, 1)).cpu().numpy()
    ins_big = torch.bincount(out[1][:n][(flags[:n] & L.MSG_INS) != 0].to(torch.int64),
                             minlength=n_local).cpu().numpy()
    ins_hot = comm.sum_vec(ins_big[base:base + nh])  # (collective) a split owner's inserts over every rank
    ins_big = ins_big.copy()
    ins_big[base:base + nh] = ins_hot
    ok_ins = bool(st_ref == 0 and np.array_equal(ins_big[loc_sorted], ins_ref[:k]))
    g64 = torch.from_numpy(chk_glob[order].astype(np.int64)).to(dev)
    ok_root = bool(np.array_equal(last["root"][g64].cpu().numpy(), r_ref[:k]) and
                   np.array_equal(last["present"][g64].cpu().numpy(), p_ref[:k]))
    ok_diff = bool(torch.equal(last["diff"][torch.from_numpy(loc_sorted).to(dev)], diff_ref[:k]))
    # the split owners' full trees (collective), leaf for leaf
    full = dd.merge_trees(srv.store.tree(), base, nh) if nh else None
    ok_tree = all(_leaves_equal(full, h, ref.tree(), int(np.searchsorted(chk_glob[order], hot[h])))
                  for h in range(nh))
    if full is not None:
        full.free()
    # selections: a cold owner's rows are all here; a split owner's merged
    # list holds every rank's rows -- this rank checks the ones it holds
    off_ref_np = off_ref.cpu().numpy()
    ok_sel, n_sel = True, 0
    mask40 = (1 << 40) - 1
    for q in range(k):
        lq = int(loc_sorted[q])
        want = sel_ref[int(off_ref_np[q]):int(off_ref_np[q + 1])]
        n_sel += int(want.numel())
        if lq < base:
            a_, b_ = int(last["off"][lq]), int(last["off"][lq + 1])
            got = last["sid"][a_:b_]
            if got.numel() != want.numel():
                ok_sel = False
                continue
            if got.numel() and not torch.equal(out[0][got - id_base][:, :46], rows[want][:, :46]):
                ok_sel = False
        else:
            h = lq - base
            a_, b_ = int(last["hoff"][h]), int(last["hoff"][h + 1])
            got = last["hid"][a_:b_]
            if got.numel() != want.numel():
                ok_sel = False
                continue
            mine = (got >> 40) == rank
            if bool(mine.any()) and not torch.equal(out[0][got[mine] & mask40][:, :46], rows[want[mine]][:, :46]):
                ok_sel = False
    ok = ok_ins and ok_root and ok_diff and ok_tree and ok_sel
    detail = {"sample_owners": int(len(pick)), "split_owners_checked": nh, "rows_checked": int(rows.shape[0]),
              "inserted": ok_ins, "roots": ok_root, "diffs": ok_diff, "split_trees": ok_tree, "selections": ok_sel,
              "selected_rows": n_sel, "check_s": time.perf_counter() - t_chk}
    ref.free()
    client_ref.free()
    del rows, own, kp, j, f_ref, known
    parity = comm.min(1 if ok else 0) == 1
    ms = elapsed / steps * 1e3
    tot_ms, launches = prof_dom[dom]
    avg_s = tot_ms / launches / 1e3
    if dom in DIST_ALG:
        alg = DIST_ALG[dom] * n
    else:
        per_msg, per_leaf = SERVER_ALG[dom]
        alg = per_msg * n + per_leaf * srv.store.tree().n_leaves
    res = {
        "value": world * n_per_gpu * steps / elapsed, "ms_per_step": ms, "steps": steps, "warmup": warmup,
        "config": {"workload": "config5: sync server (index.ts:138-202 addMessages + getMessages), %d msgs over %d "
                               "owners (%d msgs / %d owners per GPU, weak scaling: 1B over 1M at 8 GPUs), owner sizes "
                               "Zipf(1.2), equal-millis bursts, 1 %% upper-case nodes, 10 %% exact redeliveries, "
                               "shuffled; owners by murmur3(userId) mod %d (evm_dist_directory), %d hot owners "
                               "(> %.2f of a rank's fair share) split over every rank by timestamp hash "
                               "(evm_dist_hot_owners/split), routed over %s (evm_dist_route), getMessages with "
                               "full-tree diffs and merged selections (evm_dist_merge_trees/merge_select), roots "
                               "all-gathered" % (n_per_gpu * world, O, n_per_gpu, owners_per_gpu, world, nh, share,
                                                 dd.transport),
                   "messages_per_gpu": n_per_gpu, "owners_total": O, "owners_per_gpu": owners_per_gpu,
                   "split_owners": [int(x) for x in hot[:16]], "n_split_owners": nh,
                   "rows_received_this_rank": int(n), "rows_received_max_rank": n_recv_max,
                   "parallelism": "owner-sharded (murmur3 mod %d) + hot owners split by timestamp hash, %s"
                                  % (world, dd.transport)},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": alg / avg_s / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": alg / avg_s / HBM_PEAK, "traffic": traffic_of(dom, "config5n"),
                     "kernel_ms_avg": avg_s * 1e3, "alg_bytes_per_launch": alg,
                     "kernel_share_of_step": tot_ms / (ms * steps)},
        "pipeline": {"alg_bytes_per_msg": SERVER_PIPELINE_BYTES,
                     "pipeline_hbm_frac": SERVER_PIPELINE_BYTES * n_per_gpu / (elapsed / steps) / HBM_PEAK,
                     "kernels_ms_per_step": {kk: v[0] for kk, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:16]},
                     "all_kernels_ms_per_step": sum(v[0] for v in prof.values()), "allocs_in_timed_steps": allocs},
        "route": {"ms_per_step": route_avg, "bytes_per_msg": ROUTE_BYTES,
                  "imbalance_max_over_mean": n_recv_max / max(1.0, n_per_gpu)},
        "parity_checked": parity, "self_check_rank%d" % rank: detail, "setup_s": setup_s,
    }
    srv.close()
    client.free()
    del ts_in, owner_in, out, flags
    return res


def config5_loopback(a, world, device=0):
    """config5_rank on `world` loopback ranks sharing one GPU (evm_dist_hub):
    the directory, hot-owner split, exchange, merged selections and gathers
    run exactly as at N GPUs -- a correctness rehearsal, never a scaling number."""
    from evolu_amd.engine import run_loopback

    comm = ThreadComm(world)

    def fn(r, eng, dd):
        try:
            return config5_rank(eng, dd, comm.bind(r), a.c5_owners, a.c5_messages, a.steps, a.warmup, a.c5_sample,
                                a.c5_share, dist_ingest=not getattr(a, "c4_take", False))
        except BaseException:
            comm.bar.abort()
            raise

    results = run_loopback(world, fn, device)
    res = results[0]
    for r in range(1, world):
        res.update({k: v for k, v in results[r].items() if k.startswith("self_check_rank")})
    out = {"metric": METRIC + " [loopback rehearsal, not a multi-GPU measurement]", "value": res.pop("value"),
           "unit": "msgs/s", "n_gpus": 1, "loopback_ranks": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": res.pop("ms_per_step"), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u64", "data": "synthetic (device generator evs_config5_shape, SURVEY 8(d) config 5)",
           "cpu_baseline": None}
    res.pop("steps"), res.pop("warmup")
    out.update(res)
    return out


def client_split_rank(eng, dd, comm, n_per_gpu=10_000_000, cells_per_gpu=1000, steps=5, warmup=1, seed=5):
    """BASELINE config 5 on the client at N GPUs: ONE owner's applyMessages
    batch (applyMessages.ts:26-131) of world x n_per_gpu messages over
    world x cells_per_gpu cells with config 5's adversarial structure
    (synth.client_adversarial per slice: equal-millis bursts, stale and exact
    redeliveries, upper-case nodes), each rank holding its slice, split over
    the ranks by cell through the C ABI (sharded.split_apply: the global PK
    check by timestamp hash, every cell's rows on its rank in batch order,
    flags back to the source rows, global winners, the partial trees merged).
    Self-check: the whole batch gathered and applied unsharded on this GPU --
    this slice's flags, every winner and the tree, leaf for leaf."""
    import numpy as np
    import torch

    from evolu_amd import _lib as L
    from evolu_amd import synth
    from evolu_amd.sharded import split_apply

    rank, world = dd.rank, dd.world
    dev = torch.device("cuda", eng.device)
    C = cells_per_gpu * world
    t_setup = time.perf_counter()
    ts_np, cell_np = synth.client_adversarial(n_per_gpu, C, seed_config=seed + 1000 * rank)
    ts, cell = eng.dev(ts_np), eng.dev(cell_np.view(np.int32))
    del ts_np, cell_np
    empty = eng.tree_new(1)
    setup_s = time.perf_counter() - t_setup
    last = {}

    def step(keep=False):
        flags, winner, tree, st = split_apply(eng, dd, ts, cell, C, tree_in=empty)
        if st != L.EVM_OK:
            raise RuntimeError("split_apply status %d" % st)
        if keep:
            last.update(flags=flags, winner=winner, tree=tree)
        else:
            tree.free()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.prof_enable(True)
    eng.prof_reset()
    step()
    torch.cuda.synchronize(dev)
    prof = eng.prof_report()
    eng.prof_enable(False)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    elapsed = comm.max(time.perf_counter() - t0)
    step(keep=True)
    # ---- self-check: the whole batch, unsharded
    all_ts = torch.cat(comm.all_gather(ts))
    all_cell = torch.cat(comm.all_gather(cell))
    f_ref, w_ref, t_ref, st_ref = eng.apply_batch(eng.tree_new(1), all_ts, all_cell, C, raise_on_error=False)
    ok_st = st_ref == L.EVM_OK
    ok_flags = ok_st and bool(torch.equal(last["flags"], f_ref[rank * n_per_gpu:(rank + 1) * n_per_gpu]))
    ok_win = ok_st and bool(torch.equal(last["winner"], w_ref.to(torch.int64)))
    ok_tree = ok_st and _leaves_equal(last["tree"], 0, t_ref, 0)
    last["tree"].free()
    if t_ref is not None:
        t_ref.free()
    ok = ok_flags and ok_win and ok_tree
    parity = comm.min(1 if ok else 0) == 1
    ms = elapsed / steps * 1e3
    return {"config": {"workload": "config5-C: applyMessages of ONE owner's batch of %d msgs (%d per GPU) over %d "
                                   "cells, equal-millis bursts + stale/exact redeliveries + upper-case nodes "
                                   "(synth.client_adversarial per slice), split over %d rank(s) by cell through "
                                   "evm_dist_* (global PK check by timestamp hash, flags returned to the source rows, "
                                   "winners and tree merged)" % (n_per_gpu * world, n_per_gpu, C, world),
                       "messages_per_gpu": n_per_gpu, "cells_total": C,
                       "parallelism": "one owner split by cell over %d rank(s), %s" % (world, dd.transport)},
            "value": world * n_per_gpu * steps / elapsed, "unit": "msgs/s", "ms_per_step": ms, "steps": steps,
            "setup_s": setup_s,
            "kernels_ms_per_step": {kk: v[0] for kk, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:12]},
            "parity_checked": parity,
            "self_check_rank%d" % rank: {"flags": ok_flags, "winners": ok_win, "tree": ok_tree,
                                         "batch_rows": int(all_ts.shape[0])}}


def client_split_loopback(a, world, device=0):
    from evolu_amd.engine import run_loopback

    comm = ThreadComm(world)

    def fn(r, eng, dd):
        try:
            return client_split_rank(eng, dd, comm.bind(r), a.c5c_messages, a.c5c_cells, a.steps, a.warmup)
        except BaseException:
            comm.bar.abort()
            raise

    results = run_loopback(world, fn, device)
    res = results[0]
    for r in range(1, world):
        res.update({k: v for k, v in results[r].items() if k.startswith("self_check_rank")})
    return dict(res, metric=METRIC + " [client config 5 split, loopback rehearsal]", loopback_ranks=world)


def adversarial_leg(eng, a):
    """BASELINE config 5 on the client side (synth.client_adversarial): one
    owner, 10M messages over 1,000 cells from 64 nodes, equal-millis bursts
    (ties broken by counter and node), 10 % redeliveries (half stale: XOR
    toggles; the rest exact copies of the cell max: no-ops decided by node
    ranks inside the walk), ~1 % upper-case nodes.  Pipelined exactly like
    the headline; tc_redos must stay 0 (no batch falls back to the exact walk
    path)."""
    import collections

    import torch

    from evolu_amd import synth

    n, C = a.messages, a.cells
    ts_np, cell_np = synth.client_adversarial(n, C, 64, seed_config=5)
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    del ts_np
    empty = eng.tree_new(1)
    depth = max(1, a.depth)
    outs = [(torch.empty(n, dtype=torch.uint8, device=ts.device), torch.empty(C, dtype=torch.int32, device=ts.device))
            for _ in range(depth)]

    def run(k_steps):
        q = collections.deque()
        for k in range(k_steps):
            if len(q) == depth:
                q.popleft().wait()[2].free()
            q.append(eng.apply_batch_async(empty, ts, cell, C, *outs[k % depth]))
        while q:
            q.popleft().wait()[2].free()

    run(max(a.warmup, 2))
    torch.cuda.synchronize()
    eng.prof_enable(True)
    eng.prof_reset()
    for _ in range(3):
        eng.apply_batch(empty, ts, cell, C, flags=outs[0][0], winner=outs[0][1])[2].free()
    torch.cuda.synchronize()
    prof = eng.prof_report()
    dom = dominant(prof, ALG_BYTES_PER_MSG, SIDE_KERNELS)
    eng.prof_only(dom)
    eng.prof_reset()
    s0 = eng.stats()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s1 = eng.stats()
    prof_dom = eng.prof_report()
    eng.prof_enable(False)
    eng.prof_only(None)
    f = outs[0][0].cpu().numpy()
    tot_ms, launches = prof_dom[dom]
    avg_s = tot_ms / launches / 1e3
    alg = ALG_BYTES_PER_MSG[dom] * n
    ms = dt / a.steps * 1e3
    return {"workload": "client config 5 (synth.client_adversarial): 1 owner, %d msgs, %d cells, 64 nodes, equal-millis "
                        "bursts, 10 %% redeliveries, ~1 %% upper-case nodes; %d batches in flight" % (n, C, depth),
            "value": n / ms * 1e3, "unit": "msgs/s", "ms_per_step": ms, "steps": a.steps,
            "tc_batches": s1["tc_batches"] - s0["tc_batches"], "tc_redos": s1["tc_redos"] - s0["tc_redos"],
            "no_op_rows": int((f == 0).sum()), "xor_only_rows": int((f == 2).sum()), "upsert_rows": int((f == 3).sum()),
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": alg / avg_s / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": alg / avg_s / HBM_PEAK, "kernel_ms_avg": avg_s * 1e3,
                         "alg_bytes_per_launch": alg, "traffic": traffic_of(dom, "client_adversarial")},
            "pipeline_hbm_frac": 120 * n / (dt / a.steps) / HBM_PEAK,
            "kernels_ms_per_step": {k: v[0] / 3 for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:12]}}


def config5_shape_leg(eng, a, owners=100_000, n=100_000_000, seed=0xE7010005, sample=200):
    """BASELINE config 5 shape on the server: 100M messages over 100k owners,
    owner sizes Zipf(1.2) (the top owner ~18 %), equal-millis bursts on a
    1-second grid, 1 % upper-case nodes, 10 % exact redeliveries, shuffled
    (no request runs) -- generated on the device (evs_config5_shape).  One
    step = new store + addMessages (INSERT OR IGNORE) + getMessages against
    client trees holding ~90 % + every owner's root.  Self-check: `sample`
    of the smaller owners recomputed from all their rows alone by the global
    sort path (inserts and tree JSON; tests pin both paths to the oracle)."""
    import numpy as np
    import torch

    from evolu_amd import synth

    dev = torch.device("cuda", eng.device)
    gen = synth.DeviceSynth()
    t0 = time.perf_counter()
    ts, owner, keep = synth.device_config5_shape(gen, seed, owners, n, dev)
    gen_s = time.perf_counter() - t0
    first = eng.store_new(owners)
    ins, _ = first.ingest(ts, owner, 0)
    known = (keep != 0) & ((ins[:n] & 0x04) != 0)  # the client holds each known message once
    first.free()
    client = eng.merkle_insert(eng.tree_new(owners), ts[known].contiguous(), owner[known].contiguous())
    del known
    node = torch.from_numpy(np.frombuffer(b"0123456789abcdef" * owners, dtype=np.uint8).copy()).to(dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    keep_store = [None]

    def step(keep_it=False):
        store = eng.store_new(owners)
        store.ingest(ts, owner, 0, flags=flags)
        store.select(client, node)
        store.tree().roots()
        if keep_it:
            keep_store[0] = store
        else:
            store.free()

    for _ in range(max(1, a.warmup)):
        step()
    torch.cuda.synchronize()
    eng.prof_enable(True)
    eng.prof_reset()
    step()
    torch.cuda.synchronize()
    prof = eng.prof_report()
    dom = dominant(prof, SERVER_ALG)
    eng.prof_only(dom)
    eng.prof_reset()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof_dom = eng.prof_report()
    eng.prof_enable(False)
    eng.prof_only(None)
    ms = dt / a.steps * 1e3
    # self-check on the smaller owners (every row of each)
    step(keep_it=True)
    store = keep_store[0]
    counts = torch.bincount(owner.to(torch.int64), minlength=owners).cpu().numpy()
    rng = np.random.default_rng(seed & 0xFFFF)
    pool = np.flatnonzero((counts > 0) & (counts < 20_000))
    pick = np.sort(rng.choice(pool, size=min(sample, len(pool)), replace=False))
    sel = torch.isin(owner, torch.from_numpy(pick.astype(np.int32)).to(dev))
    rows = ts[sel].cpu().numpy()
    own = owner[sel].cpu().numpy().astype(np.uint32)
    fl = flags[sel].cpu().numpy()
    local = np.searchsorted(pick, own).astype(np.uint32)
    # the same owners' rows alone through the other ingest algorithm (the
    # global sort path, EVM_OPT_SERVER_PATH 2) on a fresh store
    eng.set_option(2, 2)
    try:
        ref = eng.store_new(len(pick))
        f_ref, st = ref.ingest(eng.dev(rows), eng.dev(local), 0)
        f_ref = f_ref.cpu().numpy()
    finally:
        eng.set_option(2, 0)
    ok_ins = st == 0 and np.array_equal((fl & 0x04) != 0, (f_ref & 0x04) != 0)
    ok_tree = all(store.tree().to_json(int(g)) == ref.tree().to_json(j) for j, g in enumerate(pick))
    ref.free()
    store.free()
    tot_ms, launches = prof_dom[dom]
    avg_s = tot_ms / launches / 1e3
    per_msg, per_leaf = SERVER_ALG[dom]
    n_leaves = client.n_leaves
    alg = per_msg * n + per_leaf * n_leaves
    return {"workload": "config 5 shape (server): %d msgs over %d owners, Zipf 1.2 (top owner %.1f %%), equal-millis "
                        "bursts on a 1-s grid, 1 %% upper-case nodes, 10 %% exact redeliveries, shuffled; addMessages "
                        "into an empty store + getMessages + roots per step" % (n, owners, 100.0 * counts.max() / n),
            "value": n / ms * 1e3, "unit": "msgs/s", "ms_per_step": ms, "steps": a.steps,
            "data": "synthetic (device generator evs_config5_shape, %.2f s)" % gen_s,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": alg / avg_s / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": alg / avg_s / HBM_PEAK, "kernel_ms_avg": avg_s * 1e3,
                         "alg_bytes_per_launch": alg, "traffic": traffic_of(dom, "config5")},
            "pipeline_hbm_frac": SERVER_PIPELINE_BYTES * n / (dt / a.steps) / HBM_PEAK,
            "kernels_ms_per_step": {k: v[0] for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:14]},
            "parity_checked": bool(ok_ins and ok_tree),
            "self_check": {"owners": int(len(pick)), "rows": int(len(rows)), "inserts": bool(ok_ins),
                           "trees": bool(ok_tree)}}


def config1_leg(eng, a):
    """BASELINE config 1: the todo-schema stream (100k messages, one owner),
    one applyMessages batch from an empty tree, inputs in HBM."""
    import numpy as np
    import torch

    from evolu_amd import synth

    ts_np, cell_np, cells, _ = synth.config1(100_000)
    ts, cell = eng.dev(ts_np), eng.dev(cell_np)
    empty = eng.tree_new(1)
    C = len(cells)
    flags = torch.empty(len(ts_np), dtype=torch.uint8, device=ts.device)
    winner = torch.empty(C, dtype=torch.int32, device=ts.device)

    def step():
        eng.apply_batch(empty, ts, cell, C, flags=flags, winner=winner)[2].free()

    def path_taken(fn):
        s0 = eng.stats()
        fn()
        s1 = eng.stats()
        if s1["small_batches"] > s0["small_batches"]:
            return "small-batch path: 5 kernels, one status read"
        if s1["small_fallbacks"] > s0["small_fallbacks"]:
            return "sort path (the small-batch path handed over)"
        if s1["tc_batches"] > s0["tc_batches"]:
            return "tc streaming path"
        return "sort path: radix sort by cell + segmented scan"

    for _ in range(a.warmup):
        step()
    path = path_taken(step)
    eng.prof_enable(True)
    eng.prof_reset()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    prof = eng.prof_report()
    eng.prof_enable(False)
    steps = max(a.steps, 20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    out = {"workload": "config1: examples/nextjs todo schema (index.tsx:23-34, db.ts:268-300 mutation shapes), "
                       "100000 msgs, 1 owner, %d cells, 3 nodes, send order (evolu_amd/synth.config1)" % C,
           "value": len(ts_np) / ms * 1e3, "unit": "msgs/s", "ms_per_batch": ms, "steps": steps,
           "path": path,
           "kernels_ms_per_batch": {k: v[0] / a.steps for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:10]},
           "cpu_baseline": cpu_baseline(ts_np, cell_np, a.cpu_seconds, "config-1") if a.cpu_seconds > 0 else None}
    # per-batch latency at the sizes a client applies (send.ts:107-111 one
    # mutation's messages; receive.ts:84-87 one sync's): the first k messages
    # of the stream, cells renumbered, one synchronous applyMessages each
    lat = {}
    for k in (100, 1000, 10_000, 100_000):
        k = min(k, len(ts_np))
        used, cid = np.unique(cell_np[:k], return_inverse=True)
        ts_k, cell_k = eng.dev(ts_np[:k]), eng.dev(cid.astype(np.uint32))
        fl = torch.empty(k, dtype=torch.uint8, device=ts.device)
        wn = torch.empty(len(used), dtype=torch.int32, device=ts.device)
        def one():
            eng.apply_batch(empty, ts_k, cell_k, len(used), flags=fl, winner=wn)[2].free()

        def timed():
            for _ in range(3):
                one()
            xs = []
            for _ in range(30):
                t0 = time.perf_counter()
                one()
                xs.append((time.perf_counter() - t0) * 1e3)  # (the call returns after its status read: synchronous)
            xs.sort()
            return xs

        xs = timed()
        lat[str(k)] = {"p50_ms": xs[len(xs) // 2], "p90_ms": xs[int(len(xs) * 0.9)], "cells": int(len(used)),
                       "path": path_taken(one)}
        for name, opt in (("small_path", 4), ("sort_path", 2)):  # the paths auto did not take, for comparison
            eng.set_option(1, opt)
            try:
                xs = timed()
                lat[str(k)][name + "_p50_ms"] = xs[len(xs) // 2]
            finally:
                eng.set_option(1, 0)
    out["latency_per_batch"] = lat
    return out


def reingest(eng, a, ts1, own1, owners, per_owner, request, flags):
    """The server's steady state: a second round of requests (new messages
    of the same owners: another seed's stream) ingested into a store that
    already holds the first round's owners x per_owner rows -- addMessages
    with the stored rows and trees merged (k_svo_b), then getMessages is not
    timed here.  Timed per ingest, the first ingest untimed."""
    import torch

    from evolu_amd import synth

    progress("reingest")
    ts2_np, own2_np, _ = synth.config3(owners, per_owner, seed_config=3 + 7919, request=request)
    ts2, own2 = eng.dev(ts2_np), eng.dev(own2_np)
    del ts2_np, own2_np
    f2 = torch.empty(ts2.shape[0], dtype=torch.uint8, device=ts2.device)
    reps = max(2, min(a.steps, 5))
    ms = []
    prof = None
    for r in range(reps + 1):
        st = eng.store_new(owners)
        st.ingest(ts1, own1, 0, flags=flags)
        if r == reps:
            eng.prof_enable(True)
            eng.prof_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.ingest(ts2, own2, 1 << 40, flags=f2)
        torch.cuda.synchronize()
        if r == reps:
            prof = eng.prof_report()
            eng.prof_enable(False)
        elif r > 0:
            ms.append((time.perf_counter() - t0) * 1e3)
        n_stored = st.n_messages
        st.free()
    n = ts2.shape[0]
    m = sorted(ms)[len(ms) // 2]
    dom = dominant(prof, SERVER_ALG)
    tot_ms, launches = prof[dom]
    # the store growing round after round: rounds 2, 3, 4 of
    # new messages of the same owners into one store holding 1, 2, 3 rounds
    # (rounds 2-4 from the config-4 device generator at world 1: every owner's
    # messages as one request, another seed per round -- seconds of host time
    # saved per round against synth.config3)
    progress("reingest rounds 2-4")
    gen = synth.DeviceSynth()
    rounds = []
    for k in range(3):
        t_d, o_d, _ = gen.source(0xE7040000 + k, owners, per_owner, 1, 0, ts2.device)
        rounds.append((t_d, o_d))
    # (twice: the first pass grows the memory pool to the largest store, as a
    # server's earlier rounds would have -- a timed round that first has to
    # map ~13 GB of new device memory measured the driver, up to 250 ms)
    for rep in range(2):
        st = eng.store_new(owners)
        st.ingest(ts1, own1, 0, flags=flags)
        round_ms = []
        for k, (tsk, owk) in enumerate(rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.ingest(tsk, owk, (k + 1) << 40, flags=f2)
            torch.cuda.synchronize()
            round_ms.append((time.perf_counter() - t0) * 1e3)
        stored_rounds = int(st.n_messages)
        st.free()
    del rounds
    return {"workload": "a second round of %d msgs (%d owners, new timestamps) into a store holding %d rows: "
                        "addMessages with the stored rows and trees merged" % (n, owners, ts1.shape[0]),
            "value": n / m * 1e3, "unit": "msgs/s", "ms_per_ingest_median": m, "ms_per_ingest": [round(x, 3) for x in ms],
            "stored_after": int(n_stored), "dominant_kernel": dom, "dominant_kernel_ms": tot_ms / launches,
            "rounds_2_3_4_ms": [round(x, 3) for x in round_ms],
            "rounds_vs_round_2": [round(x / round_ms[0], 3) for x in round_ms], "stored_after_round_4": stored_rounds,
            "kernels_ms": {k: v[0] for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:10]}}


def e2e_bodies(eng, ts_np, owner_np, client, node16=b"0123456789abcdef", content_bytes=16):
    """The config-3 round as the server receives it: one SyncRequest body per
    request run of ts_np (one owner each), userId = the owner as 21 hex
    chars, nodeId = node16, merkleTree = the owner's client tree (JSON by the
    device emitter), contents = content_bytes per message -- encoded on host
    threads (evm_pb_encode_requests).  -> (arena uint8, offsets uint64[R + 1])."""
    import ctypes as C

    import numpy as np
    import torch

    from evolu_amd import _lib as L

    lib = L.load()
    n = len(ts_np)
    starts = np.flatnonzero(np.r_[True, owner_np[1:] != owner_np[:-1]])
    R = len(starts)
    msg_off = np.r_[starts, n].astype(np.uint64)
    req_owner = owner_np[starts].astype(np.int64)
    users = np.frombuffer("".join("%021x" % o for o in req_owner).encode(), dtype=np.uint8)
    user_off = (np.arange(R + 1, dtype=np.uint64) * 21)
    nodes = np.frombuffer(node16 * R, dtype=np.uint8)
    node_off = np.arange(R + 1, dtype=np.uint64) * len(node16)
    jb, jo = client.to_json_batch(torch.from_numpy(req_owner.astype(np.int32)).to("cuda:%d" % eng.device))
    jb, jo = jb.cpu().numpy(), np.ascontiguousarray(jo.cpu().numpy(), dtype=np.uint64)
    content = np.arange(n * content_bytes // 8 + 1, dtype=np.uint64).view(np.uint8)
    content_off = np.arange(n + 1, dtype=np.uint64) * content_bytes
    p = lambda x: C.c_void_p(x.ctypes.data)  # noqa: E731
    ts_c = np.ascontiguousarray(ts_np)
    args = [R, p(msg_off), p(ts_c), ts_c.shape[1], p(content_off), p(content), p(users), p(user_off), p(nodes),
            p(node_off), p(jb), p(jo)]
    off = np.zeros(R + 1, dtype=np.uint64)
    L.check(lib.evm_pb_encode_requests(*args, None, p(off)), "evm_pb_encode_requests")
    arena = np.empty(int(off[-1]), dtype=np.uint8)
    L.check(lib.evm_pb_encode_requests(*args, p(arena), p(off)), "evm_pb_encode_requests")
    return arena, off


def e2e_leg(eng, ts_np, owner_np, client, device_ms, sample=8):
    """BASELINE config 3 end to end: every owner's SyncRequest body through
    evolu_amd.server.SyncServer (index.ts:204-251: parseBody, addMessages,
    getMessages, SyncResponse.toBinary) into an empty store, bodies in host
    memory to response bodies in host memory: ONE native round
    (evm_sync_round, EVM_SYNC_HOST: the bodies staged to HBM through pinned
    chunks, the round on the device, the responses back the same way), timed
    by part (SyncServer.timing: h2d, decode, users, ingest, trees, select,
    encode, d2h; the Python around it in "other").  Self-check: a
    sample of the requests through the per-request path on a fresh server
    gives the same bytes (the byte compare against the oracle's ServerDb.sync
    is tests/test_gpu_wire.py::test_e2e_bodies_vs_oracle, same generator)."""
    import numpy as np

    from evolu_amd.server import SyncServer

    progress("e2e: bodies")
    t0 = time.perf_counter()
    arena, off = e2e_bodies(eng, ts_np, owner_np, client)
    gen_s = time.perf_counter() - t0
    R = len(off) - 1
    O = int(owner_np.max()) + 1
    # one untimed round first (the context's pinned staging chunks and device
    # blocks are made once per context), then the timed round on a fresh server
    warm = SyncServer(eng, O)
    warm.sync_arena(arena, off)
    warm.close()
    srv = SyncServer(eng, O)
    t0 = time.perf_counter()
    out = srv.sync_arena(arena, off)
    wall = time.perf_counter() - t0
    timing = dict(srv.timing)
    ok = sum(1 for x in out if isinstance(x, memoryview))
    resp_bytes = sum(len(x) for x in out if isinstance(x, memoryview))
    pick = np.linspace(0, R - 1, min(sample, R)).round().astype(np.int64)
    ref = SyncServer(eng, O)
    same = True
    for k in pick:
        body = arena[int(off[k]):int(off[k + 1])].tobytes()
        (r,) = ref.sync_per_request([body])
        same = same and isinstance(r, bytes) and bytes(out[k]) == r
    ref.close()
    srv.close()
    n = len(ts_np)
    dev = e2e_device(eng, arena, off, out, O, pick, device_ms)
    return {"workload": "config 3 end to end: %d SyncRequest bodies (%d owners x %d msgs, %d-B contents, the "
                        "client's tree JSON) in host memory -> one evm_sync_round (pinned H2D, the round on the "
                        "device, pinned D2H) -> %d SyncResponse bodies in host memory, into an empty store"
                        % (R, R, n // max(R, 1), 16, R),
            "ms": wall * 1e3, "msgs_per_s": n / wall, "device_step_ms": device_ms,
            "ratio_to_device_step": wall * 1e3 / device_ms if device_ms else None,
            "ms_by_part": {k: v * 1e3 for k, v in timing.items()},
            "request_bytes": int(off[-1]), "response_bytes": int(resp_bytes), "responses": ok,
            "host_threads": os.environ.get("EVM_HOST_THREADS", "default (<= 16)"),
            "bodies_generation_s": gen_s, "self_check": {"sample": int(len(pick)), "same_bytes": bool(same)},
            "device_resident": dev}


def e2e_device(eng, arena, off, host_out, O, pick, device_ms):
    """The same round with the bodies resident in HBM (SyncServer.sync_device:
    decode, ingest, client-tree parse, selection and response encode all on
    the device; only per-body sizes, userIds and nodeIds come to the host),
    the responses left in HBM.  One untimed round on a fresh server first,
    then the timed round on another; self-check: the sampled responses equal
    the host path's bytes."""
    import numpy as np
    import torch

    from evolu_amd.server import SyncServer

    progress("e2e: device round")
    a_d = torch.from_numpy(arena).to("cuda:%d" % eng.device)
    n = len(off) - 1
    prof = None
    for rep in range(3):
        srv = SyncServer(eng, O)
        if rep == 2:  # (an untimed profiled round: the kernels' share)
            eng.prof_enable(True)
            eng.prof_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = srv.sync_device(a_d, off)
        torch.cuda.synchronize()
        if rep == 2:
            prof = eng.prof_report()
            eng.prof_enable(False)
        else:
            wall = time.perf_counter() - t0
            timing = dict(srv.timing)
        if rep < 2:
            del res
            srv.close()
    ok = sum(1 for r in res.result if r is True)
    same = True
    for k in pick:
        k = int(k)
        if res.result[k] is not True:
            same = False
            continue
        same = same and res.get(k) == bytes(host_out[k])
    resp_bytes = int(res.nbytes)
    srv.close()
    return {"ms": wall * 1e3, "ratio_to_device_step": wall * 1e3 / device_ms if device_ms else None,
            "ms_by_part": {k: v * 1e3 for k, v in timing.items()}, "responses": ok, "response_bytes": resp_bytes,
            "fallback": "device_fallback" in timing,
            "kernels_ms": {k: v[0] for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:16]},
            "self_check": {"sample": int(len(pick)), "same_bytes_as_host_path": bool(same)}}


def server_run(a, rank, world, local, owners, per_owner, zipf, request, cpu=False, leg=False):
    """Config 3 (or the Zipf stream with --zipf) on ONE GPU: server ingest of
    `owners x per_owner` messages into an empty store, then getMessages for
    every owner against a client tree built from the owner's first 90% of
    messages.  With one request per owner per batch (request >= per_owner)
    this is the reference's per-request sync (index.ts:204-216) exactly.  One
    step = ingest + select + roots.  (N GPUs: --workload config4 / config5,
    the sharded server through evm_dist_*.)"""
    import numpy as np
    import torch

    from evolu_amd import synth
    from evolu_amd.engine import Engine

    if world > 1:
        raise SystemExit("--workload server runs on one GPU; at N GPUs use --workload config4 or config5")
    if zipf > 0:
        ts_np, owner_np, _, millis = synth.config5(owners, owners * per_owner, zipf_s=zipf,
                                                   seed_config=5 + 1000 * rank, with_millis=True)
    else:
        ts_np, owner_np, millis = synth.config3(owners, per_owner, seed_config=3 + 1000 * rank, request=request)
    eng = Engine(local)
    dev = torch.device("cuda", local)
    ts_r = eng.dev(ts_np)
    lown = torch.from_numpy(owner_np.astype(np.int32)).to(dev)
    # client trees: each owner's messages minus the newest 10% (the expected diff)
    # (the client knows each owner's first 90% by timestamp)
    o64 = owner_np.astype(np.int64)
    order = np.lexsort((millis, o64))
    rank_in_owner = np.empty(len(order), dtype=np.int64)
    counts = np.bincount(o64, minlength=owners)
    rank_in_owner[order] = np.arange(len(order)) - (np.cumsum(counts) - counts)[o64[order]]
    keep = torch.from_numpy(rank_in_owner < (0.9 * counts[o64]).astype(np.int64)).to(dev)
    if zipf > 0:  # redeliveries: the client's tree holds each known message once
        first = eng.store_new(owners)
        ins, _ = first.ingest(ts_r, lown, 0)
        keep &= (ins[: len(ts_r)] & 0x04) != 0
        first.free()
    client = eng.merkle_insert(eng.tree_new(owners), ts_r[keep].contiguous(), lown[keep].contiguous())
    node = torch.from_numpy(np.frombuffer(b"0123456789abcdef" * owners, dtype=np.uint8).copy()).to(dev)
    flags = torch.empty(len(ts_r), dtype=torch.uint8, device=dev)

    def step():
        store = eng.store_new(owners)
        store.ingest(ts_r, lown, 0, flags=flags)
        diff, off, ids = store.select(client, node)
        nsel = int(ids.numel())
        store.tree().roots()
        n_leaves = store.tree().n_leaves
        store.free()
        return nsel, n_leaves

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # per-kernel breakdown (untimed): the dominant kernel
    eng.prof_enable(True)
    eng.prof_reset()
    step()
    torch.cuda.synchronize()
    prof = eng.prof_report()
    dom = dominant(prof, SERVER_ALG)
    eng.prof_only(dom)
    eng.prof_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nsel = n_leaves = 0
    step_ms = []  # per-step wall time (a step ends in a host read-back of the roots, so this adds no sync)
    step_allocs = []  # per-step growth of the engine's allocation counters (steady state: all zero)
    for _ in range(a.steps):
        c0 = eng.stats()
        s0 = time.perf_counter()
        nsel, n_leaves = step()
        step_ms.append((time.perf_counter() - s0) * 1e3)
        c1 = eng.stats()
        step_allocs.append({k: c1[k] - c0[k] for k in ("workspace_regrows", "scratch_pool_allocs", "block_allocs")})
        if os.environ.get("EVM_BENCH_VERBOSE"):
            print("step %.2f ms" % step_ms[-1], file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    prof_dom = eng.prof_report()
    eng.prof_enable(False)
    eng.prof_only(None)
    elapsed = t1 - t0
    n = owners * per_owner
    ms = elapsed / a.steps * 1e3
    tot_ms, launches = prof_dom[dom]
    avg_s = tot_ms / launches / 1e3
    per_msg, per_leaf = SERVER_ALG[dom]
    alg = per_msg * n + per_leaf * n_leaves
    roof = {"bound": "hbm", "kernel": dom, "achieved": alg / avg_s / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": alg / avg_s / HBM_PEAK, "traffic": traffic_of(dom, "config3" if zipf <= 0 else "config5"), "kernel_ms_avg": avg_s * 1e3,
            "alg_bytes_per_launch": alg, "alg_bytes": "%d B/msg + %d B/new leaf (%d leaves)" % (per_msg, per_leaf, n_leaves),
            "kernel_share_of_step": tot_ms / (ms * a.steps)}
    reqs = "one SyncRequest per owner" if request >= per_owner else "requests of %d" % request
    out = {
        "metric": METRIC, "value": n * a.steps / elapsed, "unit": "msgs/s", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic (seeded HLC streams, SURVEY 8(d) config 3/4/5)",
        "config": {"workload": ("server: addMessages + getMessages, %d owners x %d msgs, %s"
                                % (owners, per_owner, reqs)) if zipf <= 0 else
                   ("server, Zipf stream: addMessages + getMessages, %d msgs over %d owners with Zipf(%.2f) sizes"
                    % (n, owners, zipf)),
                   "messages_per_gpu": n, "owners_per_gpu": owners,
                   "selected_rows": nsel, "parallelism": "one GPU"},
        "roofline": roof,
        "pipeline": {"alg_bytes_per_msg": SERVER_PIPELINE_BYTES,
                     "pipeline_hbm_frac": SERVER_PIPELINE_BYTES * n / (elapsed / a.steps) / HBM_PEAK,
                     "kernels_ms_per_step": {k: v[0] for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])[:14]}},
        "step_ms": [round(x, 3) for x in step_ms],
        "step_allocs": step_allocs, "engine_stats": eng.stats(),
        "cpu_baseline": None,
    }
    if leg:
        for k in ("metric", "n_gpus", "higher_is_better", "scaling", "vs_baseline", "dtype"):
            out.pop(k)
    if zipf <= 0:
        if getattr(a, "reingest", 1):
            out["reingest"] = reingest(eng, a, ts_r, lown, owners, per_owner, request, flags)
        if getattr(a, "e2e", 1) and request >= per_owner:
            out["e2e"] = e2e_leg(eng, ts_np, owner_np, client, ms)
    eng.close()
    del ts_r, lown, keep, client, flags
    torch.cuda.empty_cache()
    if cpu and a.cpu_seconds > 0 and zipf <= 0:
        out["cpu_baseline"] = cpu_baseline_server(ts_np, owner_np, min(a.cpu_seconds, 10.0))
    return out


def reap_children():
    """Every process this run started has ended (subprocess.run waits for the
    CPU-baseline legs); anything still alive here is named on stderr and
    ended, so the run leaves no process behind."""
    try:
        import psutil
    except ImportError:
        return
    kids = psutil.Process().children(recursive=True)
    for c in kids:
        try:
            print("bench: reaping child pid %d (%s)" % (c.pid, " ".join(c.cmdline())[:120]), file=sys.stderr)
            c.terminate()
        except psutil.Error:
            pass
    psutil.wait_procs(kids, timeout=5)


if __name__ == "__main__":
    try:
        main()
    finally:
        reap_children()
