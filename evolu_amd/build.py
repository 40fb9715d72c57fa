"""In-tree build of libevm.so (hipcc, gfx950).  The .so travels to the GPU box."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "libevm.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("EVM_ARCH", "gfx950")

SOURCES = ["evm_engine.hip", "evm_client.hip", "evm_server.hip", "evm_clock.hip", "evm_dist.hip", "evm_json.cpp", "evm_json_dev.hip", "evm_wire_dev.hip",
           "evm_proto.cpp", "evm_sync.hip"]
HEADERS = ["evm_device.hpp", "evm_pack.hpp", "evm_prims.hpp", "evm_internal.hpp"]


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


# synthetic streams on the device (bench / test input; not part of libevm)
SYNTH_LIB = os.path.join(HERE, "libevmsynth.so")
SYNTH_SOURCES = ["evm_synth.hip"]


def _build(lib, sources, headers, extra, force, verbose):
    """Each source compiled to its own object in parallel (the two large
    kernel files dominate), then one link."""
    from concurrent.futures import ThreadPoolExecutor

    srcs = [os.path.join(CSRC, s) for s in sources]
    deps = srcs + [os.path.join(CSRC, h) for h in headers] + [os.path.join(INCLUDE, "evm.h")]
    if not force and os.path.exists(lib) and os.path.getmtime(lib) >= _newest(deps):
        return lib
    odir = os.path.join(HERE, "build", os.path.basename(lib))
    os.makedirs(odir, exist_ok=True)
    base = [HIPCC, "-O3", "--offload-arch=" + ARCH, "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-I" + INCLUDE]
    hdr_time = _newest([os.path.join(CSRC, h) for h in headers] + [os.path.join(INCLUDE, "evm.h")])

    def obj(src):
        o = os.path.join(odir, os.path.basename(src) + ".o")
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(src), hdr_time):
            cmd = base + ["-c", src, "-o", o + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
            os.replace(o + ".tmp", o)
        return o

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(obj, srcs))
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-fPIC", "-shared"] + objs + extra + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


def build_lib(force: bool = False, verbose: bool = False) -> str:
    _build(SYNTH_LIB, SYNTH_SOURCES, ["evm_device.hpp"], [], force, verbose)
    return _build(LIB, SOURCES, HEADERS, ["-ldl"], force, verbose)


if __name__ == "__main__":
    print(build_lib(force="--force" in sys.argv, verbose=True))
