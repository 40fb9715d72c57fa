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

SOURCES = ["evm_engine.hip", "evm_client.hip", "evm_server.hip", "evm_clock.hip", "evm_dist.hip", "evm_json.cpp", "evm_proto.cpp"]
HEADERS = ["evm_device.hpp", "evm_pack.hpp", "evm_prims.hpp", "evm_internal.hpp"]


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths if os.path.exists(p))


def build_lib(force: bool = False, verbose: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "evm.h")]
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _newest(deps):
        return LIB
    cmd = [HIPCC, "-O3", "--offload-arch=" + ARCH, "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-function", "-I" + INCLUDE] + srcs + ["-ldl", "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build_lib(force="--force" in sys.argv, verbose=True))
