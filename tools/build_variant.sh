#!/bin/bash
# Ablation / A-B builds of libevm.so with extra defines into _var/<name>/
# (loaded with EVM_LIB_PATH=_var/<name>/libevm.so; the default build is untouched).
#   bash tools/build_variant.sh NAME -DFOO=1 ...
set -e
name=$1; shift
C=evolu_amd/csrc
mkdir -p _var/$name
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Wno-unused-function -Iinclude "$@" \
  $C/evm_engine.hip $C/evm_client.hip $C/evm_server.hip $C/evm_clock.hip $C/evm_dist.hip $C/evm_json.cpp $C/evm_json_dev.hip $C/evm_wire_dev.hip $C/evm_proto.cpp \
  -ldl -o _var/$name/libevm.so
