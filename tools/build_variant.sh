#!/bin/bash
# Ablation / A-B builds of libevm.so into _var/<name>/ (loaded with
# EVM_LIB_PATH=_var/<name>/libevm.so; the default build is untouched).
#   bash tools/build_variant.sh NAME [-DFOO=1 ...]
#   SRC_OVERRIDE="evm_server.hip=/path/to/other.hip" bash tools/build_variant.sh NAME
# (each source compiled in parallel, then one link)
set -e
name=$1; shift
C=evolu_amd/csrc
O=_var/$name
mkdir -p $O
pids=()
for f in evm_engine.hip evm_client.hip evm_server.hip evm_clock.hip evm_dist.hip evm_json.cpp evm_json_dev.hip \
         evm_wire_dev.hip evm_proto.cpp evm_sync.hip; do
  src=$C/$f
  for ov in $SRC_OVERRIDE; do [ "${ov%%=*}" = "$f" ] && src=${ov#*=}; done
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-function -Iinclude -I$C "$@" \
    -c $src -o $O/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $O/*.o -ldl -o $O/libevm.so
rm -f $O/*.o
