#!/bin/bash
# Build experiment variants of libiddgcn_hip.so (iddgcn_hip.hip with extra -D flags, linked with the other
# sources' objects from build/, which __graft_entry__.build() leaves) for A/B timing (tools/bench_gemm.py
# loads each in turn).  usage: tools/build_variants.sh name1 "-DFLAG=1 ..." name2 "..." ...
set -e
cd "$(dirname "$0")/.."
VD=${VAR_DIR:-var_so}; mkdir -p $VD
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $(cat iddgcn_amd/csrc/device_flags.txt) \
      -c -I include $flags \
      iddgcn_amd/csrc/iddgcn_hip.hip -o $VD/$name.o && \
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $VD/$name.o build/graph_build.hip.o \
      build/similarity.hip.o build/sampling.hip.o -o $VD/$name.so && rm $VD/$name.o && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
