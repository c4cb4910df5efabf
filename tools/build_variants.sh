#!/bin/bash
# Build experiment variants of libiddgcn_hip.so (iddgcn_hip.hip only) with extra -D flags, for A/B timing
# with tools/ab_rowgemm.py.  usage: tools/build_variants.sh name1 "-DFLAG=1 ..." name2 "..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p var_so
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include $flags \
      iddgcn_amd/csrc/iddgcn_hip.hip -o var_so/$name.so && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
