#!/bin/bash
# round 6, pass z: the row GEMM's per-tile indices and coefficients DMA'd once per workgroup (wave 0) into a shared
# three-slot buffer instead of by every wave, vs the previous build; row-GEMM / model / config-3 tests.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06z}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_gemm.py --cases fwd_combine,bwd_dsig,plain,bc --rounds 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/prev.so > "$OUT/ab_shared_ic.txt" 2>&1 &&
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_config3.py tests/test_gpu_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests_subset.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
