#!/bin/bash
# round 6, pass c: the fused pass back in its pass-a form (v1); the bf16x3 row GEMM with the next tile's conversion
# issued inside its MFMA phase (product) against the same kernel converting after it (fwd_orig): per-form A/B on
# identical inputs, whole config-3 steps per build, then the headline bench line.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sigma_tn_b3.py tests/test_gpu_kernels.py tests/test_gpu_config3.py -k "b3 or bf16x3 or config3" -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_gemm.py --modes bf16x3 --rounds 3 iddgcn_amd/libiddgcn_hip.so iddgcn_amd/var/fwd_orig.so > $OUT/ab_gemm.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_sigma_tn.py 5 --config 3 iddgcn_amd/libiddgcn_hip.so iddgcn_amd/var/fwd_orig.so > $OUT/ab_step.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --also none --no-cpu-baseline --no-fold0-auc --steps 10 --warmup 3 > $OUT/bench.json.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
