#!/bin/bash
# round 6, pass g: how much the per-tile fp32 -> bf16x3 conversion costs the two headline kernels (the question behind
# "producer-written planes"): ablation builds with the conversion skipped (results wrong, timing
# only) — abl_noconv: every conversion in the row GEMM and the fused pass; abl_noconvx: the fused pass's X rows only —
# against the product on identical inputs; then the owner-E test with the gathered Adam state.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06g}
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_gemm.py --modes bf16x3 --cases fwd_combine,bwd_dsig,plain --rounds 3 iddgcn_amd/libiddgcn_hip.so iddgcn_amd/var/abl_noconv.so > $OUT/ab_gemm_noconv.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_sigma_tn.py 5 --config 3 iddgcn_amd/libiddgcn_hip.so iddgcn_amd/var/abl_noconv.so iddgcn_amd/var/abl_noconvx.so > $OUT/ab_sigma_tn_noconv.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parallel.py -k "owner_e" -x -v --timeout 300 --timeout-method thread > $OUT/tests_owner_e.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
