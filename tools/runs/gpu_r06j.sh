#!/bin/bash
# round 6, pass j: the bf16x3 row GEMM with A rows staged through registers (RB3_REGA=1, the tree) against LDS-DMA
# A rows (dma_a.so) and the round-6 kernel without its L2 prefetch (nopf.so); kernel tests; config-3 step A/B.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06j}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_gemm.py --cases fwd_combine,bwd_dsig,plain,acc,bc --rounds 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/dma_a.so tools/runs/dbg/nopf.so > "$OUT/ab_rega.txt" 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sigma_tn_b3.py tests/test_gpu_model.py tests/test_gpu_config3.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests_subset.txt" 2>&1 &&
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-other-mode --no-fold0-auc --also none --steps 10 --warmup 3 > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err"
rc=$?
echo "rc=$rc"
exit $rc
