#!/bin/bash
# round 6, pass b: the fused bf16x3 sigma' + TN kernel with the epilogue and the next tile's conversion issued behind
# its TN MFMAs — A/B against pass a's build (st3_v1) and an s_setprio variant, then the whole GPU suite, smoke and the
# headline bench line.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06b}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sigma_tn_b3.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_st3.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_sigma_tn.py 7 --config 3 iddgcn_amd/libiddgcn_hip.so iddgcn_amd/var/st3_v1.so iddgcn_amd/var/st3_prio.so > $OUT/ab_st3.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --also none --no-cpu-baseline --no-fold0-auc --steps 10 --warmup 3 > $OUT/bench.json.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
