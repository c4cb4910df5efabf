#!/bin/bash
# round 6, first pass: the fused bf16x3 sigma' + TN kernel (ABI 12) — its tests, the config-3 oracle step tests,
# smoke, the per-launch / per-step A/B against the two kernels it replaces (and the waves-4-7-TN-first variant),
# then the headline bench line.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06a}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sigma_tn_b3.py -x -v --timeout 120 --timeout-method thread > $OUT/tests_st3.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_config3.py tests/test_gpu_model.py tests/test_gpu_kernels.py -k "bf16x3 or config3 or step" -x -q --timeout 300 --timeout-method thread > $OUT/tests_cfg3.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_sigma_tn.py 7 --config 3 iddgcn_amd/libiddgcn_hip.so iddgcn_amd/var/late_tn.so > $OUT/ab_st3.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --also none --no-cpu-baseline --no-fold0-auc --steps 10 --warmup 3 > $OUT/bench.json.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
