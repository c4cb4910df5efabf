#!/bin/bash
# round 5: bf16 edge-GEMM operands (IDDGCN_GEMM_BF16) — kernel + config-5 tests, smoke, config-5 bench; fold ulp sensitivity
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05r
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_config5.py > gpurun_out/r05r/tests.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05r/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 1 --also none --no-cpu-baseline > gpurun_out/r05r/bench_cfg5.json 2> gpurun_out/r05r/bench_cfg5.err &&
IDDGCN_CFG5_CASES="sigma' bwd GEMM,sigma' bwd GEMM bf16 ops,fwd" timeout -k 10 400 python -u tools/bench_cfg5_kernels.py > gpurun_out/r05r/cfg5_kernels.txt 2>&1 &&
timeout -k 10 400 python -u tools/fold_ulp_sensitivity.py --out gpurun_out/r05r/fold_ulp_sensitivity.json > gpurun_out/r05r/fold_ulp_sensitivity.log 2>&1
