#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05g
timeout -k 10 200 python -u tools/w4_probe.py --cases plain > gpurun_out/r05g/w4_probe.txt 2>&1 &&
bash tools/pmc_gemm.sh gpurun_out/r05g/w4 bf16x3w4 plain &&
python tools/pmc_sq_summary.py gpurun_out/r05g/w4 plain > gpurun_out/r05g/summary.txt
