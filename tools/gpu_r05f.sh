#!/bin/bash
# round 5: SQ counters of the bf16x3 plain row GEMM, column-half kernel (b3) vs full-width (w4)
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/pmc_gemm.sh gpurun_out/r05f/b3 bf16x3 plain &&
bash tools/pmc_gemm.sh gpurun_out/r05f/w4 bf16x3w4 plain &&
python tools/pmc_sq_summary.py gpurun_out/r05f/b3 plain > gpurun_out/r05f/summary.txt &&
python tools/pmc_sq_summary.py gpurun_out/r05f/w4 plain >> gpurun_out/r05f/summary.txt
