#!/bin/bash
# SQ-counter passes over single edge-GEMM cases (tools/gemm_probe.py), one rocprofv3 --pmc run per
# counter group, each under its own kill timeout; stops at the first failure.
# usage (on the box, repo root): bash tools/pmc_gemm.sh <outdir> <mode> case...
OUT=${1:-gpurun_out/pmcg}; MODE=${2:-split}; shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for c in "$@"; do
  for p in 1 2; do
    if [ $p = 1 ]; then CTR=$P1; else CTR=$P2; fi
    timeout -s KILL 90 rocprofv3 --pmc $CTR -d "$OUT/${c}_$p" -o run --output-format csv -- python3 tools/gemm_probe.py ${c%%_*} $MODE 3 > "$OUT/${c}_$p.log" 2>&1 || { echo "pass $c/$p failed"; exit 1; }
  done
done
echo pmc_gemm done
