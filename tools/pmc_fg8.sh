#!/bin/bash
# SQ-counter passes over the config-5 forward edge GEMM alone (tools/fg8_probe.py, 2 launches), one rocprofv3 --pmc
# run per counter group, each under its own kill timeout; stops at the first failure.
# usage (on the box, repo root): bash tools/pmc_fg8.sh <outdir>
OUT=${1:-gpurun_out/pmc_fg8}
export TMPDIR=/tmp
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for p in 1 2; do
  if [ $p = 1 ]; then CTR=$P1; else CTR=$P2; fi
  timeout -s KILL 150 rocprofv3 --pmc $CTR -d "$OUT/fg8_$p" -o run --output-format csv -- python3 tools/fg8_probe.py 1 > "$OUT/fg8_$p.log" 2>&1 || { echo "pass $p failed"; exit 1; }
done
echo pmc_fg8 done
