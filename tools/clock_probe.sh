#!/bin/bash
# Shader clock while one edge GEMM runs back to back (tools/gemm_probe.py), read with rocm-smi --showclocks
# (reading only) a few times during the loop.  usage (box, repo root): bash tools/clock_probe.sh <outdir> <case> <mode> <reps>
OUT=${1:-gpurun_out/clk}; CASE=${2:-fwd}; MODE=${3:-exact}; REPS=${4:-1000}
mkdir -p "$OUT"
timeout -k 10 120 python3 tools/gemm_probe.py $CASE $MODE $REPS > "$OUT/${CASE}_${MODE}.log" 2>&1 &
PID=$!
for k in 1 2 3 4 5 6; do
  sleep 1
  timeout 10 rocm-smi --showclocks >> "$OUT/${CASE}_${MODE}_clk.txt" 2>&1
done
wait $PID
rc=$?
grep -h "sclk" "$OUT/${CASE}_${MODE}_clk.txt" | head -12
exit $rc
