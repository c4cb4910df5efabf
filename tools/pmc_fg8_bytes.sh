#!/bin/bash
# HBM bytes of the config-5 forward edge GEMM alone (tools/fg8_probe.py, 2 launches): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc runs, each under its own kill timeout.  usage (on the box, repo root): bash tools/pmc_fg8_bytes.sh <outdir>
OUT=${1:-gpurun_out/pmc_fg8b}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 tools/fg8_probe.py 1 > "$OUT/fetch.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 tools/fg8_probe.py 1 > "$OUT/write.log" 2>&1 &&
echo pmc_fg8_bytes done
