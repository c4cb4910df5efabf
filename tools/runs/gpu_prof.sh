#!/bin/bash
# Measurement half of a GPU pass (the tests run in their own call): smoke, the default bench line, a rocprofv3
# kernel-trace/stats run and two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the headline bench
# command, and the parity report.  Every GPU step has its own time limit; the first failure stops the script.
# usage (repo root, on the box): bash tools/gpu_prof.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 3; }
tail -6 "$OUT/smoke.log"
timeout -k 10 420 python -u bench.py > "$OUT/bench_default.json.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_default.json.log"; exit 3; }
tail -c 600 "$OUT/bench_default.json.log"; echo
B="bench.py --no-cpu-baseline --no-other-mode --also none --steps 5 --warmup 2"
timeout -k 10 120 python -u $B > "$OUT/bench_profiled_cmd.json.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B > "$OUT/bench_traced.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $B > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $B > "$OUT/pmc_write.log" 2>&1 || { echo "profile step failed"; exit 3; }
timeout -k 10 400 python -u tools/parity_report.py > "$OUT/parity_report.json" 2> "$OUT/parity.err" || { echo "parity failed"; tail "$OUT/parity.err"; exit 3; }
echo done
