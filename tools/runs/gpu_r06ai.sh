#!/bin/bash
# round 6, pass ai: nontemporal stores of the row GEMM outputs, the fused pass's dX and DistMult's do^3 (ntv.so) vs HEAD:
# the kernels alone and whole config-3 steps.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ai}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_gemm.py --cases fwd_combine,bwd_dsig,plain --rounds 3 tools/runs/dbg/prev.so tools/runs/dbg/ntv.so > "$OUT/ab_gemm_nt.txt" 2>&1 &&
timeout -k 10 500 python3 -u tools/ab_sigma_tn.py 5 --config 3 tools/runs/dbg/prev.so tools/runs/dbg/ntv.so > "$OUT/ab_sigma_tn_nt.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
