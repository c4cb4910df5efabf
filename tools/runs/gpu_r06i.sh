#!/bin/bash
# round 6, pass i: per-phase s_memtime stamps of the bf16x3 row GEMM main loop (forward with gathered combine,
# sigma' backward, plain), and the forward without its L2 prefetch DMA (A/B).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06i}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd.py tools/runs/dbg/stamp.so --case fwd_combine > "$OUT/stamp_fwd.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd.py tools/runs/dbg/stamp.so --case bwd_dsig > "$OUT/stamp_bwd.txt" 2>&1 &&
timeout -k 10 200 python3 -u tools/runs/dbg/stamp_fwd.py tools/runs/dbg/stamp.so --case plain > "$OUT/stamp_plain.txt" 2>&1 &&
timeout -k 10 300 python3 -u tools/ab_gemm.py --cases fwd_combine,bwd_dsig,plain --rounds 3 iddgcn_amd/libiddgcn_hip.so tools/runs/dbg/nopf.so > "$OUT/ab_nopf.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
