#!/bin/bash
# round 6, pass am: s_setprio for the longer wave chain.  sp1: sigma_tn_b3 waves 0-3 (stage + convert for both waves
# of their SIMD) at priority 1 for the whole loop; sp2: only around their conversions; bp1: rowgemm256_b3 waves 4-7
# (epilogue-first, the longer chain in the phase stamps) at priority 1.  The forward GEMM alone, then the fused pass
# and whole config-3 steps.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06am}
mkdir -p $OUT
D=tools/runs/dbg
timeout -k 10 300 python3 -u tools/ab_gemm.py --cases fwd_combine --rounds 3 $D/base.so $D/bp1.so > "$OUT/ab_gemm_prio.txt" 2>&1 &&
timeout -k 10 600 python3 -u tools/ab_sigma_tn.py 3 --config 3 $D/base.so $D/sp1.so $D/sp2.so $D/bp1.so > "$OUT/ab_sigma_tn_prio.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
