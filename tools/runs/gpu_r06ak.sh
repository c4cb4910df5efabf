#!/bin/bash
# round 6, pass ak: tail_seg_mfma8 (config-5 R = 8 tail reduction) with the next chunk's loads in flight under the
# current chunk's MFMAs: HEAD (prev) vs in-loop prefetch (tpf1), in-loop prefetch at 2 waves/SIMD (tpf2), the first
# chunk only loaded with the P rows (tpf3); the kernel alone, then config-5 steps.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06ak}
mkdir -p $OUT
D=tools/runs/dbg
timeout -k 10 400 python3 -u tools/bench_tailseg.py $D/prev.so $D/tpf1.so $D/tpf2.so $D/tpf3.so $D/prev.so $D/tpf2.so > "$OUT/ab_tailseg_pf.txt" 2>&1 &&
timeout -k 10 600 python3 -u tools/ab_sigma_tn.py 3 --config 5 $D/prev.so $D/tpf2.so $D/tpf1.so > "$OUT/ab_step_cfg5_pf.txt" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
