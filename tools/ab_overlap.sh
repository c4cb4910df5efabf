#!/bin/bash
# A/B inside one box: the default step vs --overlap (side-stream tail reductions), alternating, exact mode.
OUT=${1:-gpurun_out/ab_ovl}; mkdir -p $OUT
B="bench.py --no-cpu-baseline --no-other-mode --also none --steps 10 --warmup 3"
for k in 1 2; do
  timeout -k 10 120 python3 $B > $OUT/base_$k.json 2>&1 || exit 1
  timeout -k 10 120 python3 $B --overlap > $OUT/ovl_$k.json 2>&1 || exit 1
done
for f in $OUT/*.json; do python3 -c "import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"; done
