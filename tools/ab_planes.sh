set -o pipefail
mkdir -p gpurun_out/abpl
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --also none --no-other-mode > gpurun_out/abpl/on$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --also none --no-other-mode --no-planes > gpurun_out/abpl/off$i.log 2>&1 || exit 1
done
for f in gpurun_out/abpl/*.log; do python -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()})"; done
