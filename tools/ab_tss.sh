set -o pipefail
mkdir -p gpurun_out/tss
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "tail_seg or segment_reductions or tn_seg_fused" -x -q --timeout 120 --timeout-method thread > gpurun_out/tss/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_mem.py var_so/tss_off.so var_so/tss16.so var_so/tss8.so var_so/tss32.so var_so/tss_nt0.so var_so/tss_off.so var_so/tss16.so > gpurun_out/tss/bench.log 2>&1
