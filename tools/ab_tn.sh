set -o pipefail
mkdir -p gpurun_out/tn
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "tn or fused or split or planes" -x -q --timeout 120 --timeout-method thread > gpurun_out/tn/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_tn.py --rounds 4 var_so/tn_old.so var_so/tn_new.so > gpurun_out/tn/ab.log 2>&1
