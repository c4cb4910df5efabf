#!/bin/bash
# round 5: bf16x3 row GEMM with its A rows staged through registers (asm-issued global loads, converted from the
# registers into the LDS planes) instead of LDS-DMA of the fp32 row + in-LDS conversion — A/B at T = 4M
# (base = HEAD source, rega = -DB3_REGA=1), outputs compared bitwise
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r05ra
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab_gemm.py --modes bf16x3 --cases fwd_combine,bwd_dsig,plain,acc,bc --rounds 3 varx/base.so varx/rega.so > $OUT/ab.txt 2>&1
