#!/bin/bash
# --fp8 step with each fp8 GEMM backend (own kernel with the auto loader choice vs hipBLASLt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2f8e
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
for g in hip hipblaslt; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --fp8 --fp8-gemm $g > gpurun_out/r2f8e/b_${g}_$i.log 2>&1 || exit $?
echo "$g $(tail -1 gpurun_out/r2f8e/b_${g}_$i.log | cut -c100-150)"
done
done
