#!/bin/bash
# fused gate|up + SwiGLU GEMM (own kernel, variant 10) vs hipBLASLt + swiglu_fwd, in the full step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2fs
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
for f in 1 0; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --fused-swiglu $f > gpurun_out/r2fs/b_${f}_$i.log 2>&1 || exit $?
echo "fused=$f $(tail -1 gpurun_out/r2fs/b_${f}_$i.log | cut -c100-150)"
done
done
