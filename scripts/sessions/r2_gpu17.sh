#!/bin/bash
# interleaved-DMA GEMM variants: tests (variant 10 included), bf16 per-shape A/B, fp8 e2e A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2f8
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm_f8_gpu.py tests/test_gemm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2f8/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r2f8/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/gemm_nt_bench.py --variants 5:4,10:4 --rounds 5 > gpurun_out/r2f8/ab16.log 2>&1 || exit $?
cat gpurun_out/r2f8/ab16.log
for i in 1 2; do
for g in hip hipblaslt; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --fp8 --fp8-gemm $g > gpurun_out/r2f8/bench_${g}_${i}.log 2>&1 || exit $?
echo "$g $(tail -1 gpurun_out/r2f8/bench_${g}_${i}.log | cut -c1-200)"
done
done
