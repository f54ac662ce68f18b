#!/bin/bash
# lm-head chunk size A/B in the full bench (1 GiB = 16k rows, 2 GiB = 32k, 4.2 GiB = 64k = whole micro-batch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2ce
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
for mb in 1024 2048 4200; do
ND_CE_CHUNK_MB=$mb timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/r2ce/b_${mb}_${i}.log 2>&1 || exit $?
echo "$mb $(tail -1 gpurun_out/r2ce/b_${mb}_${i}.log | cut -c100-200)"
done
done
