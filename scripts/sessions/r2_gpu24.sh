#!/bin/bash
# micro-batch A/B at round-2 HEAD (same global batch 256 x 1024 per inner step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2mb
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
for mb in 64 128; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --micro-batch $mb > gpurun_out/r2mb/b_${mb}_$i.log 2>&1 || exit $?
echo "$mb $(tail -1 gpurun_out/r2mb/b_${mb}_$i.log | cut -c100-150)"
done
done
