#!/bin/bash
# re-tune the library GEMMs at the bench micro-batch (64 x 1024) on top of the existing table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp nanodiloco_amd/tuning/tunableop_gfx950.csv gpurun_out/tune/tunableop_gfx950.csv
OUT=gpurun_out/tune/tunableop_gfx950.csv timeout -k 10 900 python scripts/tune_gemms.py llama_150m.json:64 llama_1b.json:32 > gpurun_out/tune/tune.log 2>&1 || exit $?
tail -3 gpurun_out/tune/tune.log
wc -l gpurun_out/tune/tunableop_gfx950.csv
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --tuned-gemm-file gpurun_out/tune/tunableop_gfx950.csv > gpurun_out/tune/b_new_$i.log 2>&1 || exit $?
echo "new $(tail -1 gpurun_out/tune/b_new_$i.log | cut -c100-170)"
timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/tune/b_old_$i.log 2>&1 || exit $?
echo "old $(tail -1 gpurun_out/tune/b_old_$i.log | cut -c100-170)"
done
