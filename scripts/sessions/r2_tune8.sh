#!/bin/bash
# tune the fp8 (ScaledGemm) projection GEMMs on top of the shipped table, then A/B the --fp8 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune8
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp nanodiloco_amd/tuning/tunableop_gfx950.csv gpurun_out/tune8/tunableop_gfx950.csv
FP8=1 OUT=gpurun_out/tune8/tunableop_gfx950.csv timeout -k 10 900 python scripts/tune_gemms.py llama_150m.json:64 llama_1b.json:32 > gpurun_out/tune8/tune.log 2>&1 || exit $?
tail -3 gpurun_out/tune8/tune.log
grep -c Scaled gpurun_out/tune8/tunableop_gfx950.csv
for i in 1 2; do
timeout -k 10 300 python bench.py --fp8 --steps 8 --warmup 2 --tuned-gemm-file gpurun_out/tune8/tunableop_gfx950.csv > gpurun_out/tune8/b_new_$i.log 2>&1 || exit $?
echo "new $(tail -1 gpurun_out/tune8/b_new_$i.log | cut -c100-150)"
timeout -k 10 300 python bench.py --fp8 --steps 8 --warmup 2 > gpurun_out/tune8/b_old_$i.log 2>&1 || exit $?
echo "old $(tail -1 gpurun_out/tune8/b_old_$i.log | cut -c100-150)"
done
