#!/bin/bash
# round 3, session 49: TunableOp table for the 128-sequence micro-batch shapes, merged, A/B vs the shipped table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3av
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp nanodiloco_amd/tuning/tunableop_gfx950.csv $O/old.csv
OUT=$O/tuned_128.csv MAX_MS=30 timeout -k 10 500 python -u scripts/tune_gemms.py llama_150m.json:128 > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
tail -2 $O/tune.log
python scripts/merge_tuning.py $O/tuned_128.csv > $O/merge.log 2>&1 || { cat $O/merge.log; exit 1; }
cp nanodiloco_amd/tuning/tunableop_gfx950.csv $O/merged.csv
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 3 > $O/b_new_$r.log 2>&1 || exit 1
  echo "new r=$r $(tail -1 $O/b_new_$r.log | cut -c90-150)"
  timeout -k 10 300 python bench.py --steps 8 --warmup 3 --tuned-gemm-file $O/old.csv > $O/b_old_$r.log 2>&1 || exit 1
  echo "old r=$r $(tail -1 $O/b_old_$r.log | cut -c90-150)"
done
