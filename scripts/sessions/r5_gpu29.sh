#!/bin/bash
# round 5: TunableOp table for the 131,072-token micro-batch (the bench's 128-sequence micro-batches; the shipped
# table only had 8k / 32k / 65k rows), merged with the shipped table, then an interleaved bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ac
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=$PWD/$O/tuned_131k.csv MAX_MS=60 timeout -k 10 900 python scripts/tune_gemms.py llama_150m.json:128 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -3 $O/tune.log
python3 - <<'PY'
import os
O = "gpurun_out/r5ac"
base = open("nanodiloco_amd/tuning/tunableop_gfx950.csv").read().splitlines()
new = open(os.path.join(O, "tuned_131k.csv")).read().splitlines()
have = {l.split(",")[1] for l in base if l.startswith("Gemm")}
add = [l for l in new if l.startswith("Gemm") and l.split(",")[1] not in have]
val_b = [l for l in base if l.startswith("Validator")]
val_n = [l for l in new if l.startswith("Validator")]
print("validators equal:", val_b == val_n)
for l in add: print("new:", l)
open(os.path.join(O, "merged.csv"), "w").write("\n".join(base + add) + "\n")
PY
for rd in 1 2 3; do
  for arm in old new; do
    extra=""; [ $arm = new ] && extra="--tuned-gemm-file $PWD/$O/merged.csv"
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 $extra > $O/b_${arm}_$rd.log 2>&1 || { tail -5 $O/b_${arm}_$rd.log; exit 1; }
    echo "$arm r$rd $(tail -1 $O/b_${arm}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("tuned_gemm"))')"
  done
done
