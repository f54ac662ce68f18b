#!/bin/bash
# CLI trainer on the reference's default 10M model (REF configs/llama_default.json, micro-batch 8 as
# in the reference): --hip-graph auto (default) vs off; prints the last logged tokens/s of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for hg in auto off; do
  timeout -k 10 300 python -m nanodiloco_amd --llama-config-file configs/llama_default.json --batch-size 256 \
    --per-device-batch-size 8 --total-steps 20 --inner-steps 10 --warmup-steps 2 --wandb off --log-every 5 \
    --hip-graph $hg --log-file gpurun_out/tr_$hg.jsonl > gpurun_out/tr_$hg.log 2>&1 || { tail -20 gpurun_out/tr_$hg.log; exit 1; }
  python - "$hg" gpurun_out/tr_$hg.jsonl <<'PY'
import json, sys
r = [json.loads(l) for l in open(sys.argv[2]) if "tokens_per_s" in l][-1]
print(f"hip-graph {sys.argv[1]:5s}: {r['tokens_per_s']:.0f} tok/s  loss {r['loss']:.3f}")
PY
done
