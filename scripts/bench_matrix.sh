#!/bin/bash
# A list of bench.py configurations run back to back on one GPU box, one JSON summary line each.
# Usage: CONFIGS=$'name1|args1\nname2|args2' bash scripts/bench_matrix.sh   (each run has its own limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
while IFS='|' read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 ${T:-400} python bench.py $args > gpurun_out/bm_$name.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bm_$name.log; echo "$name rc=$rc"; exit $rc; fi
  python - "$name" gpurun_out/bm_$name.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"{sys.argv[1]:14s} {d['value']:10.0f} tok/s {d['ms_per_step']:9.2f} ms/step  "
      f"{d['model_tflops_per_gpu']:7.1f} TF  mb={d['config']['micro_batch']} {d['config']['model']} {d['dtype']}")
PY
done <<< "$CONFIGS"
