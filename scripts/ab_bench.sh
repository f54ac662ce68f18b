#!/bin/bash
# Interleaved bench A/B on one GPU box: runs `bench.py $COMMON $A` and `bench.py $COMMON $B`
# alternately ROUNDS times (each under its own time limit), prints value/ms_per_step per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in A B; do
    if [ $arm = A ]; then args="$A"; else args="$B"; fi
    timeout -k 10 ${T:-300} python bench.py ${COMMON:---steps 6 --warmup 2} $args > gpurun_out/ab_${arm}_$r.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab_${arm}_$r.log; echo "arm $arm rc=$rc"; exit $rc; fi
    python - "$arm" "$r" gpurun_out/ab_${arm}_$r.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"arm {sys.argv[1]} round {sys.argv[2]}: {d['value']:.0f} tok/s  {d['ms_per_step']:.2f} ms/step")
PY
  done
done
