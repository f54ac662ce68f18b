#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for f in 1 0; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --fused-swiglu $f > gpurun_out/ab/b_${f}_${i}.log 2>&1 || exit $?
    echo "fused=$f run=$i $(tail -1 gpurun_out/ab/b_${f}_${i}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
