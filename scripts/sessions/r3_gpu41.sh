#!/bin/bash
# round 3, session 41: plain-GEMM routing A/B (hipBLASLt everywhere vs own kernel for K <= 1024), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ao
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bias_gpu.py > $O/pytest_bias.log 2>&1; echo "bias rc $?"; tail -3 $O/pytest_bias.log
for r in 1 2; do
  for g in blas short; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --proj-gemm $g > $O/bench_${g}_$r.log 2>&1 || exit 1
    echo "$g $r $(tail -1 $O/bench_${g}_$r.log | cut -c1-120)"
  done
done
