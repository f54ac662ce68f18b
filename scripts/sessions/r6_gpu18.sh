#!/bin/bash
# round 6 session 18: the group-agreed RCCL fallback (parallel/rccl.py communicator_or_fallback) on the GPU:
# the own-communicator tests (one-rank collectives, torchrun bench, init timeout with a missing peer), the
# multi-rank GPU+gloo rehearsals, then the default bench (must still report comm_impl rccl)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_rccl_gpu.py tests/test_multirank_gpu.py -x -v --timeout 200 --timeout-method thread > $O/rccl_tests.log 2>&1 || { tail -40 $O/rccl_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/rccl_tests.log | tail -12
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
