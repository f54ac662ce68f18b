#!/bin/bash
# round 5: own RCCL communicator on one GPU (tests/_rccl_check.py, bench default = one-rank RCCL group)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -15 $O/test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/rccl_$r.log 2>&1 || { tail -3 $O/rccl_$r.log; exit 1; }
  tail -1 $O/rccl_$r.log | cut -c1-900
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --backend none > $O/none_$r.log 2>&1 || { tail -3 $O/none_$r.log; exit 1; }
  tail -1 $O/none_$r.log | cut -c1-300
done
