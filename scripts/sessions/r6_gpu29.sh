#!/bin/bash
# round 6 session 29: bench with the --mlp-coef flag (default and 0) and the bench-contract GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $O/b_default.log 2>&1 || { tail -20 $O/b_default.log; exit 1; }
tail -1 $O/b_default.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["mlp_saved_form"], d["comm_impl"])'
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --mlp-coef 0 > $O/b_gu.log 2>&1 || { tail -20 $O/b_gu.log; exit 1; }
tail -1 $O/b_gu.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["mlp_saved_form"], d["final_loss"])'
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
