#!/bin/bash
# round 3, session 5: ping-pong GEMM ablations (no waits / nt stores) after the store-count fix
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --check-only > $O/check.log 2>&1; echo "check exit $?" >> $O/check.log
tail -3 $O/check.log
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --ablate 0,1,8,16,32 --rounds 7 > $O/ablate.log 2>&1 && tail -4 $O/ablate.log
