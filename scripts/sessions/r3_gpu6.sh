#!/bin/bash
# round 3, session 6: ping-pong GEMM start stagger A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --check-only > $O/check.log 2>&1; echo "check exit $?" >> $O/check.log
tail -2 $O/check.log
timeout -k 10 300 python -u scripts/gemm_pp_bench.py --ablate 0,8,64 --stagger 500,1000,2000,4000,8000 --rounds 5 > $O/stagger.log 2>&1 && tail -5 $O/stagger.log
