#!/bin/bash
# round 3, session 8: LDS-staged full-line C stores vs direct half-line stores (ping-pong GEMM)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --check-only > $O/check.log 2>&1; echo "check exit $?" >> $O/check.log
tail -2 $O/check.log
timeout -k 10 300 python -u scripts/gemm_pp_bench.py --ablate 0,8,256,288 --rounds 5 > $O/abl.log 2>&1 && tail -4 $O/abl.log
