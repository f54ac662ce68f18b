#!/bin/bash
# round 3, session 3: ping-pong GEMM diagnostics + timing A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_pp_bench.py --rounds 3 > $O/pp.log 2>&1; echo "pp exit $?" >> $O/pp.log
tail -40 $O/pp.log
