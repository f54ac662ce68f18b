#!/bin/bash
# round 3, session 29: ping-pong GEMM tile-group size on the N=1024 shapes (o fwd, gu dgrad) vs hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ac
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/gemm_pp_bench.py --gms 1,2,4,8,16 --rounds 5 > $O/gms.log 2>&1; rc=$?; cat $O/gms.log; exit $rc
