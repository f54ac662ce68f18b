#!/bin/bash
# round 3, session 9: VGPR-staged k-step ping-pong GEMM (impl 2): numerics, A/B vs impl 1 and hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 200 python -u scripts/gemm_pp_bench.py --check-only --impl 3 > $O/check3.log 2>&1; rc=$?; echo "check exit $rc" >> $O/check3.log
tail -22 $O/check3.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_pp_bench.py --impls 1,3 --rounds 5 > $O/ab.log 2>&1 && tail -5 $O/ab.log
