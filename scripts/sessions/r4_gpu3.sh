#!/bin/bash
# round 4, session 3: w128 v2 (whole-line DMA pieces, operand-split pipelining): numerics, ablations,
# per-shape A/B against hipBLASLt / ping-pong at 131,072 tokens
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4d}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_w128_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/w128_probe.py ablate --abl ${ABL:-1,2,4,8,16,31} > $O/ablate.log 2>&1
rc=$?; cat $O/ablate.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/gemm_pp_bench.py --tokens 131072 --rounds 3 > $O/bench.log 2>&1
rc=$?; tail -11 $O/bench.log; exit $rc
