#!/bin/bash
# round 6 session 28: final validation at HEAD -- the whole GPU suite, smoke(), the default bench and --fp8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_bf16.log 2>&1 || { tail -20 $O/bench_bf16.log; exit 1; }
tail -1 $O/bench_bf16.log | cut -c1-220
timeout -k 10 300 python -u bench.py --fp8 --steps 20 --warmup 5 > $O/bench_fp8.log 2>&1 || { tail -20 $O/bench_fp8.log; exit 1; }
tail -1 $O/bench_fp8.log | cut -c1-220
