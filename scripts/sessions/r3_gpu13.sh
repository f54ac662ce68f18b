#!/bin/bash
# round 3, session 13: HEAD validation after the GEMM cleanup: full GPU suite, smoke, bench (bf16 / fp8 / 1B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3m
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/pytest.log
tail -4 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-220 || exit 1
timeout -k 10 300 python bench.py --fp8 > $O/bench_fp8.log 2>&1 && tail -1 $O/bench_fp8.log | cut -c1-220 || exit 1
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --model llama_1b.json --micro-batch 32 > $O/bench_1b.log 2>&1 && tail -1 $O/bench_1b.log | cut -c1-220
