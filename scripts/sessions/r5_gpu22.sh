#!/bin/bash
# round 5: wgrad split planning by the makespan model + model-gated grouping: tests, 150M / 1B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" tests/test_gemm_pp_f8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --steps 8 --warmup 2 > $O/b150.log 2>&1 || { tail -5 $O/b150.log; exit 1; }
echo "150m $(tail -1 $O/b150.log | cut -c1-120)"
for rd in 1 2; do
  for p in old cost; do
    ND_WGRAD_PLAN=$p timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 > $O/b1_${p}_$rd.log 2>&1 || { tail -5 $O/b1_${p}_$rd.log; exit 1; }
    echo "1b plan=$p r$rd $(tail -1 $O/b1_${p}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --fp8 > $O/b1_fp8.log 2>&1 || { tail -5 $O/b1_fp8.log; exit 1; }
echo "1b fp8 $(tail -1 $O/b1_fp8.log | cut -c1-120)"
