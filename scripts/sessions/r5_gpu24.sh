#!/bin/bash
# round 5: bf16-only makespan plan -- wgrad / fp8 tests, 1B bf16 + fp8 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" tests/test_gemm_pp_f8_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "" "--fp8"; do
  timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 $a > $O/b1$a.log 2>&1 || { tail -5 $O/b1$a.log; exit 1; }
  echo "1b $a $(tail -1 $O/b1$a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
