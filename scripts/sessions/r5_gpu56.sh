#!/bin/bash
# round 5 closing validation: full GPU suite + smoke + bf16 bench, --fp8, Llama-1B bf16 / --fp8 at H=500
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bd
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
v() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["micro_batch"], d["residual_dtype"], d.get("model_tflops_per_gpu"))'; }
timeout -k 10 300 python bench.py > $O/b150.log 2>&1 || { tail -5 $O/b150.log; exit 1; }
echo "150m bf16 $(v $O/b150.log)"
timeout -k 10 300 python bench.py --fp8 > $O/b150_fp8.log 2>&1 || { tail -5 $O/b150_fp8.log; exit 1; }
echo "150m fp8 $(v $O/b150_fp8.log)"
timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 > $O/b1b.log 2>&1 || { tail -5 $O/b1b.log; exit 1; }
echo "1b bf16 H500 $(v $O/b1b.log)"
timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --fp8 > $O/b1b_fp8.log 2>&1 || { tail -5 $O/b1b_fp8.log; exit 1; }
echo "1b fp8 H500 $(v $O/b1b_fp8.log)"
