#!/bin/bash
# round 5: full GPU suite + smoke after the bf16-residual commit; --residual-dtype bf16 with --fp8 and on Llama-1B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ay
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
v() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["residual_dtype"])'; }
for r in fp32 bf16; do
  timeout -k 10 300 python bench.py --fp8 --residual-dtype $r > $O/f8_$r.log 2>&1 || { tail -5 $O/f8_$r.log; exit 1; }
  echo "fp8 $(v $O/f8_$r.log)"
done
for r in fp32 bf16; do
  timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --residual-dtype $r > $O/b1_$r.log 2>&1 || { tail -5 $O/b1_$r.log; exit 1; }
  echo "1b $(v $O/b1_$r.log)"
done
