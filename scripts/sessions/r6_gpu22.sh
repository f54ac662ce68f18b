#!/bin/bash
# round 6 session 22: coefficient form of the fused SwiGLU pair (ND_MLP_COEF / ops.gemm.set_mlp_coef): its GPU tests and
# the SwiGLU kernel tests, the kernel-level A/B, then the bench step (bf16 and --fp8) with the form set by the
# environment, interleaved over 3 rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_mlp_coef_gpu.py tests/test_gemm_pp_gpu.py tests/test_gemm_pp_f8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/mlp_coef_ab.py > $O/kernels.log 2>&1 || { tail -20 $O/kernels.log; exit 1; }
cat $O/kernels.log | grep form
for r in 1 2 3; do
  for f in 0 1; do
    ND_MLP_COEF=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bf16_c${f}_r$r.log 2>&1 || { tail -20 $O/bf16_c${f}_r$r.log; exit 1; }
    echo "bf16 coef=$f round $r: $(tail -1 $O/bf16_c${f}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for r in 1 2; do
  for f in 0 1; do
    ND_MLP_COEF=$f timeout -k 10 300 python -u bench.py --fp8 --steps 20 --warmup 5 > $O/fp8_c${f}_r$r.log 2>&1 || { tail -20 $O/fp8_c${f}_r$r.log; exit 1; }
    echo "fp8 coef=$f round $r: $(tail -1 $O/fp8_c${f}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
