#!/bin/bash
# round 3, session 12: ping-pong wgrad kernel -- numerics (existing wgrad tests: default = new kernel)
# and the per-shape A/B against the round-2 kernel (dma0), then an end-to-end A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_pp_gpu.py -k "wgrad or rope" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest exit $rc" >> $O/pytest.log
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/wgrad_env_ab.py --variants ,dma0 --rounds 5 > $O/ab.log 2>&1 && tail -6 $O/ab.log || exit 1
for r in 1 2; do
for v in "" dma0; do
  ND_WGRAD_VARIANT=$v timeout -k 10 200 python bench.py --steps 6 --warmup 2 > $O/b.log 2>&1 || { echo "bench failed $v"; tail -5 $O/b.log; exit 1; }
  echo "wgrad=${v:-pp} $(tail -1 $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
done
