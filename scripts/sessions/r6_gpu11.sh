#!/bin/bash
# round 6 session 11: LDS-DMA bursts in the attention kernels too (K/V tiles of the forward / dQ, Q / dO of dK/dV):
# attention tests, then in-process A/B against the same source built with -DND_DMA_BURST=0 (raw kernels, step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or flash" --timeout 200 --timeout-method thread > $O/attn_tests.log 2>&1 || { tail -40 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "deterministic" --timeout 200 --timeout-method thread > $O/det_tests.log 2>&1 || { tail -40 $O/det_tests.log; exit 1; }
tail -1 $O/det_tests.log
ALT=nanodiloco_amd/_lib/alt/libnd_kernels_burst0b.so
echo "== alt = burst0b (speedup = alt/wt: >1 means the library WITHOUT the bursts is SLOWER)"
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what attnk --rounds 5 --iters 10 > $O/ab_attnk.log 2>&1 || { tail -20 $O/ab_attnk.log; exit 1; }
grep speedup $O/ab_attnk.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what step --rounds 7 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep speedup $O/ab_step.log
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
echo "bench bf16 $(b $O/bench.log)"
