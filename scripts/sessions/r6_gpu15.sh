#!/bin/bash
# round 6 session 15: the first K/V (Q/dO) LDS-DMA tiles issued before the attention kernels' prologue loads
# (ND_ATTN_EARLY): attention + determinism tests, in-process A/B against -DND_ATTN_EARLY=0, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or flash or deterministic" --timeout 200 --timeout-method thread > $O/attn_tests.log 2>&1 || { tail -40 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
ALT=nanodiloco_amd/_lib/alt/libnd_kernels_early0.so
echo "== alt = early0 (speedup = alt/wt: >1 means the library WITHOUT the early DMA is SLOWER)"
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what attnk --rounds 7 --iters 10 > $O/ab_attnk.log 2>&1 || { tail -20 $O/ab_attnk.log; exit 1; }
grep speedup $O/ab_attnk.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what step --rounds 7 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep speedup $O/ab_step.log
timeout -k 10 200 python -u scripts/attn_stamps.py --lib nanodiloco_amd/_lib/alt/libnd_kernels_stamp.so > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
