#!/bin/bash
# round 6 session 4: (1) the attention prologue-load wait fix (settle(): no compiler vmcnt inside the tile loops,
# which also drained the iteration's own LDS-DMA prefetch) -- attention GPU tests, kernel and step A/B against
# the round-5 placement (x512); (2) dK/dV grid order 1 (key blocks of one head grouped on an XCD) on top of it;
# (3) the forward's two S chains interleaved (x256); stamps of the fixed kernels; 3 interleaved bench rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
A=nanodiloco_amd/_lib/alt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in x512 ord1 x256; do
  echo "== alt = $v (speedup = alt/wt: >1 means the alt library is SLOWER than the working tree)"
  timeout -k 10 180 python -u scripts/ab_kernels.py --alt $A/libnd_kernels_$v.so --what attnk --rounds 7 --iters 10 > $O/ab_$v.log 2>&1 || { tail -20 $O/ab_$v.log; exit 1; }
  grep attn_ $O/ab_$v.log
done
for v in x512 ord1; do
  timeout -k 10 300 python -u scripts/ab_kernels.py --alt $A/libnd_kernels_$v.so --what step --rounds 5 --iters 3 > $O/ab_step_$v.log 2>&1 || { tail -20 $O/ab_step_$v.log; exit 1; }
  echo "step alt=$v: $(grep fwd_bwd $O/ab_step_$v.log)"
done
timeout -k 10 120 python -u scripts/attn_stamps.py --lib $A/libnd_kernels_stamp.so > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/d_$rd.log 2>&1 || { tail -5 $O/d_$rd.log; exit 1; }
  echo "order0 r$rd $(b $O/d_$rd.log)"
  ND_ATTN_DKDV_ORDER=1 timeout -k 10 300 python bench.py > $O/o_$rd.log 2>&1 || { tail -5 $O/o_$rd.log; exit 1; }
  echo "order1 r$rd $(b $O/o_$rd.log)"
done
