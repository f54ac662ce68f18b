#!/bin/bash
# round 5: (1) serial kernel profile of the bench step with / without the one-rank process group;
# (2) dswiglu epilogue prefetch depth A/B (PF 6 = working tree vs 8 / 10)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
for arm in none rccl; do
  args=""; [ $arm = none ] && args="--backend none"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$arm -o run -- python3 bench.py --steps 3 --warmup 1 --wgrad-overlap 0 $args > $O/prof_$arm.log 2>&1 || { tail -5 $O/prof_$arm.log; exit 1; }
  tail -1 $O/prof_$arm.log | cut -c1-160
done
for pf in 8 10; do
  timeout -k 10 300 python scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_pf$pf.so --what epi --rounds 5 > $O/epi_pf$pf.log 2>&1 || { tail -5 $O/epi_pf$pf.log; exit 1; }
  echo "alt = PF $pf"; grep "dswiglu\|down_dgrad" $O/epi_pf$pf.log
done
