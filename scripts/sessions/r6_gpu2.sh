#!/bin/bash
# round 6 session 2: full GPU suite at the working tree (own-RCCL failure paths, PYTHONPATH-appending
# children), attention A/B of the softmax-priority (16) and forward-occupancy-3 (32) variants, attention
# LDS / issue PMC at HEAD, one default 1-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for v in x16 x32; do
  echo "== alt = ND_ATTN_X $v (speedup = alt/wt: >1 means the variant is SLOWER than the product build)"
  timeout -k 10 180 python -u scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_$v.so --what attnk --rounds 5 --iters 10 > $O/ab_$v.log 2>&1 || { tail -20 $O/ab_$v.log; exit 1; }
  grep attn_ $O/ab_$v.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o sq -- python3 scripts/attn_pmc.py --iters 3 > $O/pmc_sq.log 2>&1 || { tail -5 $O/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o lds -- python3 scripts/attn_pmc.py --iters 3 > $O/pmc_lds.log 2>&1 || { tail -5 $O/pmc_lds.log; exit 1; }
find $O/pmc -name "*counter_collection.csv" | sort
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 120 python -u scripts/attn_stamps.py --lib nanodiloco_amd/_lib/alt/libnd_kernels_stamp.so > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
