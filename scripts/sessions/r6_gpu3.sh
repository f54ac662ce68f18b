#!/bin/bash
# round 6 session 3: dK/dV stamps with the DMA issue split (Q/dO pieces vs statistics), with the key blocks of one
# head grouped on an XCD (ND_ATTN_DKDV_ORDER=1) and with the next tile's pieces spread over the steps
# (ND_ATTN_X=128); kernel A/B of the spread (x128) and of the just-in-time-fragment 3-wave dK/dV (x64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
A=nanodiloco_amd/_lib/alt
timeout -k 10 120 python -u scripts/attn_stamps.py --lib $A/libnd_kernels_stamp.so > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
ND_ATTN_DKDV_ORDER=1 timeout -k 10 120 python -u scripts/attn_stamps.py --lib $A/libnd_kernels_stamp.so > $O/stamps_order1.log 2>&1 || { tail -20 $O/stamps_order1.log; exit 1; }
echo "== ND_ATTN_DKDV_ORDER=1"; grep -A11 dkdv $O/stamps_order1.log
timeout -k 10 120 python -u scripts/attn_stamps.py --lib $A/libnd_kernels_stamp128.so > $O/stamps_spread.log 2>&1 || { tail -20 $O/stamps_spread.log; exit 1; }
echo "== spread"; grep -A11 dkdv $O/stamps_spread.log
for v in x128 x64; do
  echo "== alt = ND_ATTN_X $v (speedup = alt/wt: >1 means the variant is SLOWER than the product build)"
  timeout -k 10 180 python -u scripts/ab_kernels.py --alt $A/libnd_kernels_$v.so --what attnk --rounds 5 --iters 10 > $O/ab_$v.log 2>&1 || { tail -20 $O/ab_$v.log; exit 1; }
  grep attn_ $O/ab_$v.log
done
