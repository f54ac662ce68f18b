#!/bin/bash
# round 5: in-step sweep of the existing launch-time knobs at HEAD (2 interleaved rounds, bf16 bench, 8 steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5t
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
arms=("default|" "gm1|ND_GEMM_PP_GM=1" "gm2|ND_GEMM_PP_GM=2" "gm8|ND_GEMM_PP_GM=8" "attn_order0|ND_ATTN_ORDER=0"
      "thr4|ND_ATTN_THR=4" "thr12|ND_ATTN_THR=12" "ppvar32|ND_GEMM_PP_VARIANT=32" "ppvar1024|ND_GEMM_PP_VARIANT=1024"
      "mb64|MB=64" "ovl2|OVL=2")
for rd in 1 2; do
  for a in "${arms[@]}"; do
    name=${a%%|*}; envs=${a#*|}
    extra=""
    case "$envs" in MB=*) extra="--micro-batch ${envs#MB=}"; envs="";; OVL=*) extra="--wgrad-overlap ${envs#OVL=}"; envs="";; esac
    env $envs timeout -k 10 200 python bench.py --steps 8 --warmup 2 $extra > $O/${name}_$rd.log 2>&1 || { tail -5 $O/${name}_$rd.log; exit 1; }
    echo "$name r$rd $(tail -1 $O/${name}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
