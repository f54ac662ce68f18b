#!/bin/bash
# round 5: TunableOp at 131k tokens with a 1 GiB rotating buffer (cold operands, as in the step), then the check
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ae
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=1024 PYTORCH_TUNABLEOP_VERBOSE=1 OUT=$PWD/$O/tuned.csv MAX_MS=100 timeout -k 10 900 python scripts/tune_gemms.py llama_150m.json:128 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep -v Validator $O/tuned.csv
python3 - <<'PY'
O = "gpurun_out/r5ae"
base = open("nanodiloco_amd/tuning/tunableop_gfx950.csv").read().splitlines()
new = open(O + "/tuned.csv").read().splitlines()
have = {l.split(",")[1] for l in base if l.startswith("Gemm")}
add = [l for l in new if l.startswith("Gemm") and "131072" in l and l.split(",")[1] not in have]
open(O + "/merged.csv", "w").write("\n".join(base + add) + "\n")
PY
timeout -k 10 300 python scripts/tuned_check.py $O/merged.csv > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
grep -v amdgpu.ids $O/check.log | grep -v "^\[("
