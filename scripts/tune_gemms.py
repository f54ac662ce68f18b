#!/usr/bin/env python3
"""Tune the library GEMMs of the training step with PyTorch TunableOp and write the winners to
nanodiloco_amd/tuning/tunableop_gfx950.csv (loaded at start-up by ops.tuned_gemm).

Runs forward + backward of each listed (model, micro-batch) configuration once with tuning on, so
every projection / lm-head GEMM shape the trainer and bench.py issue is searched.  One GPU, a few
minutes.  Usage:  python scripts/tune_gemms.py [llama_150m.json:32 llama_150m.json:8 ...]
(FP8=1: build the models with --fp8 projections, so the hipBLASLt fp8 GEMMs are tuned too.)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.config import resolve_llama_config  # noqa: E402
from nanodiloco_amd.models import LlamaForCausalLM  # noqa: E402
from nanodiloco_amd.ops.tuned_gemm import DEFAULT_FILE  # noqa: E402


def main():
    specs = sys.argv[1:] or ["llama_150m.json:32", "llama_150m.json:8", "llama_1b.json:32"]
    seq = int(os.environ.get("SEQ", 1024))
    out = os.environ.get("OUT", DEFAULT_FILE)
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_max_tuning_duration(int(os.environ.get("MAX_MS", 40)))
    tunable.set_filename(out)
    ops.set_backend("hip")
    for spec in specs:
        name, mb = spec.split(":")
        cfg = resolve_llama_config(name)
        t0 = time.time()
        fp8 = os.environ.get("FP8", "0") == "1"  # also tune the fp8 projections' _scaled_mm (ScaledGemm)
        m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=fp8).init_weights(0)
        ids = torch.randint(0, cfg.vocab_size, (int(mb), seq), device="cuda")
        o = m(ids, labels=ids)
        o.loss.backward()
        torch.cuda.synchronize()
        print(f"tuned {spec} in {time.time() - t0:.0f}s", flush=True)
        del m, o
        torch.cuda.empty_cache()
    print("tuned", len(tunable.get_results()), "GEMM shapes; TunableOp writes", out, "at exit")


if __name__ == "__main__":
    main()
