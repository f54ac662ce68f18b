#!/usr/bin/env python3
"""Cluster launcher: the capability equivalent of the reference's Modal entrypoints
(REF/scripts/train_modal.py:246-282 -- small_single_node, large_multi_node, benchmark, main;
prepare_configs :184-242), for MI355X nodes driven by plain torchrun (no Modal / cloud SDK).

  python scripts/launch.py prepare-configs --out configs/generated
  python scripts/launch.py small-single-node                      # all local GPUs, bs 128, lr 1e-3, 5000 steps
  python scripts/launch.py large-multi-node --nnodes 2 --node-rank 0 --master-addr 10.0.0.1
  python scripts/launch.py benchmark --nnodes 1                   # 200 steps, JSONL metrics with comm timings
  python scripts/launch.py main --fault-tolerant --min-nodes 1    # restarts + elastic worker count (below)

Fault tolerance: ``--fault-tolerant`` adds ``--max-restarts`` (default 3) and makes the trainer
checkpoint every outer step into ``--checkpoint-dir`` and restart with ``--resume auto`` (the newest COMPLETE
checkpoint).  ``--min-nodes M`` (< ``--nnodes``) switches torchrun to an elastic c10d rendezvous
(``--nnodes M:N``) and the trainer to ``--elastic-resume``: after a lost node the job continues on the
surviving DiLoCo workers.  ``--dry-run`` prints the command only.

Every subcommand starts ``torchrun ... -m nanodiloco_amd`` as a child process and exits with its code.
Extra arguments after ``--`` are forwarded to the trainer.  (The reference's multi-node path passes
an invalid ``--steps`` flag; here it is ``--total-steps``.)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LLAMA_DEFAULT = {"architectures": ["LlamaForCausalLM"], "hidden_size": 128, "intermediate_size": 512,
                 "num_attention_heads": 4, "num_hidden_layers": 6, "rms_norm_eps": 1e-05, "use_cache": False}
LLAMA_LARGE = {"architectures": ["LlamaForCausalLM"], "hidden_size": 256, "intermediate_size": 1024,
               "num_attention_heads": 8, "num_hidden_layers": 12, "rms_norm_eps": 1e-05, "use_cache": False}
RUN_DEFAULT = {"nodes": 2, "location": "mi355x", "backend": "nccl", "measure_comms": True}


def prepare_configs(out_dir: str):
    os.makedirs(out_dir, exist_ok=True)
    for name, cfg in (("llama_default.json", LLAMA_DEFAULT), ("llama_large.json", LLAMA_LARGE),
                      ("wandb_default.json", RUN_DEFAULT)):
        with open(os.path.join(out_dir, name), "w") as f:
            json.dump(cfg, f, indent=2)
    print(f"configs written to {out_dir}")


def _gpus() -> int:
    try:
        import torch
        return max(1, torch.cuda.device_count())
    except Exception:
        return 1


def torchrun_cmd(a, trainer_args):
    elastic = bool(a.min_nodes) and a.min_nodes < a.nnodes
    restarts = a.max_restarts if a.max_restarts is not None else (3 if (a.fault_tolerant or elastic) else 0)
    nnodes = f"{a.min_nodes}:{a.nnodes}" if elastic else str(a.nnodes)
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nnodes={nnodes}",
           f"--nproc-per-node={a.nproc_per_node or _gpus()}", f"--max-restarts={restarts}"]
    if elastic:  # the worker count may change between restarts: c10d rendezvous, no fixed node rank
        cmd += ["--rdzv-backend=c10d", f"--rdzv-endpoint={a.master_addr}:{a.master_port}", f"--rdzv-id={a.run_id}"]
    elif a.nnodes > 1:
        cmd += [f"--node-rank={a.node_rank}", f"--master-addr={a.master_addr}", f"--master-port={a.master_port}"]
    else:
        cmd += ["--master-addr=127.0.0.1", f"--master-port={a.master_port}"]
    extra = []
    if a.fault_tolerant or elastic:
        ck = a.checkpoint_dir or os.path.join(ROOT, "runs", f"{a.cmd}_ckpt")
        extra = ["--checkpoint-dir", ck, "--checkpoint-every", "1", "--resume", "auto"]
        if elastic:
            extra += ["--elastic-resume", "true"]
    return cmd + ["-m", "nanodiloco_amd"] + trainer_args + extra + a.extra


def _torchrun(a, trainer_args):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    cmd = torchrun_cmd(a, trainer_args)
    print("+", " ".join(cmd), flush=True)
    if a.dry_run:
        return 0
    return subprocess.call(cmd, cwd=ROOT, env=env)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    pc = sub.add_parser("prepare-configs")
    pc.add_argument("--out", default=os.path.join(ROOT, "configs", "generated"))
    for name in ("small-single-node", "large-multi-node", "benchmark", "main"):
        p = sub.add_parser(name)
        p.add_argument("--nnodes", type=int, default=1 if name == "small-single-node" else 2)
        p.add_argument("--node-rank", type=int, default=int(os.environ.get("NODE_RANK", 0)))
        p.add_argument("--master-addr", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
        p.add_argument("--master-port", type=int, default=int(os.environ.get("MASTER_PORT", 29500)))
        p.add_argument("--nproc-per-node", type=int, default=0)
        p.add_argument("--max-restarts", type=int, default=None, help="torchrun restarts (default 0; 3 with --fault-tolerant)")
        p.add_argument("--fault-tolerant", action="store_true",
                       help="checkpoint every outer step and restart from the newest complete checkpoint")
        p.add_argument("--min-nodes", type=int, default=0, help="elastic: continue with as few as this many nodes")
        p.add_argument("--checkpoint-dir", default=None)
        p.add_argument("--run-id", default="nanodiloco")
        p.add_argument("--dry-run", action="store_true", help="print the torchrun command only")
        p.add_argument("--llama-config", default=os.path.join(ROOT, "configs", "llama_default.json"))
        p.add_argument("--run-config", default=os.path.join(ROOT, "configs", "wandb_default.json"))
        p.add_argument("--dataset-path", default="/vol/datasets/PrimeIntellect/c4-tiny/en/save_to_disk")
        p.add_argument("extra", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    if a.cmd == "prepare-configs":
        return prepare_configs(a.out)
    if a.extra and a.extra[0] == "--":
        a.extra = a.extra[1:]
    common = ["--llama-config-file", a.llama_config, "--wandb-config-file", a.run_config,
              "--dataset-path", a.dataset_path]
    if a.cmd == "small-single-node":      # REF train_modal.py:246-255
        args = common + ["--batch-size=128", "--lr=1e-3", "--total-steps=5000"]
    elif a.cmd == "large-multi-node":     # REF :258-267
        args = common + ["--batch-size=1024", "--lr=4e-4", "--total-steps=10000"]
    elif a.cmd == "benchmark":            # REF :164-181 (200 steps), with real comm metrics
        args = common + ["--batch-size=512", "--lr=4e-4", "--total-steps=200", "--log-file",
                         os.path.join(ROOT, "runs", "benchmark.jsonl")]
    else:                                 # REF :276-282
        args = common + ["--batch-size=512", "--lr=4e-4", "--total-steps=10000"]
    sys.exit(_torchrun(a, args))


if __name__ == "__main__":
    main()
