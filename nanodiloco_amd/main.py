"""CLI entrypoint: ``python -m nanodiloco_amd`` (or ``-m nanodiloco_amd.main``) under torchrun.

Accepts exactly the reference's 13 kebab-case flags with the same defaults
(REF/nanodiloco/main.py:41-56; cyclopts derives them from ``train_model``'s kwargs) plus
non-breaking extensions.  Example (8 DiLoCo workers, one per MI355X):

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m nanodiloco_amd.main \
        --llama-config-file configs/llama_150m.json --inner-steps 100 --per-device-batch-size 64
"""
from __future__ import annotations

import argparse
import dataclasses
import sys
from typing import List, Optional

from .trainer import TrainArgs, Trainer


TRISTATE = {"hip_graph"}  # on | off | auto; the bare flag means "on"
AUTO_INT = {"per_device_batch_size"}  # an int or "auto"


def _int_or_auto(s: str):
    return "auto" if s.lower() == "auto" else int(s)


def _bool(s: str) -> bool:
    return s.lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="nanodiloco_amd", description="MI355X-native DiLoCo trainer")
    for f in dataclasses.fields(TrainArgs):
        flag = "--" + f.name.replace("_", "-")
        default = f.default
        if f.name in AUTO_INT:
            p.add_argument(flag, type=_int_or_auto, default=default)
        elif f.type in (bool, "bool"):
            p.add_argument(flag, type=_bool, nargs="?", const=True, default=default)
        elif f.type in (int, "int"):
            p.add_argument(flag, type=int, default=default)
        elif f.type in (float, "float"):
            p.add_argument(flag, type=float, default=default)
        elif f.name in TRISTATE:
            p.add_argument(flag, type=str, nargs="?", const="on", default=default)  # bare flag = on
        else:
            p.add_argument(flag, type=str, default=default)
    return p


def parse_args(argv: Optional[List[str]] = None) -> TrainArgs:
    ns = build_parser().parse_args(argv)
    return TrainArgs(**vars(ns))


def main(argv: Optional[List[str]] = None):
    from .parallel.dist import destroy_distributed

    print("Training Diloco with nanodiloco_amd...", flush=True)
    args = parse_args(argv if argv is not None else sys.argv[1:])
    try:
        Trainer(args).train()
    except BaseException:
        destroy_distributed(abort=True)
        raise
    destroy_distributed()


if __name__ == "__main__":
    main()
