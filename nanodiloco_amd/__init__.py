"""nanodiloco_amd: an MI355X-native DiLoCo trainer (capabilities of SJCaldwell/NanoDiloco).

Importing the package is light (no transformers / datasets / wandb); the CLI lives in
``nanodiloco_amd.main``.
"""
__version__ = "0.1.0"

import os as _os

# HIP hardware queues per process, read once when the HIP runtime initialises (so: before the first GPU
# call).  The compute stream, the weight-gradient side stream and every communicator stream (c10d's and the
# own RCCL communicator's, plus RCCL's internal ones) should each own a queue: with HIP's default of 4 the
# communicators' streams share the compute streams' queues and the overlapped backward ran 2-6 % slower
# (bench.py one-rank group vs none: 330.6 / 340.6 vs 323.6 ms per step; with 16 queues 324.3 vs 323.8 --
# round 5, docs/DESIGN.md §4).  Raised only if lower; 16 stays far below the 32 the pool allows.
if int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    _os.environ["GPU_MAX_HW_QUEUES"] = "16"

from .config import LlamaConfig, load_config_from_file, default_llama_config, default_run_config  # noqa: E402
from .models import LlamaForCausalLM, ParamStore  # noqa: E402


def __getattr__(name):
    # Lazy exports so `import nanodiloco_amd` does not initialise torch.distributed machinery.
    if name == "Diloco":
        from .parallel.diloco import Diloco
        return Diloco
    if name == "main":
        from .main import main
        return main
    if name == "train_model":
        from .trainer import train_model
        return train_model
    raise AttributeError(name)


__all__ = ["LlamaConfig", "LlamaForCausalLM", "ParamStore", "Diloco", "main", "train_model", "load_config_from_file",
           "default_llama_config", "default_run_config"]
