"""nanodiloco_amd: an MI355X-native DiLoCo trainer (capabilities of SJCaldwell/NanoDiloco).

Importing the package is light (no transformers / datasets / wandb); the CLI lives in
``nanodiloco_amd.main``.
"""
__version__ = "0.1.0"

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
