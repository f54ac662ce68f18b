from .param_store import ParamStore
from .llama import LlamaForCausalLM, CausalLMOutput

__all__ = ["ParamStore", "LlamaForCausalLM", "CausalLMOutput"]
