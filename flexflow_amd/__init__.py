"""flexflow_amd -- MI355X-native SpecInfer hot path (libffmi.so).

Import order matters on ROCm: load libffmi.so before torch so both share one
HIP runtime (same SONAME libamdhip64.so.7).
"""
from . import ffmi  # noqa: F401
from .checkpoint import convert_hf_model, llama_config_from_hf  # noqa: F401
from .serve import (Comm, GenerationResult, HashModel, Model, RequestManager,  # noqa: F401
                    generate, set_device)
from .tokenizer import LlamaTokenizer, load_tokenizer  # noqa: F401

__all__ = ["ffmi", "convert_hf_model", "llama_config_from_hf", "Comm", "GenerationResult", "HashModel", "Model", "RequestManager",
           "generate", "set_device", "LlamaTokenizer", "load_tokenizer"]
