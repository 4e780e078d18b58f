"""Checkpoints in the reference's on-disk format.

The reference serves LLaMA from a folder of raw tensors, one file per HF
parameter, written by FlexFlowLLAMA.convert_hf_model
(python/flexflow/serve/models/llama.py:274-285: the HF name without "model.",
numpy ``tofile`` of the tensor, plus ``lm_head.weight``) and read by
FileDataLoader (src/runtime/file_loader.cc:217-361, 363-389).  The model
config comes from the HF ``config.json`` (inference/models/llama.h:30-79).
``Model(..., weights_folder=...)`` loads such a folder in the C++ runtime.
"""
import json
import os
from typing import Mapping, Union

import numpy as np


def convert_hf_weight_name(name: str) -> str:
    """llama.py:274-275."""
    return name.replace("model.", "")


def convert_hf_model(model_or_state_dict, dst_folder: str, dtype=np.float16) -> list:
    """Write every parameter as one raw file (llama.py:277-285).

    Accepts an HF ``LlamaForCausalLM`` (anything with ``named_parameters``
    and an ``lm_head``) or a mapping name -> array.  ``dtype`` is the file
    element type (fp16 as the reference's half-precision serving uses, or
    fp32; the loader takes either).  Returns the written file names."""
    os.makedirs(dst_folder, exist_ok=True)
    if hasattr(model_or_state_dict, "named_parameters"):
        items = [(n, p.detach().cpu().float().numpy())
                 for n, p in model_or_state_dict.named_parameters()]
        lm = getattr(model_or_state_dict, "lm_head", None)
        if lm is not None:
            items.append(("lm_head.weight", lm.weight.detach().cpu().float().numpy()))
    else:
        items = [(n, np.asarray(v)) for n, v in model_or_state_dict.items()]
    written = []
    for name, arr in dict(items).items():  # (lm_head may appear twice)
        fname = convert_hf_weight_name(name)
        np.ascontiguousarray(arr, dtype=dtype).tofile(os.path.join(dst_folder, fname))
        written.append(fname)
    return written


def llama_config_from_hf(src: Union[str, Mapping]) -> dict:
    """LLAMAConfig (llama.h:30-79) from an HF config.json path, a folder
    holding one, or an already-parsed dict."""
    if isinstance(src, str):
        path = os.path.join(src, "config.json") if os.path.isdir(src) else src
        with open(path) as f:
            src = json.load(f)
    c = dict(src)
    heads = int(c["num_attention_heads"])
    # newer HF configs keep theta and the scaling under "rope_parameters"
    rp = c.get("rope_parameters") if isinstance(c.get("rope_parameters"), Mapping) else {}
    theta = c.get("rope_theta", rp.get("rope_theta", 10000.0))
    cfg = dict(num_layers=int(c["num_hidden_layers"]), vocab_size=int(c["vocab_size"]),
               num_heads=heads, num_kv_heads=int(c.get("num_key_value_heads") or heads),
               hidden=int(c["hidden_size"]), intermediate=int(c["intermediate_size"]),
               rms_eps=float(c["rms_norm_eps"]), rope_theta=float(theta))
    # llama3 RoPE scaling: the reference reads it under "scaling_factor",
    # HF configs under "rope_scaling" or "rope_parameters"
    sc = c.get("scaling_factor") or c.get("rope_scaling") or rp
    kind = sc.get("rope_type", sc.get("type")) if isinstance(sc, Mapping) else None
    if kind not in (None, "default", "llama3"):
        # the reference applies only plain and llama3 RoPE (inc_multihead_self_attention.cu:
        # 703-722); loading another scaling (linear, dynamic, yarn, ...) unscaled would
        # decode wrongly without any error
        raise ValueError(f"unsupported rope scaling type {kind!r} (supported: default, llama3)")
    if kind == "llama3":
        cfg.update(rope_llama3=1, rope_factor=float(sc["factor"]),
                   rope_low_freq_factor=float(sc["low_freq_factor"]),
                   rope_high_freq_factor=float(sc["high_freq_factor"]),
                   rope_original_max_pos=int(sc["original_max_position_embeddings"]))
    return cfg
