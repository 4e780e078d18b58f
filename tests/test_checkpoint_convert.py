"""convert_hf_model (python/flexflow/serve/models/llama.py:274-285 restated)
writes the reference's per-tensor files from an HF LlamaForCausalLM, and
llama_config_from_hf reads its config.json (llama.h:30-79).  CPU only; the
GPU side loads the same files (test_gpu_checkpoint.py).

The HF model lives in a child process: torch brings its own HIP runtime,
and two HIP runtimes in one process abort at exit.
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import flexflow_amd as fa
from test_gpu_checkpoint import CFG, SEED, seeded_state

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys
    import numpy as np
    import torch
    import transformers
    from flexflow_amd.checkpoint import convert_hf_model
    cfg, src, dst = eval(sys.argv[1]), sys.argv[2], sys.argv[3]
    hf_cfg = transformers.LlamaConfig(
        vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden"],
        intermediate_size=cfg["intermediate"], num_hidden_layers=cfg["num_layers"],
        num_attention_heads=cfg["num_heads"], num_key_value_heads=cfg["num_kv_heads"],
        rms_norm_eps=cfg["rms_eps"], rope_theta=cfg["rope_theta"], tie_word_embeddings=False)
    hf = transformers.LlamaForCausalLM(hf_cfg)
    st = dict(np.load(src))
    with torch.no_grad():
        for n, p in hf.named_parameters():
            p.copy_(torch.from_numpy(st[n]))
    convert_hf_model(hf, dst)
    hf_cfg.save_pretrained(dst)
""")


def test_hf_model_conversion_writes_the_reference_files(tmp_path):
    pytest.importorskip("transformers")
    st = seeded_state(CFG, SEED)
    np.savez(tmp_path / "st.npz", **st)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", CHILD, repr(CFG), str(tmp_path / "st.npz"),
                        str(tmp_path / "hf")], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    want = fa.convert_hf_model(st, str(tmp_path / "st"))
    got = sorted(f for f in os.listdir(tmp_path / "hf") if f.endswith(".weight"))
    assert got == sorted(want)
    assert "embed_tokens.weight" in got and "layers.0.self_attn.q_proj.weight" in got
    for name in want:
        a = np.fromfile(tmp_path / "hf" / name, np.uint16)
        b = np.fromfile(tmp_path / "st" / name, np.uint16)
        assert np.array_equal(a, b), name
    assert fa.llama_config_from_hf(str(tmp_path / "hf")) == CFG


@pytest.mark.parametrize("kind", ["linear", "dynamic", "yarn"])
def test_unsupported_rope_scaling_is_rejected(kind):
    """Only plain and llama3 RoPE exist in the reference
    (inc_multihead_self_attention.cu:703-722): another scaling type must fail
    loudly instead of loading unscaled."""
    hf = dict(num_attention_heads=4, num_hidden_layers=1, vocab_size=64, hidden_size=64,
              intermediate_size=128, rms_norm_eps=1e-6, rope_theta=10000.0,
              rope_scaling={"rope_type": kind, "factor": 2.0})
    with pytest.raises(ValueError, match="rope scaling"):
        fa.llama_config_from_hf(hf)
    hf["rope_scaling"] = {"rope_type": "default"}
    assert "rope_llama3" not in fa.llama_config_from_hf(hf)
