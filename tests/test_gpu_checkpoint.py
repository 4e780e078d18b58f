"""Checkpoints in the reference's format (file_loader.cc:217-389; one raw
file per HF tensor as convert_hf_model writes them) load into the GPU model.

Pinned against the seeded synthetic path, which the oracle and the HF
golden fixtures pin: the same tensors written as fp16 files or as fp32 files
must give bit-identical tokens.  (That convert_hf_model of an HF
LlamaForCausalLM writes exactly these files is a CPU test,
test_checkpoint_convert.py: torch must not share this process with libffmi.)  A GQA checkpoint (2 KV heads) must equal the
MHA checkpoint with those K/V heads replicated (file_loader.cc:292-302).
"""
import os

import numpy as np
import pytest

import flexflow_amd as fa
import oracle_lib as O

pytestmark = pytest.mark.gpu

CFG = dict(num_layers=2, vocab_size=1000, num_heads=4, num_kv_heads=4, hidden=256,
           intermediate=512, rms_eps=1e-6, rope_theta=10000.0)
SEED = 31


def tensor_names(cfg):
    H, F, V = cfg["hidden"], cfg["intermediate"], cfg["vocab_size"]
    out = [("model.embed_tokens.weight", (V, H), 0), ("model.norm.weight", (H,), 1),
           ("lm_head.weight", (V, H), 0)]
    for l in range(cfg["num_layers"]):
        p = f"model.layers.{l}."
        out += [(p + "input_layernorm.weight", (H,), 1),
                (p + "post_attention_layernorm.weight", (H,), 1)]
        out += [(p + f"self_attn.{x}_proj.weight", (H, H), 0) for x in "qkvo"]
        out += [(p + "mlp.gate_proj.weight", (F, H), 0), (p + "mlp.up_proj.weight", (F, H), 0),
                (p + "mlp.down_proj.weight", (H, F), 0)]
    return out


def seeded_state(cfg, seed):
    return {n: O.gen_weight(n, seed, kind, int(np.prod(shape))).reshape(shape)
            for n, shape, kind in tensor_names(cfg)}


def run(cfg, prompts, **kw):
    rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=64,
                           max_sequence_length=128)
    m = fa.Model(cfg, "inc", max_requests=4, max_tokens=64, max_seq_len=128, **kw)
    res = fa.generate(rm, m, prompts, max_length=48)
    m.close()
    return [r.output_tokens for r in res]


def prompts(seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(3, 1000, size=int(rng.integers(5, 20))).tolist() for _ in range(3)]


@pytest.mark.parametrize("dtype", [np.float16, np.float32])
def test_reference_format_folder_equals_synthetic_weights(tmp_path, dtype):
    st = seeded_state(CFG, SEED)
    names = fa.convert_hf_model(st, str(tmp_path), dtype=dtype)
    assert "layers.1.mlp.down_proj.weight" in names and "lm_head.weight" in names
    assert os.path.getsize(tmp_path / "embed_tokens.weight") == 1000 * 256 * np.dtype(dtype).itemsize
    ps = prompts(1)
    assert run(CFG, ps, weights_folder=str(tmp_path)) == run(CFG, ps, weight_seed=SEED)


def test_gqa_checkpoint_equals_replicated_mha(tmp_path):
    gqa = dict(CFG, num_kv_heads=2)
    st = seeded_state(CFG, SEED)
    d = CFG["hidden"] // CFG["num_heads"]
    st_gqa = dict(st)
    for l in range(CFG["num_layers"]):
        for x in "kv":
            n = f"model.layers.{l}.self_attn.{x}_proj.weight"
            st_gqa[n] = st[n][:2 * d]          # kv heads 0, 1
            rep = np.concatenate([st[n][:d], st[n][:d], st[n][d:2 * d], st[n][d:2 * d]])
            st[n] = rep                         # query heads 0,1 -> kv 0; 2,3 -> kv 1
    fa.convert_hf_model(st_gqa, str(tmp_path / "gqa"))
    fa.convert_hf_model(st, str(tmp_path / "mha"))
    ps = prompts(3)
    assert run(gqa, ps, weights_folder=str(tmp_path / "gqa")) == \
        run(CFG, ps, weights_folder=str(tmp_path / "mha"))


def test_missing_or_truncated_file_fails_loudly(tmp_path):
    st = seeded_state(CFG, SEED)
    fa.convert_hf_model(st, str(tmp_path))
    os.remove(tmp_path / "layers.1.mlp.up_proj.weight")
    with pytest.raises(fa.ffmi.FFMIError, match="up_proj"):
        fa.Model(CFG, "inc", max_requests=2, max_tokens=16, max_seq_len=64,
                 weights_folder=str(tmp_path))
    fa.convert_hf_model(st, str(tmp_path))
    with open(tmp_path / "norm.weight", "r+b") as f:
        f.truncate(100)
    with pytest.raises(fa.ffmi.FFMIError, match="norm.weight"):
        fa.Model(CFG, "inc", max_requests=2, max_tokens=16, max_seq_len=64,
                 weights_folder=str(tmp_path))


def test_full_precision_checkpoint_equals_synthetic(tmp_path):
    """--use-full-precision loads the fp32 files as they are (file_loader.cc
    with DT_FLOAT): the fp32 model from the folder gives the same tokens as
    the seeded fp32 model (identical weights, identical arithmetic), and a GQA
    folder equals its replicated MHA twin"""
    st = seeded_state(CFG, SEED)
    fa.convert_hf_model(st, str(tmp_path / "mha"), dtype=np.float32)
    ps = prompts(5)
    a = run(CFG, ps, weights_folder=str(tmp_path / "mha"), full_precision=True)
    assert a == run(CFG, ps, weight_seed=SEED, full_precision=True)
    d = CFG["hidden"] // CFG["num_heads"]
    st_gqa = dict(st)
    for l in range(CFG["num_layers"]):
        for x in "kv":
            n = f"model.layers.{l}.self_attn.{x}_proj.weight"
            st_gqa[n] = st[n][:2 * d]
            st[n] = np.concatenate([st[n][:d], st[n][:d], st[n][d:2 * d], st[n][d:2 * d]])
    fa.convert_hf_model(st_gqa, str(tmp_path / "gqa"), dtype=np.float32)
    fa.convert_hf_model(st, str(tmp_path / "rep"), dtype=np.float32)
    assert run(dict(CFG, num_kv_heads=2), ps, weights_folder=str(tmp_path / "gqa"),
               full_precision=True) == run(CFG, ps, weights_folder=str(tmp_path / "rep"),
                                           full_precision=True)
