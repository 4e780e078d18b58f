"""Generate golden fixtures with HF transformers (the reference's own alignment
oracle: tests/inference/huggingface_inference.py, inference_alignment_test.py).

Run HERE only (needs transformers + torch CPU; /root/reference is not read).
The fixtures (small .npz, arrays only) are committed; tests load them with
numpy.load(allow_pickle=False).

Weights are not stored: both this script and the oracle / GPU generator derive
every tensor from the same counter-based splitmix64 spec (see
oracle/oracle.h: orc_gen_weight), so a fixture is (config, seed, prompt) ->
(greedy tokens, logits, per-layer hidden states).

    python tests/golden/gen_golden.py
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

M64 = (1 << 64) - 1
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
C1 = np.uint64(0xBF58476D1CE4E5B9)
C2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(s: str) -> int:
    h = 1469598103934665603
    for b in s.encode():
        h ^= b
        h = (h * 1099511628211) & M64
    return h


def gen_weight(name: str, seed: int, kind: int, n: int) -> np.ndarray:
    """numpy twin of orc_gen_weight (bit-identical fp32 values)."""
    key = np.uint64((seed ^ fnv1a64(name)) & M64)
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = key + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * C1
        z = (z ^ (z >> np.uint64(27))) * C2
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    t = np.float32(2.0) * u - np.float32(1.0)
    center, amp = (np.float32(1.0), np.float32(0.1)) if kind == 1 else (
        np.float32(0.0), np.float32(0.034641016))
    return (center + t * amp).astype(np.float32)


CONFIGS = {
    # d = 64 (tree / spec / inc all supported by the reference for d=64)
    "tiny_d64": dict(num_layers=2, vocab_size=512, num_heads=2, num_kv_heads=2,
                     hidden=128, intermediate=256, rms_eps=1e-6,
                     rope_theta=10000.0, seed=20250117, prompt_len=12, n_new=16),
    # d = 128 (LLaMA-7B/65B head size)
    "tiny_d128": dict(num_layers=2, vocab_size=1000, num_heads=2, num_kv_heads=2,
                      hidden=256, intermediate=512, rms_eps=1e-6,
                      rope_theta=10000.0, seed=11, prompt_len=9, n_new=16),
}


def build_hf(cfg):
    import torch
    from transformers import LlamaConfig, LlamaForCausalLM

    hc = LlamaConfig(vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden"],
                     intermediate_size=cfg["intermediate"],
                     num_hidden_layers=cfg["num_layers"],
                     num_attention_heads=cfg["num_heads"],
                     num_key_value_heads=cfg["num_kv_heads"],
                     rms_norm_eps=cfg["rms_eps"], rope_theta=cfg["rope_theta"],
                     max_position_embeddings=512, tie_word_embeddings=False,
                     attention_bias=False, mlp_bias=False)
    hc._attn_implementation = "eager"
    model = LlamaForCausalLM(hc).float().eval()
    sd = model.state_dict()
    seed = cfg["seed"]
    new = {}
    for name, t in sd.items():
        kind = 1 if name.endswith("norm.weight") else 0
        w = gen_weight(name, seed, kind, t.numel()).reshape(tuple(t.shape))
        new[name] = torch.from_numpy(w)
    model.load_state_dict(new)
    return model


def make_prompt(cfg):
    # BOS(1) + ids uniform in [3, vocab) from numpy default_rng(seed) (bench.py
    # uses splitmix64 for its 128-token prompts; fixtures only need determinism)
    rng = np.random.default_rng(cfg["seed"])
    ids = rng.integers(3, cfg["vocab_size"], size=cfg["prompt_len"] - 1)
    return np.concatenate([[1], ids]).astype(np.int32)


def main():
    import torch

    torch.manual_seed(0)
    for tag, cfg in CONFIGS.items():
        model = build_hf(cfg)
        prompt = make_prompt(cfg)
        with torch.no_grad():
            out = model(torch.from_numpy(prompt[None].astype(np.int64)),
                        output_hidden_states=True)
            logits = out.logits[0].float().numpy()
            hidden = np.stack([h[0].float().numpy() for h in out.hidden_states[1:]])
            seq = list(prompt.tolist())
            for _ in range(cfg["n_new"]):
                lg = model(torch.tensor([seq])).logits[0, -1]
                seq.append(int(torch.argmax(lg)))
        greedy = np.array(seq[len(prompt):], dtype=np.int32)
        path = os.path.join(HERE, f"{tag}.npz")
        np.savez_compressed(path, config=np.array(json.dumps(cfg)),
                            prompt=prompt, greedy=greedy,
                            logits=logits.astype(np.float32),
                            hidden=hidden.astype(np.float32))
        print(tag, "greedy:", greedy.tolist())


if __name__ == "__main__":
    main()
