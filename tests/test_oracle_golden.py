"""Pin the CPU oracle against HF-transformers golden fixtures (fp32), and
check its fp16 mode stays within the reference's half-precision tolerance.

HF transformers is the reference's own alignment oracle
(tests/inference/huggingface_inference.py; per-layer tolerance atol=1e-2 with
<=5% mismatches in tests/inference/inference_alignment_test.py:193-204).
"""
import numpy as np
import pytest

import oracle_lib as O

TAGS = ["tiny_d64", "tiny_d128"]


def test_weight_generator_matches_numpy_twin():
    from golden.gen_golden import gen_weight
    for name, kind in [("model.embed_tokens.weight", 0), ("model.norm.weight", 1),
                       ("model.layers.3.mlp.down_proj.weight", 0)]:
        a = O.gen_weight(name, 1234, kind, 4099)
        b = gen_weight(name, 1234, kind, 4099)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_f16_rounding_matches_numpy():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s
                        for s in (1e-7, 1e-5, 1e-3, 1.0, 1e3, 6e4)])
    x = np.concatenate([x, np.float32([65519.0, 65520.0, 7e4, 0.0, -0.0, 5.96e-8, 2.98e-8])])
    ours = np.array([O.lib().orc_f2h(float(v)) for v in x], np.uint16)
    ref = x.astype(np.float16).view(np.uint16)
    assert np.array_equal(ours, ref)


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_fp32_matches_hf_logits_and_hidden(tag):
    cfg, g = O.load_golden(tag)
    m = O.Model(cfg, cfg["seed"], fp16=0)
    prompt = g["prompt"]
    logits = m.forward(0, prompt, 0)
    np.testing.assert_allclose(logits, g["logits"], rtol=1e-4, atol=2e-5)
    L = cfg["num_layers"]
    for j in range(L):
        ours = m.hidden(j if j < L - 1 else L, len(prompt))
        np.testing.assert_allclose(ours, g["hidden"][j], rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_fp32_greedy_matches_hf(tag):
    cfg, g = O.load_golden(tag)
    m = O.Model(cfg, cfg["seed"], fp16=0)
    toks = m.greedy(0, g["prompt"], cfg["n_new"])
    assert toks.tolist() == g["greedy"].tolist()


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_fp16_within_half_tolerance(tag):
    # the reference's half-precision alignment bar: atol 1e-2 w/ <=5% mismatch
    cfg, g = O.load_golden(tag)
    m = O.Model(cfg, cfg["seed"], fp16=1)
    logits = m.forward(0, g["prompt"], 0)
    bad = np.abs(logits - g["logits"]) > 1e-2
    assert bad.mean() <= 0.05


def test_oracle_batched_decode_matches_per_request():
    cfg, g = O.load_golden("tiny_d64")
    m1 = O.Model(cfg, cfg["seed"], fp16=1, max_requests=3, max_seq=64)
    m2 = O.Model(cfg, cfg["seed"], fp16=1, max_requests=3, max_seq=64)
    prompts = [[1, 5, 9, 33], [1, 7], [1, 2, 3, 4, 5, 6]]
    for r, p in enumerate(prompts):
        m1.forward(r, p, 0)
        m2.forward(r, p, 0)
    nxt = [11, 12, 13]
    pos = [len(p) for p in prompts]
    lb = m1.decode_batch([0, 1, 2], nxt, pos)
    for r in range(3):
        ls = m2.forward(r, [nxt[r]], pos[r])
        np.testing.assert_array_equal(lb[r], ls[0])


# ------------------------------------------------- reference half compute type
def _np_dot_ref16(a, b, block):
    """numpy twin of the ORC_REF16 accumulator: per MMA step of `block`
    products, an fp32 sum added to a half accumulator with one rounding."""
    acc = np.float16(0)
    for k0 in range(0, len(a), block):
        s = np.float32(0)
        for x, y in zip(a[k0:k0 + block], b[k0:k0 + block]):
            s = np.float32(s + np.float32(x) * np.float32(y))
        acc = np.float16(np.float32(acc) + s)
    return np.float32(acc)


@pytest.mark.parametrize("block", [16, 32])
def test_ref16_linear_matches_numpy_twin(block):
    rng = np.random.default_rng(block)
    X = O.round16(rng.standard_normal((3, 200)))
    W = O.round16(rng.uniform(-0.1, 0.1, (5, 200)))
    O.set_ref_block(block)
    try:
        Y = O.linear(X, W, fp16=O.REF16)
    finally:
        O.set_ref_block(16)
    ref = np.array([[_np_dot_ref16(x, w, block) for w in W] for x in X], np.float32)
    assert np.array_equal(Y, ref)
    # the half accumulator is measurably coarser than fp32 accumulation
    assert not np.array_equal(Y, O.linear(X, W, fp16=1))


def test_ref16_prompt_attention_matches_numpy_twin():
    """inc_multihead_self_attention.cu:98-366: half(alpha16 * acc16(q.k)),
    causal -inf fill, half softmax, half-accumulated P.V."""
    rng = np.random.default_rng(7)
    d, start, T = 64, 3, 5
    nk = start + T
    q = O.round16(rng.standard_normal((T, d)))
    K = O.round16(rng.standard_normal((nk, d)))
    V = O.round16(rng.standard_normal((nk, d)))
    out = O.attention_prompt_ref16(q, K, V, start)
    alpha = np.float32(np.float16(1.0 / np.sqrt(np.float32(d))))
    for t in range(T):
        pos = start + t
        sc = np.array([np.float16(alpha * _np_dot_ref16(q[t], K[j], 16)) for j in range(pos + 1)],
                      np.float32)
        p = np.exp(sc - sc.max(), dtype=np.float32)
        p = np.concatenate([p / np.float32(p.astype(np.float64).sum()), np.zeros(nk - pos - 1,
                                                                                  np.float32)])
        p = O.round16(p)
        ref = np.array([_np_dot_ref16(p, V[:, i], 16) for i in range(d)], np.float32)
        np.testing.assert_array_equal(out[t], ref)


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_ref16_within_half_tolerance(tag):
    # the reference's own semantics (half compute type, prompt path) against
    # HF fp32 under its half-precision alignment bar
    cfg, g = O.load_golden(tag)
    m = O.Model(cfg, cfg["seed"], fp16=O.REF16)
    logits = m.forward_ex(0, g["prompt"], 0, 1)
    bad = np.abs(logits - g["logits"]) > 1e-2
    assert bad.mean() <= 0.05
    assert not np.array_equal(logits, O.Model(cfg, cfg["seed"], fp16=1).forward(0, g["prompt"], 0))


def test_oracle_forward_multi_equals_per_request_forwards():
    """orc_model_forward_multi (the CPU port of a verify / beam step used by
    bench.py's cpu_baseline) batches the dense layers over several requests'
    blocks: bit-identical to one orc_model_forward per request."""
    cfg = dict(num_layers=2, vocab_size=500, num_heads=4, num_kv_heads=4, hidden=128,
               intermediate=256, rms_eps=1e-6, rope_theta=10000.0)
    a = O.Model(cfg, 3, fp16=1, max_requests=3, max_seq=64)
    b = O.Model(cfg, 3, fp16=1, max_requests=3, max_seq=64)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(3, 500, size=n).astype(np.int32) for n in (9, 14, 5)]
    for r, p in enumerate(prompts):
        a.forward(r, p, 0)
        b.forward(r, p, 0)
    blocks = [rng.integers(3, 500, size=n).astype(np.int32) for n in (3, 1, 6)]
    ref = np.vstack([a.forward(r, blk, len(prompts[r])) for r, blk in enumerate(blocks)])
    got = b.forward_multi([0, 1, 2], [3, 1, 6], [len(p) for p in prompts], np.concatenate(blocks))
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))


def test_token_chain_init_scale_and_chain():
    """weight_init 2 (token chain, oracle.h orc_chain_embed_scale): the
    embedding scale keeps the chain's margin at depth and width -- 128 up to
    LLaMA-7B's residual noise, doubled per doubling beyond (65B: 512) -- and a
    small model's greedy pick at every position is perm^-1 of its input token,
    perm(v) = (7919 v + 17) mod vocab."""
    assert O.chain_embed_scale(2, 768, 3072) == 128.0  # LLaMA-68M
    assert O.chain_embed_scale(32, 4096, 11008) == 128.0  # 7B
    assert O.chain_embed_scale(80, 8192, 22016) == 512.0  # 65B
    assert O.chain_embed_scale(33, 4096, 11008) == 256.0
    cfg = dict(num_layers=2, vocab_size=500, num_heads=4, num_kv_heads=4, hidden=128,
               intermediate=256, rms_eps=1e-6, rope_theta=10000.0)
    m = O.Model(cfg, 3, fp16=1, max_requests=1, max_seq=64, weight_init=2)
    toks = np.random.default_rng(1).integers(3, 500, size=40).astype(np.int32)
    ids, _ = O.softmax_argmax(m.forward(0, toks, 0))
    inv = {(7919 * v + 17) % 500: v for v in range(500)}
    assert [inv[int(t)] for t in toks] == ids.tolist()
