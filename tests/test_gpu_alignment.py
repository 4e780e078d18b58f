"""Model-level alignment on the GPU: per-layer hidden states and logits of the
MI355X path against HF transformers (the reference's own alignment oracle)
and against the CPU oracle, and greedy tokens against the reference's half
compute-type semantics.

Rules:
- vs HF fp32 (tests/golden): the reference's half-precision alignment bar,
  atol 1e-2 with <= 5% of elements outside it
  (tests/inference/inference_alignment_test.py:193-204);
- vs the oracle's fp16 mode (same rounding points, fp32 accumulation in a
  different order): logits within 2 fp16 ulp or 2e-3 absolute on >= 99.9% of
  elements;
- vs the oracle's ORC_REF16 mode (the reference's cuBLAS half compute type in
  every dense layer and its cuBLAS/cuDNN prompt attention): the GPU path
  accumulates in fp32, so greedy tokens are compared teacher-forced and the
  agreement bound is the measured one, stated in each test.

Measured fractions are appended to gpurun_out/parity_report.jsonl.
"""
import os

import numpy as np
import pytest

import flexflow_amd as fa
import oracle_lib as O
from hip_util import report, ulp_diff

pytestmark = pytest.mark.gpu

TAGS = ["tiny_d64", "tiny_d128"]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))




def prefill_capture(cfg, seed, prompt, mode="inc", **kw):
    """One prefill step of `prompt` (BOS first) with tensor capture; returns
    the model (captured tensors of that step)."""
    n = len(prompt)
    rm = fa.RequestManager(max_requests_per_batch=1, max_tokens_per_batch=max(16, n),
                           max_sequence_length=max(64, n + 2))
    m = fa.Model(cfg, mode, max_requests=1, max_tokens=max(16, n), max_seq_len=max(64, n + 2),
                 weight_seed=seed, **kw)
    m.set_debug(True)
    fa.generate(rm, m, [list(prompt[1:])], max_length=n + 1)
    return m


def half_alignment(ours, ref, atol=1e-2, frac=0.05):
    bad = np.abs(ours - ref) > atol
    return float(bad.mean()), bad.mean() <= frac


@pytest.mark.parametrize("tag", TAGS)
def test_logits_and_hidden_align_with_hf(tag):
    """inference_alignment_test.py:193-204 on every decoder layer output, the
    final norm and the logits of the prefill step."""
    cfg, g = O.load_golden(tag)
    m = prefill_capture(cfg, cfg["seed"], g["prompt"].tolist())
    L = cfg["num_layers"]
    logits = m.debug_tensor("logits")
    assert logits.shape == g["logits"].shape
    fr, ok = half_alignment(logits, g["logits"])
    assert ok, fr
    worst = fr
    for j in range(L):
        h = m.debug_tensor("hidden", j if j < L - 1 else L)
        fr, ok = half_alignment(h, g["hidden"][j])
        assert ok, (j, fr)
        worst = max(worst, fr)
    report("logits_hidden_vs_hf", tag=tag, worst_mismatch_frac=worst,
           max_abs_logit_err=float(np.abs(logits - g["logits"]).max()))
    m.close()


def close_ulp(ours, ref, ulp=2, atol=2e-3, frac=0.999):
    d = ulp_diff(ours.astype(np.float16), ref.astype(np.float16))
    ok = (d <= ulp) | (np.abs(ours - ref) <= atol)
    return float(ok.mean()), float((d == 0).mean())


@pytest.mark.parametrize("tag", TAGS)
def test_logits_match_oracle_fp16(tag):
    cfg, g = O.load_golden(tag)
    prompt = g["prompt"].tolist()
    m = prefill_capture(cfg, cfg["seed"], prompt)
    ref = O.Model(cfg, cfg["seed"], fp16=1).forward(0, prompt, 0)
    ok, exact = close_ulp(m.debug_tensor("logits"), ref)
    report("logits_vs_oracle_fp16", tag=tag, within_2ulp=ok, exact=exact)
    assert ok >= 0.999, ok
    m.close()


# ------------------------------------------------ LLaMA-7B widths, 2 layers
LLAMA_7B_W = dict(num_layers=2, vocab_size=32000, num_heads=32, num_kv_heads=32, hidden=4096,
                  intermediate=11008, rms_eps=1e-6, rope_theta=10000.0)
LLAMA_68M = dict(num_layers=2, vocab_size=32000, num_heads=12, num_kv_heads=12, hidden=768,
                 intermediate=3072, rms_eps=1e-6, rope_theta=10000.0)
SEED_7B = 20250117


def prompts(n, V, lo, hi, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(3, V, size=int(rng.integers(lo, hi))).tolist() for _ in range(n)]


@pytest.fixture(scope="module")
def oracle_7b():
    return O.Model(LLAMA_7B_W, SEED_7B, fp16=1, max_requests=1, max_seq=160)


def teacher_forced_exact(oracle, seq, n_prompt, tie_ulp=2):
    """(#exact greedy picks, #tokens); a non-exact pick must be a tie within
    tie_ulp fp16 ulp of the two tokens' fp16 softmax probabilities."""
    lg = oracle.forward(0, np.array(seq[:-1], np.int32), 0)[n_prompt - 1:]
    ids, _ = O.softmax_argmax(lg, fp16=1)
    gen = seq[n_prompt:]
    exact = 0
    for t, tok in enumerate(gen):
        if ids[t] == tok:
            exact += 1
            continue
        row = lg[t]
        p = np.exp(row - row.max())
        p16 = (p / p.sum()).astype(np.float16)
        assert ulp_diff(p16[tok], p16[ids[t]]) <= tie_ulp, (t, tok, int(ids[t]))
    return exact, len(gen)


def stats(ours, ref):
    d = np.abs(ours - ref)
    return dict(exact=float((ours.astype(np.float16) == ref.astype(np.float16)).mean()),
                within_2ulp=close_ulp(ours, ref)[0], max_abs=float(d.max()),
                p999_abs=float(np.quantile(d, 0.999)), max_ref=float(np.abs(ref).max()),
                frac_gt_1e2=float((d > 1e-2).mean()),
                frac_bad=float((d > np.maximum(1e-2, 4 * ulp16(ref))).mean()))


def ulp16(x):
    return np.spacing(np.abs(np.asarray(x)).astype(np.float16)).astype(np.float32)


def test_llama7b_width_prefill_logits_match_oracle(oracle_7b):
    """Full LLaMA-7B widths (H 4096, F 11008, V 32000) through every bench
    GEMM plan of a 40-token prefill (X_PACKED | W_STREAM weights, split-K
    slabs combined by the attention prologue and the residual norm).  Over
    K = 4096 / 11008 the fp32 reorderings flip single fp16 roundings of
    intermediates, which then propagate through the layers, so the bar is the
    reference's own alignment rule (atol 1e-2, <= 5% outside; widened to 4
    fp16 ulp where |x| > 8, where 1e-2 is about one ulp) made 5x stricter
    (<= 1% outside), with the measured spread reported (measured: logits max
    |d| 0.008 at |x| <= 7.7, none outside; layer-1 output max |d| 0.0195 at
    |x| <= 15.8, 0.2% outside)."""
    prompt = [1] + prompts(1, 32000, 39, 40, 5)[0]
    m = prefill_capture(LLAMA_7B_W, SEED_7B, prompt)
    ref = oracle_7b.forward(0, prompt, 0)
    st = {"logits": stats(m.debug_tensor("logits"), ref)}
    for j in range(2):
        st[f"hidden{j}"] = stats(m.debug_tensor("hidden", j), oracle_7b.hidden(j, len(prompt)))
    report("llama7b_width_prefill_logits", **st)
    for k, v in st.items():
        assert v["frac_bad"] <= 0.01, (k, v)
    m.close()


@pytest.mark.parametrize("mode", ["incr", "spec"])
def test_llama7b_width_batch8_tokens_match_oracle(oracle_7b, mode):
    """Config B/C shapes at 2 layers: 8 requests decoded together (T = 8
    decode steps; SpecInfer verify steps T = 8 x 21 with the 68M SSM) and
    every request's greedy tokens checked teacher-forced against the oracle."""
    B = 8
    ps = prompts(B, 32000, 20, 40, 11)
    max_len = 64
    kw = dict(max_requests_per_batch=B, max_tokens_per_batch=256, max_sequence_length=128)
    if mode == "incr":
        llm = fa.Model(LLAMA_7B_W, "inc", max_requests=B, max_tokens=256, max_seq_len=128,
                       weight_seed=SEED_7B)
        rm = fa.RequestManager(**kw)
    else:
        vt = 256 + 23 * B
        llm = fa.Model(LLAMA_7B_W, "tree", max_requests=B, max_tokens=vt, max_seq_len=128,
                       max_tree_tokens=23, weight_seed=SEED_7B)
        ssm = fa.Model(LLAMA_68M, "beam", max_requests=B, max_tokens=vt, max_seq_len=128,
                       max_tree_tokens=23, weight_seed=68)
        rm = fa.RequestManager(spec_tree_width=(1, 1, 3), max_spec_tree_token_num=23, **kw)
        rm.register_ssm_model(ssm)
    res = fa.generate(rm, llm, ps, max_length=max_len, spec=mode == "spec")
    exact = total = 0
    for p, r in zip(ps, res):
        assert len(r.output_tokens) == max_len
        e, n = teacher_forced_exact(oracle_7b, r.output_tokens, len(p) + 1)
        exact += e
        total += n
    report("llama7b_width_batch8_tokens", mode=mode, exact=exact, total=total)
    # measured 280 / 280 in both modes (rounds 2 and 3); one noise-level tie
    # allowed (each mismatch is checked as a <= 2-ulp tie above)
    assert exact >= total - 1, (exact, total)
    llm.close()


def test_llama7b_width_tokens_vs_reference_half_semantics():
    """GPU greedy tokens against the reference's OWN numerics (ORC_REF16:
    cuBLAS half compute type in every dense layer, cuBLAS/cuDNN prompt
    attention, the generation kernel for decode steps), teacher-forced:
    each GPU token compared with what the reference would pick after the same
    prefix.  The GPU accumulates in fp32, so this is a measured
    agreement, not bit-exactness; the bound below is the measured 63 / 66
    less one token, and the oracle's own fp32-accumulate mode shows the same
    gap."""
    ref = O.Model(LLAMA_7B_W, SEED_7B, fp16=O.REF16, max_requests=1, max_seq=160)
    ps = prompts(3, 32000, 20, 30, 17)
    llm = fa.Model(LLAMA_7B_W, "inc", max_requests=4, max_tokens=64, max_seq_len=128,
                   weight_seed=SEED_7B)
    rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=64,
                           max_sequence_length=128)
    res = fa.generate(rm, llm, ps, max_length=48)
    agree = total = 0
    for p, r in zip(ps, res):
        seq = r.output_tokens
        lg = ref.teacher_forced_ref(seq, len(p) + 1)
        ids, _ = O.softmax_argmax(lg, fp16=1)
        gen = np.array(seq[len(p) + 1:])
        agree += int((ids[:len(gen)] == gen).sum())
        total += len(gen)
    report("llama7b_width_tokens_vs_ref16", agree=agree, total=total)
    assert total - agree <= 4, (agree, total)
    llm.close()
