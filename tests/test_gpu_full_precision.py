"""Full precision: the reference's --use-full-precision
(inference/spec_infer/spec_infer.cc:102, incr_decoding.cc:77;
ffmi_model_opts.full_precision, runtime/llama_f32.cpp, kernels/f32.hip):
weights, activations, KV cache and softmax in fp32.

The reference runs its exact-diff invariants in this mode
(tests/inference/cpp_inference_tests.sh: the first 30 tokens identical
:104-129, SpecInfer == incremental decoding :183-189, TP = 1 vs TP > 1
:203-217).  GPU and oracle (fp32 mode, pinned to HF transformers fp32 by
test_oracle_golden.py) share every operation and differ only in fp32
summation order, ~1e-7 relative; on the bench's random-weight LLaMA-7B the
top-2 logit gap falls inside that noise at ~1e-5 of positions, so the
reference's bars are demanded literally here -- a divergence is accepted only
at an fp32-level tie (the oracle's gap between the two picks <= 1e-4, reported
if it ever happens).
"""
import ctypes

import os

import numpy as np
import pytest

import flexflow_amd as fa
import flexflow_amd.ffmi as F
import oracle_lib as O
import peer_tasks as PT
from hip_util import Buf, report
from peer_group import run_group
from spec_configs import SPEC, spec_setup

pytestmark = pytest.mark.gpu

SEED = 20250117
LLAMA_7B = dict(num_layers=32, vocab_size=32000, num_heads=32, num_kv_heads=32, hidden=4096,
                intermediate=11008, rms_eps=1e-6, rope_theta=10000.0)
LLAMA_68M = dict(num_layers=2, vocab_size=32000, num_heads=12, num_kv_heads=12, hidden=768,
                 intermediate=3072, rms_eps=1e-6, rope_theta=10000.0)
FP32_TIE = 1e-4  # oracle logit gap below which two fp32 runs may pick differently


@pytest.mark.parametrize("T,N,K", [(1, 16, 32), (5, 48, 96), (8, 4096, 4096), (24, 2304, 768),
                                   (33, 272, 1376), (64, 1000, 3072), (3, 40, 64), (168, 1536, 4096),
                                   (577, 96, 1376), (1024, 512, 4096)])
def test_linear_f32_against_fp64(T, N, K):
    """ffmi_linear_f32 against an fp64 product: every element within the fp32
    error bound of a K-term sum (2e-6 * sum|x w|, the measured MFMA f32 error
    is ~3.5e-7 at K 4096), and bit-identical on a second call (fixed order)."""
    rng = np.random.default_rng(T * 7 + N + K)
    X = rng.uniform(-1, 1, (T, K)).astype(np.float32)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float32)
    ref = X.astype(np.float64) @ W.astype(np.float64).T
    mag = np.abs(X).astype(np.float64) @ np.abs(W).astype(np.float64).T
    bx, bw, by = Buf(X), Buf(W), Buf.empty((T, N), np.float32)
    L = F.lib()
    assert L.ffmi_linear_f32(bx.ptr, bw.ptr, by.ptr, T, N, K, None) == 0
    y1 = by.get()
    assert L.ffmi_linear_f32(bx.ptr, bw.ptr, by.ptr, T, N, K, None) == 0
    y2 = by.get()
    err = np.abs(y1 - ref)
    assert np.all(err <= 2e-6 * mag + 1e-30), float((err / mag).max())
    assert np.array_equal(y1.view(np.uint32), y2.view(np.uint32))


OFF = int(os.environ.get("FFMI_RANDOM_SEED_OFFSET", "0"))  # fresh seeds for one-off sweeps


@pytest.mark.parametrize("seed", range(12 * int(os.environ.get("FFMI_RANDOM_SCALE", "1"))))
def test_linear_f32_random_shapes(seed):
    """ffmi_linear_f32 at random shapes (T 1-1100, N 1-6000 ragged, K a
    multiple of 32 up to 8192) under the same bound and determinism as
    test_linear_f32_against_fp64."""
    rng = np.random.default_rng(8800 + OFF + seed)
    T = int(np.exp(rng.uniform(0, np.log(1100))))
    N = int(rng.integers(1, 6000))
    K = 32 * int(np.exp(rng.uniform(0, np.log(256))))
    X = rng.uniform(-1, 1, (T, K)).astype(np.float32)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float32)
    ref = X.astype(np.float64) @ W.astype(np.float64).T
    mag = np.abs(X).astype(np.float64) @ np.abs(W).astype(np.float64).T
    bx, bw, by = Buf(X), Buf(W), Buf.empty((T, N), np.float32)
    L = F.lib()
    assert L.ffmi_linear_f32(bx.ptr, bw.ptr, by.ptr, T, N, K, None) == 0, (T, N, K)
    y1 = by.get()
    assert L.ffmi_linear_f32(bx.ptr, bw.ptr, by.ptr, T, N, K, None) == 0
    err = np.abs(y1 - ref)
    assert np.all(err <= 2e-6 * mag + 1e-30), (T, N, K, float((err / mag).max()))
    assert np.array_equal(y1.view(np.uint32), by.get().view(np.uint32))


def ulps32(a, b):
    """distance in fp32 ulps (monotonic int mapping)"""
    def key(x):
        u = np.asarray(x, np.float32).view(np.int32).astype(np.int64)
        return np.where(u < 0, -(u & 0x7FFFFFFF), u)
    return np.abs(key(a) - key(b))


@pytest.mark.parametrize("H", [768, 4096])
def test_rmsnorm_f32_against_oracle(H):
    """ffmi_rmsnorm_f32 / ffmi_residual_rmsnorm_f32 vs the oracle's fp32 mode
    (the same fp32 operations; only the fp64 sum of squares is reordered):
    within 1 ulp, >= 99% bit-identical, the residual sum bit-exact"""
    rng = np.random.default_rng(H)
    T, eps = 13, 1e-6
    x1 = rng.standard_normal((T, H)).astype(np.float32)
    x2 = rng.standard_normal((T, H)).astype(np.float32)
    w = rng.uniform(0.5, 1.5, H).astype(np.float32)
    L = F.lib()
    b1, b2, bw = Buf(x1), Buf(x2), Buf(w)
    out, res = Buf.empty((T, H), np.float32), Buf.empty((T, H), np.float32)
    assert L.ffmi_rmsnorm_f32(b1.ptr, bw.ptr, out.ptr, T, H, ctypes.c_float(eps), None) == 0
    d = ulps32(out.get(), O.rmsnorm(x1, w, eps, fp16=0))
    assert d.max() <= 1 and (d == 0).mean() >= 0.99, (int(d.max()), float((d == 0).mean()))
    assert L.ffmi_residual_rmsnorm_f32(b1.ptr, b2.ptr, bw.ptr, res.ptr, out.ptr, T, H,
                                       ctypes.c_float(eps), None) == 0
    rr, ro = O.residual_rmsnorm(x1, x2, w, eps, fp16=0)
    assert np.array_equal(res.get(), rr)
    d = ulps32(out.get(), ro)
    assert d.max() <= 1 and (d == 0).mean() >= 0.99


def test_silu_mul_f32_against_oracle():
    """SigmoidSiluMulti on fp32: the device expf against the host's (each
    within ~1 ulp of exp) carried through 1/(1 + e), a * sg and * b: <= 4 ulp,
    >= 90% bit-identical"""
    rng = np.random.default_rng(9)
    a = (4 * rng.standard_normal(50000)).astype(np.float32)
    b = rng.standard_normal(50000).astype(np.float32)
    ba, bb, bo = Buf(a), Buf(b), Buf.empty((50000,), np.float32)
    assert F.lib().ffmi_silu_mul_f32(ba.ptr, bb.ptr, bo.ptr, 50000, None) == 0
    d = ulps32(bo.get(), O.silu_mul(a, b, fp16=0))
    assert d.max() <= 4 and (d == 0).mean() >= 0.9, (int(d.max()), float((d == 0).mean()))


@pytest.mark.parametrize("k", [1, 3])
def test_arg_topk_f32_against_oracle(k):
    """softmax + arg-top-k on fp32 probabilities, lowest index among equal
    probabilities (planted exact ties, also across the top-k boundary)"""
    rng = np.random.default_rng(k)
    T, V = 24, 32000
    z = rng.standard_normal((T, V)).astype(np.float32)
    for t in range(0, T, 3):  # ties: the row's max copied to a lower and a higher index
        j = int(z[t].argmax())
        z[t, (j + 7) % V] = z[t, j]
        z[t, (j + V - 5) % V] = z[t, j]
    bz, bi, bp = Buf(z), Buf.empty((T, k), np.int32), Buf.empty((T, k), np.float32)
    assert F.lib().ffmi_arg_topk_f32(bz.ptr, T, V, k, bi.ptr, bp.ptr, None) == 0
    ids, probs = O.softmax_topk(z, k, fp16=0)
    assert np.array_equal(bi.get(), ids)
    assert ulps32(bp.get(), probs).max() <= 2


def oracle_greedy(om, prompts, n_new):
    """the fp32 oracle's own greedy continuation of every prompt (BOS
    included), batched: the prompts in one multi-request step, then one
    decode step per token; returns (sequences, logits rows [B][n_new][V])"""
    B = len(prompts)
    counts = [len(p) for p in prompts]
    lg = om.forward_multi(list(range(B)), counts, [0] * B, np.concatenate(prompts))
    last = lg[np.cumsum(counts) - 1]
    seqs = [list(p) for p in prompts]
    rows = []
    for step in range(n_new):
        ids, _ = O.softmax_argmax(last, fp16=0)
        rows.append(last)
        for s, i in zip(seqs, ids):
            s.append(int(i))
        if step + 1 < n_new:
            last = om.decode_batch(list(range(B)), [s[-1] for s in seqs],
                                   [len(s) - 1 for s in seqs])
    return seqs, np.stack(rows, 1)


def compare(gpu, ref, rows, n_prompts):
    """per sequence: identical, or the first divergence an fp32 tie of the
    oracle row there; returns (identical count, divergences)"""
    same, div = 0, []
    for b, (g, r) in enumerate(zip(gpu, ref)):
        if list(g) == list(r):
            same += 1
            continue
        t = next(i for i in range(min(len(g), len(r))) if g[i] != r[i])
        row = rows[b][t - n_prompts[b]]
        gap = float(row[r[t]] - row[g[t]])
        div.append(dict(seq=b, pos=t - n_prompts[b], gpu=int(g[t]), oracle=int(r[t]), gap=gap))
        assert gap <= FP32_TIE, div[-1]
    return same, div


def run(cfg, ps, max_length, spec, B, mtb=256, seq=256):
    """spec: False (incr decoding), True / a tests/spec_configs.py name"""
    kw = dict(max_requests=B, max_seq_len=seq, full_precision=True)
    if spec:
        rm, ssms, vt, tt = spec_setup("w113" if spec is True else spec, LLAMA_68M, B, mtb, seq,
                                      full_precision=True)
        llm = fa.Model(cfg, "tree", max_tokens=vt, max_tree_tokens=tt, weight_seed=SEED, **kw)
        res = fa.generate(rm, llm, ps, max_length=max_length, spec=True)
        for m in ssms:
            m.close()
    else:
        llm = fa.Model(cfg, "inc", max_tokens=mtb, weight_seed=SEED, **kw)
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=seq)
        res = fa.generate(rm, llm, ps, max_length=max_length)
    llm.close()
    return [r.output_tokens for r in res], rm.stats().llm_steps


def prompts(n, lo, hi, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(3, 32000, size=int(rng.integers(lo, hi))).tolist() for _ in range(n)]


def test_full_precision_2layer_teacher_forced_logits():
    """2 layers at LLaMA-7B widths: one prefill step over 4 prompts, logits
    against the fp32 oracle within 1e-4 (the HF-alignment tolerance the oracle
    itself meets against transformers, test_oracle_golden.py)"""
    cfg = dict(LLAMA_7B, num_layers=2)
    ps = [[1] + p for p in prompts(4, 33, 34, 3)]  # equal lengths: the prefill is the last step
    m = fa.Model(cfg, "inc", max_requests=4, max_tokens=256, max_seq_len=256, weight_seed=SEED,
                 full_precision=True)
    m.set_debug(True)
    fa.generate(fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=256,
                                  max_sequence_length=256), m, [p[1:] for p in ps],
                max_length=max(map(len, ps)) + 1)
    lg = m.debug_tensor("logits")
    m.close()
    om = O.Model(cfg, SEED, fp16=0, max_requests=4, max_seq=256)
    ref = om.forward_multi([0, 1, 2, 3], [len(p) for p in ps], [0] * 4, np.concatenate(ps))
    assert lg.shape == ref.shape
    err = np.abs(lg - ref)
    report("full_precision_2L_logits", max_abs_err=float(err.max()),
           logit_std=float(ref.std()), rows=int(ref.shape[0]))
    assert err.max() <= 1e-4, float(err.max())


@pytest.fixture(scope="module")
def bench_7b():
    """LLaMA-7B, 32 layers, fp32 (27 GB on the GPU and on the host oracle):
    8 prompts, 40 new tokens, incr decoding and SpecInfer with the fp32 68M SSM"""
    ps = prompts(8, 8, 24, 77)
    n_prompts = [len(p) + 1 for p in ps]
    NEW = 40
    max_length = max(n_prompts) + NEW
    incr, incr_steps = run(LLAMA_7B, ps, max_length, False, 8)
    spec, spec_steps = {}, {}
    for name in SPEC:  # (1,1,3), tree width 4, 4 SSMs
        spec[name], spec_steps[name] = run(LLAMA_7B, ps, max_length, name, 8)
    om = O.Model(LLAMA_7B, SEED, fp16=0, max_requests=8, max_seq=2 * max_length)
    # every request continues to max_length: the oracle runs the longest
    # continuation for all and the comparison uses each sequence's length
    ref, rows = oracle_greedy(om, [[1] + p for p in ps], max_length - min(n_prompts))
    ref = [r[:max_length] for r in ref]
    return dict(ps=ps, n_prompts=n_prompts, incr=incr, spec=spec, ref=ref, rows=rows,
                incr_steps=incr_steps, spec_steps=spec_steps)


def test_full_precision_7b_incr_equals_oracle(bench_7b):
    """the reference's bar (cpp_inference_tests.sh:104-129: first 30 tokens
    identical) on the 32-layer bench model: every token of every request"""
    b = bench_7b
    same, div = compare(b["incr"], b["ref"], b["rows"], b["n_prompts"])
    report("full_precision_7b_32L_incr_vs_oracle", identical=same, requests=len(b["ps"]),
           divergences=div, tokens=sum(len(s) - n for s, n in zip(b["incr"], b["n_prompts"])))
    assert same + len(div) == len(b["ps"])


@pytest.mark.parametrize("spec", list(SPEC))
def test_full_precision_7b_spec_equals_incr(bench_7b, spec):
    """SpecInfer == incremental decoding (cpp_inference_tests.sh:183-189), with
    widths (1,1,3), tree width 4 and 4 SSMs"""
    b = bench_7b
    same = sum(a == c for a, c in zip(b["spec"][spec], b["incr"]))
    report(f"full_precision_7b_32L_spec_vs_incr_{spec}", identical=same, requests=len(b["ps"]),
           incr_steps=b["incr_steps"], spec_steps=b["spec_steps"][spec])
    if same < len(b["ps"]):  # only at an fp32 tie of the oracle's row
        compare(b["spec"][spec], b["ref"], b["rows"], b["n_prompts"])


def test_full_precision_tp8_processes_equal_tp1():
    """TP = 8 (8 rank processes, o / down all-reduced in fp32 over the xGMI
    transport) against TP = 1, incremental decoding and SpecInfer: the
    reference's TP-invariance diff (cpp_inference_tests.sh:203-217)"""
    ps = prompts(3, 8, 16, 5)
    max_length = max(map(len, ps)) + 1 + 32
    out = {}
    for spec in (False, True):
        g = run_group(8, PT.tp_generate_f32_task, (LLAMA_7B, SEED, ps, max_length, spec, LLAMA_68M),
                      max_bytes=(256 + 23 * 3 + 16) * 4096 * 4, timeout=900)
        for r in range(8):
            assert g[r]["tokens"] == g[0]["tokens"], r
        one, _ = run(LLAMA_7B, ps, max_length, spec, 3, seq=128)  # the ranks' cache size
        out[spec] = (g[0]["tokens"], one)
    same = {("spec" if k else "incr"): sum(a == b for a, b in zip(*v)) for k, v in out.items()}
    report("full_precision_7b_tp8_vs_tp1", requests=len(ps), **same)
    assert out[False][0] == out[False][1], same
    assert out[True][0] == out[True][1], same


def test_full_precision_negative_control_rope_fault():
    """The literal fp32 bars must FAIL a real bug: 4 layers at LLaMA-7B widths,
    4 prompts, 16 new tokens.  Clean: every token equals the fp32 oracle's
    greedy decode.  Layer 2's RoPE one position off for decode tokens
    (ffmi_model_debug_fault FFMI_FAULT_ROPE_POS on the DT_FLOAT handles): at
    least one request must leave the oracle's sequence at a pick whose oracle
    logit gap is far beyond an fp32 tie (FP32_TIE)."""
    cfg = dict(LLAMA_7B, num_layers=4)
    ps = prompts(4, 16, 17, 31)
    n_prompt = 17  # with BOS
    NEW = 16
    m = fa.Model(cfg, "inc", max_requests=4, max_tokens=256, max_seq_len=128, weight_seed=SEED,
                 full_precision=True)
    runs = {}
    for fault in (False, True):
        m.debug_fault(F.FAULT_ROPE_POS if fault else F.FAULT_NONE, 2, n_prompt)
        res = fa.generate(fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=256,
                                            max_sequence_length=128), m, ps,
                          max_length=n_prompt + NEW)
        runs[fault] = [r.output_tokens for r in res]
    m.debug_fault(F.FAULT_NONE)
    m.close()
    om = O.Model(cfg, SEED, fp16=0, max_requests=4, max_seq=128)
    ref, rows = oracle_greedy(om, [[1] + p for p in ps], NEW)
    same, div = compare(runs[False], ref, rows, [n_prompt] * 4)
    gaps = []
    for b, (g, r) in enumerate(zip(runs[True], ref)):
        if list(g) != list(r):
            t = next(i for i in range(len(g)) if g[i] != r[i])
            row = rows[b][t - n_prompt]
            gaps.append(float(row[r[t]] - row[g[t]]))
    report("full_precision_negative_control_rope_layer2", clean_identical=same,
           clean_divergences=div, faulted_divergence_gaps=gaps)
    assert same == 4, div
    assert gaps and max(gaps) > 100 * FP32_TIE, ("fault NOT detected", gaps)
