"""Parity at the bench's own workload: bench.py's LLaMA-7B (32 layers, its
seed) and LLaMA-68M SSM, its 8 prompts (BOS + 127 splitmix64 ids), its
max_tokens_per_batch 1024 -- so the prefill is ONE T = 1024 step, which takes
the M-split GEMM's fixed prefill plan (gemm.hip mid_plan, >= 4 row blocks)
and the two-launch attention path -- and 64 decoded tokens per request
(decode reaches context 192), incremental decoding and SpecInfer (widths
(1,1,3), 8 SSM steps per verify, T = 168 verify steps).  Configs B and C of
BASELINE.json at the size bench.py measures them (spec_infer.cc:295-340,457;
SURVEY.md §8(d)).

Checks, all against the teacher-forced CPU oracle and the tie rule of
parity_rules.py (a 3-sigma test of the two competing logits against the
reordering noise at that position):
- incr decoding: every GPU pick equals the oracle's or is such a tie;
- SpecInfer: identical to incr decoding, or its own sequence passes the same
  rule (verify GEMMs at T = 168 and decode GEMMs at T = 8 sum in other
  orders);
- the T = 1024 prefill step, op by op (inference_alignment_test.py:20-370):
  cumulative drift within the oracle's own reordering floor, and each
  kernel's local error (the oracle's op on the GPU's own input) within 2 fp16
  ulp, norms bit-exact -- on requests 0 and 7 (the first and last 128-row
  blocks of the step);
- negative control: the same check on a model with a deliberate bug (layer
  16's RoPE one position off for decode tokens, ffmi_model_debug_fault) MUST
  report a non-tie mismatch -- the rule has teeth.
Measured figures go to gpurun_out/parity_report.jsonl.
"""
import os
import sys
import time

import numpy as np
import pytest

import flexflow_amd as fa
import flexflow_amd.ffmi as F
import oracle_lib as O
from hip_util import report, ulp_diff
from parity_rules import assert_ties, classify, picks, tie_budget
from spec_configs import SPEC, spec_setup

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import LLAMA_68M, LLAMA_7B, make_prompts  # noqa: E402

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

B, P, NEW, MTB, TREE = 8, 128, 64, 1024, 23
SEED, SSM_SEED = 20250117, 68  # bench.py's seeds
MAX_SEQ = 512  # bench.py: max(512, prefill + decode + 1)
SPARE = B  # oracle KV slot for fresh runs
ALT0 = B + 1  # oracle KV slots B+1.. : request i's prompt under the reordered dot
PER_OP_REQS = (0, 7)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def progress(msg):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_workload_progress.log"), "a") as f:
        f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def bench_prompts():
    return make_prompts(B, P - 1, LLAMA_7B["vocab_size"])  # + BOS = P tokens, as bench.py


def rm_kw():
    return dict(max_requests_per_batch=B, max_tokens_per_batch=MTB, max_spec_tree_token_num=TREE,
                max_sequence_length=MAX_SEQ)


@pytest.fixture(scope="module")
def oracle():
    t = time.time()
    m = O.Model(LLAMA_7B, SEED, fp16=1, max_requests=2 * B + 1, max_seq=P + NEW + 8)
    progress(f"oracle LLaMA-7B built in {time.time() - t:.1f}s ({O.lib().orc_num_threads()} "
             "threads)")
    return m


OPS = ["attn_norm", "qkv", "attn_out", "o_proj", "ffn_norm", "mlp_act", "down"]


@pytest.fixture(scope="module")
def gpu():
    """The GPU runs: the T = 1024 prefill step captured op by op, then incr
    decoding and SpecInfer of the bench's prompts to P + NEW tokens."""
    ps = bench_prompts()
    out = {"prompts": ps}
    llm = fa.Model(LLAMA_7B, "inc", max_requests=B, max_tokens=MTB, max_seq_len=MAX_SEQ,
                   weight_seed=SEED)
    # the prefill alone (max_length P + 1: the prefill step is the last step)
    llm.set_debug(True)
    res = fa.generate(fa.RequestManager(**rm_kw()), llm, ps, max_length=P + 1)
    assert all(len(r.output_tokens) == P + 1 for r in res)
    rows = np.concatenate([np.arange(P * i, P * (i + 1)) for i in PER_OP_REQS])
    cap = {}
    for l in range(LLAMA_7B["num_layers"]):
        for op in OPS:
            cap[(op, l)] = llm.debug_tensor(op, l)[rows]
        cap[("hidden", l)] = llm.debug_tensor("hidden", l)[rows]
    cap[("embed", 0)] = llm.debug_tensor("embed", 0)[rows]
    cap["logits"] = llm.debug_tensor("logits")[rows]
    out["prefill"] = cap
    out["prefill_T"] = B * P
    llm.set_debug(False)
    progress("GPU T=1024 prefill captured")
    out["incr"] = [r.output_tokens for r in
                   fa.generate(fa.RequestManager(**rm_kw()), llm, ps, max_length=P + NEW)]
    llm.close()
    # SpecInfer: widths (1,1,3) (the bench's), tree width 4, 4 SSMs
    # (tests/spec_configs.py)
    for name in SPEC:
        rm, ssms, vt, tt = spec_setup(name, LLAMA_68M, B, MTB, MAX_SEQ)
        tree = fa.Model(LLAMA_7B, "tree", max_requests=B, max_tokens=vt, max_seq_len=MAX_SEQ,
                        max_tree_tokens=tt, weight_seed=SEED)
        out["spec", name] = [r.output_tokens for r in fa.generate(rm, tree, ps,
                                                                  max_length=P + NEW, spec=True)]
        st = rm.stats()
        out["spec_llm_steps", name] = st.llm_steps
        out["spec_tree_tokens", name] = st.tree_tokens_verified / max(1, st.request_verifies)
        tree.close()
        for m in ssms:
            m.close()
        progress(f"GPU spec {name} done")
    return out


@pytest.fixture(scope="module")
def teacher(oracle):
    return Teacher(oracle)


class Teacher:
    """Teacher-forced oracle along GPU sequences that share the bench's
    prompts: each prompt is run once in its own KV slot, each continuation
    from position P on top of it; the reordered-dot run (the noise estimate)
    only for sequences that have a mismatch, in the spare slot."""

    def __init__(self, oracle):
        self.o = oracle
        self.prompt_last = {}
        self.alt_last = {}

    def logits(self, i, seq):
        """oracle logits predicting seq[P:] (rows [NEW][V])"""
        if i not in self.prompt_last:
            self.prompt_last[i] = self.o.forward(i, np.array(seq[:P], np.int32), 0)[-1]
        cont = self.o.forward(i, np.array(seq[P:-1], np.int32), P)
        return np.vstack([self.prompt_last[i][None], cont])

    def alt_logits(self, i, seq):
        """the same rows with the oracle's dots reordered (the noise run); the
        prompt's reordered KV stays cached in slot ALT0 + i (the oracle is
        T-invariant: prefix + continuation == one forward)"""
        O.set_dot_variant(1)
        try:
            if i not in self.alt_last:
                self.alt_last[i] = self.o.forward(ALT0 + i, np.array(seq[:P], np.int32), 0)[-1]
            cont = self.o.forward(ALT0 + i, np.array(seq[P:-1], np.int32), P)
        finally:
            O.set_dot_variant(0)
        return np.vstack([self.alt_last[i][None], cont])

    def check(self, i, seq):
        lg = self.logits(i, seq)
        gen = np.array(seq[P:])
        ids = picks(lg)
        miss = np.nonzero(ids != gen)[0]
        verdicts = []
        if len(miss):
            lg1 = self.alt_logits(i, seq)
            for t in miss:
                v = classify(lg[t], lg1[t], gen[t], ids[t])
                v["pos"] = int(t)
                verdicts.append(v)
        first = int(miss[0]) if len(miss) else len(gen)
        return first, verdicts, len(gen)


def test_bench_workload_incr_decoding_vs_oracle(teacher, gpu):
    """Config B at the bench's size: 8 x 128-token prompts in one T = 1024
    prefill step, then 63 batched T = 8 decode steps (context 129-191)."""
    tf = teacher
    firsts, verdicts, total = [], [], 0
    for i, (p, seq) in enumerate(zip(gpu["prompts"], gpu["incr"])):
        assert len(seq) == P + NEW and seq[1:P] == p
        first, v, n = tf.check(i, seq)
        firsts.append(first)
        verdicts += v
        total += n
        progress(f"incr request {i}: first mismatch {first}/{n}, {v}")
    report("bench_workload_incr_b8_p128_n64", free_run_agree=firsts,
           free_run_ge_30=sum(f >= 30 for f in firsts), mismatches=verdicts,
           exact=total - len(verdicts), total=total, tie_budget=tie_budget(total))
    assert_ties(verdicts, total)


@pytest.mark.parametrize("spec", list(SPEC))
def test_bench_workload_spec_infer_vs_incr_and_oracle(teacher, gpu, spec):
    """Config C at the bench's size: SpecInfer with the 68M SSM, T = 168
    verify steps (widths (1,1,3)); with tree width 4 (T = 216) and with
    config E's 4 SSMs (merged trees up to 64 tokens per request); identical to
    incr decoding or oracle-checked by the rule."""
    tf = teacher
    same, firsts, verdicts = 0, [], []
    for i, (a, b) in enumerate(zip(gpu["incr"], gpu["spec", spec])):
        assert len(a) == len(b) == P + NEW
        if a == b:
            same += 1
            continue
        first, v, n = tf.check(i, b)
        firsts.append(first)
        verdicts += v
        progress(f"spec request {i} differs from incr: first oracle mismatch {first}/{n}, {v}")
    total = B * NEW  # the run's picks (sequences equal to incr decoding were checked there)
    report(f"bench_workload_spec_b8_p128_n64_{spec}", spec_equals_incr=same, requests=B,
           free_run_agree_of_differing=firsts, mismatches=verdicts,
           llm_steps=gpu["spec_llm_steps", spec],
           tree_tokens_per_request_verify=gpu["spec_tree_tokens", spec],
           tie_budget=tie_budget(total))
    assert_ties(verdicts, total)


def within(ours, ref, ulp=2):
    d = ulp_diff(ours.astype(np.float16), ref.astype(np.float16))
    return dict(within_2ulp=float((d <= ulp).mean()), exact=float((d == 0).mean()),
                max_abs=float(np.abs(ours - ref).max()))


def rope_rows(x, d, tab):
    """apply_rotary_embedding_hf on every head of rows at positions 0..n-1
    (the oracle's rope_apply order), rounded to fp16"""
    n = x.shape[0]
    h = d // 2
    xs = x.reshape(n, -1, d).astype(np.float32)
    cs = tab[:n].reshape(n, 1, h, 2)
    c, s = cs[..., 0], cs[..., 1]
    a, b = xs[..., :h], xs[..., h:]
    out = np.concatenate([(a * c) - (b * s), (a * s) + (b * c)], axis=2)
    return O.round16(out).reshape(n, -1)


def test_bench_workload_prefill_T1024_per_op_drift(oracle, gpu):
    """The T = 1024 prefill step op by op, requests 0 and 7 (rows 0-127 and
    896-1023 of the step).  Bars as test_gpu_fulldepth's per-op test: local
    ops within 2 fp16 ulp on >= 99.9% (norms bit-exact); cumulative drift
    within the envelope of the oracle's own reordering floor."""
    cap, H, d = gpu["prefill"], LLAMA_7B["hidden"], 128
    L = LLAMA_7B["num_layers"]
    eps = LLAMA_7B["rms_eps"]
    tab = O.rope_table(P, d, LLAMA_7B["rope_theta"])
    summary, worst_ratio = {}, 9.0
    for k, i in enumerate(PER_OP_REQS):
        sl = slice(P * k, P * (k + 1))
        toks = np.array(gpu["prompts"][i], np.int32)
        toks = np.concatenate([[1], toks]).astype(np.int32)
        O.set_dot_variant(1)
        try:
            alt_logits = oracle.forward(SPARE, toks, 0)
            alt = {(op, l): oracle.op(op, l) for l in range(L) for op in OPS}
        finally:
            O.set_dot_variant(0)
        ref_logits = oracle.forward(SPARE, toks, 0)
        cum_first_out = None
        for l in range(L):
            for op in OPS:
                ref = oracle.op(op, l)
                st = within(cap[(op, l)][sl], ref)
                fl = within(alt[(op, l)], ref)
                worst_ratio = min(worst_ratio, st["within_2ulp"] / max(fl["within_2ulp"], 1e-9))
                if cum_first_out is None and st["within_2ulp"] < 1.0:
                    cum_first_out = dict(layer=l, op=op, **st)
        lg = cap["logits"][sl]
        bad = float((np.abs(lg - ref_logits) > 1e-2).mean())
        floor_bad = float((np.abs(alt_logits - ref_logits) > 1e-2).mean())
        floor_max = float(np.abs(alt_logits - ref_logits).max())
        gpu_max = float(np.abs(lg - ref_logits).max())
        # local: each kernel on the GPU's own input
        local = {}
        for l in (0, 15, 31):
            p = f"model.layers.{l}."
            W = lambda name, rows: oracle.weight(p + name).reshape(rows, -1)  # noqa: E731
            g = {op: cap[(op, l)][sl] for op in OPS}
            res_in = cap[("embed", 0)][sl] if l == 0 else cap[("hidden", l - 1)][sl]
            loc = {"attn_norm": O.rmsnorm(res_in, oracle.weight(p + "input_layernorm.weight"), eps)}
            wqkv = np.concatenate([W("self_attn.q_proj.weight", H), W("self_attn.k_proj.weight", H),
                                   W("self_attn.v_proj.weight", H)])
            loc["qkv"] = O.linear(g["attn_norm"], wqkv)
            qr = rope_rows(g["qkv"][:, :H], d, tab)
            kr = rope_rows(g["qkv"][:, H:2 * H], d, tab)
            vv = g["qkv"][:, 2 * H:]
            att = np.zeros((P, H), np.float32)
            scale = float(np.float32(1) / np.sqrt(np.float32(d)))
            for hd in range(H // d):
                c = slice(hd * d, (hd + 1) * d)
                for t in range(P):
                    att[t, c] = O.attention_row(qr[t, c], kr[:t + 1, c], vv[:t + 1, c],
                                                np.ones(t + 1, np.uint8), scale)
            loc["attn_out"] = att
            loc["o_proj"] = O.linear(g["attn_out"], W("self_attn.o_proj.weight", H))
            r1 = O.round16(res_in + g["o_proj"])
            loc["ffn_norm"] = O.rmsnorm(r1, oracle.weight(p + "post_attention_layernorm.weight"), eps)
            gate = O.linear(g["ffn_norm"], W("mlp.gate_proj.weight", LLAMA_7B["intermediate"]))
            up = O.linear(g["ffn_norm"], W("mlp.up_proj.weight", LLAMA_7B["intermediate"]))
            loc["mlp_act"] = O.silu_mul(gate, up)
            loc["down"] = O.linear(g["mlp_act"], W("mlp.down_proj.weight", H))
            local[l] = {op: within(g[op], loc[op]) for op in OPS}
        summary[i] = dict(first_op_beyond_2ulp=cum_first_out, logits_frac_outside_1e2=bad,
                          floor_frac_outside_1e2=floor_bad, logits_max=gpu_max,
                          floor_max=floor_max, local={str(k): v for k, v in local.items()})
        progress(f"per-op T=1024 request {i}: logits {bad:.4f} vs floor {floor_bad:.4f}")
        for l, ops in local.items():
            for op, st in ops.items():
                if op in ("attn_norm", "ffn_norm"):
                    assert st["exact"] == 1.0, (i, l, op, st)
                assert st["within_2ulp"] >= 0.999, (i, l, op, st)
        assert bad <= 1.25 * floor_bad + 0.01, (i, bad, floor_bad)
        assert gpu_max <= 1.5 * floor_max, (i, gpu_max, floor_max)
    report("bench_workload_prefill_T1024_per_op", requests=list(PER_OP_REQS),
           worst_within_2ulp_ratio_to_floor=worst_ratio, **{str(k): v for k, v in summary.items()})
    assert worst_ratio >= 0.8, worst_ratio


def test_negative_control_rope_fault_is_detected(oracle):
    """The rule must FAIL a real bug.  LLaMA-7B (bench weights), 4 requests
    of 24-token prompts, 24 decoded tokens, every layer's RoPE rotating every
    decode-phase token (position >= 25) exactly one position too far
    (ffmi_model_debug_fault FFMI_FAULT_ROPE_POS, layer -1: a wrong abs_depth,
    inc_multihead_self_attention.cu:664-738): at least one GPU pick must differ
    from the teacher-forced oracle by MORE than the tie rule allows.  The same
    run without the fault passes the rule (the control's control).
    (The same one-position shift in ONE layer of 32 moves the logits by less
    than the reordering noise at most positions -- round 5 measured 3
    mismatches, all ties -- so the token rule alone cannot see it; the per-op
    local check below does.)"""
    rng = np.random.default_rng(404)
    ps = [rng.integers(3, 32000, size=24).tolist() for _ in range(4)]
    n_prompt = 25  # with BOS
    kw = dict(max_requests_per_batch=4, max_tokens_per_batch=128, max_sequence_length=128)
    llm = fa.Model(LLAMA_7B, "inc", max_requests=4, max_tokens=128, max_seq_len=128,
                   weight_seed=SEED)
    runs = {}
    for fault in (False, True):
        llm.debug_fault(F.FAULT_ROPE_POS if fault else F.FAULT_NONE, -1, n_prompt)
        runs[fault] = [r.output_tokens for r in
                       fa.generate(fa.RequestManager(**kw), llm, ps, max_length=n_prompt + 24)]
    llm.debug_fault(F.FAULT_NONE)
    llm.close()
    out = {}
    for fault, seqs in runs.items():
        verdicts = []
        for seq in seqs:
            toks = np.array(seq[:-1], np.int32)
            lg = oracle.forward(SPARE, toks, 0)[n_prompt - 1:]
            gen = np.array(seq[n_prompt:])
            ids = picks(lg)
            miss = np.nonzero(ids != gen)[0]
            if len(miss):
                O.set_dot_variant(1)
                try:
                    lg1 = oracle.forward(SPARE, toks, 0)[n_prompt - 1:]
                finally:
                    O.set_dot_variant(0)
                # every position is a valid per-position test: later ones
                # follow the GPU's (teacher-forced) sequence
                verdicts += [dict(pos=int(t), **classify(lg[t], lg1[t], gen[t], ids[t]))
                             for t in miss]
        out[fault] = verdicts
    report("negative_control_rope_all_layers", clean=out[False], faulted=out[True],
           faulted_non_ties=sum(not v["tie"] for v in out[True]))
    progress(f"negative control: clean {out[False]}, faulted {len(out[True])} mismatches")
    assert_ties(out[False], 4 * 24)
    assert any(not v["tie"] for v in out[True]), ("fault NOT detected", out[True])


def test_negative_control_rope_fault_one_layer_local_check(oracle):
    """The one-layer form of the RoPE bug, caught where it lives: layer 16's
    RoPE one position off from position 10 on, in the bench model's T = 1024
    prefill; layer 16's attention output on the GPU's own captured qkv, against
    the oracle's attention with the true rotation (the local check of
    test_bench_workload_prefill_T1024_per_op_drift), must leave the 2-ulp band
    on more than 0.1% of the elements; layer 15 (no fault) must stay in it."""
    ps = bench_prompts()
    llm = fa.Model(LLAMA_7B, "inc", max_requests=B, max_tokens=MTB, max_seq_len=MAX_SEQ,
                   weight_seed=SEED)
    llm.debug_fault(F.FAULT_ROPE_POS, 16, 10)
    llm.set_debug(True)
    fa.generate(fa.RequestManager(**rm_kw()), llm, ps, max_length=P + 1)
    H, d = LLAMA_7B["hidden"], 128
    tab = O.rope_table(P, d, LLAMA_7B["rope_theta"])
    scale = float(np.float32(1) / np.sqrt(np.float32(d)))
    res = {}
    for l in (15, 16):
        qkv = llm.debug_tensor("qkv", l)[:P]
        got = llm.debug_tensor("attn_out", l)[:P]
        qr, kr, vv = rope_rows(qkv[:, :H], d, tab), rope_rows(qkv[:, H:2 * H], d, tab), qkv[:, 2 * H:]
        att = np.zeros((P, H), np.float32)
        for hd in range(H // d):
            c = slice(hd * d, (hd + 1) * d)
            for t in range(P):
                att[t, c] = O.attention_row(qr[t, c], kr[:t + 1, c], vv[:t + 1, c],
                                            np.ones(t + 1, np.uint8), scale)
        res[l] = within(got, att)
    llm.debug_fault(F.FAULT_NONE)
    llm.close()
    report("negative_control_rope_layer16_local", layer15=res[15], layer16=res[16])
    assert res[15]["within_2ulp"] >= 0.999, res[15]
    assert res[16]["within_2ulp"] < 0.999, ("fault NOT detected", res[16])


def test_negative_control_residual_rounding_fault_is_detected(oracle):
    """A rounding-point bug must fail the per-op local check: the residual
    RMSNorm kernel squaring the unrounded fp32 residual sum
    (ffmi_model_debug_fault FFMI_FAULT_RESID_ROUND; the reference rounds it to
    half first, residual_rms_norm_kernels.cu:112-114).  The bench model's
    T = 1024 prefill is captured with the fault; both norms of every layer,
    all 1024 rows, are checked as test_bench_workload_prefill_T1024_per_op
    checks them (the oracle's norm on the GPU's own captured input, bit-exact
    demanded): at least one must NOT be bit-exact.  The shift is below an ulp
    of most outputs (the rms moves by ~1e-5 relative and crosses an fp16
    rounding boundary in ~0.3% of rows), so the 2-ulp bar alone would pass it
    -- the bit-exact norm bar is what catches it."""
    ps = bench_prompts()
    llm = fa.Model(LLAMA_7B, "inc", max_requests=B, max_tokens=MTB, max_seq_len=MAX_SEQ,
                   weight_seed=SEED)
    llm.debug_fault(F.FAULT_RESID_ROUND)
    llm.set_debug(True)
    fa.generate(fa.RequestManager(**rm_kw()), llm, ps, max_length=P + 1)
    rows = np.arange(B * P)  # every row of the step, every layer (the rms moves
    # across an fp16 rounding boundary in only ~0.3% of rows)
    eps = LLAMA_7B["rms_eps"]
    res = {}
    for l in range(LLAMA_7B["num_layers"]):
        p = f"model.layers.{l}."
        res_in = (llm.debug_tensor("embed", 0) if l == 0 else llm.debug_tensor("hidden", l - 1))[rows]
        g = {op: llm.debug_tensor(op, l)[rows] for op in ("attn_norm", "o_proj", "ffn_norm")}
        loc_attn = O.rmsnorm(res_in, oracle.weight(p + "input_layernorm.weight"), eps)
        r1 = O.round16(res_in + g["o_proj"])
        loc_ffn = O.rmsnorm(r1, oracle.weight(p + "post_attention_layernorm.weight"), eps)
        for name, ours, ref in (("attn_norm", g["attn_norm"], loc_attn),
                                ("ffn_norm", g["ffn_norm"], loc_ffn)):
            st = within(ours, ref)
            st["rows_not_exact"] = int((ours != ref).any(axis=1).sum())
            res[f"{name}_{l}"] = st
    llm.debug_fault(F.FAULT_NONE)
    llm.close()
    bad = {k: v for k, v in res.items() if v["exact"] < 1.0}
    report("negative_control_residual_rounding", rows=B * P, norms=len(res),
           norms_not_exact=len(bad), rows_not_exact=sum(v["rows_not_exact"] for v in bad.values()),
           worst_within_2ulp=min(v["within_2ulp"] for v in res.values()), not_exact=bad)
    progress(f"residual-rounding control: {len(bad)} norms not bit-exact")
    # (layer 0's attn_norm has no residual add: the embedding alone)
    assert any(k != "attn_norm_0" for k in bad), ("fault NOT detected", res)
    assert res["attn_norm_0"]["exact"] == 1.0, res["attn_norm_0"]
