"""Randomised end-to-end GPU parity: small LLaMA models of random shape
(1-3 layers, 1-8 heads of d = 64 or 128 -- and 32 in incremental decoding --
random FFN width and vocabulary,
RoPE theta, RMS eps), random scheduler limits (batch slots, token budget) and
random request mixes (1-10 prompts of 1-60 tokens, queued past the slots),
random max_sequence_length (64, 128 or 256; max_length up to its last
allowed value), through the MI355X path:

  * incremental decoding: every request's tokens teacher-forced through the
    oracle under the tie rule of tests/parity_rules.py (a mismatch must be a
    <= 2-ulp probability tie or an oracle logit gap within 3 sigma_pair of
    the row's fp32-reordering noise), the ties of a test capped at max(2, 3%)
    of its picks (first run: 5 ties in 4281 picks; a 150-seed sweep found
    3-7-ulp ties that only the sigma_pair part admits);
  * SpecInfer with 1-2 random SSMs (the multi-SSM merge under
    FFMI_SPEC_EXT_MULTI_SSM) and random tree widths up to 4: its tokens under
    the same rule -- so SpecInfer equals incremental decoding up to ties;
  * the full-precision path (fp32, incr or SpecInfer): equal to the fp32
    oracle's free-running greedy decode up to fp32-level ties.
"""
import os

import numpy as np
import pytest

import flexflow_amd as fa
from hip_util import report

pytestmark = pytest.mark.gpu

WIDTHS = [(1, 1, 3), (3,), (2, 1, 1), (1, 1, 4), (2, 2), ()]
# FFMI_RANDOM_SEEDS: more seeds for a one-off sweep (the suite runs 20 / 10)
SEEDS = int(os.environ.get("FFMI_RANDOM_SEEDS", "20"))
OFF = int(os.environ.get("FFMI_RANDOM_SEED_OFFSET", "0"))  # fresh seeds for one-off sweeps


def check_all(cfg, seed, ps, res, ml, what):
    """every request teacher-forced through the oracle under the one tie rule
    of tests/parity_rules.py (a mismatch must be a <= 2-ulp probability tie
    or an oracle logit gap within 3 sigma_pair of the row's fp32-reordering
    noise, the oracle re-run with its dots reordered), and the test's ties
    capped at max(2, 3%) of its picks"""
    import oracle_lib as O
    from parity_rules import assert_ties, classify, picks
    verdicts, total = [], 0
    for p, r in zip(ps, res):
        seq = r.output_tokens
        assert len(seq) == ml, what
        n0 = len(p) + 1
        m = O.Model(cfg, seed, fp16=1, max_requests=1, max_seq=len(seq) + 1)
        z0 = m.forward(0, np.array(seq[:-1], np.int32), 0)[n0 - 1:]
        gen, o = seq[n0:], picks(z0)
        mism = [t for t in range(len(gen)) if o[t] != gen[t]]
        if mism:
            O.set_dot_variant(1)
            try:
                m1 = O.Model(cfg, seed, fp16=1, max_requests=1, max_seq=len(seq) + 1)
                z1 = m1.forward(0, np.array(seq[:-1], np.int32), 0)[n0 - 1:]
            finally:
                O.set_dot_variant(0)
            verdicts += [dict(classify(z0[t], z1[t], gen[t], o[t]), pos=t) for t in mism]
        total += len(gen)
    report("random_model_ties", where=str(what)[:120], ties=len(verdicts), total=total)
    assert_ties(verdicts, total)


def random_cfg(rng, vocab=None, inc=False):
    """inc: incremental decoding only, where d = 32 is a third head size (the
    reference's inc kernels take 32 / 64 / 128, tree and beam 64 / 128)"""
    heads = int(rng.choice([1, 2, 4, 8]))
    d = int(rng.choice([32, 64, 128] if inc else [64, 128]))
    return dict(num_layers=int(rng.integers(1, 4)),
                vocab_size=int(vocab or rng.integers(100, 5000)),
                num_heads=heads, num_kv_heads=heads, hidden=heads * d,
                intermediate=32 * int(rng.integers(2, 48)),
                rms_eps=float(rng.choice([1e-6, 1e-5])),
                rope_theta=float(rng.choice([10000.0, 500000.0])))


def random_requests(rng, V, msl=128):
    """1-10 prompts of up to min(60, msl / 2) tokens and a max_length below
    max_sequence_length (the reference rejects max_length >= it)"""
    n = int(rng.integers(1, 11))
    ps = [rng.integers(3, V, size=int(rng.integers(1, min(61, msl // 2)))).tolist() for _ in range(n)]
    max_length = min(msl - 1, max(len(p) for p in ps) + 1 + int(rng.integers(8, 40)))
    return ps, max_length


@pytest.mark.parametrize("seed", range(SEEDS))
def test_random_model_incr_decoding_vs_oracle(seed):
    rng = np.random.default_rng(9000 + OFF + seed)
    cfg = random_cfg(rng, inc=True)
    msl = int(rng.choice([64, 128, 256]))
    ps, ml = random_requests(rng, cfg["vocab_size"], msl)
    B = int(rng.choice([1, 2, 3, 4, 8]))
    mtb = int(rng.choice([8, 16, 32, 64, 128]))
    rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                           max_sequence_length=msl)
    m = fa.Model(cfg, "inc", max_requests=B, max_tokens=mtb, max_seq_len=msl,
                 weight_seed=100 + seed)
    try:
        res = fa.generate(rm, m, ps, max_length=ml)
    finally:
        m.close()
    check_all(cfg, 100 + seed, ps, res, ml, (cfg, B, mtb))


@pytest.mark.parametrize("seed", range(SEEDS))
def test_random_model_spec_infer_vs_oracle(seed):
    rng = np.random.default_rng(9500 + OFF + seed)
    cfg = random_cfg(rng)
    V = cfg["vocab_size"]
    msl = int(rng.choice([64, 128, 256]))
    ps, ml = random_requests(rng, V, msl)
    B = int(rng.choice([1, 2, 4, 8]))
    mtb = int(rng.choice([32, 64, 128]))
    widths = WIDTHS[int(rng.integers(0, len(WIDTHS)))]
    nssm = int(rng.integers(1, 3))
    tree = 64 if nssm > 1 else 33
    ext = fa.ffmi.SPEC_EXT_WIDTH4 | (fa.ffmi.SPEC_EXT_MULTI_SSM if nssm > 1 else 0)
    vt = mtb + tree * B
    rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                           max_sequence_length=msl, spec_tree_width=widths,
                           max_spec_tree_token_num=tree, spec_extensions=ext)
    llm = fa.Model(cfg, "tree", max_requests=B, max_tokens=vt, max_seq_len=msl,
                   max_tree_tokens=tree, weight_seed=200 + seed)
    # SSMs: random smaller models over the same vocabulary, or (agreeing
    # fully) the LLM's own shape and weights, for long accepted paths
    ssms = []
    for k in range(nssm):
        same = rng.random() < 0.3
        scfg = cfg if same else random_cfg(rng, vocab=V)
        ssms.append(fa.Model(scfg, "beam", max_requests=B, max_tokens=vt, max_seq_len=msl,
                             max_tree_tokens=tree, weight_seed=200 + seed if same else 300 + k))
        rm.register_ssm_model(ssms[-1])
    try:
        res = fa.generate(rm, llm, ps, max_length=ml, spec=True)
    except fa.ffmi.FFMIError as e:  # a prompt the SSM cannot load in time (the
        assert "SSM loaded less" in str(e)  # reference asserts): not a parity case
        pytest.skip("SSM prompt behind the LLM for this random mix")
    finally:
        llm.close()
        for s in ssms:
            s.close()
    check_all(cfg, 200 + seed, ps, res, ml, (cfg, B, mtb, widths, nssm))


@pytest.mark.parametrize("seed", range(max(1, SEEDS // 2)))
def test_random_model_chained_ssm_steps_equal_stepwise(seed, monkeypatch):
    """The chained speculation phase (beam steps staged from placeholder
    results, the middle steps grouped into one graph launch -- FFMI_CHAIN_GROUP
    drawn at random) against the stepwise loop (FFMI_SSM_CHAIN=0) on a random
    model and request mix: identical tokens and identical step, commit and
    tree-token counts (the same kernels on the same inputs)."""
    rng = np.random.default_rng(9700 + OFF + seed)
    cfg = random_cfg(rng)
    V = cfg["vocab_size"]
    msl = int(rng.choice([64, 128, 256]))
    ps, ml = random_requests(rng, V, msl)
    B = int(rng.choice([1, 2, 4, 8]))
    mtb = int(rng.choice([32, 64, 128]))
    widths = WIDTHS[int(rng.integers(0, len(WIDTHS) - 1))]  # (not incr decoding)
    nssm = int(rng.integers(1, 3))
    tree = 64 if nssm > 1 else 33
    ext = fa.ffmi.SPEC_EXT_WIDTH4 | (fa.ffmi.SPEC_EXT_MULTI_SSM if nssm > 1 else 0)
    vt = mtb + tree * B
    scfgs = []
    for k in range(nssm):
        same = rng.random() < 0.3
        scfgs.append((cfg, 400 + seed) if same else (random_cfg(rng, vocab=V), 500 + k))
    group = str(int(rng.choice([1, 2, 3, 6])))

    def run(chain):
        monkeypatch.setenv("FFMI_SSM_CHAIN", "1" if chain else "0")
        monkeypatch.setenv("FFMI_CHAIN_GROUP", group)
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=msl, spec_tree_width=widths,
                               max_spec_tree_token_num=tree, spec_extensions=ext)
        llm = fa.Model(cfg, "tree", max_requests=B, max_tokens=vt, max_seq_len=msl,
                       max_tree_tokens=tree, weight_seed=400 + seed)
        ssms = [fa.Model(c, "beam", max_requests=B, max_tokens=vt, max_seq_len=msl,
                         max_tree_tokens=tree, weight_seed=sd) for c, sd in scfgs]
        for m in ssms:
            rm.register_ssm_model(m)
        try:
            res = fa.generate(rm, llm, ps, max_length=ml, spec=True)
        except fa.ffmi.FFMIError as e:  # (as test_random_model_spec_infer_vs_oracle)
            assert "SSM loaded less" in str(e)
            return None
        finally:
            llm.close()
            for m in ssms:
                m.close()
        st = rm.stats()
        return [r.output_tokens for r in res], {
            f: getattr(st, f) for f in ("llm_steps", "ssm_steps", "tokens_committed",
                                        "tree_tokens_verified", "request_verifies")}, \
            st.ssm_phases_chained

    a, b = run(False), run(True)
    if a is None or b is None:
        assert a is None and b is None
        pytest.skip("SSM prompt behind the LLM for this random mix")
    assert a[2] == 0 and b[2] > 0  # (the stepwise run chained nothing, the other did)
    assert b[0] == a[0], (cfg, B, mtb, widths, nssm, group)
    assert b[1] == a[1], (cfg, B, mtb, widths, nssm, group)


def oracle_free_running(cfg, seed, prompt, max_length):
    """the fp32 oracle's own greedy continuation of one prompt (BOS
    included) and its logit rows"""
    import oracle_lib as O
    om = O.Model(cfg, seed, fp16=0, max_requests=1, max_seq=max_length + 1)
    seq = list(prompt)
    last = om.forward_multi([0], [len(seq)], [0], np.array(seq, np.int32))[-1:]
    rows = []
    while len(seq) < max_length:
        ids, _ = O.softmax_argmax(last, fp16=0)
        rows.append(last[0])
        seq.append(int(ids[0]))
        if len(seq) < max_length:
            last = om.decode_batch([0], [seq[-1]], [len(seq) - 1])
    return seq, rows


@pytest.mark.parametrize("seed", range(max(1, SEEDS // 2)))
def test_random_model_full_precision_vs_oracle(seed):
    """The full-precision path (fp32 end to end, the reference's
    --use-full-precision where its exact-diff bars live) at random shapes:
    incremental decoding and SpecInfer (fp32 SSMs, widths up to 4, 1-2 SSMs)
    equal to the fp32 oracle's free-running greedy decode, a divergence
    accepted only at an fp32-level tie (oracle gap <= 1e-4,
    test_gpu_full_precision's rule)."""
    rng = np.random.default_rng(9900 + OFF + seed)
    cfg = random_cfg(rng)
    V = cfg["vocab_size"]
    ps, ml = random_requests(rng, V)
    B = int(rng.choice([1, 2, 4, 8]))
    mtb = int(rng.choice([32, 64, 128]))
    spec = bool(rng.integers(0, 2))
    kw = dict(max_requests=B, max_seq_len=128, full_precision=True)
    ssms = []
    if spec:
        widths = WIDTHS[int(rng.integers(0, len(WIDTHS)))]
        nssm = int(rng.integers(1, 3))
        tree = 64 if nssm > 1 else 33
        ext = fa.ffmi.SPEC_EXT_WIDTH4 | (fa.ffmi.SPEC_EXT_MULTI_SSM if nssm > 1 else 0)
        vt = mtb + tree * B
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=128, spec_tree_width=widths,
                               max_spec_tree_token_num=tree, spec_extensions=ext)
        m = fa.Model(cfg, "tree", max_tokens=vt, max_tree_tokens=tree, weight_seed=400 + seed, **kw)
        for k in range(nssm):
            ssms.append(fa.Model(random_cfg(rng, vocab=V), "beam", max_tokens=vt,
                                 max_tree_tokens=tree, weight_seed=500 + k, **kw))
            rm.register_ssm_model(ssms[-1])
    else:
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=128)
        m = fa.Model(cfg, "inc", max_tokens=mtb, weight_seed=400 + seed, **kw)
    try:
        res = fa.generate(rm, m, ps, max_length=ml, spec=spec)
    except fa.ffmi.FFMIError as e:
        assert spec and "SSM loaded less" in str(e)
        pytest.skip("SSM prompt behind the LLM for this random mix")
    finally:
        m.close()
        for s in ssms:
            s.close()
    for p, r in zip(ps, res):
        ref, rows = oracle_free_running(cfg, 400 + seed, [1] + list(p), ml)
        g = r.output_tokens
        assert len(g) == ml
        if g != ref:
            t = next(i for i in range(ml) if g[i] != ref[i])
            row = rows[t - (len(p) + 1)]
            assert float(row[ref[t]] - row[g[t]]) <= 1e-4, (t, cfg, spec)


@pytest.mark.parametrize("seed", range(2))
def test_random_model_long_context_vs_oracle(seed):
    """Long contexts through the model: max_sequence_length 1024, prompts of
    300-900 tokens loaded in 256-token chunks next to decoding requests, 16
    new tokens each (incremental decoding), every pick teacher-forced through
    the oracle under the tie rule."""
    rng = np.random.default_rng(9700 + OFF + seed)
    cfg = random_cfg(rng)
    V = cfg["vocab_size"]
    ps = [rng.integers(3, V, size=int(rng.integers(300, 900))).tolist() for _ in range(3)]
    ml = max(len(p) for p in ps) + 17
    rm = fa.RequestManager(max_requests_per_batch=3, max_tokens_per_batch=256,
                           max_sequence_length=1024)
    m = fa.Model(cfg, "inc", max_requests=3, max_tokens=256, max_seq_len=1024,
                 weight_seed=700 + seed)
    try:
        res = fa.generate(rm, m, ps, max_length=ml)
    finally:
        m.close()
    check_all(cfg, 700 + seed, ps, res, ml, (cfg, "long"))
