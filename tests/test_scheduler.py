"""RequestManager (continuous batching + SpecInfer tree scheduler) on CPU.

Uses the library's hash test double: a model whose next token is a hash of
exactly the token context its attention would see under the packed KV-slot /
bitmask rules.  Mirrors the reference's own invariants:
  * incr decoding == plain greedy decoding of the hash "LM";
  * SpecInfer tokens == incr-decoding tokens
    (tests/inference/cpp_inference_tests.sh:183-189);
  * SpecInfer needs far fewer LLM steps when the SSM agrees
    (cpp_inference_tests.sh:155-181: incr steps >= 1.5 x spec steps).
"""
import os

import numpy as np
import pytest

import flexflow_amd as fa

M64 = (1 << 64) - 1


def mix64(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def next_tok(ctx, V):
    h = 0x243F6A8885A308D3
    for t in ctx:
        h = mix64((h + t + 1) & M64)
    return (h >> 17) % V


def expected(prompt, max_length, V, bos=1, eos=()):
    toks = [bos] + list(prompt)
    while len(toks) < max_length:
        toks.append(next_tok(toks, V))
        if toks[-1] in eos:
            toks.pop()
            break
    return toks


def prompts(n, V, lo=3, hi=40, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.integers(3, V, size=int(rng.integers(lo, hi))).tolist() for _ in range(n)]


V = 997


def run_incr(ps, max_length, batch=4, max_tokens=16, eos=(), msl=128):
    rm = fa.RequestManager(max_requests_per_batch=batch, max_tokens_per_batch=max_tokens,
                           max_sequence_length=msl, eos_token_ids=eos)
    llm = fa.HashModel(V, "inc", max_requests=batch, max_seq_len=msl)
    res = fa.generate(rm, llm, ps, max_length=max_length)
    return res, rm.stats()


def run_spec(ps, max_length, batch=4, max_tokens=64, widths=(1, 1, 3), disagree=0,
             tree_tokens=23, ssms=None, ext=0, eos=(), msl=128):
    """ssms: [(salt, disagree_pct)] per SSM (default one SSM, salt 1234)."""
    rm = fa.RequestManager(max_requests_per_batch=batch, max_tokens_per_batch=max_tokens,
                           max_sequence_length=msl, spec_tree_width=widths,
                           max_spec_tree_token_num=tree_tokens, spec_extensions=ext,
                           eos_token_ids=eos)
    llm = fa.HashModel(V, "tree", max_requests=batch, max_seq_len=msl,
                       max_tree_tokens=tree_tokens)
    for salt, dis in ssms or [(1234, disagree)]:
        rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=batch, max_seq_len=msl,
                                           max_tree_tokens=tree_tokens, salt=salt,
                                           disagree_pct=dis))
    res = fa.generate(rm, llm, ps, max_length=max_length)
    return res, rm.stats()


@pytest.mark.parametrize("batch,max_tokens", [(1, 8), (4, 16), (8, 128), (3, 5)])
def test_incr_decoding_matches_greedy(batch, max_tokens):
    ps = prompts(7, V)
    res, st = run_incr(ps, 70, batch=batch, max_tokens=max_tokens)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 70, V)
    assert st.llm_steps > 0


def test_incr_decoding_eos_stops_and_is_dropped():
    ps = prompts(4, V, seed=3)
    # pick an eos that occurs in one of the greedy continuations
    full = expected(ps[0], 70, V)
    eos = full[len(ps[0]) + 5]
    res, _ = run_incr(ps, 70, eos=(eos,))
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 70, V, eos=(eos,))


@pytest.mark.parametrize("disagree", [0, 30, 100])
@pytest.mark.parametrize("widths", [(1, 1, 3), (), (3,), (1, 2), (2, 1, 1)])
def test_spec_infer_equals_incr(disagree, widths):
    ps = prompts(6, V, seed=11)
    res, st = run_spec(ps, 90, widths=widths, disagree=disagree)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 90, V), (disagree, widths)
    assert st.llm_steps > 0 and st.ssm_steps == 8 * st.llm_steps or st.ssm_steps > 0


def test_spec_infer_prompt_chunking_and_queueing():
    # more requests than slots, prompts longer than the token budget
    ps = prompts(9, V, lo=30, hi=60, seed=5)
    res, _ = run_spec(ps, 100, batch=3, max_tokens=24, disagree=20)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 100, V)


def test_spec_infer_step_efficiency():
    # reference CI bar: incr LLM steps >= 1.5 x spec-infer LLM steps
    ps = prompts(4, V, seed=7)
    _, s_inc = run_incr(ps, 100, batch=4, max_tokens=64)
    res, s_spec = run_spec(ps, 100, batch=4, max_tokens=64, disagree=0)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 100, V)
    assert s_inc.llm_steps >= 1.5 * s_spec.llm_steps
    # with a perfect SSM every verify accepts a full 8-deep branch + bonus
    mv = 64 + 23 * 4
    assert sum(len(r.input_tokens) for r in res) <= mv - len(res)  # one prompt-load step each
    for r in res:
        assert len(r.input_tokens) <= 64  # the SSM loads each prompt in its admission batch
        assert r.llm_decoding_steps == expected_verify_steps(len(r.input_tokens), 100, 64, 4)


def expected_verify_steps(in_len, max_length, max_tokens, batch=1, tree_tokens=23):
    """Per-request llm_decoding_steps of a one-request SpecInfer run whose SSM
    always agrees with the LLM, restated from the reference's accounting:
    0 at admission (request_manager.cc:1488) and +1 per verify batch the
    request is in (:1958).
      * The LLM loads the prompt in chunks of the verify budget
        (max_tokens + tree_tokens x batch, :152-156) minus one slot per waiting
        request (:1938-1946, :2137-2141); the last chunk yields the first new
        token.
      * Each later verify commits the full MAX_BEAM_DEPTH (8) branch plus the
        bonus token, the depth capped by the tokens left (:1355-1369) --
      * unless the SSM loaded the prompt over three or more beam batches
        (max_tokens at admission, then max_tokens - 1 each): the reference
        feeds every beam prompt chunk the LAST n tokens of the request, not
        the ones at its depths (`request.tokens[size - num_tokens_in_batch +
        j]`, :1873-1875), which is right only for the final chunk; a middle
        chunk caches the wrong ids, and (hash model) the SSM never agrees
        again: one token per verify.  Reproduced, not fixed."""
    chunks = -(-in_len // (max_tokens + tree_tokens * batch - 1))
    left = max(0, max_length - (in_len + 1))
    per_verify = 1 if in_len > 2 * max_tokens - 1 else 9
    return chunks + -(-left // per_verify)


@pytest.mark.parametrize("plen,max_length,max_tokens", [
    (5, 30, 64), (5, 64, 64), (5, 100, 64), (20, 30, 64), (20, 90, 64), (40, 50, 64),
    (5, 100, 16), (14, 60, 16), (20, 60, 16), (29, 60, 16),  # SSM loads in <= 2 batches
    (30, 32, 8), (50, 100, 8), (45, 80, 16), (90, 120, 16)])  # >= 3: wrong SSM prompt
def test_spec_infer_llm_decoding_steps_per_request(plen, max_length, max_tokens):
    ps = [list(range(3, 3 + plen))]
    res, st = run_spec(ps, max_length, batch=1, max_tokens=max_tokens, disagree=0)
    r = res[0]
    assert r.output_tokens == expected(ps[0], max_length, V)
    want = expected_verify_steps(len(r.input_tokens), max_length, max_tokens)
    assert r.llm_decoding_steps == want
    assert st.llm_steps == want  # one request: one verify launch per step
    assert r.ttft_us > 0  # from registration; latency_us counts from admission


def test_spec_infer_ssm_prompt_behind_is_an_error():
    # max_tokens 8: the SSM loads 8 + 8 x 7 = 64 prompt tokens per iteration,
    # the LLM 30 per verify; a 71-token prompt trips the reference's assert
    # (request_manager.cc:1425) -- here a reported error, not an abort
    with pytest.raises(fa.ffmi.FFMIError, match="SSM loaded less"):
        run_spec([list(range(3, 73))], 100, batch=1, max_tokens=8, disagree=0)


def test_request_limits_rejected():
    rm = fa.RequestManager(max_sequence_length=32)
    assert rm.register_new_request(list(range(3, 40)), max_length=10) == 0  # prompt too long
    assert rm.register_new_request([5, 6], max_length=32) == 0  # max_length >= max_seq
    assert rm.register_new_request([5, 6], max_length=31) > 0


def test_tree_width_limit():
    with pytest.raises(fa.ffmi.FFMIError):
        fa.RequestManager(spec_tree_width=(4,))  # MAX_BEAM_WIDTH = 3 (request_manager.cc:168)
    with pytest.raises(fa.ffmi.FFMIError):
        fa.RequestManager(spec_tree_width=(2, 2))  # 4 nodes/layer > 3 (request_manager.cc:1685)
    # the flagged width-4 extension (BASELINE config C): widths and branches <= 4
    W4 = fa.ffmi.SPEC_EXT_WIDTH4
    for w in [(4,), (1, 1, 4), (2, 2), (1, 4, 1)]:
        fa.RequestManager(spec_tree_width=w, spec_extensions=W4)
    for w in [(5,), (2, 3), (4, 2)]:
        with pytest.raises(fa.ffmi.FFMIError):
            fa.RequestManager(spec_tree_width=w, spec_extensions=W4)
    with pytest.raises(fa.ffmi.FFMIError):
        fa.RequestManager(spec_extensions=8)  # unknown extension bit


W4 = fa.ffmi.SPEC_EXT_WIDTH4
MULTI = fa.ffmi.SPEC_EXT_MULTI_SSM


@pytest.mark.parametrize("disagree", [0, 30, 100])
@pytest.mark.parametrize("widths", [(1, 1, 4), (4,), (2, 2), (1, 4), (2, 1, 2)])
def test_spec_infer_width4_equals_incr(disagree, widths):
    """Config C as BASELINE states it (tree width 4): SpecInfer reproduces
    incremental decoding exactly, including trees that branch twice ((2, 2):
    the parent-link verify walk)."""
    ps = prompts(6, V, seed=11)
    res, st = run_spec(ps, 90, widths=widths, disagree=disagree, tree_tokens=40, ext=W4)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 90, V), (disagree, widths)
    assert st.llm_steps > 0


@pytest.mark.parametrize("widths", [(1, 1, 3), (1, 1, 4)])
@pytest.mark.parametrize("ssms", [
    [(1234, 0), (99, 0)],                      # two agreeing SSMs: identical trees
    [(1234, 30), (99, 30)],                    # partly different trees
    [(1234, 30), (99, 60), (7, 90), (5, 100)],  # config E: 4 SSMs, merged up to the cap
    [(1, 100), (2, 100), (3, 100), (4, 100)],
])
def test_spec_infer_multi_ssm_equals_incr(widths, ssms):
    """Config E's 4x SSMs: the merged token tree (merge_dfs_trees restated
    with path identity) verifies to exactly the incremental-decoding tokens;
    merged trees beyond max_spec_tree_token_num (64) are cut in layer order."""
    ps = prompts(6, V, seed=13)
    res, st = run_spec(ps, 90, widths=widths, tree_tokens=64, ssms=ssms, ext=W4 | MULTI,
                       max_tokens=64)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 90, V), (widths, ssms)
    assert st.ssm_steps > 0 and st.llm_steps > 0


def test_multi_ssm_merge_keeps_the_agreeing_branch():
    """A perfect SSM merged with SSMs that never agree: the union still holds
    the perfect chain, so every verify accepts it (as many LLM steps as the
    perfect SSM alone), whatever the SSM order."""
    ps = prompts(4, V, seed=7)
    _, alone = run_spec(ps, 100, disagree=0, tree_tokens=64, ext=MULTI)
    for ssms in ([(1234, 0), (5, 100), (6, 100)], [(5, 100), (6, 100), (1234, 0)]):
        res, st = run_spec(ps, 100, tree_tokens=64, ssms=ssms, ext=MULTI)
        for p, r in zip(ps, res):
            assert r.output_tokens == expected(p, 100, V)
        assert st.llm_steps == alone.llm_steps
        assert st.ssm_steps == 3 * alone.ssm_steps


def test_multi_ssm_needs_the_extension_flag():
    with pytest.raises(fa.ffmi.FFMIError, match="UNSUPPORTED|unsupported"):
        run_spec(prompts(2, V), 40, ssms=[(1, 0), (2, 0)])


@pytest.mark.parametrize("tree_tokens", [23, 48])
def test_multi_ssm_chunked_prompts_and_queueing(tree_tokens):
    """The extensions under the scheduler's other paths: more requests than
    batch slots and prompts longer than the token budget, loaded in chunks by
    the LLM and by every SSM.  Round 5 found two batch-capacity bugs here, both
    the reference's own accounting: a verify batch that overflowed (prompt
    chunks budgeted at MAX_BEAM_DEPTH + 1 tokens per running request, trees
    larger than that; the reference asserts, :2137-2147) and verified tokens
    dropped from request.tokens once the next init batch held
    max_tokens_per_batch tokens (:1402-1404)."""
    ps = prompts(9, V, lo=30, hi=60, seed=5)
    res, st = run_spec(ps, 100, batch=3, max_tokens=24, tree_tokens=tree_tokens,
                       ssms=[(1234, 20), (99, 40), (7, 100)], ext=MULTI)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 100, V), tree_tokens
    assert st.ssm_steps > 0


def test_spec_infer_verifies_root_plus_budget_nodes():
    """max_spec_tree_token_num counts the tree's nodes BELOW the root: widths
    (1,1,3) over 8 beam steps grow 1 + 1 + 1 + 3 x 6 = 21 nodes with the root,
    and under the reference's default llama budget of 20 the reference
    verifies them all (the root's KV slot is in the committed range, so the
    models' tail of max_spec_tree_token_num slots holds the 20 below it).  A
    perfectly agreeing SSM then commits 9 tokens per verify, as with a budget
    of 23; a budget of 19 cuts the last leaf."""
    ps = prompts(4, V, lo=5, hi=9, seed=21)
    st = {}
    for budget in (19, 20, 23):
        res, st[budget] = run_spec(ps, 120, tree_tokens=budget, disagree=0)
        for p, r in zip(ps, res):
            assert r.output_tokens == expected(p, 120, V), budget
    # 20 places exactly what 23 does (no tree is cut), 19 cuts one leaf per
    # full tree
    assert st[20].tree_tokens_verified == st[23].tree_tokens_verified
    assert st[20].llm_steps == st[23].llm_steps
    assert st[19].tree_tokens_verified < st[20].tree_tokens_verified


def test_spec_infer_ssm_capacity_checked_up_front():
    """An SSM sized by max_tokens_per_batch alone (64) can be handed an init
    batch of max_requests x 9 verified tokens (8 x 9 = 72) once acceptance is
    high.  serve_spec_infer checks every SSM's capacity against the largest
    batch the scheduler can build before the first step, with a message,
    instead of failing partway through a serve; a model of that size runs."""
    ps = prompts(8, V, lo=5, hi=9, seed=2)
    rm = fa.RequestManager(max_requests_per_batch=8, max_tokens_per_batch=64,
                           max_sequence_length=128, spec_tree_width=(1, 1, 3))
    llm = fa.HashModel(V, "tree", max_requests=8, max_seq_len=128)
    rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=8, max_seq_len=128,
                                       max_tokens=64))
    with pytest.raises(fa.ffmi.FFMIError, match="holds 64 tokens per step"):
        fa.generate(rm, llm, ps, max_length=100)
    rm = fa.RequestManager(max_requests_per_batch=8, max_tokens_per_batch=64,
                           max_sequence_length=128, spec_tree_width=(1, 1, 3))
    rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=8, max_seq_len=128,
                                       max_tokens=72))
    res = fa.generate(rm, llm, ps, max_length=100)
    for p, r in zip(ps, res):
        assert r.output_tokens == expected(p, 100, V)


def test_requests_registered_before_the_last_ssm():
    """Requests registered while fewer SSMs were registered get one beam tree
    per SSM when the serve starts (each SSM writes its own)."""
    ps = prompts(3, V, seed=4)
    rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=64,
                           max_sequence_length=128, spec_tree_width=(1, 1, 3),
                           spec_extensions=MULTI)
    llm = fa.HashModel(V, "tree", max_requests=4, max_seq_len=128)
    rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=4, max_seq_len=128, salt=1))
    guids = [rm.register_new_request(p, max_length=80) for p in ps]
    rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=4, max_seq_len=128, salt=2,
                                       disagree_pct=50))
    rm.serve_spec_infer(llm)
    for p, g in zip(ps, guids):
        assert rm.get_generation_result(g).output_tokens == expected(p, 80, V)


@pytest.mark.parametrize("seed", range(12))
def test_chained_ssm_steps_equal_stepwise(seed, monkeypatch):
    """Chained beam steps (the speculation phase's 8 steps staged from
    placeholder results and launched back to back, the bookkeeping replayed
    on the results; the hash model runs them as the GPU model does) against
    the stepwise loop (FFMI_SSM_CHAIN=0): identical tokens, LLM and SSM step
    counts, tree tokens verified and commits, for random batches, widths,
    SSM counts and queueing.  Phases where a loading prompt shares a step
    with running requests of another width run stepwise (the reference's
    ArgTopK k rule makes the scheduler read past such a step's results)."""
    rng = np.random.default_rng(9000 + OFF + seed)
    widths = WIDTHS[int(rng.integers(0, len(WIDTHS)))]
    nssm = int(rng.integers(1, 4))
    kw = dict(batch=int(rng.integers(1, 6)), max_tokens=int(rng.integers(24, 96)),
              widths=widths, tree_tokens=int(rng.choice([23, 40, 64])),
              ssms=[(int(rng.integers(1, 10 ** 6)), int(rng.choice([0, 30, 100])))
                    for _ in range(nssm)],
              ext=W4 | MULTI)
    ps = prompts(int(rng.integers(1, 9)), V, lo=2, hi=30, seed=seed)
    ml = int(rng.integers(40, 110))
    monkeypatch.setenv("FFMI_SSM_CHAIN", "0")
    ref, st0 = run_spec(ps, ml, **kw)
    monkeypatch.setenv("FFMI_SSM_CHAIN", "1")
    res, st1 = run_spec(ps, ml, **kw)
    assert [r.output_tokens for r in res] == [r.output_tokens for r in ref]
    assert [r.output_tokens for r in res] == [expected(p, ml, V) for p in ps]
    for f in ("llm_steps", "ssm_steps", "tokens_committed", "tree_tokens_verified",
              "request_verifies"):
        assert getattr(st1, f) == getattr(st0, f), f
    assert st0.ssm_phases_chained == 0
    assert st1.ssm_phases_chained > 0


def test_spec_infer_ignores_eos_like_the_reference():
    """SpecInfer completes a request on max_length only: the verify path never
    checks EOS (request_manager.cc:1251-1253), unlike incremental decoding
    (:650-655, :771-774).  The same holds here, one SSM or several."""
    ps = prompts(4, V, seed=3)
    eos = expected(ps[0], 70, V)[len(ps[0]) + 5]
    for ssms, ext in (([(1234, 20)], 0), ([(1234, 20), (99, 40)], MULTI)):
        res, _ = run_spec(ps, 70, ssms=ssms, ext=ext, eos=(eos,))
        for p, r in zip(ps, res):
            assert r.output_tokens == expected(p, 70, V)  # EOS not applied
    inc, _ = run_incr(ps, 70, eos=(eos,))
    assert inc[0].output_tokens == expected(ps[0], 70, V, eos=(eos,))
    assert len(inc[0].output_tokens) < 70


OFF = int(os.environ.get("FFMI_RANDOM_SEED_OFFSET", "0"))  # fresh seeds for one-off sweeps
WIDTHS = [(1, 1, 3), (3,), (1, 2), (2, 1, 1), (1, 1, 4), (4,), (2, 2), (1, 4), (2, 1, 2), ()]


@pytest.mark.parametrize("block", range(10))
def test_spec_infer_randomized_configs_equal_incr(block):
    """Randomised scheduler configurations (batch slots, token budget, tree
    widths up to 4, tree budget, 1-4 SSMs with different agreement, 1-10
    requests, prompt lengths, max_length): SpecInfer reproduces incremental
    decoding exactly.  Configurations whose prompts the SSM cannot load in
    time raise the reported FFMI error (the reference asserts) and are
    skipped."""
    import random
    checked = 0
    for seed in range(OFF + block * 40, OFF + block * 40 + 40):
        r = random.Random(seed)
        batch = r.choice([1, 2, 3, 4, 8])
        mt = r.choice([8, 16, 24, 32, 64, 128])
        widths = r.choice(WIDTHS)
        nssm = r.choice([1, 1, 2, 3, 4])
        tree = r.choice([16, 23, 27, 32, 48, 64])
        ssms = [(r.randrange(1, 10000), r.choice([0, 10, 30, 60, 100])) for _ in range(nssm)]
        ps = prompts(r.randint(1, 10), V, lo=2, hi=max(3, min(2 * mt, 60)), seed=seed)
        ml = min(127, max(r.choice([40, 70, 100, 127]), max(len(p) for p in ps) + 3))
        try:
            res, _ = run_spec(ps, ml, batch=batch, max_tokens=mt, widths=widths,
                              tree_tokens=tree, ssms=ssms, ext=W4 | (MULTI if nssm > 1 else 0))
        except fa.ffmi.FFMIError as e:
            assert "SSM loaded less" in str(e), (seed, str(e))
            continue
        for p, q in zip(ps, res):
            assert q.output_tokens == expected(p, ml, V), seed
        checked += 1
    assert checked >= 25


@pytest.mark.parametrize("seed", range(8))
def test_incr_decoding_randomized_configs(seed):
    """Incremental decoding under random slots / token budgets / EOS: equal
    to greedy decoding with the EOS dropped (request_manager.cc:771-774)."""
    import random
    r = random.Random(1000 + OFF + seed)
    ps = prompts(r.randint(1, 12), V, lo=1, hi=50, seed=OFF + seed)
    ml = r.choice([60, 90, 127])
    full = expected(ps[0], ml, V)
    eos = (full[len(ps[0]) + r.randint(1, 8)],) if r.random() < 0.7 else ()
    res, _ = run_incr(ps, ml, batch=r.choice([1, 2, 3, 5, 8]), max_tokens=r.choice([4, 7, 16, 64]),
                      eos=eos)
    for p, q in zip(ps, res):
        assert q.output_tokens == expected(p, ml, V, eos=eos), seed


@pytest.mark.parametrize("block", range(4))
def test_spec_infer_randomized_sequence_limits(block):
    """Random max_sequence_length (48-512) with max_length up to its last
    allowed value (the reference rejects max_length >= max_sequence_length,
    request_manager.cc:386-391), long prompts loaded in chunks, random trees
    and SSMs: SpecInfer == incremental decoding == greedy, so commits and
    tree slots near the end of each request's cache rows stay exact."""
    import random
    checked = 0
    for seed in range(OFF + 50000 + block * 25, OFF + 50000 + block * 25 + 25):
        r = random.Random(seed)
        msl = r.choice([48, 64, 100, 128, 256, 512])
        batch = r.choice([1, 2, 4, 8])
        mt = r.choice([16, 32, 64, 128])
        widths = r.choice(WIDTHS)
        nssm = r.choice([1, 1, 2, 4])
        tree = r.choice([16, 23, 27, 48, 64])
        ssms = [(r.randrange(1, 10000), r.choice([0, 10, 50, 100])) for _ in range(nssm)]
        ps = prompts(r.randint(1, 8), V, lo=1, hi=max(2, msl // 2), seed=seed)
        ml = r.randint(max(len(p) for p in ps) + 2, msl - 1)
        try:
            res, _ = run_spec(ps, ml, batch=batch, max_tokens=mt, widths=widths, tree_tokens=tree,
                              ssms=ssms, ext=W4 | (MULTI if nssm > 1 else 0), msl=msl)
        except fa.ffmi.FFMIError as e:
            assert "SSM loaded less" in str(e), (seed, str(e))
            continue
        inc, _ = run_incr(ps, ml, batch=batch, max_tokens=mt, msl=msl)
        for p, q, i in zip(ps, res, inc):
            want = expected(p, ml, V)
            assert q.output_tokens == want and i.output_tokens == want, (seed, msl, ml)
        checked += 1
    assert checked >= 15
