"""The token-parity rule of the GPU tests (test infrastructure).

The reference's own bars (tests/inference/cpp_inference_tests.sh):
- half precision, free-running: the first 30 tokens of two runs identical
  (:104-129, :188-189);
- SpecInfer tokens == incr-decoding tokens (:183-189).
They compare two FlexFlow runs on trained checkpoints, whose greedy picks lead
by wide margins.  Here the GPU is compared with the CPU oracle (same rounding
points, different fp32 summation order) on synthetic weights, so a pick can
flip where two logits are closer than the reordering noise.  One rule, used by
every token-level GPU test, decides whether a GPU pick that differs from the
oracle's is such a tie:

  At the position, teacher-forced (the oracle's logits z0 along the GPU's own
  sequence; the oracle is T-invariant, so they are the free-running logits
  while the prefix agrees), the GPU picked g and the oracle o:
  - ulp: distance of the two tokens' fp16 softmax probabilities; a tie if
    <= TIE_ULP (the numerical tie of argmax over fp16 probabilities,
    argmax.cu:62-100 lowest-index rule);
  - otherwise gap = z0[o] - z0[g] must be <= TIE_SIGMA x sigma_pair, where
    sigma_pair is the standard deviation of the difference of TWO logits of
    that row under a change of fp32 summation order: the oracle re-run with
    its dots reordered (orc_set_dot_variant 1) moves every logit of the row by
    d_i, and sigma_pair = sqrt(2) x std_i(d_i) (32000 samples of the
    per-logit noise at that position, not the row maximum).  The pair's own
    move d_o - d_g is reported beside it.
  A 3-sigma test: a real kernel bug moves logits by far more than the
  reordering noise (test_gpu_bench_workload.py's negative control must FAIL
  this rule).  On shallow models sigma_pair is tiny and the rule reduces to
  the <= 2-ulp probability tie of test_gpu_e2e.py.
  - or gap <= two fp16 ulps of the logits: the logits are fp16 (the
    lm_head output, as the reference's), so a reordering that moves a
    rounding moves a logit by a whole ulp, and when the two logits move one
    ulp each in opposite directions, a two-ulp gap closes (equal logits then
    go to the lower index).  sigma_pair, a standard deviation over the row,
    misses that quantum when few logits of the row move (a 150-seed sweep of
    tests/test_gpu_random_models.py met gaps of one and two logit ulps, 3-7
    probability ulps, at sigma_pair ~ 0.0006, every logit of the reordered
    oracle within one ulp).

Ceiling on the number of ties: a bug that moves logits by 1-3 sigma_pair at
many positions would pass the per-position test, so every token test also
caps the ties at max(2, TIE_MAX_FRAC of its picks) (measured at the bench
workload: 6 / 512 incr decoding, 9 / 512 SpecInfer), or at the count the
measured noise itself predicts where a test has it for every row
(expected_flips: sum over rows of Phi(-gap / sigma_pair)).
"""
import math

import numpy as np

from hip_util import ulp_diff

TIE_ULP = 2
TIE_SIGMA = 3.0
TIE_MAX_FRAC = 0.03


def p16_row(row):
    p = np.exp(row - row.max())
    return (p / p.sum()).astype(np.float16)


def classify(row0, row1, g, o):
    """row0: oracle logits at the position; row1: the same with reordered
    dots (None: no noise estimate, the ulp rule alone)"""
    p16 = p16_row(row0)
    out = dict(gpu=int(g), oracle=int(o), ulp=int(ulp_diff(p16[g], p16[o])),
               gap=float(row0[o] - row0[g]))
    if row1 is not None:
        d = (row1 - row0).astype(np.float64)
        out["sigma_pair"] = float(np.sqrt(2.0) * d.std())
        out["pair_move"] = float(d[o] - d[g])
        out["row_max_move"] = float(np.abs(d).max())
    out["logit_ulp"] = float(np.spacing(np.float16(max(abs(row0[o]), abs(row0[g])))))
    out["tie"] = bool(out["ulp"] <= TIE_ULP or out["gap"] <= 2 * out["logit_ulp"] or
                      ("sigma_pair" in out and out["gap"] <= TIE_SIGMA * out["sigma_pair"]))
    return out


def picks(logits):
    """the oracle's greedy picks: argmax of fp16 softmax, lowest index"""
    import oracle_lib as O
    ids, _ = O.softmax_argmax(np.ascontiguousarray(logits, np.float32), fp16=1)
    return ids


def tie_budget(total):
    """ties allowed among `total` picks"""
    return max(2, int(math.ceil(TIE_MAX_FRAC * total)))


def assert_ties(verdicts, total, budget=None):
    """every mismatch a tie, and no more ties than the budget"""
    bad = [v for v in verdicts if not v["tie"]]
    assert not bad, bad
    cap = tie_budget(total) if budget is None else budget
    assert len(verdicts) <= cap, ("more ties than the budget", len(verdicts), cap, total)


def expected_flips(z0, z1):
    """rows z0 (reference) and z1 (the reordered run): the number of greedy
    picks the reordering noise is expected to flip, sum over rows of
    Phi(-gap / sigma_pair) with gap the top-2 distance of z0 and sigma_pair
    = sqrt(2) x std(z1 - z0) of the row"""
    z0 = np.asarray(z0, np.float64)
    d = np.asarray(z1, np.float64) - z0
    sig = np.sqrt(2.0) * d.std(axis=1)
    top = np.sort(z0, axis=1)[:, -2:]
    gap = top[:, 1] - top[:, 0]
    x = -gap / np.maximum(sig, 1e-30)
    return float(sum(0.5 * math.erfc(-v / math.sqrt(2.0)) for v in x))


def expected_flips_all(z0, z1, competitors=16):
    """expected_flips with every competitor, not the runner-up alone: for
    each row the union bound sum_j Phi(-(z0[top] - z0[j]) / sigma_pair) over
    the `competitors` next-largest logits (a third candidate within the noise
    flips a pick as well as the second; the round-5 TP test met 26 ties
    against 13.6 from the top-2 formula).  An upper estimate of the expected
    flip count, fixed before the data: the tie budget is then
    budget_from_expected(E), a Poisson 3-sigma bound."""
    z0 = np.asarray(z0, np.float64)
    d = np.asarray(z1, np.float64) - z0
    sig = np.maximum(np.sqrt(2.0) * d.std(axis=1), 1e-30)
    srt = -np.sort(-z0, axis=1)[:, :competitors + 1]
    gaps = srt[:, :1] - srt[:, 1:]
    x = gaps / sig[:, None]
    return float(0.5 * np.sum([math.erfc(v / math.sqrt(2.0)) for v in x.ravel()]))


def budget_from_expected(e):
    """ties allowed when e flips are expected: e + 3 sqrt(e) + 2"""
    return int(math.ceil(e + 3.0 * math.sqrt(e) + 2.0))

