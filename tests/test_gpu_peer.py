"""Direct xGMI all-reduce (kernels/collective.hip) across rank PROCESSES.

The reference all-reduces the row-parallel outputs with ncclAllReduce
(allreduce_kernels.cu:53-75).  Here the ranks are separate processes that
exchange through IPC-mapped buffers (tests/peer_group.py); on the one-GPU
test box they share device 0.  Bar: bit-exact against the rank-order fp32
sum rounded once (the transport's stated semantics), on every rank, over
back-to-back rounds that cycle the epochs and buffer parities; a silent peer
is an error after the timeout, never a hang.
"""
import os

import numpy as np
import pytest

import peer_tasks as PT
from peer_group import run_group

pytestmark = pytest.mark.gpu

# (count, dtype): one-shot sizes and >= 256 KiB (two-shot for n > 2), and a
# count that does not split evenly over the ranks' chunks
CASES = [(8, "f16"), (4096, "f32"), (168 * 4096, "f16"), (8 * 8192 + 24, "f16"),
         (3 * 65536 + 8, "f32")]


@pytest.mark.parametrize("n,two_shot", [(2, False), (2, True), (3, False), (4, False)])
def test_peer_allreduce_exact(n, two_shot):
    env = {"FFMI_PEER_TWO_SHOT_MIN": "0"} if two_shot else {}
    res = run_group(n, PT.ar_task, (CASES, 3), env=env, max_bytes=4 << 20)
    for it in range(3):
        for ci, (count, dtype) in enumerate(CASES):
            want = PT.expected_sum(ci, it, n, count, dtype)
            for r in range(n):
                got = res[r][(it, ci)]
                assert got.dtype == want.dtype
                np.testing.assert_array_equal(got, want, err_msg=f"rank {r} case {ci} round {it}")


def test_peer_allreduce_silent_peer_times_out():
    res = run_group(2, PT.silent_peer_task, env={"FFMI_PEER_TIMEOUT_S": "1"})
    r0 = res[0]
    assert r0["status"] != 0, r0
    assert "timeout" in r0["msg"], r0
    assert r0["seconds"] < 30, r0


# (T, H, col0, packed): a decode row, ragged rows, rows fewer than ranks (a
# rank owning none in two-shot mode), the LLaMA-7B verify batch in column
# halves, LLaMA-65B width, beyond one chunk per thread (H 16384)
ARN_CASES = [(1, 256, 0, False), (7, 512, 256, True), (3, 1024, 0, True), (21, 4096, 0, True),
             (168, 4096, 2048, True), (37, 8192, 4096, False), (5, 16384, 8192, False)]


@pytest.mark.parametrize("n,two_shot", [(2, False), (4, False), (4, True), (8, True)])
def test_peer_allreduce_rmsnorm_fused_equals_unfused(n, two_shot):
    """The all-reduce with the residual RMSNorm folded into it (model.cc:
    3421-3470; residual_rms_norm_kernels.cu:98-131) is bit-identical to the
    transport's all-reduce followed by the norm kernel: the normalised rows on
    every rank, the residual on the rows the rank updated (its T/N share in
    two-shot mode, every row in one-shot mode), other rows untouched; two
    rounds, so the epochs and buffer parities cycle."""
    env = {"FFMI_PEER_TWO_SHOT_MIN": "0" if two_shot else str(1 << 40)}
    res = run_group(n, PT.arnorm_task, (ARN_CASES, 99), env=env, max_bytes=2 << 20)
    for r in range(n):
        for c in res[r]:
            T = ARN_CASES[c["case"]][0]
            want = (T * r // n, T * (r + 1) // n) if two_shot else (0, T)
            assert tuple(c["rows"]) == want, (r, c)
            assert c["h_equal"] and c["res_equal"] and c["res_others_untouched"], (r, c)


CFG4 = dict(num_layers=2, vocab_size=1000, num_heads=4, num_kv_heads=4, hidden=256,
            intermediate=512, rms_eps=1e-6, rope_theta=10000.0)


@pytest.mark.parametrize("n,T,V,k", [(2, 168, 4096, 1), (4, 37, 32000, 3), (4, 168, 32000, 1),
                                     (8, 24, 32000, 3)])
def test_vocab_shard_topk_matches_unsharded(n, T, V, k):
    """Vocab-parallel lm_head tail (model.cc:3392-3419): every rank's global
    top-k ids and fp16 probabilities are bit-identical to the oracle's softmax
    + arg-top-k of the gathered logits (softmax.cu:262-288, arg_topk.cu:
    339-448), planted cross-shard ties included (lowest index among equal fp16
    probabilities)."""
    res = run_group(n, PT.vshard_task, (T, V, k, 1234 + n), max_bytes=1 << 20)
    ref_i, ref_p = res[0]["ref_ids"], res[0]["ref_probs"]
    for r in range(n):
        np.testing.assert_array_equal(res[r]["ids"], ref_i, err_msg=f"rank {r}")
        np.testing.assert_array_equal(res[r]["probs"], ref_p, err_msg=f"rank {r}")


CFG4V = dict(CFG4, vocab_size=1024)  # V/TP a multiple of 16: lm_head vocab-sharded
# a long down projection (K = F/TP = 2048): its row-parallel GEMM splits K
# (8 slabs) and the all-reduce's copy-in sums the slabs
CFG4F = dict(CFG4, intermediate=4096)


@pytest.mark.parametrize("tp,overlap,cfg", [(2, "1", CFG4), (2, "0", CFG4), (4, "1", CFG4),
                                            (2, "1", CFG4V), (4, "1", CFG4V), (2, "1", CFG4F),
                                            (2, "0", CFG4F)])
def test_peer_tp_model_decodes_like_unsharded(tp, overlap, cfg):
    """TP shards as separate processes over the xGMI transport (row-parallel
    GEMMs in two column halves, each all-reduced on a second stream while the
    next half computes; the step graphed): every rank emits the same tokens,
    and they are oracle-valid greedy picks of the UNSHARDED model (ties within
    2*TP fp16 ulp, as test_gpu_tp_local)."""
    from test_gpu_e2e import SSM_CFG, check_tokens_vs_oracle, prompts
    ps = prompts(4, cfg["vocab_size"], 4, 30, 7)
    res = run_group(tp, PT.model_task, (cfg, 11, ps, 56, False, SSM_CFG),
                    env={"FFMI_TP_OVERLAP": overlap}, max_bytes=1 << 20)
    for r in range(1, tp):
        assert res[r] == res[0]
    for p, toks in zip(ps, res[0]):
        assert len(toks) == 56
        check_tokens_vs_oracle(cfg, 11, toks, len(p) + 1, tie_ulp=2 * tp,
                               max_tie_frac=0.1)


@pytest.mark.parametrize("tp,two_shot,overlap", [(2, False, "1"), (4, True, "1"), (4, True, "0"),
                                                (4, False, "1"), (8, True, "1")])
def test_peer_tp_fused_norm_equals_unfused(tp, two_shot, overlap):
    """TP shards over the transport with every residual norm folded into the
    all-reduce before it (FFMI_TP_FUSED_NORM, default on; two-shot: each rank
    normalises its T/TP rows and the rows are gathered) against the separate
    norm kernel: identical tokens in incremental decoding and SpecInfer, and
    bit-identical teacher-forced logits (the debug capture, fused with
    FFMI_TP_FUSED_NORM=2)."""
    from test_gpu_e2e import SSM_CFG, prompts
    cfg = CFG4V if tp < 8 else dict(CFG4V, num_heads=8, num_kv_heads=8, hidden=512)
    ps = prompts(3, cfg["vocab_size"], 4, 30, 13)
    ts = {"FFMI_PEER_TWO_SHOT_MIN": "0" if two_shot else str(1 << 40), "FFMI_TP_OVERLAP": overlap}
    ssm = dict(SSM_CFG, vocab_size=cfg["vocab_size"])
    got = {}
    for fused in ("0", "2"):
        env = dict(ts, FFMI_TP_FUSED_NORM=fused)
        inc = run_group(tp, PT.tp_generate_task, (cfg, 11, ps, 48, False, ssm), env=env,
                        max_bytes=1 << 20)
        spec = run_group(tp, PT.model_task, (cfg, 11, ps, 48, True, ssm), env=env,
                         max_bytes=1 << 20)
        got[fused] = (inc, spec)
    (i0, s0), (i2, s2) = got["0"], got["2"]
    for r in range(tp):
        assert i2[r]["tokens"] == i0[r]["tokens"] == i0[0]["tokens"], r
        assert s2[r] == s0[r] == s0[0], r
        np.testing.assert_array_equal(i2[r]["tf_logits"].view(np.uint16),
                                      i0[r]["tf_logits"].view(np.uint16), err_msg=f"rank {r}")


OFF = int(os.environ.get("FFMI_RANDOM_SEED_OFFSET", "0"))  # fresh seeds for one-off sweeps


@pytest.mark.parametrize("seed", range(6 * int(os.environ.get("FFMI_RANDOM_SCALE", "1"))))
def test_peer_tp_random_models(seed):
    """TP 2 or 4 over the transport at random small LLaMA shapes (heads a
    multiple of TP, d 64 / 128, FFN and vocabulary random: the vocabulary
    sharded when V/TP is a multiple of 16, else the unsharded tail), random
    prompts, overlap on or off, incremental decoding or SpecInfer: every rank
    emits the same tokens, oracle-valid picks of the UNSHARDED model under
    the TP tie rule of test_peer_tp_model_decodes_like_unsharded."""
    from test_gpu_e2e import SSM_CFG, check_tokens_vs_oracle
    rng = np.random.default_rng(4100 + OFF + seed)
    tp = int(rng.choice([2, 4]))
    heads = tp * int(rng.integers(1, 3))
    d = int(rng.choice([64, 128]))
    V = int(rng.choice([16 * tp * int(rng.integers(8, 120)), int(rng.integers(200, 3000))]))
    cfg = dict(num_layers=int(rng.integers(1, 3)), vocab_size=V, num_heads=heads,
               num_kv_heads=heads, hidden=heads * d, intermediate=32 * tp * int(rng.integers(1, 12)),
               rms_eps=1e-6, rope_theta=10000.0)
    ps = [rng.integers(3, V, size=int(rng.integers(2, 40))).tolist()
          for _ in range(int(rng.integers(1, 5)))]
    ml = max(len(p) for p in ps) + 1 + int(rng.integers(8, 24))
    spec = bool(rng.integers(0, 2))
    res = run_group(tp, PT.model_task, (cfg, 11, ps, ml, spec, dict(SSM_CFG, vocab_size=V)),
                    env={"FFMI_TP_OVERLAP": str(int(rng.integers(0, 2)))}, max_bytes=1 << 20)
    for r in range(1, tp):
        assert res[r] == res[0], (cfg, tp, spec)
    for p, toks in zip(ps, res[0]):
        assert len(toks) == ml
        check_tokens_vs_oracle(cfg, 11, toks, len(p) + 1, tie_ulp=2 * tp, max_tie_frac=0.1)


@pytest.mark.parametrize("seed", range(4 * int(os.environ.get("FFMI_RANDOM_SCALE", "1"))))
def test_peer_tp_random_models_spec_extensions(seed):
    """TP 2 or 4 rank processes running the flagged extensions (tree width 4,
    four merged SSMs; tests/spec_configs.py) at random small LLaMA shapes:
    every rank emits the same tokens, oracle-valid picks of the UNSHARDED
    model under the TP tie rule."""
    from test_gpu_e2e import SSM_CFG, check_tokens_vs_oracle
    rng = np.random.default_rng(4300 + OFF + seed)
    tp = int(rng.choice([2, 4]))
    heads = tp * int(rng.integers(1, 3))
    d = int(rng.choice([64, 128]))
    V = int(16 * tp * int(rng.integers(8, 60)))
    cfg = dict(num_layers=int(rng.integers(1, 3)), vocab_size=V, num_heads=heads,
               num_kv_heads=heads, hidden=heads * d, intermediate=32 * tp * int(rng.integers(1, 12)),
               rms_eps=1e-6, rope_theta=10000.0)
    ps = [rng.integers(3, V, size=int(rng.integers(2, 40))).tolist()
          for _ in range(int(rng.integers(1, 5)))]
    ml = max(len(p) for p in ps) + 1 + int(rng.integers(8, 24))
    spec = ["w114", "ssm4"][seed % 2]
    res = run_group(tp, PT.tp_generate_task,
                    (cfg, 11, ps, ml, spec, dict(SSM_CFG, vocab_size=V)), max_bytes=2 << 20)
    for r in range(1, tp):
        assert res[r]["tokens"] == res[0]["tokens"], (cfg, tp, spec)
    for p, toks in zip(ps, res[0]["tokens"]):
        assert len(toks) == ml
        check_tokens_vs_oracle(cfg, 11, toks, len(p) + 1, tie_ulp=2 * tp, max_tie_frac=0.1)


@pytest.mark.parametrize("queues", ["1", None], ids=["one_queue", "hip_default_queues"])
def test_peer_tp2_spec_infer_equals_incr(queues):
    """SpecInfer over the transport: identical to incremental decoding of the
    same sharded model (the reference invariant, cpp_inference_tests.sh:183-189).
    Also run with HIP's default hardware queues per rank, where the compute and
    all-reduce streams really overlap, so a missing cross-stream event wait
    shows up (one queue per rank serialises the two streams)."""
    from test_gpu_e2e import SSM_CFG, prompts
    ps = prompts(3, CFG4V["vocab_size"], 5, 30, 9)
    ssm = dict(SSM_CFG, vocab_size=1024)
    env = {"GPU_MAX_HW_QUEUES": queues}
    inc = run_group(2, PT.model_task, (CFG4V, 11, ps, 60, False, ssm), env=env,
                    max_bytes=1 << 20)
    spec = run_group(2, PT.model_task, (CFG4V, 11, ps, 60, True, ssm), env=env,
                     max_bytes=1 << 20)
    assert spec[0] == spec[1] == inc[0] == inc[1]


# LLaMA-65B widths (configs D/E: hidden 8192, 64 heads of 128, FFN 22016,
# vocab 32000), one layer, sharded over 8 rank processes exactly as the
# driver's TP = 8 run shards it: per-rank qkv 3072 x 8192, o 8192 x 1024,
# gate|up 2 x 2752 x 8192, down 8192 x 2752, lm_head vocab shard 4000 x 8192
CFG65 = dict(num_layers=1, vocab_size=32000, num_heads=64, num_kv_heads=64, hidden=8192,
             intermediate=22016, rms_eps=1e-5, rope_theta=10000.0)


def test_peer_tp8_llama65b_width_decodes_like_unsharded():
    """Config D's per-rank shapes end to end: 8 ranks over the xGMI transport
    (row-parallel halves all-reduced on the second stream, vocab-sharded tail,
    graphed steps) emit identical tokens on every rank, each an oracle-valid
    greedy pick of the unsharded model (ties within 2*TP fp16 ulp)."""
    from test_gpu_e2e import SSM_CFG, check_tokens_vs_oracle, prompts
    ps = prompts(2, CFG65["vocab_size"], 4, 12, 3)
    res = run_group(8, PT.model_task, (CFG65, 11, ps, 24, False, SSM_CFG), max_bytes=8 << 20)
    for r in range(1, 8):
        assert res[r] == res[0]
    for p, toks in zip(ps, res[0]):
        assert len(toks) == 24
        check_tokens_vs_oracle(CFG65, 11, toks, len(p) + 1, tie_ulp=16,
                               max_tie_frac=0.1)


def test_peer_tp8_llama65b_width_spec_infer_equals_incr():
    """Config E's per-rank shapes: SpecInfer at LLaMA-65B widths over 8 rank
    processes (tree-verify attention of 8 local heads, row-parallel halves
    all-reduced over the transport, vocab-sharded tail, graphed verify steps)
    with the LLaMA-68M-shaped SSM replicated on every rank, as the reference
    runs its SSM at TP = 1 beside a TP LLM (spec_infer.cc:385-387).  Every
    rank emits the same tokens, and they equal incremental decoding of the
    same sharded model (cpp_inference_tests.sh:183-189).  (One SSM: the
    reference's multi-SSM merge asserts, request_manager.cc:2823-2877.)"""
    from test_gpu_e2e import prompts
    ssm = dict(num_layers=2, vocab_size=32000, num_heads=12, num_kv_heads=12, hidden=768,
               intermediate=3072, rms_eps=1e-6, rope_theta=10000.0)
    ps = prompts(3, CFG65["vocab_size"], 4, 12, 5)
    inc = run_group(8, PT.model_task, (CFG65, 11, ps, 28, False, ssm), max_bytes=8 << 20)
    spec = run_group(8, PT.model_task, (CFG65, 11, ps, 28, True, ssm), max_bytes=8 << 20)
    for r in range(8):
        assert spec[r] == spec[0] and inc[r] == inc[0], r
    assert spec[0] == inc[0]
    assert all(len(t) == 28 for t in spec[0])
