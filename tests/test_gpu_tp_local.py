"""Tensor-parallel invariance of the GPU path on ONE device.

The reference checks that TP degrees give the same tokens
(tests/inference/cpp_inference_tests.sh:203-217).  RCCL refuses two ranks on
one GPU, so here the shards run as host threads of one process over an
in-process shard group (ffmi_comm_create_local): the same sharded weights
(file_loader.cc:286-303 row/column split), the same two all-reduces per layer
(model.cc:3421-3445) and the same replicated norms / lm_head / SSM as a
one-process-per-GPU run, only the sum is done by a group kernel instead of
RCCL.  Every rank must emit identical tokens, and those must be oracle-valid
greedy sequences of the UNSHARDED model: >= 90 % exact picks, every other pick
a tie within 2*TP fp16 ulp (each of the TP row-parallel partial sums is
rounded to fp16 before the all-reduce, so the logits carry up to TP extra
roundings per layer against the unsharded fp32-accumulated GEMM).
"""
import threading

import pytest

import flexflow_amd as fa
from test_gpu_e2e import LLM_CFG, SSM_CFG, check_tokens_vs_oracle, prompts

pytestmark = pytest.mark.gpu

CFG4 = dict(num_layers=2, vocab_size=1000, num_heads=4, num_kv_heads=4, hidden=256,
            intermediate=512, rms_eps=1e-6, rope_theta=10000.0)
CFG8 = dict(num_layers=2, vocab_size=1000, num_heads=8, num_kv_heads=8, hidden=512,
            intermediate=1024, rms_eps=1e-6, rope_theta=10000.0)


def run_tp(cfg, seed, tp, ps, max_length, spec=False):
    comms = fa.Comm.local_group(tp)
    mode = "tree" if spec else "inc"
    extra = 23 * 4 if spec else 0
    models = [fa.Model(cfg, mode, max_requests=4, max_tokens=32 + extra, max_seq_len=128,
                       weight_seed=seed, tp_rank=r, tp_size=tp, comm=comms[r])
              for r in range(tp)]
    rms = []
    for r in range(tp):
        rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=32,
                               max_sequence_length=128,
                               spec_tree_width=(1, 1, 3) if spec else ())
        if spec:  # the SSM is replicated per rank (TP = 1, spec_infer.cc:385-387)
            rm.register_ssm_model(fa.Model(SSM_CFG, "beam", max_requests=4,
                                           max_tokens=32 + extra, max_seq_len=128,
                                           weight_seed=5))
        rms.append(rm)
    out, err = [None] * tp, []

    def work(r):
        try:
            fa.set_device(0)
            out[r] = fa.generate(rms[r], models[r], ps, max_length=max_length)
        except Exception as e:  # noqa: BLE001 -- reported below
            err.append((r, e))

    th = [threading.Thread(target=work, args=(r,)) for r in range(tp)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not err, err
    assert all(o is not None for o in out)
    for m in models:
        m.close()
    for c in comms:
        c.close()
    return out


@pytest.mark.parametrize("cfg,tp", [(LLM_CFG, 2), (CFG4, 2), (CFG4, 4), (CFG8, 8),
                                    (dict(CFG4, vocab_size=1024), 4)])
def test_tp_shards_decode_like_unsharded_model(cfg, tp):
    ps = prompts(4, cfg["vocab_size"], 4, 30, 7)
    res = run_tp(cfg, 11, tp, ps, 56)
    for r in range(1, tp):  # replicated lm_head + identical all-reduce sums
        assert [x.output_tokens for x in res[r]] == [x.output_tokens for x in res[0]]
    for p, x in zip(ps, res[0]):
        assert len(x.output_tokens) == 56
        check_tokens_vs_oracle(cfg, 11, x.output_tokens, len(p) + 1, tie_ulp=2 * tp,
                               max_tie_frac=0.1)


def test_tp2_spec_infer_tokens_are_greedy():
    ps = prompts(3, 1000, 5, 30, 9)
    res = run_tp(LLM_CFG, 11, 2, ps, 60, spec=True)
    assert [x.output_tokens for x in res[1]] == [x.output_tokens for x in res[0]]
    for p, x in zip(ps, res[0]):
        check_tokens_vs_oracle(LLM_CFG, 11, x.output_tokens, len(p) + 1, tie_ulp=4,
                               max_tie_frac=0.1)


@pytest.mark.parametrize("spec", [False, True])
def test_rccl_shard_graphed_overlapped_equals_eager(monkeypatch, spec):
    """The RCCL all-reduce path (no xGMI transport attached): row-parallel
    GEMMs in two column halves, each ncclAllReduce'd on the second stream
    and copied into its columns, the whole step captured in a HIP graph --
    the same schedule as over the transport.  RCCL refuses two ranks on one
    GPU, so this is shard 0 of TP = 2 over a one-rank RCCL communicator
    (ncclAllReduce of one rank still runs): graphed + overlapped, unsplit,
    and eager runs must give identical tokens."""
    cfg = dict(CFG4, vocab_size=1024)  # vocab-sharded lm_head: the tail all-reduces too
    ps = prompts(3, cfg["vocab_size"], 5, 30, 13)
    extra = 23 * 4 if spec else 0

    def run():
        uid = fa.Comm.unique_id()
        comm = fa.Comm(uid, 1, 0)
        m = fa.Model(cfg, "tree" if spec else "inc", max_requests=4, max_tokens=32 + extra,
                     max_seq_len=128, weight_seed=11, tp_rank=0, tp_size=2, comm=comm)
        rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=32,
                               max_sequence_length=128, spec_tree_width=(1, 1, 3) if spec else ())
        if spec:
            rm.register_ssm_model(fa.Model(dict(SSM_CFG, vocab_size=cfg["vocab_size"]), "beam",
                                           max_requests=4, max_tokens=32 + extra,
                                           max_seq_len=128, weight_seed=5))
        out = [r.output_tokens for r in fa.generate(rm, m, ps, max_length=56)]
        m.close()
        comm.close()
        return out

    base = run()
    monkeypatch.setenv("FFMI_TP_OVERLAP", "0")
    unsplit = run()
    monkeypatch.setenv("FFMI_NO_GRAPHS", "1")
    eager = run()
    assert base == unsplit == eager
    assert all(len(t) == 56 for t in base)
