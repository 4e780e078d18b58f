"""Config E's SSMs distributed over the ranks of a TP group, world size 2
over gloo on CPU.

The reference builds every SSM as its own TP = 1 model
(inference/spec_infer/spec_infer.cc:381-435); replicating all of them on
every rank of a TP group makes each rank run every SSM's beam steps.  Here
SSM s runs on rank s % nranks only (RequestManager::set_ssm_exchange): after
its SSMs' speculation phase a rank all-gathers their per-step results with the
other ranks and replays the remote SSMs' prepare_next_batch_beam chains on
them, so every rank merges the identical trees (merge_dfs_trees,
request_manager.cc:2817-2878).  Each rank here runs the scheduler's hash test
model (libffmi_testmodel.so) as its LLM and as its own SSMs, with the
exchange over torch.distributed (gloo): the tokens, LLM steps, tree tokens and
commits must equal one process running every SSM itself, on every rank, and
each rank must run only its share of the SSM steps.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

V = 997
SSMS = [(1234, 0), (99, 40), (7, 100), (55, 20)]  # (salt, disagree %), config E's four
MULTI = 2  # FFMI_SPEC_EXT_MULTI_SSM


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _prompts(n, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    return [rng.integers(3, V, size=int(rng.integers(3, 40))).tolist() for _ in range(n)]


def _serve(rank, world, nssm, exchange, chain, batch=3, seed=11, max_length=90):
    os.environ["FFMI_SSM_CHAIN"] = "1" if chain else "0"
    import flexflow_amd as fa
    ps = _prompts(7, seed)  # more requests than slots: prompts load beside running ones
    rm = fa.RequestManager(max_requests_per_batch=batch, max_tokens_per_batch=48,
                           max_sequence_length=128, spec_tree_width=(1, 1, 3),
                           max_spec_tree_token_num=64, spec_extensions=MULTI)
    llm = fa.HashModel(V, "tree", max_requests=batch, max_seq_len=128, max_tree_tokens=64)
    keep = []
    for s, (salt, dis) in enumerate(SSMS[:nssm]):
        if world == 1 or s % world == rank:
            m = fa.HashModel(V, "beam", max_requests=batch, max_seq_len=128, max_tree_tokens=64,
                             salt=salt, disagree_pct=dis)
            keep.append(m)
            rm.register_ssm_model(m)
        else:
            rm.register_ssm_model(None)
    if world > 1:
        rm.set_ssm_exchange(exchange, world, rank)
    res = fa.generate(rm, llm, ps, max_length=max_length, spec=True)
    st = rm.stats()
    return dict(tokens=[r.output_tokens for r in res],
                **{f: getattr(st, f) for f in ("llm_steps", "ssm_steps", "tokens_committed",
                                                "tree_tokens_verified", "request_verifies",
                                                "ssm_phases_chained")})


def _rank_main(rank, world, port, out, nssm, chain):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        def allgather(b):
            parts = [None] * world
            dist.all_gather_object(parts, b)
            return parts

        r = _serve(rank, world, nssm, allgather, chain)
        with open(out.format(rank=rank), "w") as f:
            json.dump(r, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nssm,chain", [(2, True), (4, True), (3, False), (4, False)])
def test_ssms_placed_over_two_ranks_equal_all_local(nssm, chain, tmp_path):
    sys.path.insert(0, HERE)
    ref = _serve(0, 1, nssm, None, chain)  # every SSM in this process
    out = str(tmp_path / "rank{rank}.json")
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, __file__, str(r), "2", str(port), out, str(nssm),
                               str(int(chain))], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
             for r in range(2)]
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (_, e) in zip(procs, outs):
        assert p.returncode == 0, e.decode()[-3000:]
    ranks = [json.load(open(out.format(rank=r))) for r in range(2)]
    import test_scheduler as TS
    for r in ranks:
        assert r["tokens"] == ref["tokens"]
        for f in ("llm_steps", "tokens_committed", "tree_tokens_verified", "request_verifies"):
            assert r[f] == ref[f], f
    assert ref["tokens"] == [TS.expected(p, 90, V) for p in _prompts(7, 11)]
    # each rank ran its share of the SSM steps: SSM s on rank s % 2
    per_ssm = ref["ssm_steps"] // nssm
    assert ranks[0]["ssm_steps"] == per_ssm * ((nssm + 1) // 2)
    assert ranks[1]["ssm_steps"] == per_ssm * (nssm // 2)
    if chain:
        assert all(r["ssm_phases_chained"] > 0 for r in ranks)


def test_remote_ssm_placement_is_checked():
    """A model registered for an SSM another rank runs (or a placeholder for
    one this rank runs) is refused at serve time, with a message."""
    import flexflow_amd as fa
    rm = fa.RequestManager(max_requests_per_batch=2, max_tokens_per_batch=32,
                           max_sequence_length=128, spec_tree_width=(1, 1, 3),
                           spec_extensions=MULTI)
    llm = fa.HashModel(V, "tree", max_requests=2, max_seq_len=128)
    rm.register_ssm_model(None)  # SSM 0 belongs to rank 0, but this is rank 0
    rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=2, max_seq_len=128))
    rm.set_ssm_exchange(lambda b: [b, b], 2, 0)
    with pytest.raises(fa.ffmi.FFMIError, match="rank s % nranks"):
        fa.generate(rm, llm, [[5, 6, 7]], max_length=20, spec=True)


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    _rank_main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
               int(sys.argv[5]), bool(int(sys.argv[6])))
