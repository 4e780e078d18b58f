"""Tensor-parallel decomposition, world_size 2 over gloo on CPU.

The GPU path (runtime/llama_gpu.cpp, ModelImpl::init/forward) shards a
LLaMA layer exactly like the reference (file_loader.cc:286-303,
model.cc:3421-3445):
  * qkv column-parallel by heads:  rows [s*Hl, (s+1)*Hl) of q/k/v_proj;
  * o_proj row-parallel:            columns [s*Hl, (s+1)*Hl), then all-reduce;
  * gate/up column-parallel:        rows [s*Fl, (s+1)*Fl);
  * down_proj row-parallel:         columns [s*Fl, (s+1)*Fl), then all-reduce;
  * norms, residuals and embedding replicated;
  * lm_head vocab-sharded (model.cc:3392-3419): rank s holds rows
    [s*Vl, (s+1)*Vl) and the greedy / speculative tail is the sharded softmax
    top-k of ffmi_vocab_shard_topk -- three exchanges (global max; sum of
    exp against it, in double; each shard's top-k candidates with global
    ids), then the merge by fp16 probability with the lowest-index tie rule.
Here each rank runs that decomposition with the oracle's per-op kernels
(fp32 semantics) and torch.distributed collectives: the gathered logit
shards must match the HF golden fixture of the unsharded model, and every
rank's merged top-k must equal the oracle's softmax top-k of the full row.
A second test runs the bench's multi-rank control plane (bench.Ctrl) with
two processes.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_forward(rank, world, tag, out_path, port):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    import oracle_lib as O

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        cfg, g = O.load_golden(tag)
        seed = cfg["seed"]
        H, F, V = cfg["hidden"], cfg["intermediate"], cfg["vocab_size"]
        nh = cfg["num_heads"]
        d = H // nh
        Hl, Fl, hl = H // world, F // world, nh // world
        eps = cfg["rms_eps"]

        def W(name, rows, cols, kind=0):
            return O.gen_weight(name, seed, kind, rows * cols).reshape(rows, cols)

        def allreduce(x):
            t = torch.from_numpy(np.ascontiguousarray(x, np.float32))
            dist.all_reduce(t)
            return t.numpy()

        prompt = g["prompt"].astype(np.int64)
        T = len(prompt)
        tab = O.rope_table(T, d, cfg["rope_theta"]).reshape(T, d // 2, 2)
        cos, sin = tab[:, :, 0], tab[:, :, 1]

        def rope(x):  # [T][heads][d], HF rotate-half (inc...cu:664-738)
            a, b = x[..., : d // 2], x[..., d // 2:]
            c, s_ = cos[:, None, :], sin[:, None, :]
            return np.concatenate([a * c - b * s_, a * s_ + b * c], axis=-1)

        x = W("model.embed_tokens.weight", V, H)[prompt]
        s = rank
        for layer in range(cfg["num_layers"]):
            p = f"model.layers.{layer}."
            h = O.rmsnorm(x, O.gen_weight(p + "input_layernorm.weight", seed, 1, H), eps, 0)
            q = O.linear(h, W(p + "self_attn.q_proj.weight", H, H)[s * Hl:(s + 1) * Hl], 0)
            k = O.linear(h, W(p + "self_attn.k_proj.weight", H, H)[s * Hl:(s + 1) * Hl], 0)
            v = O.linear(h, W(p + "self_attn.v_proj.weight", H, H)[s * Hl:(s + 1) * Hl], 0)
            q, k = rope(q.reshape(T, hl, d)), rope(k.reshape(T, hl, d))
            v = v.reshape(T, hl, d)
            att = np.zeros((T, hl, d), np.float32)
            for hh in range(hl):
                for t in range(T):
                    vis = np.arange(T) <= t
                    att[t, hh] = O.attention_row(q[t, hh], k[:, hh], v[:, hh], vis,
                                                 1.0 / np.sqrt(d), 0)
            wo = W(p + "self_attn.o_proj.weight", H, H)[:, s * Hl:(s + 1) * Hl]
            o = allreduce(O.linear(att.reshape(T, Hl), wo, 0))
            x, h2 = O.residual_rmsnorm(
                x, o, O.gen_weight(p + "post_attention_layernorm.weight", seed, 1, H), eps, 0)
            gt = O.linear(h2, W(p + "mlp.gate_proj.weight", F, H)[s * Fl:(s + 1) * Fl], 0)
            up = O.linear(h2, W(p + "mlp.up_proj.weight", F, H)[s * Fl:(s + 1) * Fl], 0)
            a = O.silu_mul(gt, up, 0)
            wd = W(p + "mlp.down_proj.weight", H, F)[:, s * Fl:(s + 1) * Fl]
            dn = allreduce(O.linear(a, wd, 0))
            x = x + dn
        xf = O.rmsnorm(x, O.gen_weight("model.norm.weight", seed, 1, H), eps, 0)
        Vl = V // world
        lg = O.linear(xf, W("lm_head.weight", V, H)[s * Vl:(s + 1) * Vl], 0)  # [T][Vl]
        # sharded softmax top-k (ffmi_vocab_shard_topk): 1) global max
        mx = torch.from_numpy(lg.max(axis=1).astype(np.float32))
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        M = mx.numpy()
        # 2) sum of exp against the global max, double, summed over shards
        e = np.exp((lg - M[:, None]).astype(np.float32)).astype(np.float32)
        sm = torch.from_numpy(e.astype(np.float64).sum(axis=1))
        dist.all_reduce(sm)
        S = sm.numpy().astype(np.float32)
        # 3) each shard's top-k candidates (fp16 probability, lowest index)
        k = 3
        p16 = (e / S[:, None]).astype(np.float16).astype(np.float32)
        gid = np.arange(Vl) + s * Vl
        cand = np.zeros((T, k, 2), np.float32)
        for t in range(T):
            order = np.lexsort((gid, -p16[t]))[:k]
            cand[t, :, 0], cand[t, :, 1] = p16[t, order], gid[order]
        allc = [torch.zeros_like(torch.from_numpy(cand)) for _ in range(world)]
        dist.all_gather(allc, torch.from_numpy(cand))
        allc = np.concatenate([a.numpy() for a in allc], axis=1)  # [T][world*k][2]
        top = np.zeros((T, k), np.int64)
        for t in range(T):
            order = np.lexsort((allc[t, :, 1], -allc[t, :, 0]))[:k]
            top[t] = allc[t, order, 1].astype(np.int64)
        shards = [torch.zeros_like(torch.from_numpy(lg)) for _ in range(world)]
        dist.all_gather(shards, torch.from_numpy(np.ascontiguousarray(lg)))
        np.save(out_path.format(rank=rank), np.concatenate([x.numpy() for x in shards], axis=1))
        np.save(out_path.format(rank=rank) + ".top.npy", top)
    finally:
        dist.destroy_process_group()


def _run_ranks(code_args, world=2, timeout=300):
    """Each rank is its own interpreter: torch (for gloo) must not be imported
    into the pytest process, which may hold libffmi's HIP runtime."""
    procs = [subprocess.Popen([sys.executable, __file__, str(r), str(world)] + code_args,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE)
             for r in range(world)]
    outs = [p.communicate(timeout=timeout) for p in procs]
    for p, (_, e) in zip(procs, outs):
        assert p.returncode == 0, e.decode()[-3000:]


@pytest.mark.parametrize("tag", ["tiny_d64", "tiny_d128"])
def test_tp2_decomposition_matches_unsharded_golden(tag, tmp_path):
    sys.path.insert(0, HERE)
    import oracle_lib as O

    out = str(tmp_path / "logits_{rank}.npy")
    _run_ranks([tag, out, str(_free_port())])
    _, g = O.load_golden(tag)
    l0, l1 = np.load(out.format(rank=0)), np.load(out.format(rank=1))
    np.testing.assert_array_equal(l0, l1)  # the gathered shards: ranks agree exactly
    np.testing.assert_allclose(l0, g["logits"], rtol=1e-4, atol=5e-5)
    assert (l0.argmax(-1) == g["logits"].argmax(-1)).all()
    # the sharded top-k merge equals the unsharded softmax top-k, on every rank
    ids, _ = O.softmax_topk(l0, 3, fp16=1)
    for r in range(2):
        np.testing.assert_array_equal(np.load(out.format(rank=r) + ".top.npy"), ids)


_CTRL_CHILD = r"""
import sys, os
sys.path.insert(0, {root!r})
from bench import Ctrl
rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
c = Ctrl(rank, world, port)
data = c.bcast(b"uid-" + bytes([7] * 120) if rank == 0 else b"")
assert data == b"uid-" + bytes([7] * 120), data
m = c.max(float(rank * 10 + 1))
assert m == float((world - 1) * 10 + 1), m
c.barrier()
print("ok", rank)
"""


def test_bench_control_plane_two_ranks():
    port = _free_port()
    code = _CTRL_CHILD.format(root=ROOT)
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r), "2", str(port)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
             for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e.decode()[-2000:]
        assert o.decode().startswith("ok")


if __name__ == "__main__":  # rank entry point for test_tp2_decomposition_*
    _tp_forward(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]))
