"""Dense layers at the exact shapes the BASELINE configs run, with the flags
the model uses (packed activation tiles in, W_STREAM non-temporal weight
loads, the gate/up SiLU epilogue writing packed tiles out), against the CPU
oracle's fp32-accumulate restatement (linear_kernels.cu:450-582).

Shapes (SURVEY.md §8 constants):
- LLaMA-7B, TP = 1 (configs B/C): qkv 12288x4096, o 4096x4096,
  gate|up 2x11008x4096, down 4096x11008, lm_head 32000x4096;
- LLaMA-65B, TP = 8 per-rank shards (configs D/E): qkv 3072x8192,
  o 8192x1024, gate|up 2x2752x8192, down 8192x2752, lm_head vocab shard
  4000x8192;
- T = 8 (decode batch, skinny kernel), T = 168 (8 requests x 21-token
  verify trees, M-split kernel), T = 577 (the first T with >= 4 row blocks:
  the fixed prefill plan of gemm.hip mid_plan) and T = 1024 (bench.py's
  prefill step: 8 prompts x 128 tokens, max_tokens_per_batch 1024).
Tolerance as test_gpu_kernels.close16: <= 2 fp16 ulp (or 1e-4 * max |ref|)
everywhere and >= 99% of elements bit-identical (only the fp32 summation
order differs).
"""
import zlib

import numpy as np
import pytest

import flexflow_amd.ffmi as F
import oracle_lib as O
from hip_util import Buf, f16
from test_gpu_kernels import close16, pack_act_np, unpack_act_np

pytestmark = pytest.mark.gpu

SHAPES = {
    "7b_qkv": (12288, 4096, 0), "7b_o": (4096, 4096, 0), "7b_gate_up": (11008, 4096, 1),
    "7b_down": (4096, 11008, 0), "7b_lm_head": (32000, 4096, 0),
    "65b_tp8_qkv": (3072, 8192, 0), "65b_tp8_o": (8192, 1024, 0),
    "65b_tp8_gate_up": (2752, 8192, 1), "65b_tp8_down": (8192, 2752, 0),
    "65b_tp8_lm_head_shard": (4000, 8192, 0),
}


@pytest.mark.parametrize("T", [8, 168, 577, 1024])
@pytest.mark.parametrize("shape", list(SHAPES))
def test_linear_at_baseline_shapes(shape, T):
    N, K, epi = SHAPES[shape]
    L = F.lib()
    rng = np.random.default_rng(zlib.crc32(f"{shape}:{T}".encode()))
    X = f16(rng.standard_normal((T, K)))
    amp = 0.02 * np.sqrt(3.0)  # the synthetic weights' range (orc_gen_weight kind 0)
    if epi:
        Wg, Wu = f16(rng.uniform(-amp, amp, (N, K))), f16(rng.uniform(-amp, amp, (N, K)))
        gb, ub = Buf(Wg), Buf(Wu)
        Wp = Buf.empty((2 * L.ffmi_linear_packed_bytes(N, K) // 2,), np.uint16)
        F.check(L.ffmi_linear_pack_gate_up(gb.ptr, ub.ptr, N, K, Wp.ptr, None))
        del gb, ub
    else:
        W = f16(rng.uniform(-amp, amp, (N, K)))
        src = Buf(W)
        Wp = Buf.empty((L.ffmi_linear_packed_bytes(N, K) // 2,), np.uint16)
        F.check(L.ffmi_linear_pack_weight(src.ptr, N, K, Wp.ptr, None))
        del src
    Xp = Buf(pack_act_np(X))
    flags = epi | F.X_PACKED | F.W_STREAM | (F.Y_PACKED if epi else 0)
    Tp = (T + 15) // 16 * 16
    Y = Buf.empty(((Tp if epi else T), N), np.float16)
    F.check(L.ffmi_linear(Xp.ptr, Wp.ptr, Y.ptr, T, N, K, flags, None), shape)
    y = Y.get()
    if epi:
        y = unpack_act_np(y.reshape(-1), T, N)
        g = O.linear(X.astype(np.float32), Wg.astype(np.float32))
        u = O.linear(X.astype(np.float32), Wu.astype(np.float32))
        # the epilogue rounds gate and up to fp16, then runs the reference's
        # half chain (sigmoid_silu_multi.cu:41-46).  With the oracle's gate/up
        # rounded the same way, >= 99% of the outputs are bit-identical; the
        # rest must be the chain applied to gate/up values within the plain
        # GEMMs' tolerance (close16: 2 fp16 ulp or 1e-4 * max |ref|) of the
        # oracle's -- near zero the fp32 summation order moves gate/up by
        # several fp16 ulps -- i.e. within [min, max] of the chain over that
        # box, + 1 output ulp.
        g16, u16 = g.astype(np.float16), u.astype(np.float16)
        chain = lambda a, b: O.silu_mul(a.astype(np.float32), b.astype(np.float32))  # noqa: E731
        ref = chain(g16, u16).astype(np.float16)
        y16 = y.astype(np.float16)
        assert (y16 == ref).mean() >= 0.99, (y16 == ref).mean()
        sp = lambda a: np.spacing(np.abs(a).astype(np.float16)).astype(np.float32)  # noqa: E731
        dg = np.maximum(2 * sp(g16), 1e-4 * np.abs(g).max())
        du = np.maximum(2 * sp(u16), 1e-4 * np.abs(u).max())
        pts = [chain(g + a * dg, u + b * du) for a in (-1, 0, 1) for b in (-1, 0, 1)]
        lo, hi = np.min(pts, axis=0), np.max(pts, axis=0)
        yf = y16.astype(np.float32)
        slack = sp(np.maximum(np.abs(lo), np.abs(hi)))
        bad = (yf < lo - slack) | (yf > hi + slack)
        assert not bad.any(), (np.argwhere(bad)[:5], y16[bad][:5], ref[bad][:5])
    else:
        ref = O.linear(X.astype(np.float32), W.astype(np.float32), fp16=1)
        close16(y, ref)


@pytest.mark.parametrize("shape,T", [("7b_qkv", 1024), ("7b_o", 1024), ("7b_gate_up", 577),
                                     ("7b_gate_up", 1024), ("7b_lm_head", 577),
                                     ("7b_lm_head", 1024)])
def test_tile_gemm_bit_identical_to_msplit(shape, T, monkeypatch):
    """The compute-bound prefill form (gemm_tile_kernel: 256 x 256 tiles, LDS
    fed by global_load_lds) against the M-split kernel on the same inputs:
    both accumulate every output over the k-steps in sequence with the same
    MFMA, so the outputs are bit-identical where the M-split side runs
    unsplit (these shapes; where its planner splits K -- qkv / o at T = 577,
    K = 8192 -- the orders differ and test_linear_at_baseline_shapes holds
    both to the oracle)."""
    N, K, epi = SHAPES[shape]
    L = F.lib()
    rng = np.random.default_rng(zlib.crc32(f"tile:{shape}:{T}".encode()))
    X = f16(rng.standard_normal((T, K)))
    rows = 2 * N if epi else N
    W = f16(rng.uniform(-0.03, 0.03, (rows, K)))
    Wp = Buf.empty((L.ffmi_linear_packed_bytes(rows, K) // 2,), np.uint16)
    if epi:
        gb, ub = Buf(np.ascontiguousarray(W[:N])), Buf(np.ascontiguousarray(W[N:]))
        F.check(L.ffmi_linear_pack_gate_up(gb.ptr, ub.ptr, N, K, Wp.ptr, None))
    else:
        src = Buf(W)
        F.check(L.ffmi_linear_pack_weight(src.ptr, N, K, Wp.ptr, None))
    Xp = Buf(pack_act_np(X))
    Tp = (T + 15) // 16 * 16
    out = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("FFMI_TILE_GEMM", mode)
        for yp in (0, 1):
            flags = epi | F.X_PACKED | (F.Y_PACKED if yp else 0)
            Y = Buf.empty(((Tp if yp else T), N), np.float16)
            F.check(L.ffmi_linear(Xp.ptr, Wp.ptr, Y.ptr, T, N, K, flags, None), shape)
            out[mode, yp] = Y.get()
    for yp in (0, 1):
        a, b = out["0", yp].view(np.uint16), out["2", yp].view(np.uint16)
        assert np.array_equal(a, b), (yp, float((a != b).mean()))
