"""K-major packed weights (weights.hip, the default) against the round-1
tile-major block order (FFMI_W_TILE_MAJOR=1): the order in which the 1 KiB
fragments are stored changes where a load reads from, not which fragments a
GEMM multiplies or the order it sums them in, so every output must be
bit-identical -- skinny (decode / SSM) and M-split (verify) launches, the
gate/up SiLU epilogue, split-K deferred by nothing (reduce pass).

The layout switch is read once per process, so each layout runs in a fresh
`spawn` process.
"""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(1, 2304, 768, 0), (8, 4096, 1024, 0), (24, 512, 3072, 1), (8, 1376, 4096, 1),
         (168, 1376, 4096, 1), (168, 4096, 1024, 0), (100, 2304, 768, 0), (300, 512, 3072, 0)]


def _gemm_outputs(env, conn):
    try:
        os.environ.update(env)
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import flexflow_amd.ffmi as F
        from hip_util import Buf, f16
        L = F.lib()
        out = []
        for T, N, K, epi in CASES:
            rng = np.random.default_rng(T * 7 + N + K + epi)
            X = Buf(f16(rng.standard_normal((T, K))))
            rows = 2 * N if epi else N
            W = f16(rng.uniform(-0.05, 0.05, (rows, K)))
            Wp = Buf.empty((L.ffmi_linear_packed_bytes(rows, K) // 2,), np.uint16)
            if epi:
                g, u = Buf(W[:N]), Buf(W[N:])
                F.check(L.ffmi_linear_pack_gate_up(g.ptr, u.ptr, N, K, Wp.ptr, None))
            else:
                src = Buf(W)
                F.check(L.ffmi_linear_pack_weight(src.ptr, N, K, Wp.ptr, None))
            for flags in (0, F.W_STREAM):
                Y = Buf.empty((T, N), np.float16)
                F.check(L.ffmi_linear(X.ptr, Wp.ptr, Y.ptr, T, N, K, epi | flags, None))
                out.append(Y.get().view(np.uint16).tobytes())
        conn.send(("ok", out))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        conn.send(("err", repr(e)))
    finally:
        conn.close()


def _run(env):
    ctx = mp.get_context("spawn")
    a, b = ctx.Pipe()
    p = ctx.Process(target=_gemm_outputs, args=(env, b))
    p.start()
    try:
        assert a.poll(180), "layout process did not answer"
        st, res = a.recv()
    finally:
        p.join(60)
        if p.is_alive():
            p.kill()
    assert st == "ok", res
    return res


def test_kmajor_and_tile_major_weights_bit_identical():
    km = _run({"FFMI_W_TILE_MAJOR": "0"})
    tm = _run({"FFMI_W_TILE_MAJOR": "1"})
    assert len(km) == len(tm) == 2 * len(CASES)
    for i, (a, b) in enumerate(zip(km, tm)):
        assert a == b, f"case {CASES[i // 2]} flags {i % 2}"
