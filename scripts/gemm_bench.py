"""GEMM / kernel microbenchmark through the C ABI (HIP events, one process).

    python scripts/gemm_bench.py [--shapes llama7b|ssm] [--T 1,8,168]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, Timer, f16, hip  # noqa: E402

SHAPES = {
    "llama7b": [("qkv", 12288, 4096, 0), ("o", 4096, 4096, 0), ("gate_up", 11008, 4096, 1),
                ("down", 4096, 11008, 0), ("lm_head", 32000, 4096, 0)],
    "ssm": [("qkv", 2304, 768, 0), ("o", 768, 768, 0), ("gate_up", 3072, 768, 1),
            ("down", 768, 3072, 0), ("lm_head", 32000, 768, 0)],
    # per-rank shards of tensor parallelism (TP = 2, 4, 8)
    "llama7b_tp2": [("qkv", 6144, 4096, 0), ("o", 4096, 2048, 0), ("gate_up", 5504, 4096, 1),
                    ("down", 4096, 5504, 0)],
    "llama7b_tp4": [("qkv", 3072, 4096, 0), ("o", 4096, 1024, 0), ("gate_up", 2752, 4096, 1),
                    ("down", 4096, 2752, 0)],
    "llama7b_tp8": [("qkv", 1536, 4096, 0), ("o", 4096, 512, 0), ("gate_up", 1376, 4096, 1),
                    ("down", 4096, 1376, 0)],
    "llama65b_tp8": [("qkv", 3072, 8192, 0), ("o", 8192, 1024, 0), ("gate_up", 2752, 8192, 1),
                     ("down", 8192, 2752, 0)],
    # gate/up without its SiLU epilogue (epilogue-cost A/B)
    "gate_up_plain": [("gate_up_plain", 22016, 4096, 0)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="llama7b")
    ap.add_argument("--T", default="1,8,24,64,168,192")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--xpacked", action="store_true", help="pre-pack X (FFMI_X_PACKED)")
    ap.add_argument("--wstream", action="store_true",
                    help="non-temporal weight loads (FFMI_W_STREAM, as the LLaMA-7B model)")
    ap.add_argument("--ops", default="", help="comma list of op names to run (default all)")
    ap.add_argument("--same-x", action="store_true",
                    help="one activation buffer for every weight copy (L2-warm X)")
    ap.add_argument("--cold-mb", type=int, default=768,
                    help="rotate weight copies totalling this many MB (0: one hot copy)")
    args = ap.parse_args()
    L = F.lib()
    rng = np.random.default_rng(0)
    res = []
    for name, N, K, epi in SHAPES[args.shapes]:
        if args.ops and name not in args.ops.split(","):
            continue
        rows = 2 * N if epi else N
        W = f16(rng.uniform(-0.05, 0.05, (rows, K)))
        nb = L.ffmi_linear_packed_bytes(rows, K)
        src = Buf(W)
        Wp = Buf.empty((nb // 2,), np.uint16)
        if epi:
            half = rows // 2
            g, u = Buf(W[:half]), Buf(W[half:])
            F.check(L.ffmi_linear_pack_gate_up(g.ptr, u.ptr, half, K, Wp.ptr, None))
        else:
            F.check(L.ffmi_linear_pack_weight(src.ptr, N, K, Wp.ptr, None))
        del src
        # copies so that one rotation exceeds the 256 MB last-level cache
        ncopy = max(1, -(-args.cold_mb * (1 << 20) // nb)) if args.cold_mb else 1
        Wps = [Wp]
        for _ in range(ncopy - 1):
            c = Buf.empty((nb // 2,), np.uint16)
            assert hip().hipMemcpy(c.ptr, Wp.ptr, nb, 3) == 0
            Wps.append(c)
        for T in [int(t) for t in args.T.split(",")]:
            Xs = [Buf(f16(rng.standard_normal((T, K)))) for _ in range(1 if args.same_x else len(Wps))]
            flag = 0
            if args.xpacked and T > 64:
                flag = F.X_PACKED
                packed = []
                for xb in Xs:
                    xp = Buf.empty((L.ffmi_packed_activation_bytes(T, K) // 2,), np.uint16)
                    F.check(L.ffmi_pack_activations(xb.ptr, T, K, xp.ptr, None))
                    packed.append(xp)
                Xs = packed
            if args.wstream:
                flag |= F.W_STREAM
            Y = Buf.empty((T, N), np.float16)
            for i in range(len(Wps)):
                F.check(L.ffmi_linear(Xs[i % len(Xs)].ptr, Wps[i].ptr, Y.ptr, T, N, K, epi | flag, None))
            tm = Timer()
            tm.start()
            for it in range(args.iters):
                i = it % len(Wps)
                L.ffmi_linear(Xs[i % len(Xs)].ptr, Wps[i].ptr, Y.ptr, T, N, K, epi | flag, None)
            ms = tm.stop() / args.iters
            byts = 2.0 * (rows * K + T * K + T * N)
            r = dict(op=name, T=T, N=N, K=K, copies=len(Wps), us=round(ms * 1e3, 2),
                     GBps=round(byts / (ms * 1e-3) / 1e9, 1),
                     TFLOPs=round(2.0 * T * rows * K / (ms * 1e-3) / 1e12, 1))
            res.append(r)
            print(json.dumps(r), flush=True)
        del Wps, Wp
    return res


if __name__ == "__main__":
    main()
