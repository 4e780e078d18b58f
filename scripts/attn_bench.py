"""Tree-verify attention microbenchmark through the C ABI (HIP events).

LLaMA-7B shape: 32 heads x 128, 8 requests x 21 tree tokens, prefix `ctx`.
Times the one-launch path and the KV-update + attention path
(FFMI_ATTN_NO_FUSE, read per call).

    python scripts/attn_bench.py [--ctx 32,128,256] [--heads 32] [--d 128]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, Timer, f16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", default="32,128,256")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--reqs", type=int, default=8)
    ap.add_argument("--tree", type=int, default=21)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    L = F.lib()
    R, n, H, D = args.reqs, args.tree, args.heads, args.d
    T = R * n
    cfg = F.AttnCfg(F.ATTN_TREE, H, D, R, 512, 32, max(T, 16), 1.0 / np.sqrt(D), 10000.0, 1)
    h = ctypes.c_void_p()
    F.check(L.ffmi_attn_create(ctypes.byref(cfg), ctypes.byref(h)))
    b = ctypes.c_void_p()
    F.check(L.ffmi_batch_create(max(T, 16), R, ctypes.byref(b)))
    rng = np.random.default_rng(0)
    qkv = Buf(f16(rng.standard_normal((T, 3 * H * D))))
    out = Buf.empty(((T + 15) // 16 * 16, H * D), np.float16)
    chain = [((1 << n) - 1) ^ ((1 << j) - 1) for j in range(n)]
    for ctx in [int(c) for c in args.ctx.split(",")]:
        toks = (F.TokenInfo * T)(*[F.TokenInfo(5, ctx + j, r, ctx + j, ctx, ctx, n, j, 0)
                                   for r in range(R) for j in range(n)])
        work = (F.AttnWork * R)(*[F.AttnWork(r, r * n, n, ctx + n) for r in range(R)])
        cm = (F.CommitInfo * 1)()
        flat = np.zeros((R, 64), np.uint64)
        flat[:, :n] = chain
        mk = (ctypes.c_uint64 * flat.size)(*flat.ravel().tolist())
        desc = F.BatchDesc(T, R, 0, R, toks, work, cm, mk)
        F.check(L.ffmi_batch_upload(b, ctypes.byref(desc), None))
        for mode in ("fused", "split"):
            if mode == "split":
                os.environ["FFMI_ATTN_NO_FUSE"] = "1"
            else:
                os.environ.pop("FFMI_ATTN_NO_FUSE", None)
            for _ in range(3):
                F.check(L.ffmi_attn_tree(h, b, qkv.ptr, out.ptr, None))
            tm = Timer()
            tm.start()
            for _ in range(args.iters):
                L.ffmi_attn_tree(h, b, qkv.ptr, out.ptr, None)
            us = tm.stop() * 1e3 / args.iters
            kv = 2.0 * R * H * (ctx + n) * D * 2
            print(json.dumps(dict(ctx=ctx, mode=mode, us=round(us, 2),
                                  kv_GBps=round(kv / us / 1e3, 1))), flush=True)
    os.environ.pop("FFMI_ATTN_NO_FUSE", None)


if __name__ == "__main__":
    main()
