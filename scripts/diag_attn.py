"""Per-wave timeline of the verify attention kernel (FFMI_ATTN_STAMP=1).

    python scripts/diag_attn.py [--ctx 128]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("FFMI_ATTN_STAMP", "1")
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, f16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=128)
    ap.add_argument("--heads", type=int, default=32, help="heads per rank (4: LLaMA-7B at TP = 8)")
    # one mode per process: fused then split in one process segfaults on the
    # host in the split call (stamp builds only; not understood yet)
    ap.add_argument("--modes", default="fused")
    args = ap.parse_args()
    L = F.lib()
    R, n, H, D, ctx = 8, 21, args.heads, 128, args.ctx
    T = R * n
    cfg = F.AttnCfg(F.ATTN_TREE, H, D, R, 512, 32, T, 1.0 / np.sqrt(D), 10000.0, 1)
    h = ctypes.c_void_p()
    F.check(L.ffmi_attn_create(ctypes.byref(cfg), ctypes.byref(h)))
    b = ctypes.c_void_p()
    F.check(L.ffmi_batch_create(T, R, ctypes.byref(b)))
    rng = np.random.default_rng(0)
    qkv = Buf(f16(rng.standard_normal((T, 3 * H * D))))
    out = Buf.empty((T + 16, H * D), np.float16)
    chain = [((1 << n) - 1) ^ ((1 << j) - 1) for j in range(n)]
    toks = (F.TokenInfo * T)(*[F.TokenInfo(5, ctx + j, r, ctx + j, ctx, ctx, n, j, 0)
                               for r in range(R) for j in range(n)])
    work = (F.AttnWork * R)(*[F.AttnWork(r, r * n, n, ctx + n) for r in range(R)])
    flat = np.zeros((R, 64), np.uint64)
    flat[:, :n] = chain
    mk = (ctypes.c_uint64 * flat.size)(*flat.ravel().tolist())
    desc = F.BatchDesc(T, R, 0, R, toks, work, (F.CommitInfo * 1)(), mk)
    F.check(L.ffmi_batch_upload(b, ctypes.byref(desc), None))
    for mode in args.modes.split(","):
        if mode == "split":
            os.environ["FFMI_ATTN_NO_FUSE"] = "1"
        for _ in range(5):
            F.check(L.ffmi_attn_tree(h, b, qkv.ptr, out.ptr, None))
        buf = np.zeros((R * H * 8, 12), np.int64)
        m = L.ffmi_debug_attn_stamps(buf.ctypes.data, buf.shape[0])
        st = buf[:m]
        t0 = st[:, 0].min()
        us = lambda a: np.percentile(a * 10 / 1000, [0, 50, 90, 100]).round(2)  # noqa: E731
        print(f"== {mode} ctx={ctx}: waves {m}, span {(st[:, 5].max() - t0) * 10 / 1000:.2f} us")
        names = ["start", "prologue", "setup (q, masks)", "key loop", "to merge barrier",
                 "merge + store"]
        print(f"  {names[0]:18s} p0/50/90/100 {us(st[:, 0] - t0)}")
        if mode == "fused":
            seq = [(0, 6, "commits"), (6, 7, "KV update"), (7, 8, "its barrier"),
                   (8, 9, "V^T stores"), (9, 1, "drain + barrier")]
            for a, b, nm in seq:
                print(f"    {nm:16s} {us(st[:, b] - st[:, a])}")
        for i in range(1, 6):
            print(f"  {names[i]:18s} {us(st[:, i] - st[:, i - 1])}")
        pass


if __name__ == "__main__":
    main()
