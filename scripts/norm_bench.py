"""Residual RMSNorm microbenchmark through the C ABI (HIP events):
T=168, H=4096 (the verify shape), fp16 x1 + x2, packed output.

    python scripts/norm_bench.py [--rows 21,168] [--H 4096]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, Timer, f16  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", default="", help="comma list of row counts (default: 168, 24, 8)")
ap.add_argument("--H", type=int, default=4096)
args = ap.parse_args()
L = F.lib()
rng = np.random.default_rng(0)
shapes = ([(int(t), args.H) for t in args.rows.split(",")] if args.rows
          else [(168, 4096), (24, 768), (8, 4096)])
for T, H in shapes:
    x1, x2 = Buf(f16(rng.standard_normal((T, H)))), Buf(f16(rng.standard_normal((T, H))))
    w = Buf(f16(np.ones(H)))
    res, out = Buf.empty((T, H), np.float16), Buf.empty((T + 16, H), np.float16)
    for flags in (0, F.Y_PACKED):
        for _ in range(5):
            F.check(L.ffmi_rmsnorm_ex(x1.ptr, x2.ptr, w.ptr, res.ptr, out.ptr, T, H, 1e-6, flags,
                                      None))
        tm = Timer()
        tm.start()
        n = 200
        for _ in range(n):
            L.ffmi_rmsnorm_ex(x1.ptr, x2.ptr, w.ptr, res.ptr, out.ptr, T, H, 1e-6, flags, None)
        print(f"T={T} H={H} flags={flags}: {tm.stop() * 1e3 / n:.2f} us per launch", flush=True)
