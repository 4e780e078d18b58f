"""Structured-input GEMM diagnostic (M-split path): W = identity slice, so
Y[m][n] should equal X[m][n]; prints where values land."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf  # noqa: E402

L = F.lib()
for (T, N, K) in [(100, 128, 64), (100, 768, 768), (168, 256, 4096)]:
    X = (np.arange(T)[:, None] * 0.25 + (np.arange(K)[None, :] % 64) * (1 / 64.0)).astype(np.float16)
    W = np.zeros((N, K), np.float16)
    for n in range(N):
        W[n, n % K] = 1.0
    nb = L.ffmi_linear_packed_bytes(N, K)
    wb = Buf(W)
    Wp = Buf.empty((nb // 2,), np.uint16)
    F.check(L.ffmi_linear_pack_weight(wb.ptr, N, K, Wp.ptr, None))
    Xb, Yb = Buf(X), Buf.empty((T, N), np.float16)
    F.check(L.ffmi_linear(Xb.ptr, Wp.ptr, Yb.ptr, T, N, K, 0, None))
    Y = Yb.get().astype(np.float32)
    ref = X.astype(np.float32)[:, np.arange(N) % K]
    bad = np.abs(Y - ref) > 1e-3
    print(T, N, K, "bad", bad.sum(), "of", bad.size)
    if bad.any():
        m, n = np.argwhere(bad)[0]
        print(" first bad", m, n, "got", Y[m, n], "want", ref[m, n])
        print(" Y[0,:8]", Y[0, :8], "ref", ref[0, :8])
        print(" Y[1,:8]", Y[1, :8], "ref", ref[1, :8])
        print(" Y[:8,0]", Y[:8, 0], "ref", ref[:8, 0])
