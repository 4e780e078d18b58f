"""Per-wave timeline of one M-split GEMM launch (FFMI_GEMM_STAMP=1).

    python scripts/diag_stamps.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("FFMI_GEMM_STAMP", "1")
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf  # noqa: E402

L = F.lib()
rng = np.random.default_rng(0)
for name, N, K, T in [("qkv", 12288, 4096, 168), ("down", 4096, 11008, 168),
                      ("o", 4096, 4096, 168)]:
    W = (rng.uniform(-0.05, 0.05, (N, K))).astype(np.float16)
    nb = L.ffmi_linear_packed_bytes(N, K)
    wb = Buf(W)
    copies = []
    for _ in range(max(1, (768 << 20) // nb)):
        c = Buf.empty((nb // 2,), np.uint16)
        F.check(L.ffmi_linear_pack_weight(wb.ptr, N, K, c.ptr, None))
        copies.append(c)
    X0 = Buf(rng.standard_normal((T, K)).astype(np.float16))
    X = Buf.empty((L.ffmi_packed_activation_bytes(T, K) // 2,), np.uint16)
    F.check(L.ffmi_pack_activations(X0.ptr, T, K, X.ptr, None))
    Y = Buf.empty((T, N), np.float16)
    for i in range(len(copies)):
        F.check(L.ffmi_linear(X.ptr, copies[i].ptr, Y.ptr, T, N, K, F.X_PACKED, None))
    F.check(L.ffmi_linear(X.ptr, copies[0].ptr, Y.ptr, T, N, K, F.X_PACKED, None))
    buf = np.zeros((1 << 16, 8), np.int64)
    n = L.ffmi_debug_gemm_stamps(buf.ctypes.data, buf.shape[0])
    st = buf[:n]
    t0 = st[:, 0].min()
    start = st[:, 0] - t0
    pro, loop, end = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    tot = st[:, 3].max() - t0
    cu = (st[:, 5] << 16) | ((st[:, 4] >> 8) & 0xFFFF)
    ucu, cnt = np.unique(cu, return_counts=True)
    print(f"== {name} T={T}: waves {n} (WGs {n // 4}), kernel span {tot * 10 / 1000:.1f} us")

    def q(a):
        return np.percentile(a * 10 / 1000, [0, 50, 90, 100]).round(2)
    print("  start  us p0/50/90/100", q(start))
    print("  prolog us", q(pro))
    print("  k-loop us", q(loop))
    print("  epilog us", q(end))
    print("  distinct CUs", len(ucu), "waves per CU histogram", np.bincount(cnt)[1:])
    del copies
