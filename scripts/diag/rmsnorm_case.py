"""Diagnostic: one RMSNorm case against the oracle, mismatch summary."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import flexflow_amd.ffmi as F
import oracle_lib as O
from hip_util import Buf, f16, ulp_diff
L = F.lib()
for (T, H, sc, seed) in [(1088, 16160, 30.0, 0), (64, 16160, 30.0, 1), (64, 16160, 1.0, 2), (64, 8192, 30.0, 3), (64, 12000, 30.0, 4), (64, 16384, 30.0, 5), (64, 16160, 0.01, 6)]:
    rng = np.random.default_rng(seed)
    x1 = f16(rng.standard_normal((T, H)) * sc)
    w = f16(1 + rng.uniform(-0.5, 0.5, H))
    b1, bw = Buf(x1), Buf(w)
    out = Buf.empty((T, H), np.float16)
    F.check(L.ffmi_rmsnorm(b1.ptr, bw.ptr, out.ptr, T, H, 1e-6, None))
    g = out.get()
    r = O.rmsnorm(x1.astype(np.float32), w.astype(np.float32), 1e-6).astype(np.float16)
    d = ulp_diff(g, r)
    rows = np.unique(np.argwhere(d > 1)[:, 0])
    print(T, H, sc, "max ulp", int(d.max()), "frac>1", float((d > 1).mean()), "rows", len(rows), rows[:8])
    if len(rows):
        rr = rows[0]
        print("  row", rr, "gpu", g[rr, :6], "ref", r[rr, :6])
