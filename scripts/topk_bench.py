"""Softmax + argmax / top-k microbenchmark through the C ABI (HIP events):
the SSM step's top-3 (T = 24) and the verify step's argmax (T = 168) over a
32000 vocabulary.  V = 31999 / 32001 (no 16-B rows) and 128256 take the
streaming kernel, for comparison with the register-resident kernel."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, Timer, f16  # noqa: E402

L = F.lib()
rng = np.random.default_rng(0)
for T, V, k in [(24, 32000, 3), (24, 31999, 3), (168, 32000, 1), (8, 32000, 1), (8, 32000, 3), (24, 32000, 1),
                (24, 32001, 3), (168, 32001, 1), (24, 128256, 3), (168, 128256, 1)]:
    x = Buf(f16(rng.standard_normal((T, V)) * 3.0))
    ids = Buf.empty((T, k), np.int32)
    pr = Buf.empty((T, k), np.float32)
    for _ in range(5):
        F.check(L.ffmi_arg_topk(x.ptr, T, V, k, ids.ptr, pr.ptr, None))
    tm = Timer()
    tm.start()
    n = 300
    for _ in range(n):
        L.ffmi_arg_topk(x.ptr, T, V, k, ids.ptr, pr.ptr, None)
    t1 = tm.stop() * 1e3 / n
    # the split-row form (the model's: a zeroed workspace)
    nb = int(L.ffmi_arg_topk_workspace_bytes(T))
    ws = Buf(np.zeros(nb // 4, np.uint32))
    for _ in range(5):
        F.check(L.ffmi_arg_topk_ws(x.ptr, T, V, k, ids.ptr, pr.ptr, ws.ptr, nb, None))
    tm = Timer()
    tm.start()
    for _ in range(n):
        L.ffmi_arg_topk_ws(x.ptr, T, V, k, ids.ptr, pr.ptr, ws.ptr, nb, None)
    t2 = tm.stop() * 1e3 / n
    print(f"T={T} V={V} k={k}: {t1:.2f} us per launch (one workgroup per row), "
          f"{t2:.2f} us (split rows)", flush=True)
