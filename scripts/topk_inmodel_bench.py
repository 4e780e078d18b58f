"""The SSM step's tail in isolation, as the model runs it: the lm_head GEMM
(T = 24, N = 32000, K = 768) writes the logits, then the softmax top-k (k =
3) reads them -- cold, from the memory side, not L2-hot as in topk_bench.py --
and writes ids / probs either to device memory or to coherent pinned host
memory (the model's result buffer).  Per-iteration times (HIP events over 200
back-to-back pairs) for: the GEMM alone, GEMM + top-k one workgroup per row,
GEMM + split-row top-k; each with device and host outputs."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, Timer, f16, hip  # noqa: E402

L = F.lib()
H = hip()
H.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
rng = np.random.default_rng(0)
T, N, K, k = int(os.environ.get("T", 24)), 32000, 768, 3
x = Buf(f16(rng.standard_normal((T, K))))
wp = Buf(f16(rng.standard_normal(int(L.ffmi_linear_packed_bytes(N, K)) // 2) * 0.05))
y = Buf.empty((T, N), np.float16)
wsb = int(L.ffmi_linear_workspace_bytes(T, N, K, 0))
ws = Buf.empty((max(wsb, 16),), np.uint8)
ids, pr = Buf.empty((T, k), np.int32), Buf.empty((T, k), np.float32)
hptr = ctypes.c_void_p()
assert H.hipHostMalloc(ctypes.byref(hptr), T * k * 8, 0x40000000 | 0x2) == 0
hids, hpr = hptr, ctypes.c_void_p(hptr.value + T * k * 4)
nb = int(L.ffmi_arg_topk_workspace_bytes(T))
tws = Buf(np.zeros(nb // 4, np.uint32))


def gemm():
    L.ffmi_linear_ws(x.ptr, wp.ptr, y.ptr, T, N, K, 0, ws.ptr, wsb, None)


def time_it(fn, n=200):
    for _ in range(10):
        fn()
    tm = Timer()
    tm.start()
    for _ in range(n):
        fn()
    return tm.stop() * 1e3 / n


base = time_it(gemm)
print(f"T={T}: lm_head GEMM alone {base:.2f} us per launch", flush=True)
for name, out in (("device", (ids.ptr, pr.ptr)), ("host", (hids, hpr))):
    t1 = time_it(lambda: (gemm(), L.ffmi_arg_topk(y.ptr, T, N, k, out[0], out[1], None)))
    t2 = time_it(lambda: (gemm(), L.ffmi_arg_topk_ws(y.ptr, T, N, k, out[0], out[1], tws.ptr, nb,
                                                      None)))
    print(f"  + top-k, {name} outputs: one workgroup per row {t1 - base:.2f} us, "
          f"split rows {t2 - base:.2f} us (GEMM + top-k {t1:.2f} / {t2:.2f})", flush=True)
