"""In-kernel clock of the verify-size gate/up k-loop (MI355X_MICROARCH.md
'DVFS give-back' item 6): the 168 x 22016 x 4096 M-split GEMM (gate/up's
k-loop without its SiLU epilogue, the model's flags) launched back to back
for >= 2.5 s over rotating weight copies, random vs zero-filled operands;
then the stamps of the last launch give, per wave, d(s_memtime) /
d(s_memrealtime) x 100 MHz over the k-loop (FFMI_GEMM_STAMP=1 build path).

    python scripts/diag_clock.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("FFMI_GEMM_STAMP", "1")
import flexflow_amd.ffmi as F  # noqa: E402
from hip_util import Buf, Timer, hip  # noqa: E402

L = F.lib()
T, N, K = 168, 22016, 4096


def run(kind):
    rng = np.random.default_rng(0)
    if kind == "random":
        W = rng.uniform(-0.05, 0.05, (N, K)).astype(np.float16)
        X0 = rng.standard_normal((T, K)).astype(np.float16)
    else:
        W = np.zeros((N, K), np.float16)
        X0 = np.zeros((T, K), np.float16)
    nb = L.ffmi_linear_packed_bytes(N, K)
    wb = Buf(W)
    copies = []
    for _ in range(max(1, (768 << 20) // nb)):
        c = Buf.empty((nb // 2,), np.uint16)
        F.check(L.ffmi_linear_pack_weight(wb.ptr, N, K, c.ptr, None))
        copies.append(c)
    del wb
    xb = Buf(X0)
    X = Buf.empty((L.ffmi_packed_activation_bytes(T, K) // 2,), np.uint16)
    F.check(L.ffmi_pack_activations(xb.ptr, T, K, X.ptr, None))
    Y = Buf.empty((T, N), np.float16)
    flags = F.X_PACKED | F.W_STREAM
    t_end = time.time() + 2.5
    n = 0
    tm = Timer()
    tm.start()
    while time.time() < t_end:
        for _ in range(50):
            F.check(L.ffmi_linear(X.ptr, copies[n % len(copies)].ptr, Y.ptr, T, N, K, flags, None))
            n += 1
        assert hip().hipDeviceSynchronize() == 0
    us = tm.stop() * 1e3 / n
    buf = np.zeros((1 << 16, 8), np.int64)
    m = L.ffmi_debug_gemm_stamps(buf.ctypes.data, buf.shape[0])
    st = buf[:m]
    dt_rt = st[:, 2] - st[:, 1]
    ok = dt_rt > 0
    ghz = (st[ok, 7] - st[ok, 6]) / dt_rt[ok] * 100e6 / 1e9
    loop_us = dt_rt[ok] * 10 / 1000
    gbs = 2.0 * (N * K + T * K + T * N) / (us * 1e-6) / 1e9
    print(f"{kind:6s}: {n} launches, {us:.1f} us each ({gbs:.0f} GB/s); k-loop clock GHz "
          f"p10/50/90 {np.percentile(ghz, [10, 50, 90]).round(3)}, k-loop us p50 "
          f"{np.percentile(loop_us, 50):.1f}", flush=True)
    t0 = st[:, 0].min()
    q = lambda a: np.percentile(a * 10 / 1000, [0, 50, 90, 100]).round(2)  # noqa: E731
    print(f"        span {(st[:, 3].max() - t0) * 10 / 1000:.1f} us; p0/50/90/100: start "
          f"{q(st[:, 0] - t0)} prologue {q(st[:, 1] - st[:, 0])} k-loop {q(st[:, 2] - st[:, 1])} "
          f"epilogue {q(st[:, 3] - st[:, 2])} end {q(st[:, 3] - t0)}", flush=True)


for kind in ("random", "zero", "random"):
    run(kind)
