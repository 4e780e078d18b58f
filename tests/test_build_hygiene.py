"""Build hygiene of the gfx950 kernels (CPU-only: hipcc cross-compiles).

No kernel may use scratch (private memory): on these kernels scratch comes
from dynamically indexed private arrays or struct copies and puts extra
vector-memory operations into the in-order load queue (measured: the fused
attention prologue lost ~3 us to 100 B/lane of scratch).
"""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "flexflow_amd", "csrc", "kernels")
HIPCC = "/opt/rocm/bin/hipcc"


def _usage(src):
    out = subprocess.run(
        [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
         "--cuda-device-only", "-c", src, "-o", os.devnull,
         "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    kernels, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            kernels[name] = int(m.group(1))
    return kernels


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("sh") is None,
                    reason="hipcc not available")
def test_no_kernel_uses_scratch():
    srcs = sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".hip"))
    with ThreadPoolExecutor(max_workers=4) as ex:
        results = list(ex.map(_usage, srcs))
    bad = {k: v for r in results for k, v in r.items() if v}
    assert sum(len(r) for r in results) > 20
    assert not bad, f"kernels with scratch: {bad}"
