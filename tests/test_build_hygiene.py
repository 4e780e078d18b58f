"""Build hygiene of the gfx950 kernels (CPU-only: hipcc cross-compiles).

No kernel may use scratch (private memory): on these kernels scratch comes
from dynamically indexed private arrays or struct copies and puts extra
vector-memory operations into the in-order load queue (measured: the fused
attention prologue lost ~3 us to 100 B/lane of scratch).

The check reads `.private_segment_fixed_size` from the gfx950 code objects
inside the built libffmi.so (one offload bundle per translation unit in its
.hip_fatbin section) when the library is newer than every kernel source, and
otherwise recompiles the sources with hipcc's resource-usage remarks.
"""
import os
import re
import shutil
import struct
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "flexflow_amd", "csrc", "kernels")
HIPCC = "/opt/rocm/bin/hipcc"
LLVM = "/opt/rocm/llvm/bin"
LIB = os.path.join(ROOT, "flexflow_amd", "libffmi.so")


def _lib_usage(lib):
    """{kernel: scratch bytes per lane} from the built library's code objects."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib,
                        os.path.join(d, "stripped.so")], check=True, capture_output=True)
        data = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        pos, n = data.find(magic), 0
        while pos >= 0:
            (cnt,) = struct.unpack_from("<Q", data, pos + len(magic))
            p = pos + len(magic) + 8
            for _ in range(cnt):
                off, size, tlen = struct.unpack_from("<QQQ", data, p)
                p += 24
                triple = data[p:p + tlen].decode()
                p += tlen
                if not triple.endswith("gfx950"):
                    continue
                co = os.path.join(d, f"k{n}.co")
                n += 1
                with open(co, "wb") as f:
                    f.write(data[pos + off:pos + off + size])
                notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                       capture_output=True, text=True).stdout
                name = None  # metadata keys are sorted: .name precedes .private_segment_*
                for line in notes.splitlines():
                    m = re.match(r"\s+\.name:\s+(\S+)", line)
                    if m:
                        name = m.group(1)
                    m = re.search(r"\.private_segment_fixed_size:\s+(\d+)", line)
                    if m and name:
                        out[name] = int(m.group(1))
            pos = data.find(magic, pos + 1)
    return out


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
    # the library is fresh only if newer than every kernel source AND every
    # header the kernels include (a WorkDev / collective layout change)
    csrc = os.path.dirname(KDIR)
    hdrs = [os.path.join(d, f) for d in (csrc, KDIR, os.path.join(ROOT, "include"))
            for f in os.listdir(d) if f.endswith(".h")]
    fresh = os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-readelf") and \
        all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in srcs + hdrs)
    if fresh:
        results = [_lib_usage(LIB)]
    else:
        with ThreadPoolExecutor(max_workers=4) as ex:
            results = list(ex.map(_usage, srcs))
    bad = {k: v for r in results for k, v in r.items() if v}
    assert sum(len(r) for r in results) > 20
    assert not bad, f"kernels with scratch: {bad}"
