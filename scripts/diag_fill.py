import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import flexflow_amd.ffmi as F
import oracle_lib as O
from hip_util import Buf
L = F.lib()
for name, kind, n in [("model.layers.0.self_attn.q_proj.weight", 0, 100003), ("model.norm.weight", 1, 4096)]:
    buf = Buf.empty((n,), np.uint16)
    F.check(L.ffmi_fill_weight(buf.ptr, n, name.encode(), 20250117, kind, None))
    got = buf.get()
    f32 = O.gen_weight(name, 20250117, kind, n)
    ref = f32.astype(np.float16).view(np.uint16)
    bad = np.nonzero(got != ref)[0]
    print(name, "mismatch", len(bad), "of", n)
    for i in bad[:10]:
        print(i, hex(got[i]), hex(ref[i]), repr(f32[i]), np.uint16(got[i]).view(np.float16), f32[i].view(np.uint32))
