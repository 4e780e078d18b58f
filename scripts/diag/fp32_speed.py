"""Full-precision LLaMA-7B throughput on one GPU (the parity instrument's
speed, not the measured path): incremental decoding and SpecInfer, bench.py's
prompts (8 x 128 tokens), 64 new tokens, wall time of generate()."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import flexflow_amd as fa  # noqa: E402
from bench import LLAMA_68M, LLAMA_7B, make_prompts  # noqa: E402

B, P, D = 8, 128, 64
ps = make_prompts(B, P - 1, 32000)
out = {}
for spec in (False, True):
    kw = dict(max_requests=B, max_seq_len=512, full_precision=True)
    if spec:
        llm = fa.Model(LLAMA_7B, "tree", max_tokens=1024 + 23 * B, **kw)
        ssm = fa.Model(LLAMA_68M, "beam", max_tokens=1024 + 23 * B, max_tree_tokens=23,
                       weight_seed=68, **kw)
        mk = lambda: fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=1024,  # noqa: E731
                                       max_sequence_length=512, spec_tree_width=(1, 1, 3))
    else:
        llm = fa.Model(LLAMA_7B, "inc", max_tokens=1024, **kw)
        mk = lambda: fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=1024,  # noqa: E731
                                       max_sequence_length=512)
    times = []
    for rep in range(2):
        rm = mk()
        if spec:
            rm.register_ssm_model(ssm)
        t = time.time()
        fa.generate(rm, llm, ps, max_length=P + D, spec=spec)
        times.append(time.time() - t)
    out["spec" if spec else "incr"] = dict(s_per_generate=round(times[-1], 3),
                                           tokens_per_s=round(B * D / times[-1], 1))
    llm.close()
    if spec:
        ssm.close()
print(json.dumps({"full_precision_llama7b": out}))
