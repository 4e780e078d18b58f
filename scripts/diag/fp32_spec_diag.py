"""Diagnostic: fp32 SpecInfer vs incr on a 2-layer LLaMA-7B-width model,
with the SSM in either precision and graphs on / off."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import flexflow_amd as fa  # noqa: E402

CFG = dict(num_layers=2, vocab_size=32000, num_heads=32, num_kv_heads=32, hidden=4096,
           intermediate=11008, rms_eps=1e-6, rope_theta=10000.0)
SSM = dict(num_layers=2, vocab_size=32000, num_heads=12, num_kv_heads=12, hidden=768,
           intermediate=3072, rms_eps=1e-6, rope_theta=10000.0)


def run(ps, spec, fp_llm, fp_ssm):
    B, mtb, L = len(ps), 256, 40
    kw = dict(max_requests=B, max_seq_len=256)
    if spec:
        llm = fa.Model(CFG, "tree", max_tokens=mtb + 23 * B, weight_seed=1, full_precision=fp_llm, **kw)
        ssm = fa.Model(SSM, "beam", max_tokens=mtb + 23 * B, max_tree_tokens=23, weight_seed=68,
                       full_precision=fp_ssm, **kw)
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=256, spec_tree_width=(1, 1, 3))
        rm.register_ssm_model(ssm)
        res = fa.generate(rm, llm, ps, max_length=L, spec=True)
        ssm.close()
    else:
        llm = fa.Model(CFG, "inc", max_tokens=mtb, weight_seed=1, full_precision=fp_llm, **kw)
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=256)
        res = fa.generate(rm, llm, ps, max_length=L)
    llm.close()
    return [r.output_tokens for r in res], rm.stats().llm_steps


rng = np.random.default_rng(1)
ps = [rng.integers(3, 32000, size=10).tolist() for _ in range(3)]
for fp in (False, True):
    inc, _ = run(ps, False, fp, fp)
    for fs in (False, True):
        sp, st = run(ps, True, fp, fs)
        firsts = []
        for a, b in zip(inc, sp):
            firsts.append(next((i for i in range(len(a)) if a[i] != b[i]), -1))
        print(f"llm fp32={fp} ssm fp32={fs} graphs={'FFMI_NO_GRAPHS' not in os.environ}: "
              f"spec==incr {sum(a == b for a, b in zip(inc, sp))}/3 first diff {firsts} steps {st}",
              flush=True)
