"""Kernel boundaries of the LLaMA-68M SSM beam step (T = 24: 8 requests x 3
beams), on the GPU's 100 MHz realtime clock: one-wave marker kernels
(FFMI_MARKERS=768) between the kernels of the SSM's last layer and its tail
(final norm, lm_head, softmax top-k) in the last step of that size, graphed as
in production.  Each marker-to-marker interval is one kernel + one boundary;
the "(empty)" interval is a bare boundary.

    python scripts/diag_ssm_step.py [--layers 2] [--decode 32]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["FFMI_MARKERS"] = "768"
os.environ.setdefault("FFMI_MARKERS_T", "24")
import bench  # noqa: E402
import flexflow_amd as fa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2, help="LLM layers (the LLM is not measured)")
    ap.add_argument("--decode", type=int, default=32)
    args = ap.parse_args()
    cfg = dict(bench.LLAMA_7B, num_layers=args.layers)
    B, P = 8, 128
    prompts = bench.make_prompts(B, P - 1, cfg["vocab_size"])
    kw = dict(max_requests_per_batch=B, max_tokens_per_batch=1024, max_spec_tree_token_num=23,
              max_sequence_length=512)
    llm = fa.Model(cfg, "tree", max_requests=B, max_tokens=1024 + 23 * B, max_seq_len=512,
                   max_tree_tokens=23, weight_seed=20250117)
    rm = fa.RequestManager(spec_tree_width=(1, 1, 3), **kw)
    ssm = fa.Model(dict(bench.LLAMA_68M), "beam", max_requests=B, max_tokens=1024 + 23 * B,
                   max_seq_len=512, max_tree_tokens=23, weight_seed=68)
    rm.register_ssm_model(ssm)
    fa.generate(rm, llm, prompts, max_length=P + args.decode, spec=True)
    L = fa.ffmi.lib()
    mk = np.zeros(64, np.int64)
    n = L.ffmi_debug_markers(mk.ctypes.data, 64)
    mk = mk[:n]
    us = lambda t: round(t * 10 / 1000, 2)  # noqa: E731
    names = ["residual norm (down slabs)", "qkv GEMM", "attention + o", "residual norm (heads)",
             "gate/up GEMM", "down GEMM", "(empty: marker to marker)", "final norm", "lm_head",
             "softmax top-k"]
    print(f"== SSM last layer + tail, last step of T = {os.environ['FFMI_MARKERS_T']} ({n} markers)")
    for i in range(min(len(names), n - 1)):
        print(f"  {names[i]:28s} {us(mk[i + 1] - mk[i]):7.2f} us (marker to marker)")
    print(f"  total {us(mk[n - 1] - mk[0]):.2f} us")


if __name__ == "__main__":
    main()
