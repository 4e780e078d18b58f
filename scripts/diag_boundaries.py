"""Kernel boundaries of the LLaMA-7B verify step, measured on the GPU's own
100 MHz realtime clock: one-wave marker kernels (FFMI_MARKERS=4096) between
the last layer's kernels of the last full verify step (T = 168, FFMI_MARKERS_T), and the per-wave stamps of
that layer's attention (FFMI_ATTN_STAMP=1).  Marker-to-marker intervals are
kernel + boundary; for the attention the interval splits into the gap before
its first wave starts, its in-kernel span, and the gap after its last wave.

    python scripts/diag_boundaries.py [--layers 4] [--decode 32]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["FFMI_MARKERS"] = "4096"
os.environ["FFMI_ATTN_STAMP"] = "1"
os.environ.setdefault("FFMI_MARKERS_T", "168")  # a full verify batch (8 x 21 tree tokens)
import bench  # noqa: E402
import flexflow_amd as fa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
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
    buf = np.zeros((B * 32 * 8, 12), np.int64)
    m = L.ffmi_debug_attn_stamps(buf.ctypes.data, buf.shape[0])
    st = buf[:m]
    us = lambda t: round(t * 10 / 1000, 2)  # noqa: E731
    names = ["residual norm", "qkv GEMM", "attention", "o GEMM", "residual norm",
             "gate/up GEMM", "down GEMM", "(empty: marker to marker)"]
    print(f"== last layer, last verify step of T = {os.environ['FFMI_MARKERS_T']}")
    for i in range(min(len(names), n - 1)):
        print(f"  {names[i]:26s} {us(mk[i + 1] - mk[i]):7.2f} us (marker to marker)")
    a0, a1 = st[:, 0].min(), st[:, 5].max()
    print(f"  attention: marker -> first wave {us(a0 - mk[2]):.2f} us, in-kernel span {us(a1 - a0):.2f} us,"
          f" last wave -> marker {us(mk[3] - a1):.2f} us")


if __name__ == "__main__":
    main()
