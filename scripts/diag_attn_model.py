"""Per-wave timeline of the verify (or, --mode incr, decode) attention kernel
INSIDE the LLaMA-7B model (FFMI_ATTN_STAMP=1): the stamps of the last d = 128
attention launch of one generate (last layer, last step), so the prologue
sees the qkv GEMM's real split-K slabs and commits.

    python scripts/diag_attn_model.py [--layers 4] [--mode spec|incr]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FFMI_ATTN_STAMP", "1")
# stamp the last layer of the last FULL step only (T = 168 verify, 8 x 21 tree
# tokens; the last steps of a generate are shorter): FFMI_MARKERS gates it
os.environ.setdefault("FFMI_MARKERS", "4096")
os.environ.setdefault("FFMI_MARKERS_T", "168")
import bench  # noqa: E402
import flexflow_amd as fa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--decode", type=int, default=32)
    ap.add_argument("--mode", default="spec", choices=["spec", "incr"])
    ap.add_argument("--ssm", action="store_true",
                    help="stamp the 68M SSM's d = 64 beam-step attention instead (FFMI_ATTN_STAMP=64)")
    args = ap.parse_args()
    if args.mode == "incr":
        os.environ["FFMI_MARKERS_T"] = "8"  # a full decode batch
    if args.ssm:
        os.environ["FFMI_ATTN_STAMP"] = "64"
        os.environ["FFMI_MARKERS"] = "0"  # (the SSM: its last launch)
        assert args.mode == "spec"
    bench.fa = fa
    cfg = dict(bench.LLAMA_7B, num_layers=args.layers)
    B, P = 8, 128
    prompts = bench.make_prompts(B, P - 1, cfg["vocab_size"])
    kw = dict(max_requests_per_batch=B, max_tokens_per_batch=1024, max_spec_tree_token_num=23,
              max_sequence_length=512)
    spec = args.mode == "spec"
    llm = fa.Model(cfg, "tree" if spec else "inc", max_requests=B, max_tokens=1024 + 23 * B,
                   max_seq_len=512, max_tree_tokens=23, weight_seed=20250117)
    rm = fa.RequestManager(spec_tree_width=(1, 1, 3), **kw) if spec else fa.RequestManager(**kw)
    if spec:
        ssm = fa.Model(dict(bench.LLAMA_68M), "beam", max_requests=B, max_tokens=1024 + 23 * B,
                       max_seq_len=512, max_tree_tokens=23, weight_seed=68)
        rm.register_ssm_model(ssm)
    fa.generate(rm, llm, prompts, max_length=P + args.decode, spec=spec)
    L = fa.ffmi.lib()
    buf = np.zeros((B * (12 if args.ssm else 32) * 8, 12), np.int64)
    m = L.ffmi_debug_attn_stamps(buf.ctypes.data, buf.shape[0])
    st = buf[:m]
    t0 = st[:, 0].min()
    us = lambda a: np.percentile(a * 10 / 1000, [0, 50, 90, 100]).round(2)  # noqa: E731
    print(f"== in-model {args.mode} attention: waves {m}, span {(st[:, 5].max() - t0) * 10 / 1000:.2f} us")
    print(f"  {'start':18s} p0/50/90/100 {us(st[:, 0] - t0)}")
    for a, b, nm in [(0, 10, "issue loads"), (10, 11, "wait mrec/tail"), (11, 6, "barrier+commits"),
                     (6, 7, "KV update"), (7, 8, "its barrier"),
                     (8, 9, "V^T stores"), (9, 1, "drain + barrier")]:
        print(f"    {nm:16s} {us(st[:, b] - st[:, a])}")
    names = ["start", "prologue", "setup (q, masks)", "key loop", "to merge barrier",
             "merge + store"]
    for i in range(2, 6):
        print(f"  {names[i]:18s} {us(st[:, i] - st[:, i - 1])}")
    print(f"  {'end':18s} {us(st[:, 5] - t0)}")


if __name__ == "__main__":
    main()
