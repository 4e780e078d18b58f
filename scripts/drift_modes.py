#!/usr/bin/env python3
"""Reordering drift of the CPU oracle against itself, per synthetic weight
init (test infrastructure; runs on any host with ~30 GB of RAM).

The oracle runs the same prompt with its fp32 dots in three summation orders
(orc_set_dot_variant 0/1/2: dot8 / dot16 / dot32) and reports how far the
final logits and the per-layer hidden states move, how many greedy picks
flip, and the top-2 logit margins -- the noise floor every GPU-vs-oracle
token comparison sits on (tests/parity_rules.py, tests/test_gpu_token_chain.py).

  python scripts/drift_modes.py [--init 0|1|2] [--layers 32] [--tokens 64]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import oracle_lib as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", type=int, default=0, help="0 uniform, 1 depth-scaled, 2 token chain")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--tokens", type=int, default=64)
    a = ap.parse_args()
    cfg = dict(num_layers=a.layers, vocab_size=32000, num_heads=32, num_kv_heads=32, hidden=4096,
               intermediate=11008, rms_eps=1e-6, rope_theta=10000.0)
    t = time.time()
    m = O.Model(cfg, 20250117, fp16=1, max_requests=1, max_seq=a.tokens + 8, weight_init=a.init)
    print(f"built in {time.time() - t:.1f}s", flush=True)
    rng = np.random.default_rng(5)
    toks = np.array([1] + rng.integers(3, 32000, size=a.tokens - 1).tolist(), np.int32)
    lg, hid = {}, {}
    for v in (0, 1, 2):
        O.set_dot_variant(v)
        lg[v] = m.forward(0, toks, 0)
        hid[v] = [m.hidden(l, len(toks)) for l in range(a.layers + 1)]
    O.set_dot_variant(0)
    ids = {v: O.softmax_argmax(lg[v])[0] for v in lg}
    for v in (1, 2):
        d = np.abs(lg[v] - lg[0])
        print(f"dot variant {v} vs 0: logits max |d| {d.max():.4f}, frac > 1e-2 "
              f"{(d > 1e-2).mean():.4f}, greedy flips {(ids[v] != ids[0]).sum()}/{len(toks)}")
    for l in sorted(set([0, 1, 2, 4, 8, 16, a.layers - 1, a.layers]) & set(range(a.layers + 1))):
        x, y = hid[0][l], hid[1][l]
        print(f"  hidden after layer {l}: relative |d| {np.linalg.norm(x - y) / np.linalg.norm(x):.2e}")
    srt = np.sort(lg[0], axis=1)
    gap = srt[:, -1] - srt[:, -2]
    print(f"logit std {lg[0].std():.3f}; top-2 margin median {np.median(gap):.4f}, "
          f"min {gap.min():.4f}, p10 {np.percentile(gap, 10):.4f}")


if __name__ == "__main__":
    main()
