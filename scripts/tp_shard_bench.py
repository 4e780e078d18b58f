"""Per-rank compute of the TP=N SpecInfer step, on ONE GPU.

Builds the LLaMA-7B (or --model 65b: LLaMA-65B, configs D/E) verify model as shard 0 of N (heads / FFN columns /
rows of o and down) over a 1-rank communicator with no RCCL state and no
transport (Comm.peer(1, 0), never attached), so its all-reduces are no-ops and
its steps are graphed like the bench's: the numbers are the per-rank GEMM /
attention / norm time of the bench at --gpus N, WITHOUT the all-reduce cost
(tokens are meaningless).  (Round 3's first table used a 1-rank RCCL
communicator, which now takes the RCCL path and times ncclAllReduce calls.)

    python scripts/tp_shard_bench.py --tp 8 [--model 65b] [--mode incr]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import flexflow_amd as fa  # noqa: E402
from bench import LLAMA_65B, LLAMA_68M, LLAMA_7B, make_prompts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--model", choices=["7b", "65b"], default="7b")
    ap.add_argument("--mode", choices=["spec", "incr"], default="spec")
    ap.add_argument("--ssms", type=int, default=1,
                    help="SSMs on this rank (4: config E's SSMs replicated per rank; 1: this "
                         "rank's share when they are distributed one per rank)")
    args = ap.parse_args()
    cfg = LLAMA_65B if args.model == "65b" else LLAMA_7B
    spec = args.mode == "spec"
    fa.set_device(0)
    comm = fa.Comm.peer(1, 0)
    B, P, D, tree, mtb = 8, 128, 128, 23, 1024
    rm_kw = dict(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                 max_spec_tree_token_num=tree, max_sequence_length=512)
    if spec:
        llm = fa.Model(cfg, "tree", max_requests=B, max_tokens=mtb + tree * B, max_seq_len=512,
                       max_tree_tokens=tree, tp_rank=0, tp_size=args.tp, comm=comm)
        if args.ssms > 1:  # config E: merged trees up to 64 tokens
            rm_kw["max_spec_tree_token_num"] = tree = 64
            llm.close()
            llm = fa.Model(cfg, "tree", max_requests=B, max_tokens=mtb + tree * B,
                           max_seq_len=512, max_tree_tokens=tree, tp_rank=0, tp_size=args.tp,
                           comm=comm)
        ssms = [fa.Model(LLAMA_68M, "beam", max_requests=B, max_tokens=mtb + tree * B,
                         max_seq_len=512, max_tree_tokens=tree, weight_seed=68 + i)
                for i in range(args.ssms)]
        rm = fa.RequestManager(spec_tree_width=(1, 1, 3),
                               spec_extensions=fa.ffmi.SPEC_EXT_MULTI_SSM if args.ssms > 1 else 0,
                               **rm_kw)
        for ssm in ssms:
            rm.register_ssm_model(ssm)
    else:
        llm = fa.Model(cfg, "inc", max_requests=B, max_tokens=mtb, max_seq_len=512,
                       tp_rank=0, tp_size=args.tp, comm=comm)
        rm = fa.RequestManager(**rm_kw)
    prompts = make_prompts(B, P - 1, cfg["vocab_size"])
    fa.generate(rm, llm, prompts, max_length=P + D)  # warm
    t0 = time.time()
    llm_us = ssm_us = 0.0
    for _ in range(args.steps):  # timed with op profiling off, as the bench
        res = fa.generate(rm, llm, prompts, max_length=P + D)
        st = rm.stats()
        llm_us += st.llm_us
        ssm_us += st.ssm_us
    dt = (time.time() - t0) / args.steps
    llm.set_profiling(1)  # op breakdown: one more, untimed generate
    fa.generate(rm, llm, prompts, max_length=P + D)
    ops = llm.op_stats()
    llm.set_profiling(0)
    print(json.dumps({
        "model": args.model, "mode": args.mode, "tp": args.tp, "ssms": args.ssms if spec else 0,
        "s_per_generate": round(dt, 3),
        "tokens_per_s_without_allreduce": round(sum(len(r.output_tokens) - len(r.input_tokens)
                                                    for r in res) / dt, 1),
        "llm_ms": round(llm_us / 1000 / args.steps, 1),
        "ssm_ms": round(ssm_us / 1000 / args.steps, 1),
        "ops_avg_us": {k: round(1000 * v["ms"] / v["launches"], 2) for k, v in ops.items()},
    }))


if __name__ == "__main__":
    main()
