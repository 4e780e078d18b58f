"""Rank tasks for tests/peer_group.py (run inside the spawned rank processes)."""
import time

import numpy as np


def case_data(case, it, rank, count, dtype):
    rng = np.random.default_rng(1000003 * case + 7919 * it + rank)
    x = rng.standard_normal(count).astype(np.float32)
    return x.astype(np.float16) if dtype == "f16" else x


def ar_task(fa, comm, rank, n, cases, iters):
    """ffmi_allreduce over the xGMI transport, `iters` back-to-back rounds of
    every case (epochs, parities and buffer reuse all cycle)."""
    import flexflow_amd.ffmi as F
    from hip_util import Buf, sync
    L = F.lib()
    out = {}
    for it in range(iters):
        for ci, (count, dtype) in enumerate(cases):
            x = case_data(ci, it, rank, count, dtype)
            src = Buf(x)
            dst = Buf.empty(x.shape, x.dtype)
            F.check(L.ffmi_allreduce(comm.handle, src.ptr, dst.ptr, count,
                                     F.F16 if dtype == "f16" else F.F32, None), "allreduce")
            sync()
            out[(it, ci)] = dst.get()
    return out


def arnorm_task(fa, comm, rank, n, cases, seed, iters=2):
    """ffmi_allreduce_rmsnorm against ffmi_allreduce + ffmi_rmsnorm_ex on the
    same inputs, per case (T, H, col0, packed): the normalised rows `out` on
    every row and the residual on the rows the call reports as updated.
    Columns < col0 come from `prev` = the unfused all-reduce's sum."""
    import ctypes

    import flexflow_amd.ffmi as F
    from hip_util import Buf, f16, sync
    L = F.lib()
    out = []
    for it in range(iters):
        for ci, (T, H, col0, packed) in enumerate(cases):
            rng = np.random.default_rng(seed + 7919 * ci + 104729 * it)  # same on every rank
            res0 = f16(rng.standard_normal((T, H)) * 2)
            w = f16(rng.uniform(0.25, 2.0, H))
            parts = [f16(rng.standard_normal((T, H)) * 0.7) for _ in range(n)]
            flags = F.Y_PACKED if packed else 0
            hbytes = L.ffmi_packed_activation_bytes(T, H) if packed else T * H * 2
            eps = 1e-5
            s = Buf(parts[rank])
            F.check(L.ffmi_allreduce(comm.handle, s.ptr, s.ptr, T * H, F.F16, None), "allreduce")
            wb = Buf(w)
            r1, h1 = Buf(res0), Buf.empty((hbytes // 2,), np.uint16)
            F.check(L.ffmi_rmsnorm_ex(r1.ptr, s.ptr, wb.ptr, r1.ptr, h1.ptr, T, H, eps, flags, None),
                    "rmsnorm")
            inp = Buf(np.ascontiguousarray(parts[rank][:, col0:]))
            r2, h2 = Buf(res0), Buf.empty((hbytes // 2,), np.uint16)
            rows = (ctypes.c_int * 2)()
            F.check(L.ffmi_allreduce_rmsnorm(comm.handle, inp.ptr, T, H, col0,
                                             s.ptr if col0 else None, r2.ptr, wb.ptr, eps, h2.ptr,
                                             flags, rows, None), "allreduce_rmsnorm")
            sync()
            a, b = r1.get().reshape(T, H), r2.get().reshape(T, H)
            lo, hi = rows[0], rows[1]
            out.append(dict(case=ci, it=it, rows=(lo, hi),
                            h_equal=bool(np.array_equal(h1.get(), h2.get())),
                            res_equal=bool(np.array_equal(a[lo:hi].view(np.uint16),
                                                          b[lo:hi].view(np.uint16))),
                            res_others_untouched=bool(np.array_equal(
                                np.delete(b, np.s_[lo:hi], 0).view(np.uint16),
                                np.delete(res0, np.s_[lo:hi], 0).view(np.uint16)))))
    return out


def expected_sum(case, it, n, count, dtype):
    acc = np.zeros(count, np.float32)
    for r in range(n):  # rank order, fp32, rounded once
        acc = acc + case_data(case, it, r, count, dtype).astype(np.float32)
    return acc.astype(np.float16) if dtype == "f16" else acc


def silent_peer_task(fa, comm, rank, n):
    """Rank 0 all-reduces alone: its kernel must time out and report it."""
    import flexflow_amd.ffmi as F
    from hip_util import Buf, sync
    if rank != 0:
        time.sleep(4)  # keep the buffer mapped while rank 0 waits
        return "idle"
    x = Buf(np.ones(4096, np.float32))
    t0 = time.time()
    F.check(F.lib().ffmi_allreduce(comm.handle, x.ptr, x.ptr, 4096, F.F32, None), "allreduce")
    sync()
    dt = time.time() - t0
    st = F.lib().ffmi_comm_peer_status(comm.handle)
    comm.expect_error = True  # (the harness's final status check is skipped)
    return {"status": int(st), "seconds": dt,
            "msg": F.lib().ffmi_last_error().decode(errors="replace")}


def model_task(fa, comm, rank, n, cfg, seed, prompts, max_length, spec, ssm_cfg):
    """One TP shard of a LLaMA model per rank, over the xGMI transport."""
    mode = "tree" if spec else "inc"
    extra = 23 * 4 if spec else 0
    m = fa.Model(cfg, mode, max_requests=4, max_tokens=32 + extra, max_seq_len=128,
                 weight_seed=seed, tp_rank=rank, tp_size=n, comm=comm)
    rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=32,
                           max_sequence_length=128, spec_tree_width=(1, 1, 3) if spec else ())
    if spec:
        rm.register_ssm_model(fa.Model(ssm_cfg, "beam", max_requests=4, max_tokens=32 + extra,
                                       max_seq_len=128, weight_seed=5))
    res = fa.generate(rm, m, prompts, max_length=max_length)
    m.close()
    return [r.output_tokens for r in res]


def planted_logits(T, V, seed):
    """Logit rows with planted cross-shard ties: equal maxima in different
    shards, rows of near-equal logits whose fp16 probabilities tie, random
    rows."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((T, V)).astype(np.float32) * 3
    for t in range(T):
        kind = t % 4
        if kind == 0:  # the same maximum at several ids across shards
            m = x[t].max() + 1.0
            for i in rng.choice(V, 4, replace=False):
                x[t, i] = m
        elif kind == 1:  # tiny spread: the fp16 softmax rounds many ids to one p
            x[t] = rng.choice([0.0, 2.0 ** -14, 2.0 ** -13, 2.0 ** -12], V)
        elif kind == 2:  # second-best equal to best after rounding, other shard
            i, j = rng.choice(V, 2, replace=False)
            x[t, i] = x[t].max() + 2.0
            x[t, j] = x[t, i] - 2.0 ** -9
    return x.astype(np.float16)


def vshard_task(fa, comm, rank, n, T, V, k, seed):
    import flexflow_amd.ffmi as F
    from hip_util import Buf
    L = F.lib()
    x = planted_logits(T, V, seed)
    Vl = V // n
    shard = Buf(np.ascontiguousarray(x[:, rank * Vl:(rank + 1) * Vl]))
    ids, probs = Buf.empty((T, k), np.int32), Buf.empty((T, k), np.float32)
    scratch = Buf.empty((L.ffmi_vocab_shard_scratch_bytes(n, T),), np.uint8)
    F.check(L.ffmi_vocab_shard_topk(comm.handle, shard.ptr, T, Vl, k, ids.ptr, probs.ptr,
                                    scratch.ptr, None), "vocab shard topk")
    out = {"ids": ids.get(), "probs": probs.get()}
    if rank == 0:  # the oracle's softmax + arg-top-k on the gathered logits
        import oracle_lib as O
        ri, rp = O.softmax_topk(x.astype(np.float32), k, fp16=1)
        out["ref_ids"], out["ref_probs"] = ri.reshape(T, k), rp.reshape(T, k)
    return out


def tp_generate_task(fa, comm, rank, n, cfg, seed, prompts, max_length, spec, ssm_cfg,
                     tf_seqs=(), weight_init=0, fault=None, ssm_place="replicated"):
    """One TP shard per rank of a full-depth model over the xGMI transport:
    incr decoding (spec False) or SpecInfer with the SSM replicated on every
    rank (spec_infer.cc:385-387).  Then, in incr mode, a teacher-forced pass:
    the sequences `tf_seqs` (+ this run's own) as ONE prefill step with the
    logits captured (this rank's vocab shard, [T][V/n]); the row predicting
    token j + 1 of sequence s is s's j-th row of its block."""
    # fault = (kind, layer, arg, rank): a negative control on that rank's
    # shard only (ffmi_model_debug_fault FFMI_FAULT_TP_*)
    def apply_fault(m):
        if fault is not None and rank == fault[3]:
            m.debug_fault(fault[0], fault[1], fault[2])
    B = len(prompts)
    mtb = 256
    if spec:  # True or a tests/spec_configs.py name; the SSMs replicated per rank
        from spec_configs import spec_setup
        # ssm_place "distributed": SSM s on rank s % n only, results exchanged
        # (config E's placement); "replicated": every SSM on every rank
        place = (comm, rank, n) if ssm_place == "distributed" else None
        rm, ssms, vt, tt = spec_setup("w113" if spec is True else spec, ssm_cfg, B, mtb, 128,
                                      place=place, weight_init=weight_init)
        m = fa.Model(cfg, "tree", max_requests=B, max_tokens=vt, max_seq_len=128,
                     max_tree_tokens=tt, weight_seed=seed, tp_rank=rank, tp_size=n, comm=comm,
                     weight_init=weight_init)
        apply_fault(m)
        res = fa.generate(rm, m, prompts, max_length=max_length, spec=True)
        st = rm.stats()
        out = {"tokens": [r.output_tokens for r in res], "llm_steps": st.llm_steps,
               "ssm_steps": st.ssm_steps, "tree_tokens_verified": st.tree_tokens_verified,
               "ssm_us": st.ssm_us, "ssm_exchange_us": st.ssm_exchange_us}
        m.close()
        for x in ssms:
            x.close()
        return out
    nt = B + len(tf_seqs)
    m = fa.Model(cfg, "inc", max_requests=max(B, nt), max_tokens=2 * mtb, max_seq_len=128,
                 weight_seed=seed, tp_rank=rank, tp_size=n, comm=comm, weight_init=weight_init)
    apply_fault(m)
    rm = fa.RequestManager(max_requests_per_batch=max(B, nt), max_tokens_per_batch=mtb,
                           max_sequence_length=128)
    res = fa.generate(rm, m, prompts, max_length=max_length)
    toks = [r.output_tokens for r in res]
    seqs = list(tf_seqs) + toks
    assert sum(len(s) for s in seqs) <= 2 * mtb and len(set(map(len, seqs))) == 1
    m.set_debug(True)
    fa.generate(fa.RequestManager(max_requests_per_batch=nt, max_tokens_per_batch=2 * mtb,
                                  max_sequence_length=128), m, [s[1:] for s in seqs],
                max_length=len(seqs[0]) + 1)
    lg = m.debug_tensor("logits")
    m.close()
    return {"tokens": toks, "tf_logits": lg.astype(np.float16), "tf_seqs": seqs}


def tp_generate_f32_task(fa, comm, rank, n, cfg, seed, prompts, max_length, spec, ssm_cfg):
    """Full precision (--use-full-precision) TP shard per rank: incr decoding
    or SpecInfer (SSM replicated, also fp32), tokens only"""
    B = len(prompts)
    mtb = 256
    kw = dict(max_requests=B, max_seq_len=128, full_precision=True)
    if spec:
        m = fa.Model(cfg, "tree", max_tokens=mtb + 23 * B, weight_seed=seed, tp_rank=rank,
                     tp_size=n, comm=comm, **kw)
        ssm = fa.Model(ssm_cfg, "beam", max_tokens=mtb + 23 * B, max_tree_tokens=23,
                       weight_seed=68, **kw)
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=128, spec_tree_width=(1, 1, 3))
        rm.register_ssm_model(ssm)
        res = fa.generate(rm, m, prompts, max_length=max_length, spec=True)
        ssm.close()
    else:
        m = fa.Model(cfg, "inc", max_tokens=mtb, weight_seed=seed, tp_rank=rank, tp_size=n,
                     comm=comm, **kw)
        rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                               max_sequence_length=128)
        res = fa.generate(rm, m, prompts, max_length=max_length)
    m.close()
    return {"tokens": [r.output_tokens for r in res], "llm_steps": rm.stats().llm_steps}
