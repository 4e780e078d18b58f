"""SpecInfer configurations of the GPU tests.

- "w113": config C as the reference runs it: tree widths (1, 1, 3) (its
  maximum, MAX_BEAM_WIDTH = 3, request_manager.cc:168-171), one SSM, 23-token
  tree budget (spec_infer.cc:298-340);
- "w114": config C as BASELINE.json states it, tree width 4: widths (1, 1, 4),
  27-token trees, the flagged FFMI_SPEC_EXT_WIDTH4;
- "ssm4": config E's "4x SSMs": four LLaMA-68M SSMs (seeds 68..71), widths
  (1, 1, 3), trees merged by path and cut to 64 tokens
  (FFMI_SPEC_EXT_MULTI_SSM, merge_dfs_trees request_manager.cc:2817-2878).
"""
import flexflow_amd as fa

SPEC = {
    "w113": dict(widths=(1, 1, 3), ssm_seeds=(68,), tree=23, ext=0),
    "w114": dict(widths=(1, 1, 4), ssm_seeds=(68,), tree=27, ext=fa.ffmi.SPEC_EXT_WIDTH4),
    "ssm4": dict(widths=(1, 1, 3), ssm_seeds=(68, 69, 70, 71), tree=64,
                 ext=fa.ffmi.SPEC_EXT_MULTI_SSM),
}


def spec_setup(name, ssm_cfg, B, mtb, max_seq, place=None, **model_kw):
    """RequestManager with config `name`'s widths / extensions, its SSMs
    registered.  Returns (rm, ssms, vt, tree): vt = the verify batch's token
    capacity (mtb + tree * B), the LLM's max_tokens.  place = (comm, rank,
    nranks): the SSMs distributed over the TP group (SSM s on rank s % nranks,
    ffmi_rm_set_ssm_exchange_comm); otherwise every SSM is built here."""
    sc = SPEC[name]
    tree = sc["tree"]
    vt = mtb + tree * B
    rm = fa.RequestManager(max_requests_per_batch=B, max_tokens_per_batch=mtb,
                           max_sequence_length=max_seq, spec_tree_width=sc["widths"],
                           max_spec_tree_token_num=tree, spec_extensions=sc["ext"])
    ssms = []
    for i, seed in enumerate(sc["ssm_seeds"]):
        if place is not None and i % place[2] != place[1]:
            rm.register_ssm_model(None)  # another rank runs it
            continue
        m = fa.Model(ssm_cfg, "beam", max_requests=B, max_tokens=vt, max_seq_len=max_seq,
                     max_tree_tokens=tree, weight_seed=seed, **model_kw)
        ssms.append(m)
        rm.register_ssm_model(m)
    if place is not None:
        rm.set_ssm_exchange(place[0])
    return rm, ssms, vt, tree
