"""ctypes binding of libffmi.so (include/ffmi.h).

The product path: every call goes to the HIP/C++ library.  There is no CPU
fallback; importing this module without a built libffmi.so raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# FFMI_LIB_VARIANT=<suffix> loads libffmi_<suffix>.so from the same directory
# (build-flag A/B runs, e.g. scripts/gpu_ab.sh "" FFMI_LIB_VARIANT=x); the default is libffmi.so
_VARIANT = os.environ.get("FFMI_LIB_VARIANT", "")
LIB_PATH = os.path.join(_HERE, f"libffmi_{_VARIANT}.so" if _VARIANT else "libffmi.so")

c_int, c_float, c_void_p, c_size_t, c_uint64, c_int64, c_double, c_long = (
    ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
    ctypes.c_int64, ctypes.c_double, ctypes.c_long)

FFMI_OK = 0
STATUS = {0: "ok", 1: "invalid argument", 2: "hip error", 3: "rccl error", 4: "oom",
          5: "unsupported", 6: "no gfx950 device"}
ATTN_INC, ATTN_SPEC, ATTN_TREE = 0, 1, 2
MODEL_INC, MODEL_BEAM, MODEL_TREE = 0, 1, 2
# ffmi_model_debug_tensor kinds (include/ffmi.h FFMI_DBG_*)
DBG_KINDS = {"hidden": 0, "logits": 1, "attn_norm": 2, "qkv": 3, "attn_out": 4, "o_proj": 5,
             "ffn_norm": 6, "mlp_act": 7, "down": 8, "embed": 9}
DBG_HIDDEN, DBG_LOGITS = DBG_KINDS["hidden"], DBG_KINDS["logits"]
EPI_NONE, EPI_SILU_MUL = 0, 1
X_PACKED = 0x10  # FFMI_X_PACKED flag for the epilogue argument
Y_PACKED = 0x20  # FFMI_Y_PACKED
W_STREAM = 0x40  # FFMI_W_STREAM: non-temporal weight loads (speed only)
F16, F32, I32 = 0, 1, 2
# synthetic weight inits (ffmi_model_opts.weight_init) and fault kinds
WEIGHT_INITS = {"uniform": 0, "depth_scaled": 1, "token_chain": 2}
FAULT_NONE, FAULT_ROPE_POS, FAULT_RESID_ROUND, FAULT_TP_HEAD_SWAP, FAULT_TP_AR_DROP = 0, 1, 2, 3, 4
# flagged SpecInfer extensions (include/ffmi.h FFMI_SPEC_EXT_*)
SPEC_EXT_WIDTH4, SPEC_EXT_MULTI_SSM = 1, 2
ATTN_QTILE = 32
MAX_TREE = 64


class TokenInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("token_id", "pos", "req", "store_slot", "prefix_len", "tree_base",
                 "tree_len", "tree_bit")] + [("tree_vis", ctypes.c_uint64)]


class AttnWork(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("req", "q_start", "q_count", "kv_len")]


class CommitInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("src_token", "req", "depth", "pad")]


class BatchDesc(ctypes.Structure):
    _fields_ = [("num_tokens", ctypes.c_int32), ("num_work", ctypes.c_int32),
                ("num_commits", ctypes.c_int32), ("num_mask_reqs", ctypes.c_int32),
                ("tokens", ctypes.POINTER(TokenInfo)), ("work", ctypes.POINTER(AttnWork)),
                ("commits", ctypes.POINTER(CommitInfo)),
                ("masks", ctypes.POINTER(ctypes.c_uint64))]


class AttnCfg(ctypes.Structure):
    _fields_ = [("mode", c_int), ("num_heads", c_int), ("head_dim", c_int),
                ("max_requests", c_int), ("max_seq_len", c_int), ("max_tree_tokens", c_int),
                ("max_tokens", c_int), ("qk_scale", c_float), ("rope_theta", c_float),
                ("out_layout", c_int), ("rope_llama3", c_int), ("rope_factor", c_float),
                ("rope_low_freq_factor", c_float), ("rope_high_freq_factor", c_float),
                ("rope_original_max_pos", c_int), ("full_precision", c_int)]


class LlamaConfig(ctypes.Structure):
    _fields_ = [("num_layers", c_int), ("vocab_size", c_int), ("num_heads", c_int),
                ("num_kv_heads", c_int), ("hidden", c_int), ("intermediate", c_int),
                ("rms_eps", c_float), ("rope_theta", c_float), ("rope_llama3", c_int),
                ("rope_factor", c_float), ("rope_low_freq_factor", c_float),
                ("rope_high_freq_factor", c_float), ("rope_original_max_pos", c_int)]

    @classmethod
    def from_dict(cls, d):
        return cls(d["num_layers"], d["vocab_size"], d["num_heads"],
                   d.get("num_kv_heads", d["num_heads"]), d["hidden"], d["intermediate"],
                   d.get("rms_eps", 1e-6), d.get("rope_theta", 10000.0),
                   d.get("rope_llama3", 0), d.get("rope_factor", 1.0),
                   d.get("rope_low_freq_factor", 1.0), d.get("rope_high_freq_factor", 4.0),
                   d.get("rope_original_max_pos", 8192))


class ModelOpts(ctypes.Structure):
    _fields_ = [("mode", c_int), ("tp_rank", c_int), ("tp_size", c_int), ("comm", c_void_p),
                ("max_requests", c_int), ("max_tokens", c_int), ("max_seq_len", c_int),
                ("max_tree_tokens", c_int), ("weight_seed", c_uint64), ("use_graphs", c_int),
                ("weights_folder", ctypes.c_char_p), ("weight_init", c_int),
                ("full_precision", c_int)]


class RMConfig(ctypes.Structure):
    _fields_ = [("max_requests_per_batch", c_int), ("max_tokens_per_batch", c_int),
                ("max_spec_tree_token_num", c_int), ("max_sequence_length", c_int),
                ("bos_token_id", c_int), ("eos_token_ids", ctypes.POINTER(c_int)),
                ("num_eos", c_int), ("spec_tree_width", ctypes.POINTER(c_int)),
                ("num_tree_width", c_int), ("verbose", c_int), ("spec_extensions", c_int)]


class Profile(ctypes.Structure):
    _fields_ = [("llm_decoding_steps", c_int), ("ssm_decoding_steps", c_int),
                ("start_us", c_double), ("finish_us", c_double),
                ("registration_us", c_double), ("first_token_us", c_double),
                ("input_len", c_int), ("output_len", c_int)]


class OpStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", c_long), ("total_ms", c_double),
                ("bytes", c_double), ("flops", c_double)]


class ServeStats(ctypes.Structure):
    _fields_ = [("llm_steps", c_long), ("ssm_steps", c_long), ("tokens_committed", c_long),
                ("tree_tokens_verified", c_long), ("request_verifies", c_long),
                ("wall_us", c_double), ("llm_us", c_double), ("ssm_us", c_double),
                ("ssm_phases_chained", c_long), ("ssm_exchange_us", c_double)]


# ffmi_allgather_fn (include/ffmi.h): an all-gather of equal-size host blocks
ALLGATHER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t, c_void_p)

# name -> (restype, argtypes); every symbol declared in include/ffmi.h
SIGNATURES = {
    "ffmi_batch_create": (c_int, [c_int, c_int, ctypes.POINTER(c_void_p)]),
    "ffmi_batch_destroy": (None, [c_void_p]),
    "ffmi_batch_upload": (c_int, [c_void_p, ctypes.POINTER(BatchDesc), c_void_p]),
    "ffmi_attn_create": (c_int, [ctypes.POINTER(AttnCfg), ctypes.POINTER(c_void_p)]),
    "ffmi_attn_destroy": (None, [c_void_p]),
    "ffmi_attn_inc": (c_int, [c_void_p] * 5),
    "ffmi_attn_spec": (c_int, [c_void_p] * 5),
    "ffmi_attn_tree": (c_int, [c_void_p] * 5),
    "ffmi_attn_kv_ptrs": (c_int, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                  ctypes.POINTER(c_int)]),
    "ffmi_linear_packed_bytes": (c_size_t, [c_int, c_int]),
    "ffmi_linear_pack_weight": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "ffmi_linear_pack_gate_up": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "ffmi_linear": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "ffmi_linear_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "ffmi_rmsnorm_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p]),
    "ffmi_residual_rmsnorm_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                          c_int, c_float, c_void_p]),
    "ffmi_silu_mul_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ffmi_arg_topk_f32": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "ffmi_linear_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "ffmi_linear_ws": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                               c_size_t, c_void_p]),
    "ffmi_rmsnorm": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p]),
    "ffmi_residual_rmsnorm": (c_int, [c_void_p] * 5 + [c_int, c_int, c_float, c_void_p]),
    "ffmi_comm_unique_id": (c_int, [c_void_p]),
    "ffmi_comm_create": (c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "ffmi_comm_create_local": (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    "ffmi_comm_destroy": (None, [c_void_p]),
    "ffmi_comm_create_peer": (c_int, [c_int, c_int, ctypes.POINTER(c_void_p)]),
    "ffmi_comm_peer_export": (c_int, [c_void_p, c_size_t, c_void_p]),
    "ffmi_comm_peer_attach": (c_int, [c_void_p, c_void_p]),
    "ffmi_comm_peer_status": (c_int, [c_void_p]),
    "ffmi_comm_peer_detach": (c_int, [c_void_p]),
    "ffmi_vocab_shard_scratch_bytes": (c_size_t, [c_int, c_int]),
    "ffmi_vocab_shard_topk": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                      c_void_p, c_void_p, c_void_p]),
    "ffmi_allreduce": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "ffmi_allreduce_rmsnorm": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                       c_void_p, c_float, c_void_p, c_int, c_void_p, c_void_p]),
    "ffmi_embedding": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "ffmi_silu_mul": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ffmi_argmax": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "ffmi_arg_topk": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "ffmi_arg_topk_workspace_bytes": (c_size_t, [c_int]),
    "ffmi_arg_topk_ws": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                 c_size_t, c_void_p]),
    "ffmi_fill_weight": (c_int, [c_void_p, c_size_t, ctypes.c_char_p, c_uint64, c_int, c_void_p]),
    "ffmi_model_create": (c_int, [ctypes.POINTER(LlamaConfig), ctypes.POINTER(ModelOpts),
                                  ctypes.POINTER(c_void_p)]),
    "ffmi_model_destroy": (None, [c_void_p]),
    "ffmi_model_set_profiling": (c_int, [c_void_p, c_int]),
    "ffmi_model_op_stats": (c_int, [c_void_p, ctypes.POINTER(OpStat), c_int]),
    "ffmi_model_set_debug": (c_int, [c_void_p, c_int]),
    "ffmi_model_debug_tensor": (ctypes.c_long, [c_void_p, c_int, c_int, c_void_p, ctypes.c_long]),
    "ffmi_model_debug_width": (ctypes.c_long, [c_void_p, c_int]),
    "ffmi_model_debug_fault": (c_int, [c_void_p, c_int, c_int, c_int]),
    "ffmi_set_device": (c_int, [c_int]),
    "ffmi_rm_create": (c_int, [ctypes.POINTER(RMConfig), ctypes.POINTER(c_void_p)]),
    "ffmi_rm_destroy": (None, [c_void_p]),
    "ffmi_rm_register_ssm": (c_int, [c_void_p, c_void_p]),
    "ffmi_rm_register_remote_ssm": (c_int, [c_void_p]),
    "ffmi_rm_set_ssm_exchange": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "ffmi_rm_set_ssm_exchange_comm": (c_int, [c_void_p, c_void_p]),
    "ffmi_comm_allgather": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "ffmi_rm_register_output_filepath": (c_int, [c_void_p, ctypes.c_char_p]),
    "ffmi_rm_register_detokenizer": (c_int, [c_void_p, c_void_p, c_void_p]),
    "ffmi_rm_set_old_llama_tokenizer": (c_int, [c_void_p, c_int]),
    "ffmi_rm_register_request": (c_int64, [c_void_p, ctypes.POINTER(c_int), c_int, c_int, c_int,
                                           c_int]),
    "ffmi_rm_serve_incr_decoding": (c_int, [c_void_p, c_void_p]),
    "ffmi_rm_serve_spec_infer": (c_int, [c_void_p, c_void_p]),
    "ffmi_rm_get_output": (c_int, [c_void_p, c_int64, ctypes.POINTER(c_int), c_int]),
    "ffmi_rm_get_profile": (c_int, [c_void_p, c_int64, ctypes.POINTER(Profile)]),
    "ffmi_rm_get_stats": (c_int, [c_void_p, ctypes.POINTER(ServeStats)]),
    "ffmi_status_str": (ctypes.c_char_p, [c_int]),
    "ffmi_version": (ctypes.c_char_p, []),
    "ffmi_last_error": (ctypes.c_char_p, []),
    "ffmi_packed_activation_bytes": (ctypes.c_size_t, [c_int, c_int]),
    "ffmi_rmsnorm_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                c_float, c_int, c_void_p]),
    "ffmi_pack_activations": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "ffmi_debug_gemm_stamps": (ctypes.c_long, [c_void_p, ctypes.c_long]),
    "ffmi_debug_fused_residual_linear": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                                 c_int, c_int, c_void_p]),
    "ffmi_debug_fused_norm_linear": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                                             c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "ffmi_debug_attn_stamps": (ctypes.c_long, [c_void_p, ctypes.c_long]),
    "ffmi_debug_markers": (ctypes.c_long, [c_void_p, ctypes.c_long]),
}

# test doubles: libffmi_testmodel.so (include/ffmi_test.h), never the product
TEST_SIGNATURES = {
    "ffmi_test_hash_model_create": (c_int, [c_int, c_int, c_int, c_int, c_int, c_uint64, c_int,
                                            ctypes.POINTER(c_void_p)]),
    "ffmi_test_hash_model_set_capacity": (c_int, [c_void_p, c_int]),
}
TEST_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libffmi_testmodel.so")

_lib = None
_test_lib = None


def test_lib():
    """The test-double library (scheduler hash model), loaded after lib()."""
    global _test_lib
    if _test_lib is None:
        lib()
        L = ctypes.CDLL(TEST_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in TEST_SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _test_lib = L
    return _test_lib


def lib():
    """Load libffmi.so (RTLD_GLOBAL, before torch if possible so one HIP
    runtime is shared)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libffmi.so not built at {LIB_PATH}; run "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# ffmi_detokenize_fn: int (*)(const int *ids, int n, char *buf, int cap, void *ctx)
DETOKENIZE_FN = ctypes.CFUNCTYPE(c_int, ctypes.POINTER(c_int), c_int, ctypes.c_void_p, c_int,
                                 c_void_p)


class FFMIError(RuntimeError):
    pass


def check(st, what=""):
    if st != FFMI_OK:
        msg = lib().ffmi_last_error().decode(errors="replace")
        raise FFMIError(f"{what}: {STATUS.get(st, st)} [{msg}]")


def int_array(vals):
    arr = (c_int * max(1, len(vals)))(*vals)
    return arr
