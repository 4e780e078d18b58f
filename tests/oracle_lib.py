"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
the checker / CPU baseline.  Never imported by flexflow_amd/.
"""
import ctypes
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int)
_u8p = ctypes.POINTER(ctypes.c_uint8)


class OrcConfig(ctypes.Structure):
    _fields_ = [("num_layers", ctypes.c_int), ("vocab_size", ctypes.c_int),
                ("num_heads", ctypes.c_int), ("num_kv_heads", ctypes.c_int),
                ("hidden", ctypes.c_int), ("intermediate", ctypes.c_int),
                ("rms_eps", ctypes.c_float), ("rope_theta", ctypes.c_float)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            subprocess.check_call(["make", "-C", os.path.dirname(LIB_PATH)])
        L = ctypes.CDLL(LIB_PATH)
        L.orc_f2h.restype = ctypes.c_uint16
        L.orc_f2h.argtypes = [ctypes.c_float]
        L.orc_h2f.restype = ctypes.c_float
        L.orc_h2f.argtypes = [ctypes.c_uint16]
        L.orc_gen_weight.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int,
                                     ctypes.c_size_t, _f32p]
        L.orc_linear.argtypes = [_f32p, _f32p, _f32p] + [ctypes.c_int] * 4
        L.orc_rmsnorm.argtypes = [_f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_float, ctypes.c_int]
        L.orc_residual_rmsnorm.argtypes = [_f32p] * 5 + [ctypes.c_int, ctypes.c_int,
                                                         ctypes.c_float, ctypes.c_int]
        L.orc_silu_mul.argtypes = [_f32p, _f32p, _f32p, ctypes.c_size_t, ctypes.c_int]
        L.orc_rope_table.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float]
        L.orc_rope_table_llama3.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                            ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_int]
        L.orc_rope_head.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                    ctypes.c_int]
        L.orc_attention_row.argtypes = [_f32p, _f32p, _f32p, _u8p, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_float, _f32p, ctypes.c_int]
        L.orc_softmax_argmax.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         _i32p, _f32p]
        L.orc_softmax_topk.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, _i32p, _f32p]
        L.orc_model_create.restype = ctypes.c_void_p
        L.orc_model_create.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_model_create_ex.restype = ctypes.c_void_p
        L.orc_model_create_ex.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_weight_amp.restype = ctypes.c_float
        L.orc_weight_amp.argtypes = [ctypes.c_int]
        L.orc_chain_embed_scale.restype = ctypes.c_float
        L.orc_chain_embed_scale.argtypes = [ctypes.c_int] * 3
        L.orc_model_destroy.argtypes = [ctypes.c_void_p]
        L.orc_model_forward.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p,
                                        ctypes.c_int, ctypes.c_int, _f32p]
        L.orc_model_forward_ex.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, ctypes.c_int,
                                           ctypes.c_int, _f32p, ctypes.c_int]
        L.orc_set_ref_block.argtypes = [ctypes.c_int]
        L.orc_set_dot_variant.argtypes = [ctypes.c_int]
        L.orc_attention_prompt_ref16.argtypes = [_f32p, _f32p, _f32p] + [ctypes.c_int] * 3 + [
            _f32p]
        L.orc_model_decode_batch.argtypes = [ctypes.c_void_p, _i32p, _i32p, _i32p,
                                             ctypes.c_int, _f32p]
        L.orc_model_get_hidden.argtypes = [ctypes.c_void_p, ctypes.c_int, _f32p]
        L.orc_model_forward_multi.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, _i32p, _i32p,
                                              _i32p, _f32p]
        L.orc_model_get_op.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _f32p]
        L.orc_model_greedy.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p,
                                       ctypes.c_int, ctypes.c_int, _i32p]
        L.orc_model_weight.restype = ctypes.c_long
        L.orc_model_weight.argtypes = [ctypes.c_void_p, ctypes.c_char_p, _f32p]
        L.orc_num_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def fp(a):
    return a.ctypes.data_as(_f32p)


def ip(a):
    return a.ctypes.data_as(_i32p)


REF16 = 2  # oracle.h ORC_REF16: the reference's half compute type in GEMMs / prompt attention


def set_ref_block(k):
    lib().orc_set_ref_block(k)


def chain_embed_scale(num_layers, hidden, intermediate):
    """token-chain init's embedding scale (oracle.h orc_chain_embed_scale)"""
    return lib().orc_chain_embed_scale(num_layers, hidden, intermediate)


def set_dot_variant(v):
    """0: dot8 (default); 1: dot16; 2: dot32 -- other fp32 summation orders of
    the same sums (the noise floor of GPU-vs-oracle drift)"""
    lib().orc_set_dot_variant(v)


def attention_prompt_ref16(q, K, V, start):
    q = np.ascontiguousarray(q, np.float32)
    K = np.ascontiguousarray(K, np.float32)
    V = np.ascontiguousarray(V, np.float32)
    T, d = q.shape
    out = np.empty((T, d), np.float32)
    lib().orc_attention_prompt_ref16(fp(q), fp(K), fp(V), T, start, d, fp(out))
    return out


def round16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def gen_weight(name, seed, kind, n):
    out = np.empty(n, np.float32)
    lib().orc_gen_weight(name.encode(), seed, kind, n, fp(out))
    return out


def linear(X, W, fp16=1):
    X = np.ascontiguousarray(X, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    T, K = X.shape
    N = W.shape[0]
    Y = np.empty((T, N), np.float32)
    lib().orc_linear(fp(X), fp(W), fp(Y), T, N, K, fp16)
    return Y


def rmsnorm(X, w, eps, fp16=1):
    X = np.ascontiguousarray(X, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    out = np.empty_like(X)
    lib().orc_rmsnorm(fp(X), fp(w), fp(out), X.shape[0], X.shape[1], eps, fp16)
    return out


def residual_rmsnorm(X1, X2, w, eps, fp16=1):
    X1 = np.ascontiguousarray(X1, np.float32)
    X2 = np.ascontiguousarray(X2, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    res = np.empty_like(X1)
    out = np.empty_like(X1)
    lib().orc_residual_rmsnorm(fp(X1), fp(X2), fp(w), fp(res), fp(out), X1.shape[0],
                               X1.shape[1], eps, fp16)
    return res, out


def silu_mul(A, B, fp16=1):
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    out = np.empty_like(A)
    lib().orc_silu_mul(fp(A), fp(B), fp(out), A.size, fp16)
    return out


def rope_table(max_pos, d, theta, llama3=None):
    """llama3: None or (factor, low_freq_factor, high_freq_factor, original_max_pos)."""
    tab = np.zeros((max_pos, d), np.float32)
    if llama3:
        lib().orc_rope_table_llama3(fp(tab), max_pos, d, theta, 1, *llama3)
    else:
        lib().orc_rope_table(fp(tab), max_pos, d, theta)
    return tab


def attention_row(q, K, V, visible, scale, fp16=1):
    q = np.ascontiguousarray(q, np.float32)
    K = np.ascontiguousarray(K, np.float32)
    V = np.ascontiguousarray(V, np.float32)
    vis = np.ascontiguousarray(visible, np.uint8)
    d = q.shape[0]
    out = np.empty(d, np.float32)
    lib().orc_attention_row(fp(q), fp(K), fp(V), vis.ctypes.data_as(_u8p), K.shape[0], d,
                            scale, fp(out), fp16)
    return out


def softmax_argmax(logits, fp16=1):
    logits = np.ascontiguousarray(logits, np.float32)
    T, V = logits.shape
    ids = np.empty(T, np.int32)
    probs = np.empty(T, np.float32)
    lib().orc_softmax_argmax(fp(logits), T, V, fp16, ip(ids), fp(probs))
    return ids, probs


def softmax_topk(logits, k, fp16=1):
    logits = np.ascontiguousarray(logits, np.float32)
    T, V = logits.shape
    ids = np.empty((T, k), np.int32)
    probs = np.empty((T, k), np.float32)
    lib().orc_softmax_topk(fp(logits), T, V, k, fp16, ip(ids), fp(probs))
    return ids, probs


class Model:
    """Oracle LLaMA (llama.cc restatement), one KV cache row per request."""

    def __init__(self, cfg, seed, fp16=1, max_requests=4, max_seq=512, weight_init=0):
        self.cfg = dict(cfg)
        c = OrcConfig(cfg["num_layers"], cfg["vocab_size"], cfg["num_heads"],
                      cfg.get("num_kv_heads", cfg["num_heads"]), cfg["hidden"],
                      cfg["intermediate"], cfg.get("rms_eps", 1e-6),
                      cfg.get("rope_theta", 10000.0))
        # weight_init 1: depth-scaled o/down projections (oracle.h)
        self.h = lib().orc_model_create_ex(ctypes.byref(c), seed, fp16, max_requests, max_seq,
                                           int(weight_init))
        if not self.h:
            raise RuntimeError("orc_model_create failed")
        self.fp16 = fp16

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_model_destroy(self.h)
            self.h = None

    def forward(self, req, tokens, start_pos):
        tokens = np.ascontiguousarray(tokens, np.int32)
        T = tokens.shape[0]
        logits = np.empty((T, self.cfg["vocab_size"]), np.float32)
        rc = lib().orc_model_forward(self.h, req, ip(tokens), T, start_pos, fp(logits))
        assert rc == 0
        return logits

    def forward_ex(self, req, tokens, start_pos, prompt_phase):
        tokens = np.ascontiguousarray(tokens, np.int32)
        T = tokens.shape[0]
        logits = np.empty((T, self.cfg["vocab_size"]), np.float32)
        rc = lib().orc_model_forward_ex(self.h, req, ip(tokens), T, start_pos, fp(logits),
                                        int(prompt_phase))
        assert rc == 0
        return logits

    def teacher_forced_ref(self, seq, n_prompt, req=0):
        """Logits the reference would compute along `seq`: the prompt
        (seq[:n_prompt]) in one prompt-phase step, then every later token in
        its own decode step (generation kernel), as incr_decoding runs it
        (request_manager.cc:713-1135).  Returns the logits rows that pick
        seq[n_prompt:] ([len(seq) - n_prompt][V])."""
        rows = [self.forward_ex(req, seq[:n_prompt], 0, 1)[-1]]
        for i in range(n_prompt, len(seq) - 1):
            rows.append(self.forward_ex(req, seq[i:i + 1], i, 0)[0])
        return np.stack(rows)

    def decode_batch(self, reqs, tokens, pos):
        reqs = np.ascontiguousarray(reqs, np.int32)
        tokens = np.ascontiguousarray(tokens, np.int32)
        pos = np.ascontiguousarray(pos, np.int32)
        T = tokens.shape[0]
        logits = np.empty((T, self.cfg["vocab_size"]), np.float32)
        rc = lib().orc_model_decode_batch(self.h, ip(reqs), ip(tokens), ip(pos), T, fp(logits))
        assert rc == 0
        return logits

    def forward_multi(self, reqs, counts, start, tokens, logits=True):
        """several requests' token blocks in one step (orc_model_forward_multi)"""
        reqs = np.ascontiguousarray(reqs, np.int32)
        counts = np.ascontiguousarray(counts, np.int32)
        start = np.ascontiguousarray(start, np.int32)
        tokens = np.ascontiguousarray(tokens, np.int32)
        out = np.empty((int(counts.sum()), self.cfg["vocab_size"]), np.float32) if logits else None
        rc = lib().orc_model_forward_multi(self.h, len(reqs), ip(reqs), ip(counts), ip(start),
                                           ip(tokens), fp(out) if logits else None)
        assert rc == 0
        return out

    def hidden(self, layer, T):
        out = np.empty((T, self.cfg["hidden"]), np.float32)
        lib().orc_model_get_hidden(self.h, layer, fp(out))
        return out

    OPS = {"attn_norm": 2, "qkv": 3, "attn_out": 4, "o_proj": 5, "ffn_norm": 6, "mlp_act": 7,
           "down": 8, "embed": 9}  # include/ffmi.h FFMI_DBG_*

    def op(self, which, layer):
        """per-op tensor of the last forward, [T][width] (see OPS)"""
        k = self.OPS[which]
        T = lib().orc_model_get_op(self.h, k, layer, None)
        assert T > 0, (which, layer)
        H, F = self.cfg["hidden"], self.cfg["intermediate"]
        width = {3: 3 * H, 7: F}.get(k, H)
        out = np.empty((T, width), np.float32)
        lib().orc_model_get_op(self.h, k, layer, fp(out))
        return out

    def greedy(self, req, prompt, n_new):
        prompt = np.ascontiguousarray(prompt, np.int32)
        out = np.empty(n_new, np.int32)
        rc = lib().orc_model_greedy(self.h, req, ip(prompt), prompt.shape[0], n_new, ip(out))
        assert rc == 0
        return out

    def weight(self, name):
        n = lib().orc_model_weight(self.h, name.encode(), None)
        assert n > 0, name
        out = np.empty(n, np.float32)
        lib().orc_model_weight(self.h, name.encode(), fp(out))
        return out


def load_golden(tag):
    path = os.path.join(ROOT, "tests", "golden", f"{tag}.npz")
    z = np.load(path, allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    return cfg, {k: z[k] for k in z.files if k != "config"}
