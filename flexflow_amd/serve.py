"""Serving API over libffmi.so, mirroring the reference's RequestManager /
FFModel::generate surface (include/flexflow/request_manager.h:119-358,
python/flexflow/serve/serve.py LLM/SSM).  All work happens in the C++
runtime and HIP kernels; this file only marshals arguments.
"""
import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Union

from . import ffmi as F


class Model:
    """A LLaMA model on one GPU (one TP shard).  mode: "inc" (incremental
    decoding LLM), "tree" (SpecInfer verify LLM) or "beam" (SSM)."""

    MODES = {"inc": F.MODEL_INC, "beam": F.MODEL_BEAM, "tree": F.MODEL_TREE}

    def __init__(self, config: dict, mode: str = "inc", *, max_requests=8, max_tokens=128,
                 max_seq_len=512, max_tree_tokens=23, weight_seed=20250117, tp_rank=0,
                 tp_size=1, comm=None, weights_folder: Optional[str] = None,
                 weight_init: Union[int, str] = 0, full_precision: bool = False):
        """weights_folder: a checkpoint in the reference's per-tensor format
        (see checkpoint.convert_hf_model); None: seeded synthetic weights,
        `weight_init` "uniform" (0, the bench's), "depth_scaled" (1) or
        "token_chain" (2) -- include/ffmi.h ffmi_model_opts.  full_precision:
        the reference's --use-full-precision (every tensor fp32,
        runtime/llama_f32.cpp); default the fp16 model."""
        L = F.lib()
        self.config = dict(config)
        self.mode = mode
        cfg = F.LlamaConfig.from_dict(config)
        opts = F.ModelOpts(self.MODES[mode], tp_rank, tp_size, comm.handle if comm else None,
                           max_requests, max_tokens, max_seq_len, max_tree_tokens, weight_seed, 0,
                           weights_folder.encode() if weights_folder else None,
                           F.WEIGHT_INITS.get(weight_init, weight_init), int(full_precision))
        h = ctypes.c_void_p()
        F.check(L.ffmi_model_create(ctypes.byref(cfg), ctypes.byref(opts), ctypes.byref(h)),
                "ffmi_model_create")
        self.handle = h

    def set_profiling(self, level: int):
        F.check(F.lib().ffmi_model_set_profiling(self.handle, level), "set_profiling")

    def op_stats(self):
        n = F.lib().ffmi_model_op_stats(self.handle, None, 0)
        arr = (F.OpStat * max(n, 1))()
        F.lib().ffmi_model_op_stats(self.handle, arr, n)
        return {a.name.decode(): dict(launches=a.launches, ms=a.total_ms, bytes=a.bytes,
                                      flops=a.flops) for a in arr[:n]}

    def set_debug(self, enable: bool = True):
        """Keep the last step's per-layer hidden states and logits
        (--inference-debugging, operator.h:271-360); steps run eager."""
        F.check(F.lib().ffmi_model_set_debug(self.handle, int(enable)), "set_debug")

    def debug_tensor(self, which: str, layer: int = 0):
        """A captured tensor of the last step as fp32 [T][width]:
        'hidden' (layer l < num_layers: residual stream after layer l;
        layer == num_layers: final norm output), 'logits' (this rank's vocab
        shard under a vocab-sharded lm_head), or an op of layer l: 'embed',
        'attn_norm', 'qkv', 'attn_out', 'o_proj', 'ffn_norm', 'mlp_act',
        'down' (include/ffmi.h FFMI_DBG_*; shard widths under TP)."""
        import numpy as np
        kind = F.DBG_KINDS[which]
        width = F.lib().ffmi_model_debug_width(self.handle, kind)
        if width <= 0:
            raise F.FFMIError(f"debug_tensor({which}): no such tensor")
        buf = np.empty(1024 * width, np.float32)
        T = F.lib().ffmi_model_debug_tensor(self.handle, kind, layer,
                                            buf.ctypes.data_as(ctypes.c_void_p), buf.size)
        if T < 0:
            raise F.FFMIError(f"debug_tensor({which}, {layer}): nothing captured")
        return buf[:T * width].reshape(T, width).copy()

    def debug_fault(self, kind: int, layer: int = 0, arg: int = 0):
        """Negative-control fault injection (tests only): F.FAULT_ROPE_POS
        makes `layer`'s RoPE rotate positions >= arg as position + 1;
        F.FAULT_NONE clears every fault (include/ffmi.h)."""
        F.check(F.lib().ffmi_model_debug_fault(self.handle, kind, layer, arg), "debug_fault")

    def close(self):
        if getattr(self, "handle", None):
            F.lib().ffmi_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


def set_device(dev: int):
    F.check(F.lib().ffmi_set_device(dev), "set_device")


class HashModel(Model):
    """Scheduler test double (CPU only, see ffmi_test_hash_model_create)."""

    def __init__(self, vocab=1000, mode="inc", *, max_requests=8, max_seq_len=512,
                 max_tree_tokens=23, salt=0, disagree_pct=0, max_tokens=None):
        self.mode = mode
        h = ctypes.c_void_p()
        F.check(F.test_lib().ffmi_test_hash_model_create(vocab, self.MODES[mode], max_requests,
                                                    max_seq_len, max_tree_tokens, salt,
                                                    disagree_pct, ctypes.byref(h)),
                "hash model")
        self.handle = h
        if max_tokens is not None:  # a GPU model's token capacity per step
            F.check(F.test_lib().ffmi_test_hash_model_set_capacity(h, max_tokens), "capacity")


class Comm:
    """RCCL communicator for tensor parallelism (one process per GPU)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        F.check(F.lib().ffmi_comm_unique_id(buf), "unique id")
        return buf.raw

    def __init__(self, uid: bytes, nranks: int, rank: int):
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(uid, 128)
        F.check(F.lib().ffmi_comm_create(buf, nranks, rank, ctypes.byref(h)), "comm create")
        self.handle = h

    @classmethod
    def local_group(cls, nranks: int):
        """In-process shard group: one communicator per host thread stepping
        a TP shard on this process's device (ffmi_comm_create_local)."""
        arr = (ctypes.c_void_p * nranks)()
        F.check(F.lib().ffmi_comm_create_local(nranks, arr), "local group")
        out = []
        for r in range(nranks):
            c = cls.__new__(cls)
            c.handle = ctypes.c_void_p(arr[r])
            out.append(c)
        return out

    @classmethod
    def peer(cls, nranks: int, rank: int):
        """A communicator with the direct xGMI transport only (no RCCL
        state): export() its exchange buffer, all-gather the handles over the
        caller's control plane, then attach() them (ffmi_comm_create_peer)."""
        c = cls.__new__(cls)
        h = ctypes.c_void_p()
        F.check(F.lib().ffmi_comm_create_peer(nranks, rank, ctypes.byref(h)), "peer comm")
        c.handle = h
        return c

    def export(self, max_bytes: int) -> bytes:
        """Allocate this rank's exchange buffer (4 x max_bytes) and return its
        64-byte IPC handle (ffmi_comm_peer_export)."""
        buf = ctypes.create_string_buffer(64)
        F.check(F.lib().ffmi_comm_peer_export(self.handle, max_bytes, buf), "peer export")
        return buf.raw

    def attach(self, handles) -> None:
        """Map every rank's exchange buffer (handles in rank order) and run the
        collective self-test (ffmi_comm_peer_attach)."""
        blob = b"".join(handles)
        buf = ctypes.create_string_buffer(blob, len(blob))
        F.check(F.lib().ffmi_comm_peer_attach(self.handle, buf), "peer attach")

    def detach(self) -> None:
        F.check(F.lib().ffmi_comm_peer_detach(self.handle), "peer detach")

    def status(self) -> None:
        F.check(F.lib().ffmi_comm_peer_status(self.handle), "peer status")

    def close(self):
        if getattr(self, "handle", None):
            F.lib().ffmi_comm_destroy(self.handle)
            self.handle = None


@dataclass
class GenerationResult:
    guid: int
    input_tokens: List[int]
    output_tokens: List[int]
    llm_decoding_steps: int = 0
    ssm_decoding_steps: int = 0
    latency_us: float = 0.0
    ttft_us: float = 0.0
    output_text: str = ""  # tokenizer.decode(output_tokens) when one is registered


class RequestManager:
    def __init__(self, max_requests_per_batch=8, max_tokens_per_batch=128,
                 max_spec_tree_token_num=23, max_sequence_length=512, bos_token_id=1,
                 eos_token_ids=(), spec_tree_width=(), verbose=False, spec_extensions=0):
        """spec_extensions: F.SPEC_EXT_WIDTH4 (tree widths / branches up to 4;
        the reference allows 3) | F.SPEC_EXT_MULTI_SSM (several SSMs, trees
        merged); 0 keeps the reference's limits (include/ffmi.h)."""
        self._eos = F.int_array(list(eos_token_ids))
        self._widths = F.int_array(list(spec_tree_width))
        cfg = F.RMConfig(max_requests_per_batch, max_tokens_per_batch, max_spec_tree_token_num,
                         max_sequence_length, bos_token_id, self._eos, len(eos_token_ids),
                         self._widths, len(spec_tree_width), int(verbose), int(spec_extensions))
        h = ctypes.c_void_p()
        F.check(F.lib().ffmi_rm_create(ctypes.byref(cfg), ctypes.byref(h)), "rm create")
        self.handle = h
        self.guids: List[int] = []
        self._ssms = []
        self._bos = bos_token_id
        self.max_sequence_length = max_sequence_length
        self.tokenizer = None
        self._add_special = {}

    def close(self):
        if getattr(self, "handle", None):
            F.lib().ffmi_rm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()

    def register_ssm_model(self, ssm: Optional[Model]):
        """ssm=None: an SSM that another rank of the TP group runs (config E's
        placement, set_ssm_exchange): every rank registers the same SSMs in
        the same order, SSM s as a model on rank s % nranks only."""
        if ssm is None:
            F.check(F.lib().ffmi_rm_register_remote_ssm(self.handle), "register remote ssm")
        else:
            F.check(F.lib().ffmi_rm_register_ssm(self.handle, ssm.handle), "register ssm")
        self._ssms.append(ssm)

    def set_ssm_exchange(self, exchange, nranks: int = 1, rank: int = 0):
        """Distributed SSMs (include/ffmi.h ffmi_rm_set_ssm_exchange): after
        its SSMs' beam steps each rank exchanges their results and replays
        the other ranks' SSMs' bookkeeping.  `exchange` is a Comm (its all-
        gather over the TP transport) or a callable all_gather(bytes) ->
        list of every rank's bytes (e.g. torch.distributed over gloo)."""
        if isinstance(exchange, Comm):
            F.check(F.lib().ffmi_rm_set_ssm_exchange_comm(self.handle, exchange.handle),
                    "ssm exchange")
            self._xch = exchange
            return

        def fn(_ctx, mine, nbytes, out):
            try:
                parts = exchange(ctypes.string_at(mine, nbytes))
                if len(parts) != nranks or any(len(p) != nbytes for p in parts):
                    return 1
                ctypes.memmove(out, b"".join(parts), nbytes * nranks)
                return 0
            except Exception:  # never unwind a Python error through C++
                return 1

        self._xch = F.ALLGATHER_FN(fn)  # kept alive with the manager
        F.check(F.lib().ffmi_rm_set_ssm_exchange(self.handle, nranks, rank,
                                                 ctypes.cast(self._xch, ctypes.c_void_p), None),
                "ssm exchange")

    def register_output_filepath(self, path: Optional[str]):
        """RequestManager::register_output_filepath (request_manager.cc:246-249):
        completed requests are appended in the reference's record format."""
        F.check(F.lib().ffmi_rm_register_output_filepath(
            self.handle, path.encode() if path else None), "output filepath")

    def register_tokenizer(self, tokenizer, bos_token_id=None, eos_token_ids=None):
        """The text of each output record is tokenizer.decode(tokens), as the
        reference's tokenizer_->Decode (request_manager.cc:786-789).  Any
        object with decode(list[int]) -> str: a `tokenizers.Tokenizer`, an HF
        tokenizer, or a test double; or a path, resolved like the reference's
        register_tokenizer (request_manager.cc:181-217, tokenizer.json first,
        then tokenizer.model; flexflow_amd.tokenizer).  A tokenizer with
        encode(str) also lets register_new_request take text prompts.  BOS/EOS
        stay as configured at creation."""
        if isinstance(tokenizer, (str, os.PathLike)):
            from .tokenizer import load_tokenizer
            tokenizer = load_tokenizer(os.fspath(tokenizer), self._bos)
        self.tokenizer = tokenizer
        F.check(F.lib().ffmi_rm_set_old_llama_tokenizer(
            self.handle, int(bool(getattr(tokenizer, "old_llama_tokenizer", False)))), "tokenizer")
        if tokenizer is None:
            self._detok = None
            F.check(F.lib().ffmi_rm_register_detokenizer(self.handle, None, None), "detok")
            return
        cache = {}

        def fn(ids, n, buf, cap, _ctx):
            try:
                key = tuple(ids[:n])
                if buf is None or cap == 0:  # length query
                    cache.clear()
                    cache[key] = tokenizer.decode(list(key)).encode("utf-8")
                    return len(cache[key])
                data = cache.get(key)
                if data is None:
                    data = tokenizer.decode(list(key)).encode("utf-8")
                m = min(cap, len(data))
                ctypes.memmove(buf, data, m)
                return m
            except Exception:  # never unwind a Python error through C++
                return 0

        self._detok = F.DETOKENIZE_FN(fn)  # kept alive with the manager
        F.check(F.lib().ffmi_rm_register_detokenizer(
            self.handle, ctypes.cast(self._detok, ctypes.c_void_p), None), "detok")

    def register_new_request(self, prompt: Union[str, List[int], None], max_length=-1,
                             max_new_tokens=-1, add_special_tokens=True,
                             benchmarking_tokens=-1) -> int:
        """Token ids, or text encoded by the registered tokenizer without
        special tokens (request_manager.cc:369-373; BOS is prepended by the
        request manager when add_special_tokens is set).

        benchmarking_tokens >= 0 is the reference's synthetic-prompt mode
        (:362-369): the prompt is that many copies of token 15 and `prompt` is
        ignored; it must be below max_sequence_length (the reference asserts).
        Deviation: max_new_tokens counts from that prompt here, where the
        reference leaves max_length unset in this mode."""
        if benchmarking_tokens >= 0:
            if benchmarking_tokens >= self.max_sequence_length:
                raise ValueError("Benchmarking tokens exceed max sequence length")
            prompt = [15] * benchmarking_tokens
        if isinstance(prompt, str):
            if self.tokenizer is None or not hasattr(self.tokenizer, "encode"):
                raise ValueError("text prompt needs a tokenizer with encode() "
                                 "(register_tokenizer); the reference asserts "
                                 "'Tokenizer is null!'")
            prompt = self.tokenizer.encode(prompt)
        arr = F.int_array(list(prompt))
        g = F.lib().ffmi_rm_register_request(self.handle, arr, len(prompt), max_length,
                                             max_new_tokens, int(add_special_tokens))
        if g > 0:
            self.guids.append(g)
            self._add_special[g] = bool(add_special_tokens)
        return g

    def serve_incr_decoding(self, llm: Model):
        F.check(F.lib().ffmi_rm_serve_incr_decoding(self.handle, llm.handle), "serve incr")

    def serve_spec_infer(self, llm: Model):
        F.check(F.lib().ffmi_rm_serve_spec_infer(self.handle, llm.handle), "serve spec")

    def get_generation_result(self, guid: int) -> GenerationResult:
        L = F.lib()
        n = L.ffmi_rm_get_output(self.handle, guid, None, 0)
        buf = (ctypes.c_int * max(n, 1))()
        L.ffmi_rm_get_output(self.handle, guid, buf, n)
        p = F.Profile()
        F.check(L.ffmi_rm_get_profile(self.handle, guid, ctypes.byref(p)), "profile")
        out = list(buf[:n])
        text = ""
        if self.tokenizer is not None:
            try:
                text = self.tokenizer.decode(out)
            except Exception:  # a decode-less test double
                text = ""
            # the old LLaMA tokenizer's "<s> " prefix (request_manager.cc:776-781)
            if (getattr(self.tokenizer, "old_llama_tokenizer", False) and
                    self._add_special.get(guid, True) and out and out[0] == self._bos):
                text = "<s> " + text
        return GenerationResult(guid, out[:p.input_len], out, p.llm_decoding_steps,
                                p.ssm_decoding_steps, p.finish_us - p.start_us,
                                p.first_token_us - p.registration_us, text)

    def stats(self) -> F.ServeStats:
        s = F.ServeStats()
        F.check(F.lib().ffmi_rm_get_stats(self.handle, ctypes.byref(s)), "stats")
        return s


def generate(rm: RequestManager, llm: Model, prompts, max_length=-1, max_new_tokens=-1,
             spec: Optional[bool] = None):
    """FFModel::generate (request_manager.cc:2880-2911): register, serve, collect."""
    guids = [rm.register_new_request(p, max_length=max_length, max_new_tokens=max_new_tokens)
             for p in prompts]
    if spec is None:
        spec = llm.mode == "tree"
    if spec:
        rm.serve_spec_infer(llm)
    else:
        rm.serve_incr_decoding(llm)
    return [rm.get_generation_result(g) if g > 0 else None for g in guids]
