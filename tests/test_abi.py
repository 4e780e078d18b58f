"""The C-ABI library loads (no GPU needed) and exports every symbol that
include/ffmi.h declares; the Python binding covers them all."""
import ctypes
import os
import re

import flexflow_amd.ffmi as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header="ffmi.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ffmi_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(F.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_test_doubles_live_outside_the_product_library():
    """The scheduler hash model (include/ffmi_test.h) is exported by
    libffmi_testmodel.so only; libffmi.so carries no test symbols."""
    prod = ctypes.CDLL(F.LIB_PATH)
    test = ctypes.CDLL(F.TEST_LIB_PATH)
    names = declared_functions("ffmi_test.h")
    assert names == ["ffmi_test_hash_model_create", "ffmi_test_hash_model_set_capacity"]
    for n in names:
        assert hasattr(test, n) and not hasattr(prod, n), n
    assert set(names) <= set(F.TEST_SIGNATURES)


def test_binding_covers_header():
    names = set(declared_functions())
    assert names <= set(F.SIGNATURES), sorted(names - set(F.SIGNATURES))


def test_status_strings_and_version():
    L = F.lib()
    assert L.ffmi_version().startswith(b"ffmi")
    assert L.ffmi_status_str(0) == b"ok"
    assert L.ffmi_status_str(6) == b"no gfx950 device"


def test_invalid_arguments_return_status_not_abort():
    L = F.lib()
    assert L.ffmi_linear(None, None, None, 1, 16, 32, 0, None) == 1
    assert L.ffmi_rmsnorm(None, None, None, 1, 8, 1e-6, None) == 1
    # the full-precision linear: null operands, then an in_dim off the k-block
    assert L.ffmi_linear_f32(None, None, None, 1, 16, 32, None) == 1
    assert L.ffmi_linear_f32(None, None, None, 1, 16, 48, None) == 5
    cfg = F.AttnCfg(0, 2, 96, 1, 16, 0, 16, 0.1, 10000.0, 0)  # head_dim 96 unsupported
    h = ctypes.c_void_p()
    assert L.ffmi_attn_create(ctypes.byref(cfg), ctypes.byref(h)) == 5
    # head_dim 32: incremental decoding only, as the reference's kernels
    # (inc...cu:911-926 take 32 / 64 / 128; tree_inc...cu:562-572 and
    # spec_inc...cu:431-441 64 / 128)
    for mode in (F.ATTN_TREE, F.ATTN_SPEC):
        cfg = F.AttnCfg(mode, 2, 32, 1, 16, 8, 16, 0.1, 10000.0, 0)
        assert L.ffmi_attn_create(ctypes.byref(cfg), ctypes.byref(h)) == 5
    # the all-reduce + residual norm with null operands
    assert L.ffmi_allreduce_rmsnorm(None, None, 8, 256, 0, None, None, None, 1e-6, None, 0, None,
                                    None) == 1
    # the top-k with a caller workspace: null operands
    assert L.ffmi_arg_topk_ws(None, 4, 32000, 1, None, None, None, 0, None) == 1


def test_full_precision_model_opts_and_no_device():
    """ffmi_model_opts.full_precision (the reference's --use-full-precision)
    routes creation to the fp32 model, which fails with NO_DEVICE here (no
    GPU) rather than falling back to anything on the host."""
    L = F.lib()
    cfg = F.LlamaConfig.from_dict(dict(num_layers=1, vocab_size=64, num_heads=2, num_kv_heads=2,
                                       hidden=128, intermediate=256))
    opts = F.ModelOpts(F.MODEL_INC, 0, 1, None, 1, 16, 64, 0, 1, 0, None, 0, 1)
    assert opts.full_precision == 1
    h = ctypes.c_void_p()
    assert L.ffmi_model_create(ctypes.byref(cfg), ctypes.byref(opts), ctypes.byref(h)) == 6
