"""llama3 RoPE scaling of the oracle's table against a numpy restatement of
the reference's formula (inc_multihead_self_attention.cu:701-725): f32
arithmetic, freq = pos * (1.0 / pow(theta, 2i/d)) in the float/double mix,
and the wavelength taken of the position-scaled freq, as the reference does.
"""
import numpy as np
import pytest

import oracle_lib as O


def ref_table(max_pos, d, theta, llama3=None):
    f32 = np.float32
    h = d // 2
    ex = (f32(2) * np.arange(h, dtype=f32) / f32(d)).astype(f32)
    inv = 1.0 / np.power(f32(theta), ex).astype(np.float64)
    tab = np.zeros((max_pos, h, 2), f32)
    pi = f32(3.141592654)
    for p in range(max_pos):
        freq = (p * inv).astype(f32)
        if llama3:
            factor, lo, hi, orig = (f32(llama3[0]), f32(llama3[1]), f32(llama3[2]),
                                    f32(llama3[3]))
            low_wl, high_wl = f32(orig / lo), f32(orig / hi)
            with np.errstate(divide="ignore"):
                wl = (f32(2) * pi / freq).astype(f32)
            out = freq.copy()
            for i in range(h):
                if wl[i] < high_wl:
                    continue
                if wl[i] > low_wl:
                    out[i] = f32(freq[i] / factor)
                else:
                    sm = f32(f32(f32(orig / wl[i]) - lo) / f32(hi - lo))
                    a = f32(f32(f32(f32(1) - sm) * freq[i]) / factor)
                    out[i] = f32(a + f32(sm * freq[i]))
            freq = out
        tab[p, :, 0] = np.cos(freq.astype(np.float64)).astype(f32)
        tab[p, :, 1] = np.sin(freq.astype(np.float64)).astype(f32)
    return tab.reshape(max_pos, d)


@pytest.mark.parametrize("llama3", [None, (8.0, 1.0, 4.0, 64), (32.0, 1.0, 4.0, 8192)])
@pytest.mark.parametrize("d", [64, 128])
def test_oracle_rope_table_matches_reference_formula(d, llama3):
    ours = O.rope_table(300, d, 500000.0 if llama3 else 10000.0, llama3)
    ref = ref_table(300, d, 500000.0 if llama3 else 10000.0, llama3)
    # powf (numpy vs libm) may differ by 1 ulp, and cos/sin of freq ~ pos
    # then by ~pos * 2^-24: a tolerance that scales with the position (a
    # wrong scaling branch moves freq by the factor, orders of magnitude more)
    tol = 1e-6 + 4e-7 * np.arange(300, dtype=np.float32)[:, None]
    assert np.all(np.abs(ours - ref) <= tol)


def test_llama3_scaling_changes_only_long_wavelengths():
    base = O.rope_table(200, 128, 500000.0)
    l3 = O.rope_table(200, 128, 500000.0, (8.0, 1.0, 4.0, 64))
    assert np.array_equal(base[0], l3[0])            # pos 0: freq 0 either way
    # high-frequency pairs (wavelength < 16 at pos 100) are untouched
    assert np.array_equal(base[100, :8], l3[100, :8])
    assert not np.array_equal(base[100], l3[100])


def test_llama_config_from_hf_reads_llama3_scaling(tmp_path):
    import json

    import flexflow_amd as fa
    base = dict(num_hidden_layers=2, vocab_size=1000, num_attention_heads=4,
                num_key_value_heads=2, hidden_size=256, intermediate_size=512,
                rms_norm_eps=1e-5)
    sc = dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
              original_max_position_embeddings=8192)
    want = dict(num_layers=2, vocab_size=1000, num_heads=4, num_kv_heads=2, hidden=256,
                intermediate=512, rms_eps=1e-5, rope_theta=500000.0, rope_llama3=1,
                rope_factor=8.0, rope_low_freq_factor=1.0, rope_high_freq_factor=4.0,
                rope_original_max_pos=8192)
    for c in (dict(base, rope_theta=500000.0, rope_scaling=sc),           # HF <= 4.4x
              dict(base, rope_parameters=dict(sc, rope_theta=500000.0)),  # HF 5.x
              dict(base, rope_theta=500000.0, scaling_factor=sc)):       # reference key
        (tmp_path / "config.json").write_text(json.dumps(c))
        assert fa.llama_config_from_hf(str(tmp_path)) == want
    plain = fa.llama_config_from_hf(dict(base))
    assert plain["rope_theta"] == 10000.0 and "rope_llama3" not in plain
