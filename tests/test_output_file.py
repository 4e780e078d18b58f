"""Output-file records and detokenization (RequestManager::register_output_filepath,
request_manager.cc:246-249; record formats :813-840 incremental decoding and
:1303-1330 SpecInfer), on CPU with the hash test double.

The reference's own regression script compares the "token IDs:" lines of the
incr_decoding and spec_infer output files (tests/inference/
cpp_inference_tests.sh:183-189); that comparison is restated here.
"""
import re

import pytest

import flexflow_amd as fa
from test_scheduler import V, expected, prompts

RECORD = re.compile(r"\[Profile\] guid\((\d+)\) llm_decoding_steps\((\d+)\) "
                    r"latency\((\d+\.\d{3})\)(?: ttft\((-?\d+\.\d{3})\))?\n"
                    r"token IDs: ([0-9,]*)\n")


class WordTok:
    """decode(ids) -> text, like tokenizers.Tokenizer / HF tokenizers."""

    def decode(self, ids):
        return " ".join(f"w{t}" for t in ids)


def serve(tmp_path, name, spec, ps, max_length, tok=None):
    path = tmp_path / name
    kw = dict(max_requests_per_batch=4, max_sequence_length=128)
    if spec:
        rm = fa.RequestManager(max_tokens_per_batch=64, spec_tree_width=(1, 1, 3),
                               max_spec_tree_token_num=23, **kw)
        llm = fa.HashModel(V, "tree", max_requests=4, max_seq_len=128, max_tree_tokens=23)
        rm.register_ssm_model(fa.HashModel(V, "beam", max_requests=4, max_seq_len=128,
                                           max_tree_tokens=23, salt=7, disagree_pct=30))
    else:
        rm = fa.RequestManager(max_tokens_per_batch=16, **kw)
        llm = fa.HashModel(V, "inc", max_requests=4, max_seq_len=128)
    rm.register_output_filepath(str(path))
    if tok is not None:
        rm.register_tokenizer(tok)
    res = fa.generate(rm, llm, ps, max_length=max_length)
    return path.read_text(), res


def parse(text, tok=None):
    """Records in file order: (guid, steps, latency, ttft, ids, decoded text)."""
    out, pos = [], 0
    while pos < len(text):
        m = RECORD.match(text, pos)
        assert m, f"bad record at byte {pos}: {text[pos:pos + 80]!r}"
        ids = [int(x) for x in m.group(5).split(",")]
        pos = m.end()
        body = tok.decode(ids) if tok else ""
        assert text.startswith(body, pos)
        pos += len(body)
        out.append((int(m.group(1)), int(m.group(2)), float(m.group(3)), m.group(4), ids, body))
    return out


@pytest.mark.parametrize("spec", [False, True])
def test_output_records_match_results(tmp_path, spec):
    ps = prompts(6, V, seed=21)
    text, res = serve(tmp_path, "out.txt", spec, ps, 60)
    recs = parse(text)
    assert len(recs) == len(ps)
    by_guid = {r.guid: r for r in res}
    for guid, steps, lat, ttft, ids, body in recs:
        r = by_guid[guid]
        assert ids == r.output_tokens and steps == r.llm_decoding_steps and lat >= 0
        assert (ttft is None) == spec  # ttft only in the incr record (:822-824)
        assert body == ""  # no tokenizer registered: empty text, no newline


def test_spec_and_incr_files_agree_like_the_reference_script(tmp_path):
    """cpp_inference_tests.sh:183-189: the token-ID lines of the spec_infer and
    incr_decoding output files are identical (ordered by guid)."""
    ps = prompts(8, V, seed=5)
    tok = WordTok()
    t_incr, _ = serve(tmp_path, "incr.txt", False, ps, 70, tok)
    t_spec, _ = serve(tmp_path, "spec.txt", True, ps, 70, tok)
    a = sorted(parse(t_incr, tok), key=lambda r: r[0])
    b = sorted(parse(t_spec, tok), key=lambda r: r[0])
    assert [r[4] for r in a] == [r[4] for r in b] == [expected(p, 70, V) for p in ps]
    assert [r[5] for r in a] == [tok.decode(r[4]) for r in a]


def test_records_append_and_can_be_turned_off(tmp_path):
    ps = prompts(2, V, seed=9)
    path = tmp_path / "o.txt"
    rm = fa.RequestManager(max_requests_per_batch=4, max_tokens_per_batch=16,
                           max_sequence_length=128)
    llm = fa.HashModel(V, "inc", max_requests=4, max_seq_len=128)
    rm.register_output_filepath(str(path))
    fa.generate(rm, llm, ps, max_length=30)
    fa.generate(rm, llm, ps, max_length=30)
    assert len(parse(path.read_text())) == 4  # appended, like std::ios::app
    rm.register_output_filepath(None)
    fa.generate(rm, llm, ps, max_length=30)
    assert len(parse(path.read_text())) == 4


def test_hf_tokenizers_object_as_detokenizer(tmp_path):
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers.models import WordLevel
    from tokenizers.pre_tokenizers import Whitespace
    vocab = {f"t{i}": i for i in range(V)}
    vocab["[UNK]"] = V
    tk = tokenizers.Tokenizer(WordLevel(vocab, unk_token="[UNK]"))
    tk.pre_tokenizer = Whitespace()
    ps = prompts(3, V, seed=4)
    text, res = serve(tmp_path, "tk.txt", False, ps, 40, tk)
    recs = parse(text, tk)
    assert [r[5] for r in recs] == [tk.decode(r[4]) for r in recs]
    assert all(r[5].startswith("t1 ") for r in recs)  # BOS = token 1
