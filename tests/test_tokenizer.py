"""Tokenizer loading and text prompts (RequestManager::register_tokenizer,
request_manager.cc:181-217; prompt encoding :358-373; output text :772-789),
on CPU with the hash test double.

No LLaMA tokenizer files ship offline, so the fixtures are built here: a
SentencePiece model trained on a synthetic corpus (the `tokenizer.model`
path) and a WordLevel `tokenizers` JSON (the `tokenizer.json` path).  What is
checked is the reference's resolution order, BOS handling and the "<s> "
prefix rule, not a particular vocabulary.
"""
import pytest

import flexflow_amd as fa

spm = pytest.importorskip("sentencepiece")
tokenizers = pytest.importorskip("tokenizers")


def _corpus(path, n=1500):
    import random
    rng = random.Random(5)
    syll = ["ka", "lo", "mi", "ne", "su", "ta", "ri", "po", "de", "fa", "gu", "he"]
    with open(path, "w") as f:
        for _ in range(n):
            words = ["".join(rng.choice(syll) for _ in range(rng.randint(1, 4)))
                     for _ in range(rng.randint(3, 12))]
            f.write(" ".join(words) + "\n")


@pytest.fixture(scope="module")
def sp_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("sp")
    _corpus(d / "corpus.txt")
    spm.SentencePieceTrainer.train(input=str(d / "corpus.txt"), model_prefix=str(d / "tokenizer"),
                                   vocab_size=120, model_type="bpe", bos_id=1, eos_id=2,
                                   unk_id=0, pad_id=-1, hard_vocab_limit=False,
                                   minloglevel=2)
    (d / "corpus.txt").unlink()
    return d


def _hf_json(path, V):
    from tokenizers.models import WordLevel
    from tokenizers.pre_tokenizers import Whitespace
    vocab = {f"t{i}": i for i in range(V)}
    tk = tokenizers.Tokenizer(WordLevel(vocab, unk_token="t0"))
    tk.pre_tokenizer = Whitespace()
    tk.save(str(path))
    return tk


def _serve(tok, prompts, V, max_length=24, spec=False):
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
    rm.register_tokenizer(tok)
    return rm, fa.generate(rm, llm, prompts, max_length=max_length)


def test_directory_prefers_tokenizer_json(sp_dir, tmp_path):
    d = tmp_path / "both"
    d.mkdir()
    (d / "tokenizer.model").write_bytes((sp_dir / "tokenizer.model").read_bytes())
    _hf_json(d / "tokenizer.json", 50)
    assert not fa.load_tokenizer(str(d)).old_llama_tokenizer      # tokenizer.json first
    (d / "tokenizer.json").unlink()
    assert fa.load_tokenizer(str(d)).old_llama_tokenizer          # then tokenizer.model
    (d / "tokenizer.model").unlink()
    with pytest.raises(FileNotFoundError):
        fa.load_tokenizer(str(d))


@pytest.mark.parametrize("spec", [False, True])
def test_sentencepiece_text_prompts(sp_dir, spec):
    tok = fa.load_tokenizer(str(sp_dir))
    V = tok._sp.get_piece_size()
    texts = ["kalo mine suta", "ripo defa guhe kaka", "lo"]
    rm, res = _serve(str(sp_dir), texts, V, spec=spec)
    for text, r in zip(texts, res):
        ids = tok.encode(text)
        assert 1 not in ids                                      # encoded without BOS
        assert r.input_tokens == [1] + ids                       # BOS from the manager
        assert len(r.output_tokens) == 24
        # SentencePiece drops BOS on decode; the reference prefixes "<s> "
        assert r.output_text == "<s> " + tok._sp.decode(r.output_tokens)
        assert r.output_text.startswith("<s> " + tok._sp.decode(ids))


def test_hf_json_text_prompts(tmp_path):
    V = 300
    tk = _hf_json(tmp_path / "tokenizer.json", V)
    rm, res = _serve(str(tmp_path / "tokenizer.json"), ["t5 t17 t250", "t3"], V)
    for text, r in zip(["t5 t17 t250", "t3"], res):
        assert r.input_tokens == [1] + tk.encode(text, add_special_tokens=False).ids
        assert r.output_text == tk.decode(r.output_tokens, skip_special_tokens=False)
        assert r.output_text.startswith("t1 " + text)


def test_text_prompt_without_tokenizer_is_an_error():
    rm = fa.RequestManager(max_requests_per_batch=1, max_tokens_per_batch=16)
    with pytest.raises(ValueError):
        rm.register_new_request("hello")


def test_benchmarking_tokens_prompt():
    """request_manager.cc:358-369: BOS + benchmarking_tokens copies of 15."""
    V = 997
    rm = fa.RequestManager(max_requests_per_batch=2, max_tokens_per_batch=16,
                           max_sequence_length=128)
    llm = fa.HashModel(V, "inc", max_requests=2, max_seq_len=128)
    g = rm.register_new_request(None, max_length=40, benchmarking_tokens=20)
    rm.serve_incr_decoding(llm)
    r = rm.get_generation_result(g)
    assert r.input_tokens == [1] + [15] * 20 and len(r.output_tokens) == 40
    with pytest.raises(ValueError):
        rm.register_new_request(None, benchmarking_tokens=128)


def test_bos_prefix_only_with_add_special_tokens(sp_dir, tmp_path):
    """The "<s> " prefix needs add_special_tokens (request_manager.cc:776-781):
    a caller-supplied BOS with add_special_tokens=False gets the bare text, in
    the result and in the output-file record."""
    tok = fa.load_tokenizer(str(sp_dir))
    V = tok._sp.get_piece_size()
    rm = fa.RequestManager(max_tokens_per_batch=16, max_requests_per_batch=4,
                           max_sequence_length=128)
    rm.register_tokenizer(str(sp_dir))
    out = tmp_path / "out.txt"
    rm.register_output_filepath(str(out))
    ids = tok.encode("kalo mine suta")
    g_plain = rm.register_new_request([1] + ids, max_length=20, add_special_tokens=False)
    g_special = rm.register_new_request(ids, max_length=20)
    rm.serve_incr_decoding(fa.HashModel(V, "inc", max_requests=4, max_seq_len=128))
    plain, special = rm.get_generation_result(g_plain), rm.get_generation_result(g_special)
    assert plain.output_tokens[0] == 1 and special.output_tokens[0] == 1
    assert plain.output_text == tok._sp.decode(plain.output_tokens)
    assert special.output_text == "<s> " + tok._sp.decode(special.output_tokens)
    text = out.read_text()
    assert special.output_text in text
    assert "\n" + plain.output_text + "[Profile]" in text or text.endswith("\n" + plain.output_text)
