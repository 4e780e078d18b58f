"""LLaMA tokenizer loading for the serving front end.

Restates RequestManager::register_tokenizer for ModelType::LLAMA
(request_manager.cc:181-217): a directory resolves to `tokenizer.json` if it
exists, else `tokenizer.model`; a file path is used as given.  The reference
reads tokenizer.json with tokenizers-cpp (`Tokenizer::FromBlobJSON`, the HF
`tokenizers` library underneath) and tokenizer.model with SentencePiece
(`FromBlobSentencePiece`, flagging `old_llama_tokenizer`).  tokenizers-cpp is
an empty submodule in the reference tree; here the same two libraries are
used directly from Python (`tokenizers`, `sentencepiece`).

Text semantics kept from the reference:
- prompts are encoded WITHOUT special tokens; the request manager prepends BOS
  itself when add_special_tokens is set (request_manager.cc:358-373);
- on completion a trailing EOS is dropped before decoding (:772-775, in the
  C++ request manager here);
- SentencePiece drops BOS when decoding, so the reference prefixes "<s> " to
  the text when the old LLaMA tokenizer is in use, the request was registered
  with add_special_tokens and its tokens start with BOS (:776-781).  That rule
  belongs to the request manager (it knows add_special_tokens per request):
  RequestManager applies it, decode() here is the bare Decode.
Whether tokenizers-cpp's Encode/Decode skip special tokens is not visible in
the reference tree (empty submodule): the HF path here encodes without and
decodes with special tokens, and that choice is parity-unpinned.
"""
import os
from typing import List


class LlamaTokenizer:
    """encode(text) -> ids (no BOS), decode(ids) -> text, as the request
    manager's tokenizer_ is used."""

    def __init__(self, path: str, bos_token_id: int = 1):
        self.bos_token_id = bos_token_id
        if os.path.isdir(path):
            json_path = os.path.join(path, "tokenizer.json")
            model_path = os.path.join(path, "tokenizer.model")
        else:
            json_path = model_path = path
        if os.path.isfile(json_path) and json_path.endswith(".json"):
            import tokenizers
            self._hf = tokenizers.Tokenizer.from_file(json_path)
            self._sp = None
            self.old_llama_tokenizer = False
            self.path = json_path
        elif os.path.isfile(model_path):
            import sentencepiece
            self._sp = sentencepiece.SentencePieceProcessor(model_file=model_path)
            self._hf = None
            self.old_llama_tokenizer = True
            self.path = model_path
        else:
            # the reference prints "Failed to open file" and asserts
            raise FileNotFoundError(f"no tokenizer.json or tokenizer.model at {path}")

    def encode(self, text: str) -> List[int]:
        if self._sp is not None:
            return list(self._sp.encode(text))
        return list(self._hf.encode(text, add_special_tokens=False).ids)

    def decode(self, ids: List[int]) -> str:
        ids = list(ids)
        if self._sp is not None:
            return self._sp.decode(ids)
        return self._hf.decode(ids, skip_special_tokens=False)


def load_tokenizer(path: str, bos_token_id: int = 1) -> LlamaTokenizer:
    return LlamaTokenizer(path, bos_token_id)
