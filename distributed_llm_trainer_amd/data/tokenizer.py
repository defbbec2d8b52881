"""Tokenizer resolution that works offline.

The reference calls ``GPT2TokenizerFast.from_pretrained("gpt2")``
(``tinystories.py:30``), which on an offline box silently yields an unusable
tokenizer.  Resolution order here:

1. ``DLT_TOKENIZER_DIR`` / a local directory path -> ``GPT2TokenizerFast.from_pretrained(dir)``;
2. the HF hub name (works when the files are already in the local HF cache);
3. ``"byte"`` -> a dependency-free byte-level tokenizer (vocab 256, ids 0..255;
   used by tests and for smoke runs on real text without network access).

A tokenizer whose vocabulary is empty is rejected instead of being used (offline, this
image's transformers returns a GPT-2 tokenizer with ``vocab_size == 0`` whose ``encode``
yields no ids).  When no usable GPT-2 tokenizer exists, ``get_tokenizer`` falls back to
the byte tokenizer with a loud warning (``DLT_TOKENIZER_STRICT=1``: raise instead), so
the real-data CLIs still run offline; the ids stay < 256, inside the model's vocabulary.
"""
from __future__ import annotations

import os
from typing import List


class ByteTokenizer:
    vocab_size = 256
    eos_token_id = 0

    def encode(self, text: str) -> List[int]:
        return list(text.encode("utf-8"))

    def decode(self, ids) -> str:
        return bytes(int(i) & 0xFF for i in ids).decode("utf-8", errors="replace")


def get_tokenizer(name: str = "gpt2"):
    if name == "byte":
        return ByteTokenizer()
    local = os.environ.get("DLT_TOKENIZER_DIR")
    candidates = [c for c in (local, name) if c]
    err = None
    for cand in candidates:
        try:
            from transformers import GPT2TokenizerFast
            tok = GPT2TokenizerFast.from_pretrained(cand, local_files_only=not cand.startswith("http"))
            if len(tok) == 0 or tok.vocab_size < 256 or not tok.encode("hello world"):
                raise RuntimeError(f"unusable vocabulary (vocab_size={tok.vocab_size})")
            tok.model_max_length = 10 ** 9
            return tok
        except Exception as e:  # noqa: BLE001
            err = e
    msg = (f"could not load tokenizer {name!r} offline ({err}). Point DLT_TOKENIZER_DIR at a directory with "
           "the GPT-2 tokenizer files, pre-tokenise to a .bin token file, or use tokenizer 'byte'.")
    if os.environ.get("DLT_TOKENIZER_STRICT") == "1":
        raise RuntimeError(msg)
    import warnings
    warnings.warn(msg + " Falling back to the byte-level tokenizer (ids 0..255).", RuntimeWarning, stacklevel=2)
    return ByteTokenizer()
