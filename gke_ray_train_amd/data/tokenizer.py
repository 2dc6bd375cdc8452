"""Tokenizers: the reference's character tokenizer and an offline byte-level tokenizer with
Llama-3-style chat special tokens (no HF Hub access on this machine).

``CharTokenizer`` reproduces reference ray-jobs/pytorch_llm_ray.py:20-55 exactly (sorted unique
characters, JSON vocab with ``char_to_idx`` / ``idx_to_char`` / ``vocab_size``). One documented
fix: ``encode(..., unk=-1)`` keeps the reference's -1 for unknown characters by default (which
would crash an embedding lookup); pass ``unk=<id>`` to map them to a valid id instead.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, List, Optional

import numpy as np


class CharTokenizer:
    def __init__(self, vocab_file_path: Optional[str] = None):
        self.char_to_idx: Dict[str, int] = {}
        self.idx_to_char: Dict[int, str] = {}
        self.vocab_size = 0
        if vocab_file_path and os.path.exists(vocab_file_path):
            self.load_vocab(vocab_file_path)

    def fit_on_text(self, text: str):
        chars = sorted(set(text))
        self.char_to_idx = {c: i for i, c in enumerate(chars)}
        self.idx_to_char = {i: c for i, c in enumerate(chars)}
        self.vocab_size = len(chars)

    def encode(self, text: str, unk: int = -1) -> List[int]:
        return [self.char_to_idx.get(c, unk) for c in text]

    def encode_np(self, text: str, unk: int = -1) -> np.ndarray:
        """Vectorised encode for large corpora (same result as ``encode``)."""
        if not text:
            return np.zeros(0, dtype=np.int64)
        codes = np.frombuffer(text.encode("utf-32-le"), dtype=np.uint32)
        keys = np.array([ord(c) for c in self.char_to_idx], dtype=np.uint32)
        vals = np.array(list(self.char_to_idx.values()), dtype=np.int64)
        order = np.argsort(keys)
        keys, vals = keys[order], vals[order]
        pos = np.clip(np.searchsorted(keys, codes), 0, len(keys) - 1)
        out = np.where(keys[pos] == codes, vals[pos], unk)
        return out.astype(np.int64)

    def decode(self, ids: Iterable[int]) -> str:
        return "".join(self.idx_to_char.get(int(i), "") for i in ids)

    def save_vocab(self, file_path: str):
        os.makedirs(os.path.dirname(file_path) or ".", exist_ok=True)
        with open(file_path, "w", encoding="utf-8") as f:
            json.dump({"char_to_idx": self.char_to_idx, "idx_to_char": self.idx_to_char,
                       "vocab_size": self.vocab_size}, f, ensure_ascii=False, indent=2)

    def load_vocab(self, file_path: str):
        with open(file_path, "r", encoding="utf-8") as f:
            d = json.load(f)
        self.char_to_idx = d["char_to_idx"]
        self.idx_to_char = {int(k): v for k, v in d["idx_to_char"].items()}
        self.vocab_size = d["vocab_size"]


class ByteTokenizer:
    """Byte-level tokenizer embedded in a model vocabulary of ``vocab_size`` ids.

    ids 0..255 = bytes, then the special tokens; remaining ids are unused (so it can drive a
    Llama-2 (32000) or Llama-3 (128256) embedding without a real BPE vocabulary). Provides the
    HF-tokenizer surface the SFT path needs: ``__call__``, ``encode``/``decode``,
    ``apply_chat_template`` (Llama-3 header format), ``pad_token``/``eos_token``, ``padding_side``,
    ``save_pretrained``.
    """

    SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>",
                "<|pad|>"]

    def __init__(self, vocab_size: int = 32000):
        assert vocab_size >= 256 + len(self.SPECIALS)
        self.vocab_size = vocab_size
        self.special_ids = {t: 256 + i for i, t in enumerate(self.SPECIALS)}
        self.bos_token, self.eos_token = "<|begin_of_text|>", "<|end_of_text|>"
        self.bos_token_id = self.special_ids[self.bos_token]
        self.eos_token_id = self.special_ids[self.eos_token]
        self.pad_token = None
        self.pad_token_id = None
        self.padding_side = "right"
        self.model_max_length = 1 << 30

    def __setattr__(self, k, v):
        object.__setattr__(self, k, v)
        if k == "pad_token" and v is not None and hasattr(self, "special_ids"):
            object.__setattr__(self, "pad_token_id", self.special_ids.get(v, self.eos_token_id))

    def convert_tokens_to_ids(self, tok):
        return self.special_ids[tok]

    def encode(self, text: str, add_special_tokens: bool = False) -> List[int]:
        out = [self.bos_token_id] if add_special_tokens else []
        i = 0
        while i < len(text):
            hit = None
            if text[i] == "<":
                for t, tid in self.special_ids.items():
                    if text.startswith(t, i):
                        hit = (t, tid)
                        break
            if hit:
                out.append(hit[1])
                i += len(hit[0])
            else:
                j = text.find("<", i + 1)
                j = len(text) if j < 0 else j
                out.extend(text[i:j].encode("utf-8"))
                i = j
        return out

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        inv = {v: k for k, v in self.special_ids.items()}
        buf, out = bytearray(), []
        for t in (int(x) for x in ids):
            if t < 256:
                buf.append(t)
            else:
                out.append(buf.decode("utf-8", "replace"))
                buf = bytearray()
                if not skip_special_tokens and t in inv:
                    out.append(inv[t])
        out.append(buf.decode("utf-8", "replace"))
        return "".join(out)

    def __call__(self, text, truncation=False, max_length=None, return_tensors=None, **_):
        ids = self.encode(text, add_special_tokens=False)
        if truncation and max_length:
            ids = ids[:max_length]
        if return_tensors == "pt":
            import torch
            t = torch.tensor([ids], dtype=torch.long)
            return {"input_ids": t, "attention_mask": torch.ones_like(t)}
        return {"input_ids": ids, "attention_mask": [1] * len(ids)}

    def apply_chat_template(self, messages, tokenize=False, add_generation_prompt=False):
        s = self.bos_token
        for m in messages:
            s += f"<|start_header_id|>{m['role']}<|end_header_id|>\n\n{m['content']}<|eot_id|>"
        if add_generation_prompt:
            s += "<|start_header_id|>assistant<|end_header_id|>\n\n"
        return self.encode(s) if tokenize else s

    def save_pretrained(self, path: str):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
            json.dump({"tokenizer_class": "GrtByteTokenizer", "vocab_size": self.vocab_size,
                       "special_tokens": self.special_ids, "pad_token": self.pad_token,
                       "padding_side": self.padding_side}, f, indent=2)

    @classmethod
    def from_pretrained(cls, path_or_name, **_):
        p = os.path.join(str(path_or_name), "tokenizer_config.json")
        if os.path.exists(p):
            with open(p) as f:
                d = json.load(f)
            t = cls(d["vocab_size"])
            if d.get("pad_token"):
                t.pad_token = d["pad_token"]
            t.padding_side = d.get("padding_side", "right")
            return t
        from ..models.llama import CONFIGS
        v = CONFIGS.get(str(path_or_name), {}).get("vocab_size", 32000)
        return cls(v)
