"""Synthetic Wikitext-2-raw corpus (no network on this machine).

The reference downloads ``wikitext-2-raw-v1`` with HF datasets and writes ``wiki.{train,valid,
test}.tokens`` as the paragraphs joined by "\\n" (reference ray-jobs/prepare_wikitext2_ray_job.py:
51-73). Here the same three files are produced from a deterministic generator with Wikitext's
shape: `` = Title = `` / `` = = Section = = `` headings, blank lines, long paragraphs of
Zipf-distributed words, `` @-@ `` / `` @,@ `` tokens, numbers and a few non-ASCII characters, at the
real split sizes (~10.9 M / 1.1 M / 1.3 M characters). Character vocabulary ~ 150-280 symbols, like
the real corpus, so BasicLLM's char vocab V is in the reference's range.
"""
from __future__ import annotations

import os

import numpy as np

SPLIT_CHARS = {"train": 10_900_000, "validation": 1_140_000, "test": 1_290_000}
FILES = {"train": "wiki.train.tokens", "validation": "wiki.valid.tokens", "test": "wiki.test.tokens"}

_SYL = ["an", "ar", "as", "at", "be", "ca", "ce", "co", "de", "di", "el", "en", "er", "es", "ha", "he", "in", "is",
        "it", "la", "le", "li", "lo", "ma", "me", "mi", "ne", "no", "on", "or", "ou", "ra", "re", "ri", "ro", "sa",
        "se", "si", "so", "st", "ta", "te", "th", "ti", "to", "tr", "un", "ur", "us", "ve", "wa", "we", "wi"]
_EXTRA = list("éèáóöüñçøåæíúàâêîôûßłšžčć–—’“”°£€½×") + ["ā", "ī", "ō", "ū", "ş", "ğ", "ı", "ž"]
_FUNC = ["the", "of", "and", "in", "to", "a", "was", "is", "for", "on", "as", "by", "with", "he", "that", "at",
         "from", "his", "it", "an", "were", "which", "are", "this", "also", "be", "had", "first", "one", "their"]


def _make_vocab(rng, n=30000):
    words = []
    for _ in range(n):
        k = rng.integers(1, 5)
        w = "".join(_SYL[i] for i in rng.integers(0, len(_SYL), size=k))
        if rng.random() < 0.02:
            w = w[: rng.integers(1, max(2, len(w)))] + _EXTRA[rng.integers(0, len(_EXTRA))] + w[1:]
        if rng.random() < 0.15:
            w = w.capitalize()
        words.append(w)
    return _FUNC + words


def generate_split(split: str, seed: int = 0, n_chars: int = None) -> str:
    n_chars = n_chars or SPLIT_CHARS[split]
    rng = np.random.default_rng(seed + {"train": 0, "validation": 1, "test": 2}[split])
    vocab = _make_vocab(np.random.default_rng(seed))
    ranks = np.arange(1, len(vocab) + 1)
    p = 1.0 / ranks ** 1.05
    p /= p.sum()
    out, total = [], 0
    while total < n_chars:
        title = " ".join(vocab[i].capitalize() for i in rng.choice(len(vocab), size=rng.integers(1, 4), p=p))
        lines = ["", f" = {title} = ", ""]
        for _ in range(rng.integers(2, 7)):
            if rng.random() < 0.4:
                sec = " ".join(vocab[i] for i in rng.choice(len(vocab), size=rng.integers(1, 3), p=p)).title()
                lines += [f" = = {sec} = = ", ""]
            ws = [vocab[i] for i in rng.choice(len(vocab), size=rng.integers(40, 220), p=p)]
            for j in range(len(ws)):
                r = rng.random()
                if r < 0.05:
                    ws[j] += " ,"
                elif r < 0.08:
                    ws[j] += " ."
                elif r < 0.09:
                    ws[j] = f"{rng.integers(1, 3000)}"
                elif r < 0.095:
                    ws[j] = f"{rng.integers(1, 99)} @,@ {rng.integers(100, 999)}"
                elif r < 0.10:
                    ws[j] += " @-@ " + vocab[rng.integers(0, 500)]
                elif r < 0.103:
                    ws[j] = f"( {ws[j]} )"
            lines += [" " + " ".join(ws) + " . ", ""]
        chunk = "\n".join(lines)
        out.append(chunk)
        total += len(chunk)
    return "".join(out)[:n_chars]


def prepare(dir_path: str, seed: int = 0, scale: float = 1.0, overwrite: bool = False) -> dict:
    """Idempotently write the three split files (skip when all exist and are non-empty)."""
    os.makedirs(dir_path, exist_ok=True)
    paths = {s: os.path.join(dir_path, f) for s, f in FILES.items()}
    if not overwrite and all(os.path.exists(p) and os.path.getsize(p) > 0 for p in paths.values()):
        return paths
    for s, p in paths.items():
        text = generate_split(s, seed=seed, n_chars=int(SPLIT_CHARS[s] * scale))
        tmp = p + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            f.write(text)
        os.replace(tmp, p)  # atomic: readers never see a partial file
    return paths
