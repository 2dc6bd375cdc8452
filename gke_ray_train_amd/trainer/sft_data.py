"""SFT data: synthetic text-to-SQL corpus, chat formatting, tokenisation, padding collator and the
length-grouped sampler.

Reference: gretelai/synthetic_text_to_sql rows formatted with the Llama-3 chat template
(system / "### Database Schema / ### User Question / ### SQL Query" / assistant), shuffled with
seed 42 and cut to 1000 train / 200 eval samples (ray-jobs/fine_tune_llama_ray.py:256-293). With no
network, rows are generated with the same columns (id, sql_context, sql_prompt, sql,
sql_complexity, domain) and realistic CREATE TABLE / SELECT shapes; ``sql_complexity`` includes
"window functions" so the inference comparison's filter (:87-102) finds samples.
"""
from __future__ import annotations

import math
import random
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import Sampler

SYSTEM_PROMPT = ("You are a precise SQL query generation assistant. Given a database schema and a user question, "
                 "you MUST generate only the SQL query that directly answers the question. Do not include any other "
                 "explanatory text, markdown formatting, or any conversational preamble.")

_DOMAINS = ["retail", "healthcare", "finance", "education", "logistics", "energy", "media", "agriculture", "sports",
            "government"]
_COMPLEX = ["basic SQL", "aggregation", "single join", "subqueries", "window functions", "multiple_joins", "set operations",
            "CTEs"]
_COLS = ["id", "name", "city", "amount", "price", "quantity", "created_at", "status", "region", "score", "category",
         "revenue", "age", "department", "salary", "country", "rating", "duration"]


def _table(rng, dom):
    t = f"{dom}_{rng.choice(['orders', 'items', 'events', 'users', 'records', 'accounts', 'sales'])}"
    cols = rng.sample(_COLS, rng.randint(3, 7))
    if "id" not in cols:
        cols.insert(0, "id")
    types = {c: ("INT" if c in ("id", "quantity", "age") else "DECIMAL(10,2)" if c in ("amount", "price", "revenue", "salary", "score", "rating")
                 else "DATE" if c == "created_at" else "VARCHAR(50)") for c in cols}
    ddl = f"CREATE TABLE {t} ({', '.join(f'{c} {types[c]}' for c in cols)});"
    rows = ", ".join("(" + ", ".join(str(rng.randint(1, 999)) if types[c] != "VARCHAR(50)" and types[c] != "DATE"
                                     else f"'{c}_{rng.randint(1, 9)}'" if types[c] == "VARCHAR(50)" else "'2023-0%d-1%d'" % (rng.randint(1, 9), rng.randint(0, 9))
                                     for c in cols) + ")" for _ in range(rng.randint(1, 3)))
    return t, cols, types, ddl + f" INSERT INTO {t} VALUES {rows};"


def synthetic_text_to_sql(n: int, seed: int = 0, split: str = "train") -> List[Dict[str, str]]:
    rng = random.Random(seed * 7919 + (0 if split == "train" else 1))
    out = []
    for i in range(n):
        dom = rng.choice(_DOMAINS)
        cx = rng.choice(_COMPLEX)
        t, cols, types, ctx = _table(rng, dom)
        num = [c for c in cols if types[c].startswith(("INT", "DECIMAL")) and c != "id"] or ["id"]
        cat = [c for c in cols if types[c] == "VARCHAR(50)"] or ["id"]
        a, g = rng.choice(num), rng.choice(cat)
        if cx == "aggregation":
            q, s = f"What is the total {a} for each {g}?", f"SELECT {g}, SUM({a}) FROM {t} GROUP BY {g};"
        elif cx == "window functions":
            q = f"Rank each row by {a} within its {g}."
            s = f"SELECT {g}, {a}, RANK() OVER (PARTITION BY {g} ORDER BY {a} DESC) AS rnk FROM {t};"
        elif cx == "subqueries":
            q = f"List the rows whose {a} is above the average {a}."
            s = f"SELECT * FROM {t} WHERE {a} > (SELECT AVG({a}) FROM {t});"
        elif cx == "CTEs":
            q = f"Using a CTE, find the maximum {a} per {g}."
            s = f"WITH m AS (SELECT {g}, MAX({a}) AS mx FROM {t} GROUP BY {g}) SELECT * FROM m;"
        else:
            q, s = f"How many rows in {t} have {a} greater than {rng.randint(1, 500)}?", \
                f"SELECT COUNT(*) FROM {t} WHERE {a} > {rng.randint(1, 500)};"
        out.append({"id": i, "domain": dom, "sql_complexity": cx, "sql_prompt": q, "sql_context": ctx, "sql": s,
                    "sql_explanation": f"Computes {q[0].lower() + q[1:]}"})
    return out


def format_chat_sample(sample: Dict[str, str], tokenizer, with_answer: bool = True) -> Dict[str, str]:
    user = (f"### Database Schema:\n{sample.get('sql_context', '')}\n\n### User Question:\n{sample.get('sql_prompt', '')}"
            f"\n\n### SQL Query:")
    msgs = [{"role": "system", "content": SYSTEM_PROMPT}, {"role": "user", "content": user}]
    if with_answer:
        msgs.append({"role": "assistant", "content": sample.get("sql", "")})
    return {"text": tokenizer.apply_chat_template(msgs, tokenize=False, add_generation_prompt=not with_answer)}


def tokenize_texts(texts: List[str], tokenizer, max_len: int) -> List[List[int]]:
    return [tokenizer.encode(t)[:max_len] for t in texts]


def pack_sequences(seqs: List[List[int]], max_len: int, eos_id: int) -> List[List[int]]:
    """TRL ``packing=True``: concatenate with EOS separators and cut into max_len chunks."""
    flat: List[int] = []
    for s in seqs:
        flat.extend(s + [eos_id])
    return [flat[i:i + max_len] for i in range(0, len(flat) - max_len + 1, max_len)] or [flat[:max_len]]


class PadCollator:
    """Right-padding collator: labels = ids with padded positions -100 (native ``grt_pad_collate``)."""

    def __init__(self, pad_id: int, pad_to_multiple_of: int = 8, max_len: Optional[int] = None):
        self.pad_id = pad_id
        self.mult = pad_to_multiple_of
        self.max_len = max_len

    def __call__(self, seqs: List[List[int]]):
        L = max(len(s) for s in seqs)
        if self.mult:
            L = int(math.ceil(L / self.mult) * self.mult)
        if self.max_len:
            L = min(L, max(self.max_len, 1))
        B = len(seqs)
        ids = np.empty((B, L), dtype=np.int64)
        labels = np.empty((B, L), dtype=np.int64)
        mask = np.empty((B, L), dtype=np.int64)
        try:
            import ctypes
            from .. import _native
            lib = _native.runtime_lib()
            flat = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int64) for s in seqs]))
            offs = np.zeros(B + 1, dtype=np.int64)
            offs[1:] = np.cumsum([len(s) for s in seqs])
            P = ctypes.c_void_p
            lib.grt_pad_collate(P(flat.ctypes.data), P(offs.ctypes.data), None, ctypes.c_int64(B), ctypes.c_int64(L),
                                ctypes.c_int64(self.pad_id), P(ids.ctypes.data), P(labels.ctypes.data),
                                P(mask.ctypes.data))
        except OSError:
            for b, s in enumerate(seqs):
                s = s[:L]
                ids[b] = self.pad_id
                ids[b, :len(s)] = s
                labels[b] = -100
                labels[b, :len(s)] = s
                mask[b] = 0
                mask[b, :len(s)] = 1
        return {"input_ids": torch.from_numpy(ids), "labels": torch.from_numpy(labels),
                "attention_mask": torch.from_numpy(mask)}


class LengthGroupedSampler(Sampler):
    """HF ``group_by_length``: random megabatches of 50 x batch, each sorted by length (longest
    first), sharded across ranks; ``set_epoch`` reshuffles."""

    def __init__(self, lengths: List[int], batch_size: int, world: int = 1, rank: int = 0, seed: int = 42,
                 mega_mult: int = 50):
        self.lengths = lengths
        self.bs = batch_size
        self.world, self.rank = world, rank
        self.seed = seed
        self.mega = mega_mult
        self.epoch = 0

    def set_epoch(self, e):
        self.epoch = e

    def _order(self):
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        perm = torch.randperm(len(self.lengths), generator=g).tolist()
        ms = self.mega * self.bs * self.world
        megas = [perm[i:i + ms] for i in range(0, len(perm), ms)]
        order = []
        for m in megas:
            order.extend(sorted(m, key=lambda i: -self.lengths[i]))
        return order

    def __iter__(self):
        order = self._order()
        n = len(order) // self.world * self.world
        return iter(order[self.rank:n:self.world])

    def __len__(self):
        return len(self.lengths) // self.world
