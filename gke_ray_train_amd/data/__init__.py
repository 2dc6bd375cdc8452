"""Data: tokenizers, synthetic Wikitext-2 / text-to-SQL corpora, token datasets + HBM streaming
loader, and the Ray-Data-like streaming dataset."""
from .datasets import TextDataset, TokenBatchLoader, gather_windows, synthetic_tokens
from .pipeline import DataIterator, Dataset, from_items, from_numpy, from_pandas, range_, read_text
from .tokenizer import ByteTokenizer, CharTokenizer
from . import wikitext

range = range_  # noqa: A001  (ray.data.range)

__all__ = ["TextDataset", "TokenBatchLoader", "gather_windows", "synthetic_tokens", "DataIterator", "Dataset",
           "from_items", "from_numpy", "from_pandas", "range", "read_text", "ByteTokenizer", "CharTokenizer",
           "wikitext"]
