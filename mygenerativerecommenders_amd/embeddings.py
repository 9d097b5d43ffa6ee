"""Item-embedding modules — drop-in for reference ``models/embeddings/embeddings.py``
(Hydra ``_target_: ...embeddings.embeddings.LocalEmbeddingModule``), SURVEY §8 N2.

``LocalEmbeddingModule`` keeps the reference's layout (embeddings.py:40-101): two
``nn.Embedding(num_items + 1, item_embedding_dim // 2, padding_idx=0)`` tables, item and
year, concatenated, the year row of an item coming from an item -> year lookup table.
The reference fills that table at import time from a CSV at a fixed path on its
author's machine and falls back to an empty mapping (every item -> year row 0) when
the file is absent; here the mapping is a constructor argument (``item2year`` or
``movies_csv``) with the same empty default.  ``get_item_embeddings`` runs one fused
gather kernel (``gr_item_embedding_fwd``) instead of clamp + index + two embedding
lookups + cat, and one backward kernel (``gr_item_embedding_bwd``: padding rows get no
gradient, as with ``padding_idx=0``).
"""
from __future__ import annotations

import abc
import csv
from typing import Mapping, Optional

import torch

from . import _lib
from .preprocessors import _truncated_normal_


def _stream():
    return _lib.stream_handle()


class _ItemEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w0, w1, map1):
        n = ids.numel()
        d0 = w0.shape[1]
        d1 = w1.shape[1] if w1 is not None else 0
        out = torch.empty(n, d0 + d1, dtype=w0.dtype, device=w0.device)
        _lib.call("gr_item_embedding_fwd", ids.data_ptr(), n, w0.data_ptr(), w0.shape[0], d0,
                  _lib.ptr(w1), w1.shape[0] if w1 is not None else 0, d1, _lib.ptr(map1),
                  map1.numel() if map1 is not None else 0, out.data_ptr(), _stream())
        ctx.save_for_backward(ids, map1 if map1 is not None else torch.empty(0))
        ctx.meta = (w0.shape, None if w1 is None else w1.shape, map1 is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        ids, map1 = ctx.saved_tensors
        s0, s1, has_map = ctx.meta
        g = g.contiguous()
        need0 = ctx.needs_input_grad[1]
        need1 = s1 is not None and ctx.needs_input_grad[2]
        if not (need0 or need1):
            return None, None, None, None
        dw0 = torch.empty(s0, dtype=g.dtype, device=g.device) if need0 else None
        dw1 = torch.empty(s1, dtype=g.dtype, device=g.device) if need1 else None
        _lib.call("gr_item_embedding_bwd", ids.data_ptr(), ids.numel(), g.data_ptr(), s0[0],
                  s0[1], s1[0] if s1 is not None else 0, s1[1] if s1 is not None else 0,
                  map1.data_ptr() if has_map else None, map1.numel() if has_map else 0, 0,
                  _lib.ptr(dw0), _lib.ptr(dw1), _stream())
        return None, dw0, dw1, None


def item_embedding(ids: torch.Tensor, w0: torch.Tensor, w1: Optional[torch.Tensor] = None,
                   map1: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cat(w0[ids], w1[map1[clamp(ids)]]) with shape ids.shape + (d0 + d1,); padding row
    0 of either table receives no gradient."""
    _lib.require_gpu(ids, w0, w1, map1)
    for w in (w0, w1):
        if w is not None and (w.dtype != torch.float32 or w.dim() != 2):
            raise TypeError("item_embedding: tables must be 2-D float32")
    flat = ids.reshape(-1).to(torch.int64).contiguous()
    m = map1.to(torch.int64).contiguous() if map1 is not None else None
    out = _ItemEmbed.apply(flat, w0.contiguous(), None if w1 is None else w1.contiguous(), m)
    return out.view(*ids.shape, out.shape[-1])


class EmbeddingModule(torch.nn.Module):
    """embeddings.py:21-37."""

    @abc.abstractmethod
    def debug_str(self) -> str:
        pass

    @abc.abstractmethod
    def get_item_embeddings(self, item_ids: torch.Tensor) -> torch.Tensor:
        pass

    @property
    @abc.abstractmethod
    def item_embedding_dim(self) -> int:
        pass


def read_item2year(movies_csv: str) -> dict:
    """{movie_id: year} from a movies CSV with ``movie_id`` and ``year`` columns (the file
    the reference reads at import, embeddings.py:12-18)."""
    with open(movies_csv, newline="") as f:
        return {int(r["movie_id"]): int(r["year"]) for r in csv.DictReader(f)}


class LocalEmbeddingModule(EmbeddingModule):
    """embeddings.py:40-101: item and year half-width tables, concatenated."""

    def __init__(self, num_items: int, item_embedding_dim: int,
                 item2year: Optional[Mapping[int, int]] = None,
                 movies_csv: Optional[str] = None) -> None:
        super().__init__()
        if item2year is None and movies_csv is not None:
            item2year = read_item2year(movies_csv)
        item2year = dict(item2year or {})
        self._item_embedding_dim: int = item_embedding_dim
        half_dim = item_embedding_dim // 2
        self._item_emb = torch.nn.Embedding(num_items + 1, half_dim, padding_idx=0)
        self._year_emb = torch.nn.Embedding(num_items + 1, half_dim, padding_idx=0)
        max_item_id = max(item2year.keys()) if item2year else num_items
        table = torch.zeros(max_item_id + 1, dtype=torch.long)
        for item_id, year in item2year.items():
            table[item_id] = year
        self.register_buffer("year_lookup_table", table)
        self.reset_params()

    def debug_str(self) -> str:
        return f"local_emb_d{self._item_embedding_dim}"

    def reset_params(self):
        # embeddings.py:80-88: both tables (padding rows included) ~ truncated normal 0.02
        for name, params in self.named_parameters():
            if "_item_emb" in name or "_year_emb" in name:
                _truncated_normal_(params.data, mean=0.0, std=0.02)

    def lookup_year_ids(self, item_ids: torch.Tensor) -> torch.Tensor:
        """embeddings.py:90-92."""
        valid = torch.clamp(item_ids, 0, self.year_lookup_table.size(0) - 1)
        return self.year_lookup_table[valid]

    def get_item_embeddings(self, item_ids: torch.Tensor) -> torch.Tensor:
        return item_embedding(item_ids, self._item_emb.weight, self._year_emb.weight,
                              self.year_lookup_table)

    def grad_row_support(self) -> dict:
        """{year table: rows} -- the only rows of ``_year_emb`` that can receive a
        gradient: every lookup goes through ``year_lookup_table`` (ids clamped into it),
        so its distinct values, minus padding row 0 and rows past the table.  With the
        reference's empty default map that set is empty.  Feeds the data-parallel
        reducer's ``row_support`` (distributed.BucketedGradReducer): at ml-20m width the
        year table is 131,263 x 128 floats (67 MB) of which only these rows travel."""
        rows = self.year_lookup_table.unique()
        n = self._year_emb.weight.shape[0]
        rows = rows[(rows > 0) & (rows < n)]
        return {self._year_emb.weight: rows}

    @property
    def item_embedding_dim(self) -> int:
        return self._item_embedding_dim


class CategoricalEmbeddingModule(EmbeddingModule):
    """embeddings.py:104-139: items share their category's row."""

    def __init__(self, num_items: int, item_embedding_dim: int,
                 item_id_to_category_id: torch.Tensor) -> None:
        super().__init__()
        self._item_embedding_dim: int = item_embedding_dim
        self._item_emb = torch.nn.Embedding(num_items + 1, item_embedding_dim, padding_idx=0)
        self.register_buffer("_item_id_to_category_id", item_id_to_category_id)
        self.reset_params()

    def debug_str(self) -> str:
        return f"cat_emb_d{self._item_embedding_dim}"

    def reset_params(self):
        for name, params in self.named_parameters():
            if "_item_emb" in name:
                _truncated_normal_(params.data, mean=0.0, std=0.02)

    def get_item_embeddings(self, item_ids: torch.Tensor) -> torch.Tensor:
        ids = self._item_id_to_category_id[(item_ids - 1).clamp(min=0)] + 1
        return item_embedding(ids, self._item_emb.weight)

    @property
    def item_embedding_dim(self) -> int:
        return self._item_embedding_dim
