"""Negatives sampling — drop-in for reference ``models/negatives_samples/negative_sampler.py``
(Hydra ``_target_: ...negatives_samples.negative_sampler.LocalNegativesSampler``).

``LocalNegativesSampler`` draws exactly the reference's offsets (the same
``torch.randint`` call, negative_sampler.py:110-117, so the same generator state gives the
same sampled ids) and exposes the two pieces the fused loss kernel needs instead of the
(M, R, D) gathered tensor: ``sample_offsets`` and ``item_table`` (the embedding of every
catalog row, one row per offset).  ``forward`` keeps the reference's materialising
contract for callers outside the fused path.  L2 normalisation runs the
``gr_l2_normalize`` kernel (negative_sampler.py:31-37).

``InBatchNegativesSampler`` (negative_sampler.py:135-211) caches the batch's present
ids and normalised embeddings (optionally de-duplicated, by the reference's own
``torch.unique`` call) and samples offsets into that cache with the reference's draw; the
fused loss takes the cache as its table.
"""
from __future__ import annotations

import abc
from typing import List, Optional, Tuple

import torch

from . import ops


class NegativesSampler(torch.nn.Module):
    """negative_sampler.py:21-63."""

    def __init__(self, l2_norm: bool, l2_norm_eps: float) -> None:
        super().__init__()
        self._l2_norm: bool = l2_norm
        self._l2_norm_eps: float = l2_norm_eps

    def normalize_embeddings(self, x: torch.Tensor) -> torch.Tensor:
        return self._maybe_l2_norm(x)

    def _maybe_l2_norm(self, x: torch.Tensor) -> torch.Tensor:
        # x / clamp(||x||_2, min=eps) over the last dim (negative_sampler.py:31-37)
        if self._l2_norm:
            x = ops.l2_normalize(x, self._l2_norm_eps)
        return x

    @abc.abstractmethod
    def debug_str(self) -> str:
        pass

    @abc.abstractmethod
    def process_batch(self, ids: torch.Tensor, presences: torch.Tensor,
                      embeddings: torch.Tensor) -> None:
        pass

    @abc.abstractmethod
    def forward(self, positive_ids: torch.Tensor,
                num_to_sample: int) -> Tuple[torch.Tensor, torch.Tensor]:
        pass


class LocalNegativesSampler(NegativesSampler):
    """negative_sampler.py:66-131: uniform negatives over the local catalog."""

    def __init__(self, l2_norm: bool, l2_norm_eps: float, num_items: Optional[int] = None,
                 all_item_ids: Optional[List[int]] = None) -> None:
        super().__init__(l2_norm=l2_norm, l2_norm_eps=l2_norm_eps)
        # argument validation as negative_sampler.py:75-84
        if all_item_ids is None and num_items is None:
            raise ValueError("Either num_items or all_item_ids must be provided")
        elif all_item_ids and num_items and num_items != len(all_item_ids):
            raise ValueError("num_items and all_item_ids must have the same length")
        elif all_item_ids:
            num_items = len(all_item_ids)
        elif num_items:
            all_item_ids = list(range(num_items))
        self._num_items: int = len(all_item_ids)
        self.register_buffer("_all_item_ids", torch.tensor(all_item_ids))
        # set by the training step (retrieval.py:110-116)
        self._item_emb: Optional[torch.nn.Embedding] = None
        self._embeddings_module = None

    def debug_str(self) -> str:
        return f"local{f'-l2-eps{self._l2_norm_eps}' if self._l2_norm else ''}"

    def process_batch(self, ids: torch.Tensor, presences: torch.Tensor,
                      embeddings: torch.Tensor) -> None:
        pass

    @property
    def all_item_ids(self) -> torch.Tensor:
        return self._all_item_ids

    def sample_offsets(self, positive_ids: torch.Tensor, num_to_sample: int) -> torch.Tensor:
        """(…, R) uniform offsets into the catalog — the reference's own draw
        (negative_sampler.py:110-117)."""
        output_shape = positive_ids.size() + (num_to_sample,)
        return torch.randint(low=0, high=self._num_items, size=output_shape,
                             dtype=positive_ids.dtype, device=positive_ids.device)

    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        if self._embeddings_module is not None:
            return self._embeddings_module.get_item_embeddings(ids)
        if self._item_emb is None:
            raise RuntimeError("LocalNegativesSampler: set _embeddings_module (or _item_emb) "
                               "before sampling (retrieval.py:110-116)")
        return self._item_emb(ids)

    def normalized_table(self) -> torch.Tensor:
        """(V, D) normalised embedding of every catalog row (the fused loss's table)."""
        return self.normalize_embeddings(self.item_table())

    def item_table(self) -> torch.Tensor:
        """(V, D) un-normalised embedding of every catalog row, row = sampling offset.
        ``get_item_embeddings`` is a per-id function, so ``item_table()[offsets]`` equals
        the reference's ``get_item_embeddings(all_item_ids[offsets])`` and autograd
        reaches the embedding parameters through this one (V, D) tensor."""
        return self._embed(self._all_item_ids)

    def forward(self, positive_ids: torch.Tensor,
                num_to_sample: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """(sampled_ids, normalised sampled embeddings), negative_sampler.py:105-131."""
        offsets = self.sample_offsets(positive_ids, num_to_sample)
        output_shape = offsets.shape
        sampled_ids = self._all_item_ids[offsets.view(-1)].reshape(output_shape)
        return sampled_ids, self.normalize_embeddings(self._embed(sampled_ids))


class InBatchNegativesSampler(NegativesSampler):
    """negative_sampler.py:135-211: negatives drawn from the batch's own items."""

    def __init__(self, l2_norm: bool, l2_norm_eps: float, dedup_embeddings: bool) -> None:
        super().__init__(l2_norm=l2_norm, l2_norm_eps=l2_norm_eps)
        self._dedup_embeddings: bool = dedup_embeddings
        self._cached_ids: Optional[torch.Tensor] = None
        self._cached_embeddings: Optional[torch.Tensor] = None

    def debug_str(self) -> str:
        s = f"in-batch{f'-l2-eps{self._l2_norm_eps}' if self._l2_norm else ''}"
        return s + ("-dedup" if self._dedup_embeddings else "")

    def process_batch(self, ids: torch.Tensor, presences: torch.Tensor,
                      embeddings: torch.Tensor) -> None:
        """ids / presences (N') or (B, N), embeddings (..., D): caches the present rows'
        ids and normalised embeddings (negative_sampler.py:153-188); with dedup, one row
        per distinct id, the one the reference's own scatter of positions
        (``offsets[inverse] = arange``) picks."""
        assert ids.size() == presences.size()
        assert ids.size() == embeddings.size()[:-1]
        if self._dedup_embeddings:
            valid_ids = ids[presences]
            unique_ids, inverse = torch.unique(input=valid_ids, sorted=False, return_inverse=True)
            offsets = torch.empty((unique_ids.numel(),), dtype=torch.int64, device=unique_ids.device)
            offsets[inverse] = torch.arange(valid_ids.numel(), dtype=torch.int64,
                                            device=unique_ids.device)
            self._cached_embeddings = self._maybe_l2_norm(embeddings[presences][offsets, :])
            self._cached_ids = unique_ids
        else:
            self._cached_embeddings = self._maybe_l2_norm(embeddings[presences])
            self._cached_ids = ids[presences]

    def get_all_ids_and_embeddings(self) -> Tuple[torch.Tensor, torch.Tensor]:
        return self._cached_ids, self._cached_embeddings

    @property
    def all_item_ids(self) -> torch.Tensor:
        return self._cached_ids

    def sample_offsets(self, positive_ids: torch.Tensor, num_to_sample: int) -> torch.Tensor:
        """(..., R) uniform offsets into the cache -- the reference's own draw
        (negative_sampler.py:200-206)."""
        if self._cached_ids is None:
            raise RuntimeError("InBatchNegativesSampler: process_batch before sampling")
        return torch.randint(low=0, high=self._cached_ids.size(0),
                             size=positive_ids.size() + (num_to_sample,),
                             dtype=positive_ids.dtype, device=positive_ids.device)

    def normalized_table(self) -> torch.Tensor:
        """The cache, already normalised by process_batch (the reference returns it as is)."""
        return self._cached_embeddings

    def forward(self, positive_ids: torch.Tensor,
                num_to_sample: int) -> Tuple[torch.Tensor, torch.Tensor]:
        offsets = self.sample_offsets(positive_ids, num_to_sample)
        return self._cached_ids[offsets], self._cached_embeddings[offsets]
