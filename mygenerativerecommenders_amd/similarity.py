"""Similarity modules — drop-in for reference ``models/similarity/dot_product.py``
(Hydra ``_target_: ...similarity.dot_product.DotProductSimilarity``).

Inside ``SampledSoftmaxLoss`` the dot products are computed by the fused loss kernel
(``gr_sampled_softmax_fwd``); ``DotProductSimilarity`` marks that choice and keeps the
reference's standalone contract (dot_product.py:31-64) for other callers, where the
products are plain library GEMMs.
"""
from __future__ import annotations

from typing import Optional

import torch


class NDPModule(torch.nn.Module):
    """ndp_module.py: similarity between query and item embeddings."""

    def forward(self, input_embeddings: torch.Tensor, item_embeddings: torch.Tensor,
                item_sideinfo: Optional[torch.Tensor], item_ids: torch.Tensor,
                precomputed_logits: Optional[torch.Tensor] = None):
        raise NotImplementedError


class DotProductSimilarity(NDPModule):
    def debug_str(self) -> str:
        return "dp"

    def forward(self, input_embeddings: torch.Tensor, item_embeddings: torch.Tensor,
                item_sideinfo: Optional[torch.Tensor], item_ids: torch.Tensor,
                precomputed_logits: Optional[torch.Tensor] = None):
        """input (B, D) or (B*r, D); items (1, X, D) or (B, X, D) -> (B, X) (dot_product.py:44-64,
        including its return conventions: a (logits, {}) tuple for a shared item set)."""
        del item_ids
        if item_embeddings.size(0) == 1:
            return torch.mm(input_embeddings, item_embeddings.squeeze(0).t()), {}
        elif input_embeddings.size(0) != item_embeddings.size(0):
            B, X, D = item_embeddings.size()
            return torch.bmm(input_embeddings.view(B, -1, D),
                             item_embeddings.permute(0, 2, 1)).view(-1, X)
        else:
            return torch.bmm(item_embeddings, input_embeddings.unsqueeze(2)).squeeze(2)
