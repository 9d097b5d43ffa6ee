"""Output postprocessors — drop-in for reference ``models/postprocessors/postprocessors.py``
(Hydra ``_target_: ...postprocessors.postprocessors.L2NormEmbeddingPostprocessor``).

``L2NormEmbeddingPostprocessor`` (postprocessors.py:34-56) runs the
``gr_l2_normalize`` kernel forward and backward; ``LayerNormEmbeddingPostprocessor``
(postprocessors.py:59-80) is not on the path and keeps plain PyTorch.
"""
from __future__ import annotations

import abc

import torch
import torch.nn.functional as F

from . import ops


class OutputPostprocessorModule(torch.nn.Module):
    """postprocessors.py:21-31."""

    @abc.abstractmethod
    def debug_str(self) -> str:
        pass

    @abc.abstractmethod
    def forward(self, output_embeddings: torch.Tensor) -> torch.Tensor:
        pass


class L2NormEmbeddingPostprocessor(OutputPostprocessorModule):
    def __init__(self, embedding_dim: int, eps: float = 1e-6) -> None:
        super().__init__()
        self._embedding_dim: int = embedding_dim
        self._eps: float = eps

    def debug_str(self) -> str:
        return "l2"

    def forward(self, output_embeddings: torch.Tensor) -> torch.Tensor:
        return ops.l2_normalize(output_embeddings[..., : self._embedding_dim], self._eps)


class LayerNormEmbeddingPostprocessor(OutputPostprocessorModule):
    """Off the hot path (postprocessors.py:59-80): plain PyTorch."""

    def __init__(self, embedding_dim: int, eps: float = 1e-6) -> None:
        super().__init__()
        self._embedding_dim: int = embedding_dim
        self._eps: float = eps

    def debug_str(self) -> str:
        return "ln"

    def forward(self, output_embeddings: torch.Tensor) -> torch.Tensor:
        output_embeddings = output_embeddings[..., : self._embedding_dim]
        return F.layer_norm(output_embeddings, normalized_shape=(self._embedding_dim,),
                            eps=self._eps)
