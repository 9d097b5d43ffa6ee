"""Autoregressive losses — drop-in for reference ``models/losses/autoregressive_losses.py``
(Hydra ``_target_: ...losses.autoregressive_losses.SampledSoftmaxLoss``), SURVEY §8 N1.

``SampledSoftmaxLoss.jagged_forward`` keeps the reference signature and semantics
(autoregressive_losses.py:259-306) and runs as:

  offsets = sampler.sample_offsets(ids, R)            same randint as the reference
  table   = normalize(sampler.item_table())           (V, D), gr_l2_normalize
  pos     = normalize(supervision_embeddings)         (M, D), gr_l2_normalize
  loss_t  = gr_sampled_softmax_fwd(out, pos, table[offsets], ...)   one fused kernel
  loss    = sum(loss_t * w) / sum(w)

so the (M, R, D) negatives tensor and the (M, R) logits are never materialised.  The
fused path covers ``LocalNegativesSampler`` (the ml-1m / ml-20m configs,
configs/model/hstu.yaml) and ``InBatchNegativesSampler`` (table = the batch cache of
negative_sampler.py:153-188, sampled by the reference's draw over it), each with
``DotProductSimilarity``; other similarities (MoL) raise.
"""
from __future__ import annotations

import abc

import torch

from . import ops
from .negatives_sampler import InBatchNegativesSampler, LocalNegativesSampler, NegativesSampler


class AutoregressiveLoss(torch.nn.Module):
    """autoregressive_losses.py:12-38."""

    @abc.abstractmethod
    def jagged_forward(self, output_embeddings: torch.Tensor, supervision_ids: torch.Tensor,
                       supervision_embeddings: torch.Tensor, supervision_weights: torch.Tensor,
                       negatives_sampler: NegativesSampler) -> torch.Tensor:
        pass


def _is_dot_product(similarity) -> bool:
    return type(similarity).__name__ == "DotProductSimilarity"


class SampledSoftmaxLoss(AutoregressiveLoss):
    """autoregressive_losses.py:249-306."""

    def __init__(self, num_to_sample: int, softmax_temperature: float) -> None:
        super().__init__()
        self._num_to_sample: int = num_to_sample
        self._softmax_temperature: float = softmax_temperature

    def jagged_forward(self, output_embeddings: torch.Tensor, supervision_ids: torch.Tensor,
                       supervision_embeddings: torch.Tensor, supervision_weights: torch.Tensor,
                       negatives_sampler: NegativesSampler, similarity) -> torch.Tensor:
        assert output_embeddings.size() == supervision_embeddings.size()
        assert supervision_ids.size() == supervision_embeddings.size()[:-1]
        assert supervision_ids.size() == supervision_weights.size()
        if not isinstance(negatives_sampler, (LocalNegativesSampler, InBatchNegativesSampler)):
            raise NotImplementedError("SampledSoftmaxLoss: the fused path takes a "
                                      "LocalNegativesSampler or an InBatchNegativesSampler")
        if not _is_dot_product(similarity):
            raise NotImplementedError("SampledSoftmaxLoss: the fused path takes "
                                      "DotProductSimilarity")
        offsets = negatives_sampler.sample_offsets(supervision_ids, self._num_to_sample)
        table = negatives_sampler.normalized_table()
        positive_embeddings = negatives_sampler.normalize_embeddings(supervision_embeddings)
        jagged_loss = ops.sampled_softmax_loss(
            output_embeddings, positive_embeddings, table, supervision_ids, offsets,
            negatives_sampler.all_item_ids, self._softmax_temperature)
        return (jagged_loss * supervision_weights).sum() / supervision_weights.sum()
