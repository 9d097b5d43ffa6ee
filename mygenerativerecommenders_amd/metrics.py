"""Retrieval metrics — drop-in for reference ``models/metrics/retrieval.py``
(Hydra ``_target_: ...metrics.retrieval.RetrievalMetrics``), SURVEY §8 N3.

``RetrievalMetrics`` keeps the reference's update/compute contract (retrieval.py:6-68):
the rank of the target among the top-k ids (k + 1 when absent), NDCG@k = 1/log2(rank+1)
and HR@k = [rank <= k] for every k of ``at_k_list``, and MRR = mean 1/rank.  Everything
stays on the tensors' device; under ``torch.distributed`` ``compute`` all-gathers the
per-rank (top-k, target) rows first (the torchmetrics ``dist_reduce_fx="cat"`` of the
reference), so every rank returns the global metrics.  No torchmetrics dependency.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.distributed as dist


def target_ranks(top_k_ids: torch.Tensor, target_ids: torch.Tensor) -> torch.Tensor:
    """1-based position of target_ids[b] in top_k_ids[b], or k + 1 if absent
    (retrieval.py:46-53: first match of cat([top_k, target]) == target)."""
    hits = torch.cat([top_k_ids, target_ids.view(-1, 1)], dim=1) == target_ids.view(-1, 1)
    return hits.to(torch.int8).argmax(dim=1) + 1


def _gather_rows(x: torch.Tensor) -> torch.Tensor:
    """Concatenates the (rows, ...) tensors of all ranks in rank order (uneven rows ok)."""
    world = dist.get_world_size()
    n = torch.tensor([x.shape[0]], device=x.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    top = max(sizes)
    pad = torch.zeros((top,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0)


class RetrievalMetrics(torch.nn.Module):
    """retrieval.py:6-68."""

    def __init__(self, k: int, at_k_list: List[int], **kwargs) -> None:
        super().__init__()
        self.k = k
        self.at_k_list = at_k_list
        self.top_k_ids: List[torch.Tensor] = []
        self.target_ids: List[torch.Tensor] = []

    def reset(self) -> None:
        self.top_k_ids = []
        self.target_ids = []

    def update(self, top_k_ids: torch.Tensor, target_ids: torch.Tensor, **kwargs) -> None:
        self.top_k_ids.append(top_k_ids)
        self.target_ids.append(target_ids.view(-1, 1))

    def forward(self, top_k_ids: torch.Tensor, target_ids: torch.Tensor, **kwargs) -> None:
        self.update(top_k_ids, target_ids)

    def compute(self) -> Dict[str, torch.Tensor]:
        top_k = torch.cat(self.top_k_ids, dim=0)
        target = torch.cat(self.target_ids, dim=0)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            top_k = _gather_rows(top_k)
            target = _gather_rows(target)
        assert top_k.size(1) == self.k
        ranks = target_ranks(top_k, target)
        out: Dict[str, torch.Tensor] = {}
        rf = ranks.to(torch.float32)
        for at_k in self.at_k_list:
            out[f"ndcg@{at_k}"] = torch.where(ranks <= at_k, 1.0 / torch.log2(rf + 1),
                                              torch.zeros((), device=rf.device)).mean()
        for at_k in self.at_k_list:
            out[f"hr@{at_k}"] = (ranks <= at_k).to(torch.float32).mean()
        out["mrr"] = (1.0 / rf).mean()
        return out
