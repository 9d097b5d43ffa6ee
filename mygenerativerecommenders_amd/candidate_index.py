"""CandidateIndex — drop-in for reference ``models/indexing/candidate_index.py``
(Hydra ``_target_: ...indexing.candidate_index.CandidateIndex``).

``get_top_k_outputs`` (candidate_index.py:107-164) runs as ONE fused device pass
(``mips_topk``): invalid ids are excluded during selection instead of taking the top
(k + N0) and filtering with a (B, k', N0) compare, a cumsum and a host-syncing
``nonzero``.  Both give the same ids and scores; ours have a
canonical tie order and need no host sync.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .top_k import MIPSBruteForceTopK, TopKModule


class CandidateIndex(torch.nn.Module):
    def __init__(self, k: int, ids: torch.Tensor, top_k_module: TopKModule,
                 embeddings: torch.Tensor = None, invalid_ids: Optional[torch.Tensor] = None,
                 debug_path: Optional[str] = None) -> None:
        super().__init__()
        self.register_buffer("_ids", torch.as_tensor(ids).unsqueeze(0))
        self._k = min(k, self._ids.shape[1])
        if not isinstance(top_k_module, MIPSBruteForceTopK):
            raise TypeError("CandidateIndex runs the fused MIPS kernel: top_k_module must be "
                            "mygenerativerecommenders_amd.top_k.MIPSBruteForceTopK")
        self._top_k_module = top_k_module
        self._invalid_ids = invalid_ids
        self._debug_path = debug_path
        self.update_embeddings(embeddings)

    def update_embeddings(self, embeddings: torch.Tensor) -> None:
        """embeddings (1, X, D); kept as the reference's (D, X) transposed view
        (candidate_index.py:27-31) and packed for the kernel on first use."""
        if embeddings is not None:
            self._embeddings_t = embeddings.permute(2, 1, 0).squeeze(2)
        else:
            self._embeddings_t = None
        # the table may be an inference tensor rewritten in place (no version counter)
        self._top_k_module.invalidate()

    @property
    def ids(self) -> torch.Tensor:
        return self._ids

    @property
    def num_objects(self) -> int:
        return self._ids.size(1)

    @property
    def embeddings(self) -> Optional[torch.Tensor]:
        """(1, X, D) view (candidate_index.py:45-51); None before update_embeddings(),
        which is what Retrieval.retrieve tests for (retrieval.py:34)."""
        if self._embeddings_t is None:
            return None
        return self._embeddings_t.unsqueeze(2).permute(2, 1, 0).squeeze(2)

    def filter_invalid_ids(self, invalid_ids: torch.Tensor) -> "CandidateIndex":
        """candidate_index.py:53-105 (unused and broken in the reference for a (1, X)
        index).  Invalid-id filtering is fused into get_top_k_outputs instead."""
        raise NotImplementedError("pass invalid_ids= to get_top_k_outputs (fused exclusion)")

    def get_top_k_outputs(self, query_embeddings: torch.Tensor, k: int = None,
                          invalid_ids: Optional[torch.Tensor] = None
                          ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Returns (top_k_ids (B, k) int64, top_k_scores (B, k) fp32), best first.
        Items whose id appears in the row of ``invalid_ids`` (B, N0) are excluded."""
        if k is None:
            k = self._k
        if invalid_ids is None:
            invalid_ids = self._invalid_ids
        if self._embeddings_t is None:
            raise RuntimeError("CandidateIndex: call update_embeddings() first")
        scores, ids = self._top_k_module(
            query_embeddings=query_embeddings, item_embeddings_t=self._embeddings_t,
            item_ids=self._ids, k=k, sorted=True, invalid_ids=invalid_ids)
        return ids, scores

    def apply_object_filter(self) -> "CandidateIndex":
        raise NotImplementedError("not implemented.")
