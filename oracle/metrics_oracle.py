"""CPU oracle for the retrieval metrics — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, as the checker.  Pure-Python/numpy restatement of
``RetrievalMetrics.compute`` (metrics/retrieval.py:40-68): the rank of the target in the
top-k list (first match; k + 1 when absent), NDCG@k = 1/log2(rank + 1) for rank <= k,
HR@k = [rank <= k], MRR = mean 1/rank.  The reference module needs torchmetrics, which
this image lacks, so no recorded outputs pin it: parity unpinned beyond this restatement
of the reference formula.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np


def retrieval_metrics(top_k: np.ndarray, target: np.ndarray, at_k_list: List[int]) -> Dict[str, float]:
    B, k = top_k.shape
    ranks = np.empty(B, dtype=np.int64)
    for b in range(B):
        hit = np.nonzero(top_k[b] == target[b])[0]
        ranks[b] = hit[0] + 1 if len(hit) else k + 1
    out = {}
    for a in at_k_list:
        out[f"ndcg@{a}"] = float(np.mean(np.where(ranks <= a, 1.0 / np.log2(ranks + 1.0), 0.0)))
    for a in at_k_list:
        out[f"hr@{a}"] = float(np.mean(ranks <= a))
    out["mrr"] = float(np.mean(1.0 / ranks))
    return out
