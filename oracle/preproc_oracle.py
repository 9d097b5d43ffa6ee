"""CPU oracle for the input preprocessor — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  numpy restatement of
``LearnablePositionalEmbeddingInputFeaturesPreprocessor.forward``
(preprocessors/learnable_positional_embedding.py:42-58) with dropout off, and its
gradients, pinned against ``tests/golden/preproc.npz`` recorded from the reference by
``oracle/gen_golden.py``.
"""
from __future__ import annotations

import numpy as np


def preprocess(x: np.ndarray, ids: np.ndarray, pos_w: np.ndarray, scale: float,
               mask: np.ndarray | None = None):
    """y = (x * scale + pos_w[:N]) * keep * (ids != 0); ``mask`` = dropout keep/(1-p)
    factors (None: dropout off).  Returns y and the valid mask (B, N, 1)."""
    B, N, D = x.shape
    v = x.astype(np.float64) * scale + pos_w[:N].astype(np.float64)[None]
    if mask is not None:
        v = v * mask
    valid = (ids != 0)[..., None].astype(np.float64)
    return v * valid, valid


def preprocess_bwd(dy: np.ndarray, ids: np.ndarray, scale: float, n_pos: int,
                   mask: np.ndarray | None = None):
    """(dx, dpos) of preprocess for upstream dy; dpos has n_pos rows (rows >= N are 0)."""
    B, N, D = dy.shape
    g = dy.astype(np.float64) * (ids != 0)[..., None]
    if mask is not None:
        g = g * mask
    dpos = np.zeros((n_pos, D))
    dpos[:N] = g.sum(0)
    return g * scale, dpos
