"""CPU oracle for the item-embedding gather — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  numpy restatement of
``LocalEmbeddingModule.get_item_embeddings`` (embeddings/embeddings.py:90-97: clamp the id
into the year lookup table, gather the item row and the year row, concatenate) and of
the two ``nn.Embedding(padding_idx=0)`` backwards, pinned against
``tests/golden/embeddings.npz`` recorded from the reference by ``oracle/gen_golden.py``.
"""
from __future__ import annotations

import numpy as np


def year_ids(ids: np.ndarray, year_table: np.ndarray) -> np.ndarray:
    """embeddings.py:90-92: year_table[clamp(id, 0, len - 1)]."""
    return year_table[np.clip(ids, 0, year_table.shape[0] - 1)]


def get_item_embeddings(ids: np.ndarray, item_w: np.ndarray, year_w: np.ndarray,
                        year_table: np.ndarray) -> np.ndarray:
    return np.concatenate([item_w[ids], year_w[year_ids(ids, year_table)]], axis=-1)


def get_item_embeddings_bwd(ids: np.ndarray, dout: np.ndarray, item_w_rows: int,
                            year_w_rows: int, year_table: np.ndarray):
    """(d_item_w, d_year_w): scatter-add of dout's halves, row 0 (padding_idx) zero."""
    d0 = dout.shape[-1] // 2
    g = dout.reshape(-1, dout.shape[-1]).astype(np.float64)
    flat = ids.reshape(-1)
    yid = year_ids(flat, year_table)
    dw0 = np.zeros((item_w_rows, d0))
    dw1 = np.zeros((year_w_rows, dout.shape[-1] - d0))
    np.add.at(dw0, flat, g[:, :d0])
    np.add.at(dw1, yid, g[:, d0:])
    dw0[0] = 0.0
    dw1[0] = 0.0
    return dw0, dw1
