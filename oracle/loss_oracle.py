"""CPU oracle for the sampled-softmax loss — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker — never as the thing measured or shipped.

A float64 numpy restatement, forward and analytic backward, of
  * ``SampledSoftmaxLoss.jagged_forward``   autoregressive_losses.py:259-306
  * ``LocalNegativesSampler.forward``       negative_sampler.py:105-131 (given offsets)
  * ``NegativesSampler._maybe_l2_norm``     negative_sampler.py:31-37
  * ``DotProductSimilarity.forward``        dot_product.py:56-64 (bmm branches)
pinned against ``tests/golden/ssm_*.npz`` recorded from the reference itself by
``oracle/gen_golden.py`` (``tests/test_oracle_golden.py``).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

COLLISION_LOGIT = -5e4  # autoregressive_losses.py:296-300


def _l2(x: np.ndarray, eps: float):
    n = np.linalg.norm(x, axis=-1, keepdims=True)
    return x / np.maximum(n, eps), n


def _l2_bwd(x: np.ndarray, n: np.ndarray, dy: np.ndarray, eps: float) -> np.ndarray:
    """d/dx of x / max(||x||, eps): (dy - y (y.dy)) / ||x|| where ||x|| > eps, dy / eps
    otherwise (the clamp's gradient is 0 below eps)."""
    big = n > eps
    safe = np.where(big, n, 1.0)
    y = x / safe
    proj = np.sum(y * dy, axis=-1, keepdims=True)
    return np.where(big, (dy - y * proj) / safe, dy / eps)


def sampled_softmax(out: np.ndarray, sup_ids: np.ndarray, sup_emb: np.ndarray,
                    weights: np.ndarray, table: np.ndarray, table_ids: np.ndarray,
                    offsets: np.ndarray, temperature: float, l2_norm: bool = True,
                    eps: float = 1e-6, grads: bool = True) -> Dict[str, np.ndarray]:
    """Loss and gradients.  ``table`` (V, D) is the un-normalised embedding of catalog
    row v (= get_item_embeddings(all_item_ids[v])), ``table_ids[v]`` its id, ``offsets``
    (M, R) the sampled rows.  Returns loss (scalar), loss_t (M,), and when ``grads``:
    d_out (M, D), d_sup_emb (M, D), d_table (V, D) for d loss."""
    out = out.astype(np.float64)
    sup_emb = sup_emb.astype(np.float64)
    table = table.astype(np.float64)
    w = weights.astype(np.float64)
    M, D = out.shape
    R = offsets.shape[1]
    T = float(temperature)
    if l2_norm:
        pos, pos_n = _l2(sup_emb, eps)
        tab, tab_n = _l2(table, eps)
    else:
        pos, tab = sup_emb, table
    neg = tab[offsets]                                        # (M, R, D)
    pos_logit = np.sum(out * pos, axis=-1) / T                # (M,)
    neg_logit = np.einsum("mrd,md->mr", neg, out) / T         # (M, R)
    coll = table_ids[offsets] == sup_ids[:, None]
    neg_logit = np.where(coll, COLLISION_LOGIT, neg_logit)
    logits = np.concatenate([pos_logit[:, None], neg_logit], axis=1)
    mx = logits.max(axis=1, keepdims=True)
    lse = (mx + np.log(np.exp(logits - mx).sum(axis=1, keepdims=True)))[:, 0]
    loss_t = lse - pos_logit
    loss = float(np.sum(loss_t * w) / np.sum(w))
    res = {"loss": np.array(loss), "loss_t": loss_t, "lse": lse}
    if not grads:
        return res
    g = w / np.sum(w)                                         # d loss / d loss_t
    p = np.exp(logits - lse[:, None])
    dl = g[:, None] * p
    dl[:, 0] -= g
    dl_neg = np.where(coll, 0.0, dl[:, 1:])                   # where(): no grad if masked
    d_out = (dl[:, :1] * pos + np.einsum("mr,mrd->md", dl_neg, neg)) / T
    d_pos = dl[:, :1] * out / T
    d_tab = np.zeros_like(tab)
    np.add.at(d_tab, offsets.reshape(-1),
              (dl_neg[:, :, None] * out[:, None, :]).reshape(-1, D) / T)
    if l2_norm:
        d_sup = _l2_bwd(sup_emb, pos_n, d_pos, eps)
        d_table = _l2_bwd(table, tab_n, d_tab, eps)
    else:
        d_sup, d_table = d_pos, d_tab
    res.update(d_out=d_out, d_sup_emb=d_sup, d_table=d_table, d_pos=d_pos, d_tab_norm=d_tab)
    return res


def from_golden(z) -> Dict[str, np.ndarray]:
    """Runs the oracle on a ``tests/golden/ssm_*.npz`` record; d_weight maps the table
    gradient back onto embedding rows by id (the reference's Embedding.weight.grad)."""
    ids = z["all_ids"]
    table = z["weight"][ids]
    r = sampled_softmax(z["out"], z["sup_ids"], z["sup_emb"], z["weights"], table, ids,
                        z["offsets"], float(z["T"]), bool(z["l2_norm"]), float(z["eps"]))
    d_weight = np.zeros(z["weight"].shape, dtype=np.float64)
    d_weight[ids] = r["d_table"]
    r["d_weight"] = d_weight
    return r
