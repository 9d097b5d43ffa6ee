"""CPU oracle for the HSTU encoder hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker (or the timed CPU baseline) — never
as the thing measured or shipped.  The product path lives in
``mygenerativerecommenders_amd`` and fails loudly without its HIP library.

This is a from-scratch fp32 restatement (PyTorch CPU tensors, autograd for the
backward) of the reference's algorithm, parity-pinned against the golden fixtures
under ``tests/golden/hstu_*.npz`` that ``oracle/gen_golden.py`` recorded from the
reference itself (``tests/test_oracle_golden.py``).

Two variants:
  * jagged (``hstu_forward``): per-sequence dense L_b x L_b blocks — the math the
    HIP kernels implement;
  * padded (``hstu_forward_padded``): the reference's batched (B, N, N) op order,
    used as the CPU throughput baseline (SURVEY.md §8d "padded-order restatement").

Reference map (paths relative to ``src/generative_recommenders_pl/models``):
  * relative bias ........ ``sequential_encoders/hstu.py:96-128`` (+ bucket fn 579-581)
  * attention ............ ``sequential_encoders/hstu.py:134-205`` (non-cache branch)
  * STU layer ............ ``sequential_encoders/hstu.py:266-423``
  * HSTUJagged ........... ``sequential_encoders/hstu.py:439-518``
  * HSTU.forward ......... ``sequential_encoders/hstu.py:633-672``
  * cached decoding ...... ``sequential_encoders/hstu.py:151-177, 293-298, 321-322,
                            393-423`` (``hstu_forward_cached``; pinned by
                            ``tests/golden/decode_*.npz``)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

NUM_BUCKETS = 128  # hstu.py:577


def bucket_reference_semantics(delta: torch.Tensor) -> torch.Tensor:
    """hstu.py:579-581 + the clamp at hstu.py:117-123: fp32 log of |dt| clamped to 1,
    divided by 0.301, truncated, clamped to [0, 128]."""
    return torch.clamp(
        (torch.log(torch.abs(delta).clamp(min=1)) / 0.301).long(), 0, NUM_BUCKETS)


def bucket_via_thresholds(delta: torch.Tensor, thresholds: np.ndarray) -> torch.Tensor:
    """The integer-threshold form the HIP kernels use: bucket = max{b : T[b] <= |dt|}."""
    thr = torch.as_tensor(thresholds, dtype=torch.int64)
    return torch.searchsorted(thr, delta.abs().contiguous(), right=True) - 1


@dataclass
class HSTUConfig:
    N: int  # padded max length = max_sequence_len + max_output_len (hstu.py:596-605)
    D: int
    H: int
    dqk: int
    dv: int
    concat_ua: bool = False
    eps: float = 1e-6  # hstu.py:224
    softmax: bool = False  # normalization="softmax_rel_bias" (hstu.py:341-389)


def layer_params_from_state(state: Dict[str, torch.Tensor], i: int,
                            prefix: str = "_hstu._attention_layers") -> Dict[str, torch.Tensor]:
    p = f"{prefix}.{i}."
    return {
        "uvqk": state[p + "_uvqk"],
        "o_w": state[p + "_o.weight"],
        "o_b": state[p + "_o.bias"],
        "ts_w": state.get(p + "_rel_attn_bias._ts_w"),  # None: no bias module
        "pos_w": state.get(p + "_rel_attn_bias._pos_w"),
    }


def rel_bias_jagged(ts_b: torch.Tensor, L: int, N: int, pos_w: torch.Tensor,
                    ts_w: torch.Tensor, thresholds: np.ndarray) -> torch.Tensor:
    """(L, L) slice of the (N, N) bias of hstu.py:96-128 for one sequence.

    pos[i, j] = pos_w[N - 1 + j - i] (the pad/repeat/reshape trick of :106-110,124);
    query i uses the timestamp of item i + 1, with ext_ts[N] = ts[N - 1] (:113-119).
    """
    i = torch.arange(L)
    j = torch.arange(L)
    pos = pos_w[(N - 1) + j.view(1, L) - i.view(L, 1)]
    ext = torch.cat([ts_b, ts_b[N - 1:N]])
    delta = ext[1:L + 1].view(L, 1) - ts_b[:L].view(1, L)
    bucket = bucket_via_thresholds(delta, thresholds)
    return pos + ts_w[bucket]


def hstu_attention_jagged(q, k, v, offsets, ts, cfg: HSTUConfig, pos_w, ts_w,
                          thresholds) -> torch.Tensor:
    """hstu.py:134-205 restated jagged: A = silu(QK^T + bias) / N, causal j <= i."""
    H, dqk, dv, N = cfg.H, cfg.dqk, cfg.dv, cfg.N
    outs = []
    B = offsets.numel() - 1
    for b in range(B):
        s, e = int(offsets[b]), int(offsets[b + 1])
        L = e - s
        if L == 0:
            continue
        qb = q[s:e].view(L, H, dqk).transpose(0, 1)  # (H, L, dqk)
        kb = k[s:e].view(L, H, dqk).transpose(0, 1)
        vb = v[s:e].view(L, H, dv).transpose(0, 1)
        scores = qb @ kb.transpose(1, 2)  # (H, L, L)
        if ts is not None:
            scores = scores + rel_bias_jagged(ts[b], L, N, pos_w, ts_w, thresholds)
        a = F.silu(scores) / N
        a = a * torch.tril(torch.ones(L, L, dtype=a.dtype))
        outs.append((a @ vb).transpose(0, 1).reshape(L, H * dv))
    return torch.cat(outs, 0) if outs else q.new_zeros(0, H * dv)


def softmax_attention_jagged(q, k, v, offsets, ts, cfg: HSTUConfig, pos_w, ts_w,
                             thresholds) -> torch.Tensor:
    """hstu.py:371-389 (normalization="softmax_rel_bias", no cache) restated per sequence:
    one score over all heads' columns at once (einsum "bnd,bmd->bnm" of the padded
    (B, n, h dqk) q / k), plus the bias when the layer has a bias module, scaled by
    1 / sqrt(attention_dim) and normalised over ALL n keys — the padded keys (k = 0, so
    their score is the bias alone) and the future ones included — then the causal mask,
    then the product with the padded v.  Rows past L_b are dropped (dense_to_jagged)."""
    N = cfg.N
    outs = []
    for b in range(offsets.numel() - 1):
        s, e = int(offsets[b]), int(offsets[b + 1])
        L = e - s
        if L == 0:
            continue
        kb = torch.cat([k[s:e], k.new_zeros(N - L, k.shape[1])])  # (N, h dqk)
        scores = q[s:e] @ kb.t()  # (L, N)
        if pos_w is not None:
            i = torch.arange(L).view(L, 1)
            j = torch.arange(N).view(1, N)
            ext = torch.cat([ts[b], ts[b, N - 1:N]])
            delta = ext[1:L + 1].view(L, 1) - ts[b].view(1, N)
            scores = scores + (pos_w[(N - 1) + j - i] +
                               ts_w[bucket_via_thresholds(delta, thresholds)])
        a = F.softmax(scores / (cfg.dqk ** 0.5), dim=-1)
        a = a * torch.tril(torch.ones(L, N, dtype=a.dtype))
        outs.append(a[:, :L] @ v[s:e])
    return torch.cat(outs, 0) if outs else q.new_zeros(0, v.shape[1])


def stu_layer_jagged(x, offsets, ts, cfg: HSTUConfig, p, thresholds):
    """hstu.py:266-413 (eval mode, normalization='rel_bias' or 'softmax_rel_bias',
    linear_config='uvqk', linear_activation='silu')."""
    H, dv, dqk = cfg.H, cfg.dv, cfg.dqk
    normed = F.layer_norm(x, [cfg.D], eps=cfg.eps)
    h = F.silu(normed @ p["uvqk"])
    u, v, q, k = torch.split(h, [dv * H, dv * H, dqk * H, dqk * H], dim=1)
    attn_fn = softmax_attention_jagged if cfg.softmax else hstu_attention_jagged
    attn = attn_fn(q, k, v, offsets, ts, cfg, p["pos_w"], p["ts_w"], thresholds)
    a = F.layer_norm(attn, [dv * H], eps=cfg.eps)
    o_in = torch.cat([u, a, u * a], -1) if cfg.concat_ua else u * a
    return o_in @ p["o_w"].t() + p["o_b"] + x


def hstu_forward(lengths: torch.Tensor, user_embeddings: torch.Tensor,
                 ts: Optional[torch.Tensor], cfg: HSTUConfig,
                 layers: List[Dict[str, torch.Tensor]], thresholds) -> torch.Tensor:
    """hstu.py:633-672 -> 482-518: dense->jagged, layer loop, jagged->padded (rows
    >= L_b are zero)."""
    B, N, D = user_embeddings.shape
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64),
                         torch.cumsum(lengths.to(torch.int64), 0)])
    rows = [user_embeddings[b, :int(lengths[b])] for b in range(B)]
    x = torch.cat(rows, 0)
    for p in layers:
        x = stu_layer_jagged(x, offsets, ts, cfg, p, thresholds)
    out = user_embeddings.new_zeros(B, N, D)
    parts = []
    for b in range(B):
        s, e = int(offsets[b]), int(offsets[b + 1])
        pad = user_embeddings.new_zeros(N - (e - s), D)
        parts.append(torch.cat([x[s:e], pad], 0))
    out = torch.stack(parts, 0)
    return out


# ----------------------------------------------------------------------------------
# Padded (reference op-order) variant: the CPU throughput baseline.
# ----------------------------------------------------------------------------------

def rel_bias_padded(ts: torch.Tensor, N: int, pos_w, ts_w, thresholds) -> torch.Tensor:
    """hstu.py:96-128 batched: (B, N, N)."""
    i = torch.arange(N)
    pos = pos_w[(N - 1) + i.view(1, N) - i.view(N, 1)]
    ext = torch.cat([ts, ts[:, N - 1:N]], 1)
    delta = ext[:, 1:].unsqueeze(2) - ext[:, :-1].unsqueeze(1)
    bucket = bucket_reference_semantics(delta)
    return pos.unsqueeze(0) + ts_w[bucket.view(-1)].view(ts.shape[0], N, N)


def hstu_forward_padded(lengths, user_embeddings, ts, cfg: HSTUConfig, layers,
                        thresholds=None) -> torch.Tensor:
    """Same result as ``hstu_forward``; computes on the padded (B, N, ·) layout with
    the reference's batched op order (bmm over (B, H, N, N)), masking padded rows."""
    B, N, D = user_embeddings.shape
    H, dqk, dv = cfg.H, cfg.dqk, cfg.dv
    valid = (torch.arange(N).view(1, N) < lengths.view(B, 1)).to(user_embeddings.dtype)
    valid = valid.unsqueeze(-1)
    causal = torch.tril(torch.ones(N, N, dtype=user_embeddings.dtype))
    x = user_embeddings * valid
    for p in layers:
        normed = F.layer_norm(x, [D], eps=cfg.eps)
        h = F.silu(normed @ p["uvqk"])
        u, v, q, k = torch.split(h, [dv * H, dv * H, dqk * H, dqk * H], dim=-1)
        q = q * valid
        k = k * valid
        v = v * valid
        s = torch.einsum("bnhd,bmhd->bhnm", q.view(B, N, H, dqk), k.view(B, N, H, dqk))
        if ts is not None:
            s = s + rel_bias_padded(ts, N, p["pos_w"], p["ts_w"], thresholds).unsqueeze(1)
        a = F.silu(s) / N * causal
        attn = torch.einsum("bhnm,bmhd->bnhd", a, v.view(B, N, H, dv)).reshape(B, N, H * dv)
        an = F.layer_norm(attn, [dv * H], eps=cfg.eps)
        o_in = torch.cat([u, an, u * an], -1) if cfg.concat_ua else u * an
        x = (o_in @ p["o_w"].t() + p["o_b"] + x) * valid
    return x


# ----------------------------------------------------------------------------------
# Reference-op-order variant: the CPU throughput proxy.
# Same math as the two variants above, in the order the reference runs it on a CPU
# without fbgemm: per-row Python loops for every pad / unpad (ops.py:60-114 fallbacks),
# linear layers on the jagged rows, the (B, N, N) bias built with the pad/repeat
# Toeplitz trick and the fp32-log bucketisation, the float mask multiply, dropout
# before the output projection (train mode).  scripts/cpu_proxy_check.py times it
# against the reference's own HSTU module in the build container.
# ----------------------------------------------------------------------------------

def _rows_to_jagged(dense: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
    """ops.py:60-73 fallback: one slice per row, then one cat."""
    parts = []
    for b in range(offsets.numel() - 1):
        parts.append(dense[b, :offsets[b + 1] - offsets[b]])
    return torch.cat(parts, 0)


def _rows_to_padded(values: torch.Tensor, offsets: torch.Tensor, n: int) -> torch.Tensor:
    """ops.py:104-114 fallback: a zero (B, n, ...) tensor filled row by row."""
    B = offsets.numel() - 1
    out = values.new_zeros((B, n) + tuple(values.shape[1:]))
    for b in range(B):
        s, e = offsets[b], offsets[b + 1]
        out[b, :e - s] = values[s:e]
    return out


def _rel_bias_reference_order(ts: torch.Tensor, N: int, pos_w, ts_w) -> torch.Tensor:
    """hstu.py:96-128: a (N, 3N-2) Toeplitz band from the padded, repeated pos_w, its
    middle N columns; fp32-log buckets of ext_ts[i+1] - ts[j]; index_select of ts_w."""
    B = ts.shape[0]
    band = F.pad(pos_w[: 2 * N - 1], [0, N]).repeat(N)[:-N].view(1, N, 3 * N - 2)
    r = (2 * N - 1) // 2
    ext = torch.cat([ts, ts[:, N - 1:N]], 1)
    bucket = bucket_reference_semantics(ext[:, 1:].unsqueeze(2) - ext[:, :-1].unsqueeze(1))
    ts_bias = torch.index_select(ts_w, 0, bucket.view(-1)).view(B, N, N)
    return band[:, :, r:-r] + ts_bias


def hstu_forward_reference_order(lengths, user_embeddings, ts, cfg: HSTUConfig, layers,
                                 dropout_p: float = 0.0, training: bool = False) -> torch.Tensor:
    """hstu.py:633-672 -> 482-518 -> 266-413 -> 134-205 in the reference's op order."""
    B, N, D = user_embeddings.shape
    H, dqk, dv = cfg.H, cfg.dqk, cfg.dv
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64),
                         torch.cumsum(lengths.to(torch.int64), 0)])
    mask = 1.0 - torch.triu(torch.ones(N, N, dtype=torch.bool), diagonal=1).float()
    x = _rows_to_jagged(user_embeddings, offsets)
    for p in layers:
        normed = F.layer_norm(x, [D], eps=cfg.eps)
        h = F.silu(torch.mm(normed, p["uvqk"]))
        u, v, q, k = torch.split(h, [dv * H, dv * H, dqk * H, dqk * H], dim=1)
        pq = _rows_to_padded(q, offsets, N)
        pk = _rows_to_padded(k, offsets, N)
        s = torch.einsum("bnhd,bmhd->bhnm", pq.view(B, N, H, dqk), pk.view(B, N, H, dqk))
        if ts is not None:
            s = s + _rel_bias_reference_order(ts, N, p["pos_w"], p["ts_w"]).unsqueeze(1)
        s = F.silu(s) / N
        s = s * mask.unsqueeze(0).unsqueeze(0)
        pv = _rows_to_padded(v, offsets, N).reshape(B, N, H, dv)
        attn = _rows_to_jagged(torch.einsum("bhnm,bmhd->bnhd", s, pv).reshape(B, N, H * dv),
                               offsets)
        an = F.layer_norm(attn, [dv * H], eps=cfg.eps)
        o_in = torch.cat([u, an, u * an], -1) if cfg.concat_ua else u * an
        o_in = F.dropout(o_in, p=dropout_p, training=training)
        x = F.linear(o_in, p["o_w"], p["o_b"]) + x
    return _rows_to_padded(x, offsets, N)


# ----------------------------------------------------------------------------------
# Cached (incremental) decoding: the delta_x_offsets / cache branch of the reference.
# ----------------------------------------------------------------------------------

def stu_layer_cached(x, offsets, ts, cfg: HSTUConfig, p, delta=None, cache=None):
    """One layer of hstu.py:266-423 with its cache states, restated on padded tensors.

    Without ``delta``: the full layer, returning (new_outputs, (v, padded_q, padded_k,
    new_outputs)) (hstu.py:420-423).  With ``delta`` = (jagged rows, positions) and
    ``cache`` = that tuple: only the rows x[delta[0]] are re-encoded (hstu.py:293-298);
    v, padded q / k and the outputs are updated IN PLACE by index_copy_ (hstu.py:321-322,
    151-177, 415-418) — position delta[1][e] of sequence e for q / k — and the attention
    reads the updated caches."""
    H, dv, dqk, N, D = cfg.H, cfg.dv, cfg.dqk, cfg.N, cfg.D
    B = offsets.numel() - 1
    xs = x[delta[0]] if delta is not None else x
    normed = F.layer_norm(xs, [D], eps=cfg.eps)
    h = F.silu(normed @ p["uvqk"])
    u, v, q, k = torch.split(h, [dv * H, dv * H, dqk * H, dqk * H], dim=1)
    if delta is not None:
        v_c, q_c, k_c, out_c = cache
        v = v_c.index_copy_(0, delta[0], v)
        flat = delta[1] + torch.arange(0, B * N, N, dtype=delta[1].dtype)
        pq = q_c.view(B * N, -1).index_copy_(0, flat, q).view(B, N, -1)
        pk = k_c.view(B * N, -1).index_copy_(0, flat, k).view(B, N, -1)
    else:
        pq = _rows_to_padded(q, offsets, N)
        pk = _rows_to_padded(k, offsets, N)
    s = torch.einsum("bnhd,bmhd->bhnm", pq.view(B, N, H, dqk), pk.view(B, N, H, dqk))
    if ts is not None:
        s = s + rel_bias_padded(ts, N, p["pos_w"], p["ts_w"], None).unsqueeze(1)
    a = F.silu(s) / N * torch.tril(torch.ones(N, N, dtype=s.dtype))
    pv = _rows_to_padded(v, offsets, N).reshape(B, N, H, dv)
    attn = _rows_to_jagged(torch.einsum("bhnm,bmhd->bnhd", a, pv).reshape(B, N, H * dv),
                           offsets)
    if delta is not None:
        attn = attn[delta[0]]
    an = F.layer_norm(attn, [dv * H], eps=cfg.eps)
    o_in = torch.cat([u, an, u * an], -1) if cfg.concat_ua else u * an
    new = o_in @ p["o_w"].t() + p["o_b"] + xs
    if delta is not None:
        new = cache[3].index_copy_(0, delta[0], new)
    return new, (v.contiguous(), pq, pk, new)


def hstu_forward_cached(lengths, user_embeddings, ts, cfg: HSTUConfig, layers,
                        delta=None, cache=None):
    """HSTU.forward (hstu.py:633-672 -> 482-518) with return_cache_states=True:
    (y (B, N, D), [per-layer (v, padded_q, padded_k, outputs)]).  With ``delta`` /
    ``cache`` the cached step; the cache tensors are updated in place."""
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64),
                         torch.cumsum(lengths.to(torch.int64), 0)])
    x = _rows_to_jagged(user_embeddings, offsets)
    states = []
    for i, p in enumerate(layers):
        x, st = stu_layer_cached(x, offsets, ts, cfg, p, delta,
                                 cache[i] if cache is not None else None)
        states.append(st)
    return _rows_to_padded(x, offsets, cfg.N), states
