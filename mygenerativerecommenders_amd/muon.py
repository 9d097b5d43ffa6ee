"""Muon optimizer — drop-in for reference ``models/optimizers/muon.py``
(Hydra ``_target_: ...optimizers.muon.Muon``, configs/experiment/ml-1m-hstu-muon.yaml),
SURVEY §8 N4.

Same update as the reference (muon.py:3-86): SGD momentum (lerp), Nesterov blend, a
5-step quintic Newton-Schulz orthogonalisation in bf16 (a, b, c = 3.4445, -4.7750,
2.0315; X / (||X||_F + 1e-7); transposed when rows > cols), a sqrt(max(1, rows/cols))
scale, decoupled weight decay.  The MI355X shape of it: every parameter of one shape
is orthogonalised in ONE batched chain (stacked (P, m, n) bf16 GEMMs on the matrix
cores, 15 GEMM launches per shape class instead of 15 per parameter), and the momentum
/ Nesterov / decay / apply steps are multi-tensor (_foreach) launches, so a step of the
HSTU's 2 x num_blocks weight matrices costs a few dozen launches and captures in a graph.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Tuple

import torch

_NS_COEFFS = (3.4445, -4.7750, 2.0315)
# the GPU chain's combines as gr_bf16_scale_add launches (False: the reference's torch ops;
# the results are bit-identical, tests/test_gpu_next_rows.py)
FUSED_COMBINE = True


def _scale_add(x: torch.Tensor, s: float, y: torch.Tensor) -> torch.Tensor:
    """bf16(bf16(s * x) + y) in one launch (gr_bf16_scale_add): the reference's
    ``s * x + y`` on bf16 tensors with both of its roundings."""
    from . import _lib
    x, y = x.contiguous(), y.contiguous()
    out = torch.empty_like(y)
    _lib.call("gr_bf16_scale_add", x.data_ptr(), float(s), y.data_ptr(), out.data_ptr(), y.numel(),
              _lib.stream_handle())
    return out


def zeropower_via_newtonschulz5(G: torch.Tensor, steps: int) -> torch.Tensor:
    """Approximate orthogonalisation U S' V^T of G (..., m, n), in bf16 (muon.py:3-29).
    On the GPU each iteration is three GEMMs, one scale and two ``gr_bf16_scale_add``
    combines (six launches instead of eight), bit-identical to the reference's ops."""
    assert G.ndim >= 2
    a, b, c = _NS_COEFFS
    X = G.bfloat16()
    tall = G.size(-2) > G.size(-1)
    if tall:
        X = X.mT
    X = X / (X.norm(dim=(-2, -1), keepdim=True) + 1e-7)
    fused = X.is_cuda and FUSED_COMBINE
    for _ in range(steps):
        A = X @ X.mT
        if fused:
            B = _scale_add(A, b, (c * A) @ A)
            X = _scale_add(X, a, B @ X)
        else:
            B = b * A + c * A @ A
            X = a * X + B @ X
    if tall:
        X = X.mT
    return X


class Muon(torch.optim.Optimizer):
    """muon.py:46-86: lr in units of spectral norm per update; AdamW-style decay."""

    def __init__(self, params, lr: float = 0.02, weight_decay: float = 0, momentum: float = 0.95,
                 ns_steps: int = 5, nesterov: bool = True) -> None:
        defaults = dict(lr=lr, weight_decay=weight_decay, momentum=momentum, ns_steps=ns_steps,
                        nesterov=nesterov)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params: List[torch.Tensor] = group["params"]
            if not params:
                continue
            beta, lr, wd = group["momentum"], group["lr"], group["weight_decay"]
            grads, bufs = [], []
            for p in params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                st = self.state[p]
                if len(st) == 0:
                    st["momentum_buffer"] = torch.zeros_like(p)
                grads.append(p.grad)
                bufs.append(st["momentum_buffer"])
            # momentum.lerp_(grad, 1 - beta); update = grad.lerp_(momentum, beta) (Nesterov)
            torch._foreach_lerp_(bufs, grads, 1 - beta)
            if group["nesterov"]:
                torch._foreach_lerp_(grads, bufs, beta)
                updates = grads
            else:
                updates = bufs
            # one batched Newton-Schulz chain per update shape (viewed 2-D)
            classes: Dict[Tuple[int, int], List[int]] = defaultdict(list)
            mats = []
            for i, u in enumerate(updates):
                m = u.view(len(u), -1) if u.ndim == 4 else u
                mats.append(m)
                classes[tuple(m.shape[-2:])].append(i)
            out: List[torch.Tensor] = [None] * len(params)  # type: ignore[list-item]
            for (rows, cols), idx in classes.items():
                stacked = torch.stack([mats[i] for i in idx]) if len(idx) > 1 else mats[idx[0]][None]
                ortho = zeropower_via_newtonschulz5(stacked, group["ns_steps"])
                ortho = ortho * max(1, rows / cols) ** 0.5
                for k, i in enumerate(idx):
                    out[i] = ortho[k].reshape(params[i].shape)
            if wd:
                torch._foreach_mul_(params, 1 - lr * wd)
            torch._foreach_add_(params, out, alpha=-lr)
        return loss
