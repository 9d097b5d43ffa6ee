"""AdamW as one launch per parameter group (``gr_adamw_step``).

torch.optim.AdamW(fused=True, capturable=True) -- the reference's optimizer
(``configs/model/*.yaml``: AdamW, betas (0.9, 0.98), weight decay 1e-3) -- costs two
launches per step on the GPU: the step counters' ``_foreach_add_`` and the fused
multi-tensor kernel.  ``FlatAdamW`` keeps the moments in two flat fp32 buffers and runs
the same update, the counter advanced inside the same launch; the tensors' pointers
travel in the kernel arguments (up to 48 tensors per launch), as torch's tensor lists
do, so graph capture and fresh gradient tensors each step both work.  The
per-parameter state (``exp_avg`` / ``exp_avg_sq`` views into the flat buffers, ``step``)
has torch's names.  Dense fp32 CUDA tensors only; ``amsgrad`` and ``maximize`` raise.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, maximize: bool = False):
        if amsgrad or maximize:
            raise NotImplementedError("FlatAdamW: amsgrad / maximize are not supported")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError(f"FlatAdamW: invalid lr / eps / weight_decay ({lr}, {eps}, {weight_decay})")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"FlatAdamW: invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self._flat: dict = {}

    def _group_state(self, gi: int, group: dict) -> dict:
        fs = self._flat.get(gi)
        if fs is not None:
            return fs
        params = group["params"]
        dev = params[0].device
        for p in params:
            if p.device != dev or p.dtype != torch.float32 or not p.is_contiguous() or not p.is_cuda:
                raise TypeError("FlatAdamW: contiguous fp32 CUDA parameters on one device expected")
        offs = np.zeros(len(params), np.int64)
        o = 0
        for i, p in enumerate(params):
            offs[i] = o
            o += (p.numel() + 3) // 4 * 4  # 16-byte aligned moments (float4 path)
        m = torch.zeros(o, dtype=torch.float32, device=dev)
        v = torch.zeros(o, dtype=torch.float32, device=dev)
        step = torch.zeros(1, dtype=torch.float32, device=dev)
        done = torch.zeros(1, dtype=torch.int32, device=dev)
        for p, off in zip(params, offs.tolist()):
            self.state[p] = {"step": step, "exp_avg": m[off:off + p.numel()].view_as(p),
                             "exp_avg_sq": v[off:off + p.numel()].view_as(p)}
        fs = self._flat[gi] = {"m": m, "v": v, "step": step, "done": done, "offs": offs}
        return fs

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = group["params"]
            if not params or all(p.grad is None for p in params):
                continue
            fs = self._group_state(gi, group)
            n = len(params)
            pp = np.zeros(n, np.uint64)
            gp = np.zeros(n, np.uint64)
            ne = np.zeros(n, np.int64)
            for i, p in enumerate(params):
                g = p.grad
                if g is None:
                    continue
                if (g.dtype != torch.float32 or g.is_sparse or not g.is_contiguous()
                        or g.shape != p.shape or g.device != p.device):
                    raise TypeError("FlatAdamW: dense contiguous fp32 gradients expected")
                pp[i], gp[i], ne[i] = p.data_ptr(), g.data_ptr(), p.numel()
            b1, b2 = group["betas"]
            _lib.call("gr_adamw_step", pp.ctypes.data, gp.ctypes.data, fs["offs"].ctypes.data,
                      ne.ctypes.data, n, fs["m"].data_ptr(), fs["v"].data_ptr(),
                      fs["step"].data_ptr(), fs["done"].data_ptr(), float(group["lr"]), float(b1),
                      float(b2), float(group["eps"]), float(group["weight_decay"]),
                      _lib.stream_handle())
        return loss
