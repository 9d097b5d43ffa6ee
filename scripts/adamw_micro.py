"""FlatAdamW vs torch fused AdamW on one large table + small tensors (C5's AdamW group
shape): device time per step by CUDA events.   python scripts/adamw_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd.optim import FlatAdamW  # noqa: E402


def run(kind, shapes, iters=20):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in shapes]
    for p in ps:
        p.grad = torch.randn_like(p)
    if kind == "flat":
        opt = FlatAdamW(ps, lr=5e-4, betas=(0.8, 0.95), eps=1e-10, weight_decay=5e-3)
    else:
        opt = torch.optim.AdamW(ps, lr=5e-4, betas=(0.8, 0.95), eps=1e-10, weight_decay=5e-3,
                                fused=True, capturable=True)
    for _ in range(3):
        opt.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        opt.step()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for name, shapes in (("c5_group", [(131263, 256), (2000, 256)] + [(256,)] * 24 + [(4117,), (129,)] * 8),
                     ("c2", [(50, 200), (50, 50), (50,), (401,), (129,)] * 4),
                     ("big_only", [(131263, 256)])):
    for kind in ("flat", "torch", "flat", "torch"):
        print(name, kind, round(run(kind, shapes), 4), "ms", flush=True)
