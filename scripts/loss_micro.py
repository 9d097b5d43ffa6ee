"""Micro-benchmark of the fused sampled-softmax loss kernels at the ml-1m C2 shape
(M = 128 x 199 supervised positions, R = 128, D = 50, 3953-row catalog), timed by the
library's live event timing, next to the reference's materialising PyTorch chain.

    python scripts/loss_micro.py --iters 50
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--M", type=int, default=128 * 199)
    ap.add_argument("--D", type=int, default=50)
    ap.add_argument("--V", type=int, default=3953)
    ap.add_argument("--R", type=int, default=128)
    args = ap.parse_args()
    M, D, V, R, T = args.M, args.D, args.V, args.R, 0.05
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    out = torch.nn.functional.normalize(torch.randn(M, D, device=dev, generator=g), dim=-1)
    pos = torch.nn.functional.normalize(torch.randn(M, D, device=dev, generator=g), dim=-1)
    tab = torch.nn.functional.normalize(torch.randn(V, D, device=dev, generator=g), dim=-1)
    ids = torch.arange(1, V + 1, device=dev)
    sup = torch.randint(1, V + 1, (M,), device=dev, generator=g)
    offs = torch.randint(0, V, (M, R), device=dev, generator=g)
    w = torch.ones(M, device=dev) / M
    out.requires_grad_(True)
    pos.requires_grad_(True)
    tab.requires_grad_(True)

    def fused():
        lt = ops.sampled_softmax_loss(out, pos, tab, sup, offs, ids, T)
        (lt * w).sum().backward()

    def reference_chain():
        neg = tab[offs]
        pl = (pos * out).sum(-1, keepdim=True) / T
        nl = torch.bmm(neg, out.unsqueeze(2)).squeeze(2)
        nl = torch.where(sup.unsqueeze(1) == ids[offs], -5e4, nl / T)
        jl = -torch.nn.functional.log_softmax(torch.cat([pl, nl], 1), 1)[:, 0]
        (jl * w).sum().backward()

    res = {"M": M, "D": D, "V": V, "R": R}
    for name, fn in (("fused", fused), ("torch_chain", reference_chain)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = round((time.perf_counter() - t0) / args.iters * 1e3, 4)
    _lib.timing_enable(True)
    for _ in range(args.iters):
        torch.cuda._sleep(1_000_000)
        fused()
    torch.cuda.synchronize()
    _lib.timing_enable(False)
    kt = _lib.kernel_times(("sampled_softmax_fwd", "sampled_softmax_bwd", "sampled_softmax_csr",
                            "sampled_softmax_table_grad"))
    gather = M * R * D * 4
    for n, (tot, c) in kt.items():
        if c:
            avg = tot / c
            res[n] = {"avg_us": round(avg * 1e3, 2),
                      "gather_GBps": round(gather / (avg * 1e-3) / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
