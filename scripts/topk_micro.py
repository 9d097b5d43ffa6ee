"""Micro-benchmark of mips_topk at C4 shapes (per-kernel device time via the library's
event timing).  python scripts/topk_micro.py [--items 10000000] [--dim 50]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib  # noqa: E402
from mygenerativerecommenders_amd.top_k import PackedItems, mips_topk, topk_workspace_bytes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--items", type=int, default=10_000_000)
ap.add_argument("--dim", type=int, default=50)
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--k", type=int, default=200)
ap.add_argument("--n0", type=int, default=211)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--opt", action="append", default=[], help="launch option NAME=VALUE")
a = ap.parse_args()
for o in a.opt:
    _n, _v = o.split("=")
    _lib.set_option(_n, int(_v))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
E = torch.randn(a.items, a.dim, device=dev, generator=g)
E /= E.norm(dim=1, keepdim=True)
pk = PackedItems(E)
del E
Q = torch.randn(a.batch, a.dim, device=dev, generator=g)
Q /= Q.norm(dim=1, keepdim=True)
inv = torch.randint(1, a.items + 1, (a.batch, a.n0), device=dev, generator=g)
ws = torch.empty(topk_workspace_bytes(a.batch, a.items, a.dim, a.k), dtype=torch.uint8, device=dev)
for _ in range(3):
    mips_topk(Q, pk, a.k, invalid_ids=inv, index_base=1, workspace=ws)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.iters):
    mips_topk(Q, pk, a.k, invalid_ids=inv, index_base=1, workspace=ws)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.iters
_lib.timing_enable(True)
for _ in range(a.iters):
    mips_topk(Q, pk, a.k, invalid_ids=inv, index_base=1, workspace=ws)
torch.cuda.synchronize()
_lib.timing_enable(False)
kt = {n: v[0] / a.iters for n, v in _lib.kernel_times(_lib.KERNEL_NAMES).items() if v[1]}
fl = 2.0 * a.batch * a.items * a.dim
print(f"X={a.items} D={a.dim} B={a.batch}: {dt*1e3:.3f} ms/batch  {a.batch*a.items/dt/1e9:.1f} G items/s"
      f"  fallback={int(ws[:4].view(torch.int32).item())}")
if a.items >= 262144 and a.dim <= 64:  # filter path: candidate counts (workspace layout)
    al = lambda v: (v + 255) // 256 * 256  # noqa: E731  (flag | tau | tau_e | q rows | cnt)
    off_cnt = al(al(al(256 + 4 * a.batch) + 4 * a.batch) + 16 * a.batch * ((a.dim + 3) // 4))
    cnt = ws[off_cnt:off_cnt + 4 * 16 * a.batch].view(torch.int32).view(a.batch, 16).sum(1).float()
    print(f"  candidates/query: mean {cnt.mean().item():.0f} min {cnt.min().item():.0f} "
          f"max {cnt.max().item():.0f}")
for n, ms in sorted(kt.items(), key=lambda kv: -kv[1]):
    extra = f"  {fl/ms/1e9:.1f} TFLOP/s" if n in ("mips_filter", "mips_select") else ""
    print(f"  {n:24s} {ms*1e3:8.1f} us{extra}")
