"""Phase cycle breakdown of the dK/dV attention kernel (diagnostic build, -DGR_STAMP):
    GR_HSTU_LIB=vlib/libgr_stamp.so python scripts/stamp_dkv.py [--batch B --len L]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--len", type=int, default=256)
ap.add_argument("--hepi", action="store_true", help="fused silu'(h) epilogue (the product path)")
a = ap.parse_args()
B, L, d, H = a.batch, a.len, 50, 1
N = L + 11
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
rows, n_out, hv = B * L, 4 * d, d
uvqk = torch.randn(rows, n_out, device=dev, generator=g) * 0.5
q, k, v = uvqk[:, 2 * hv:3 * hv], uvqk[:, 3 * hv:], uvqk[:, hv:2 * hv]
offsets = torch.arange(0, B + 1, device=dev, dtype=torch.int64) * L
ts = (1_000_000_000 + torch.cumsum(torch.randint(0, 200_000, (B, N), device=dev, generator=g), 1))
bmap = ops.bucket_map(ts.to(torch.int64), offsets, N)
pos_w = torch.randn(2 * N - 1, device=dev, generator=g) * 0.1
ts_w = torch.randn(129, device=dev, generator=g) * 0.1
dout = torch.randn(rows, hv, device=dev, generator=g)
hpre = torch.randn(rows, n_out, device=dev, generator=g) if a.hepi else None
hp = (lambda c: hpre[:, c:].data_ptr()) if a.hepi else (lambda c: None)
dd = torch.empty(rows, n_out, device=dev)
dpw, dtw = torch.empty_like(pos_w), torch.empty_like(ts_w)
Lb = _lib.lib()
ws_n = Lb.hstu_attn_bwd_workspace_size(B, N, L, H, 128)
ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
for _ in range(3):
    _lib.call("hstu_attn_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out, n_out,
              dout.data_ptr(), hv, offsets.data_ptr(), B, N, L, H, d, d, bmap.data_ptr(),
              pos_w.data_ptr(), ts_w.data_ptr(), 128, hp(2 * hv), hp(3 * hv), hp(hv), n_out,
              dd[:, 2 * hv:].data_ptr(), dd[:, 3 * hv:].data_ptr(), dd[:, hv:].data_ptr(), n_out,
              dpw.data_ptr(), dtw.data_ptr(), ws.data_ptr(), ws_n, _lib.stream_handle())
torch.cuda.synchronize()
n_wg = ((L + 63) // 64) * B
buf = (ctypes.c_ulonglong * (n_wg * 4 * 12))()
raw = ctypes.CDLL(_lib.LIB_PATH)
assert raw.gr_stamp_read(buf, n_wg * 4 * 12) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(n_wg, 4, 12).astype(np.float64)
names = ["tile_ld", "mm_S_dP", "elementwise", "bias_hist", "mm_dV_dK", "tile_sync", "kt", "total",
         "prologue", "wave_all", "-", "-"]
tl = (ctypes.c_ulonglong * (n_wg * 4))()
assert raw.gr_timeline_read(tl, n_wg * 4) == 0
tl = np.frombuffer(tl, dtype=np.uint64).reshape(n_wg, 4).astype(np.float64)
wg_us = (tl[:, 1] - tl[:, 0]) * 0.01
for kt in sorted(set(st[:, 0, 6].astype(int))):
    sel = st[st[:, 0, 6] == kt]
    print(f"kt={kt}: " + "  ".join(f"{n}={sel[:, :, i].mean():9.0f}" for i, n in enumerate(names) if n not in ("kt", "-"))
          + f"  wg_us={wg_us[st[:, 0, 6] == kt].mean():.2f}")
