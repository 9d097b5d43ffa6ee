"""Workgroup timeline of the f32 attention backward (diagnostic build, -DGR_STAMP):
    GR_HSTU_LIB=vlib/libgr_stamp.so python scripts/timeline_bwd.py [--batch B --len L --split]
Prints per-kind workgroup durations (by key / query tile), the launch span, and how
many workgroups each CU held over time (slot occupancy)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--len", type=int, default=200)
ap.add_argument("--split", action="store_true")
ap.add_argument("--nobias", action="store_true")
a = ap.parse_args()
B, L, d, H = a.batch, a.len, 50, 1
N = L + 11
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
rows, n_out, hv = B * L, 4 * d, d
uvqk = torch.randn(rows, n_out, device=dev, generator=g) * 0.5
hpre = torch.randn(rows, n_out, device=dev, generator=g)
q, k, v = uvqk[:, 2 * hv:3 * hv], uvqk[:, 3 * hv:], uvqk[:, hv:2 * hv]
offsets = torch.arange(0, B + 1, device=dev, dtype=torch.int64) * L
ts = (1_000_000_000 + torch.cumsum(torch.randint(0, 200_000, (B, N), device=dev, generator=g), 1))
bmap = None if a.nobias else ops.bucket_map(ts.to(torch.int64), offsets, N)
pos_w = torch.randn(2 * N - 1, device=dev, generator=g) * 0.1
ts_w = torch.randn(129, device=dev, generator=g) * 0.1
dout = torch.randn(rows, hv, device=dev, generator=g)
dd = torch.empty(rows, n_out, device=dev)
dpw, dtw = torch.empty_like(pos_w), torch.empty_like(ts_w)
Lb = _lib.lib()
_lib.set_option("ATTN_BWD_SPLIT", int(a.split))
ws_n = Lb.hstu_attn_bwd_workspace_size(B, N, L, H, 128)
ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
raw = ctypes.CDLL(_lib.LIB_PATH)
n_t = (L + 63) // 64
grid = n_t * B * H
n_wg = 2 * grid  # dQ workgroups in slots [grid, 2 grid)


def run():
    _lib.call("hstu_attn_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out, n_out,
              dout.data_ptr(), hv, offsets.data_ptr(), B, N, L, H, d, d, _lib.ptr(bmap),
              pos_w.data_ptr(), ts_w.data_ptr(), 128, hpre[:, 2 * hv:].data_ptr(),
              hpre[:, 3 * hv:].data_ptr(), hpre[:, hv:].data_ptr(), n_out,
              dd[:, 2 * hv:].data_ptr(), dd[:, 3 * hv:].data_ptr(), dd[:, hv:].data_ptr(), n_out,
              dpw.data_ptr(), dtw.data_ptr(), ws.data_ptr(), ws_n, _lib.stream_handle())


for _ in range(5):
    run()
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (n_wg * 4))()
assert raw.gr_timeline_read(buf, n_wg * 4) == 0
tl = np.frombuffer(buf, dtype=np.uint64).reshape(n_wg, 4).astype(np.int64)
last = int(tl[:, 0].max())
tl = tl[tl[:, 0] > last - 100_000_000]  # this launch's workgroups (paired grids write fewer slots)
n_wg = len(tl)
TICK_US = 0.01  # s_memrealtime: 100 MHz
t0 = tl[:, 0].min()
ent = (tl[:, 0] - t0) * TICK_US
ext = (tl[:, 1] - t0) * TICK_US
dur = ext - ent
kind = tl[:, 3]
hw = tl[:, 2] & 0xFFFFFFFF
xcc = (tl[:, 2] >> 32) & 0xF
cu = (xcc << 16) | ((hw >> 8) & 0xFF)
out = {"B": B, "L": L, "split": a.split, "span_us": float(ext.max()), "n_wg": int(n_wg)}
for kd, name in ((0, "dkv"), (1, "dq")):
    sel = kind == kd
    if not sel.any():
        continue
    # the rank -> tile mapping is snake-ordered; report by duration quantiles instead
    out[name] = {"n": int(sel.sum()), "dur_mean": float(dur[sel].mean()),
                 "dur_p50": float(np.median(dur[sel])), "dur_max": float(dur[sel].max()),
                 "dur_min": float(dur[sel].min()), "entry_max": float(ent[sel].max()),
                 "exit_max": float(ext[sel].max())}
ucu = np.unique(cu)
busy = np.array([dur[cu == c].sum() for c in ucu])
nwg = np.array([(cu == c).sum() for c in ucu])
lastexit = np.array([ext[cu == c].max() for c in ucu])
out["cus_seen"] = int(len(ucu))
out["wg_per_cu"] = [int(nwg.min()), float(nwg.mean()), int(nwg.max())]
out["cu_slot_us"] = [float(busy.min()), float(busy.mean()), float(busy.max())]
out["cu_last_exit"] = [float(lastexit.min()), float(lastexit.mean()), float(lastexit.max())]
# concurrency over time (all CUs): mean resident workgroups per CU in 1 us bins
bins = np.arange(0, ext.max() + 1, 1.0)
conc = np.zeros(len(bins))
for e0, e1 in zip(ent, ext):
    conc[int(e0):int(e1) + 1] += 1
out["resident_per_cu_by_us"] = [round(float(c) / max(1, len(ucu)), 2) for c in conc[::2]]
print(json.dumps(out))
