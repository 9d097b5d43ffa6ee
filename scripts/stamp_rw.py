"""Per-wave phase timeline of the layer-boundary kernel (rowwave2_kernel) at C2, from the
diagnostic build (-DGR_STAMP, s_memrealtime = 10 ns ticks):
    GR_HSTU_LIB=stamplib/libgr_stamp.so python scripts/stamp_rw.py
Prints, for the last forward and the last backward boundary launch, the mean / max over
waves of: staging (entry -> panels in LDS), product 1, epilogue 1 + prep 2, product 2,
epilogue 2, and the spread of wave entry / exit times."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mygenerativerecommenders_amd import _lib  # noqa: E402

dev = torch.device("cuda")
B, N0, out_len, D, blocks = 128, 200, 11, 50, 4
enc = bench.build_model(N0, out_len, D, blocks, dev)
lengths, x, ts, _, dy = bench.make_batch(B, N0, out_len, D, 1, dev)
raw = ctypes.CDLL(_lib.LIB_PATH)
n = 1 << 15


def read(tag):
    buf = (ctypes.c_ulonglong * n)()
    assert raw.gr_rw_stamp_read(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).astype(np.float64)
    st = st[(st[:, 0] > 0) & (st[:, 5] > 0)]
    t0 = st[:, 0].min()
    ph = np.diff(st[:, :6], axis=1) * 0.01  # us
    names = ["stage", "mma1", "epi1+prep2", "mma2", "epi2"]
    print(f"{tag}: waves {len(st)}  span {(st[:, 5].max() - t0) * 0.01:.2f} us  "
          f"entry spread {(st[:, 0].max() - t0) * 0.01:.2f} us")
    for i, nm in enumerate(names):
        print(f"   {nm:12s} mean {ph[:, i].mean():7.2f} us  max {ph[:, i].max():7.2f} us")
    ex = (st[:, 5] - t0) * 0.01
    print(f"   exit: p10 {np.percentile(ex, 10):.2f}  p50 {np.percentile(ex, 50):.2f}  "
          f"p90 {np.percentile(ex, 90):.2f}  max {ex.max():.2f} us")


for _ in range(3):
    y, _ = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
               past_payloads={"timestamps": ts}, max_len=N0)
    y.backward(dy)
torch.cuda.synchronize()
with torch.no_grad():
    y, _ = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
               past_payloads={"timestamps": ts}, max_len=N0)
torch.cuda.synchronize()
read("boundary_fwd (last forward launch)")
y, _ = enc(past_lengths=lengths, user_embeddings=x, valid_mask=None,
           past_payloads={"timestamps": ts}, max_len=N0)
y.backward(dy)
torch.cuda.synchronize()
read("boundary_bwd (last backward launch)")
