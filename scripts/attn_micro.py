"""Micro-benchmark of the attention kernels alone (forward, dK/dV, dQ, bias reduce) at
the C2 (ml-1m) and C3 (ml-20m-like) shapes, timed by the library's live event timing.

    python scripts/attn_micro.py --shape c2 --iters 50
Run under rocprofv3 (program directly after `--`) for counters.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib, ops  # noqa: E402

SHAPES = {
    # B, N (padded), L (all sequences), d, H
    "c2": (128, 211, 200, 50, 1),
    "c3": (32, 2059, 2048, 256, 1),
    "c2b64": (64, 211, 200, 50, 1),
    "c2b32": (32, 211, 200, 50, 1),
    "c2b256": (256, 211, 200, 50, 1),
}


def flops(B, L, d, H):
    T = B * L * (L + 1) / 2 * H
    return {"attn_fwd": 2 * T * 2 * d, "attn_bwd_dkv": 2 * T * 3 * d, "attn_bwd_dq": 2 * T * d,
            "attn_bwd": 2 * T * 4 * d}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="fwd|bwd")
    ap.add_argument("--batch", type=int, default=0, help="override B")
    ap.add_argument("--len", type=int, default=0, help="override L (N = L + 11)")
    ap.add_argument("--nobias", action="store_true", help="no relative bias (timestamps absent)")
    ap.add_argument("--bf16", action="store_true", help="bf16-operand kernels")
    ap.add_argument("--split", action="store_true", help="f32 backward as separate dK/dV, dQ launches")
    ap.add_argument("--nopairs", action="store_true", help="f32 backward: one tile per workgroup")
    ap.add_argument("--pairs", type=int, default=1, help="GR_OPT_ATTN_BWD_PAIRS (0/1/2)")
    ap.add_argument("--ds", type=int, default=None, nargs="?", const=1,
                    help="f32 backward dS forms: 0 = recompute, 1 = two launches (library "
                         "default), 2 = in-launch hand-off")
    ap.add_argument("--hepi", action="store_true",
                    help="fused silu'(h) epilogue on dQ/dK/dV (as in the training step)")
    ap.add_argument("--opt", action="append", default=[], help="launch option NAME=VALUE")
    ap.add_argument("--stamp", action="store_true",
                    help="print the wide bf16 key-major kernel's phase cycles (-DGR_STAMP library)")
    args = ap.parse_args()
    for o in args.opt:
        n, v = o.split("=")
        _lib.set_option(n, int(v))
    B, N, L, d, H = SHAPES[args.shape]
    if args.batch:
        B = args.batch
    if args.len:
        L, N = args.len, args.len + 11
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    rows = B * L
    n_out = 4 * H * d
    hv = H * d
    uvqk = torch.randn(rows, n_out, device=dev, generator=g) * 0.5
    q, k, v = uvqk[:, 2 * hv:3 * hv], uvqk[:, 3 * hv:], uvqk[:, hv:2 * hv]
    offsets = torch.arange(0, B + 1, device=dev, dtype=torch.int64) * L
    ts = (1_000_000_000 + torch.cumsum(torch.randint(0, 200_000, (B, N), device=dev,
                                                     generator=g), 1)).to(torch.int64)
    bmap = ops.bucket_map(ts, offsets, N)
    pos_w = torch.randn(2 * N - 1, device=dev, generator=g) * 0.1
    ts_w = torch.randn(129, device=dev, generator=g) * 0.1
    out = torch.empty(rows, hv, device=dev)
    dout = torch.randn(rows, hv, device=dev, generator=g)
    dd = torch.empty(rows, n_out, device=dev)
    dq, dk, dvv = dd[:, 2 * hv:3 * hv], dd[:, 3 * hv:], dd[:, hv:2 * hv]
    dpw = torch.empty_like(pos_w)
    dtw = torch.empty_like(ts_w)
    L_ = _lib.lib()
    _lib.set_option("ATTN_BWD_SPLIT", int(args.split))
    _lib.set_option("ATTN_BWD_PAIRS", 0 if args.nopairs else args.pairs)
    if args.ds is not None:
        _lib.set_option("ATTN_BWD_DS", int(args.ds))  # before the workspace size query
    ws_n = (L_.hstu_attn_bwd_bf16_workspace_size(B, N, L, H, d, d, 128) if args.bf16
            else L_.hstu_attn_bwd_workspace_size_d(B, N, L, H, d, d, 128))
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)
    st = _lib.stream_handle()

    if args.nobias:
        bmap = None
    # wide bf16 heads: the forward's bf16 Q / K / V copies (made per step, as in training)
    cb = L_.hstu_attn_bf16_copies_bytes(B, N, H, d, d) if args.bf16 else 0
    copies = torch.empty(cb, dtype=torch.uint8, device=dev) if cb else None

    def fwd():
        if copies is not None:
            _lib.call("hstu_attn_bf16_copies", q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out,
                      n_out, offsets.data_ptr(), B, N, H, d, d, copies.data_ptr(), st)
        extra = (_lib.ptr(copies),) if args.bf16 else ()
        _lib.call("hstu_attn_fwd_bf16" if args.bf16 else "hstu_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out, n_out,
                  offsets.data_ptr(), B, N, L, H, d, d, _lib.ptr(bmap), pos_w.data_ptr(),
                  ts_w.data_ptr(), 128, out.data_ptr(), hv, *extra, st)

    h = torch.randn(rows, n_out, device=dev, generator=g) if args.hepi else None
    hq = h[:, 2 * hv:3 * hv].data_ptr() if args.hepi else None
    hk = h[:, 3 * hv:].data_ptr() if args.hepi else None
    hvp = h[:, hv:2 * hv].data_ptr() if args.hepi else None

    def bwd():
        _lib.call("hstu_attn_bwd_bf16" if args.bf16 else "hstu_attn_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), n_out, n_out,
                  dout.data_ptr(), hv, offsets.data_ptr(), B, N, L, H, d, d, _lib.ptr(bmap),
                  pos_w.data_ptr(), ts_w.data_ptr(), 128, hq, hk, hvp, n_out if args.hepi else 0,
                  dq.data_ptr(), dk.data_ptr(), dvv.data_ptr(), n_out, dpw.data_ptr(),
                  dtw.data_ptr(), *((_lib.ptr(copies),) if args.bf16 else ()), ws.data_ptr(), ws_n, st)

    for _ in range(3):
        fwd()
        bwd()
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    for _ in range(args.iters):
        torch.cuda._sleep(2_000_000)
        if args.only != "bwd":
            fwd()
        if args.only != "fwd":
            bwd()
    torch.cuda.synchronize()
    _lib.timing_enable(False)
    kt = _lib.kernel_times(("attn_fwd", "attn_bwd", "attn_bwd_dkv", "attn_bwd_dq", "attn_bias_reduce", "attn_bf16_copies"))
    fl = flops(B, L, d, H)
    res = {}
    for name, (tot, n) in kt.items():
        if not n:
            continue
        # per call of the op (a form may issue several launches under one name: the
        # wide-head dV / dK launches are both "attn_bwd_dkv")
        per_call = tot / args.iters
        res[name] = {"us_per_call": round(per_call * 1e3, 2), "launches_per_call": n / args.iters,
                     "tflops": round(fl.get(name, 0) / (per_call * 1e-3) / 1e12, 2) if name in fl else None}
    print(json.dumps({"shape": args.shape, "bf16": args.bf16, "B": B, "N": N, "L": L, "d": d, "H": H,
                      "kernels": res}))
    if args.stamp:
        stamp_report(B * H, (L + 127) // 128)


def stamp_report(BH, n_kt):
    """Phase cycles per wave of the wide bf16 key-major launch (last call), by kind and key
    tile: the workgroup -> (bh, key tile, kind) map is xcd_slot's (hstu_attn_bf16w.hip)."""
    import ctypes
    import numpy as np
    raw = ctypes.CDLL(_lib.LIB_PATH)
    per_seq = 2 * n_kt
    grid = ((BH + 7) // 8) * 8 * per_seq
    buf = (ctypes.c_ulonglong * (grid * 48))()
    assert raw.gr_stamp_bw_read(buf, grid * 48) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(grid, 4, 12).astype(np.float64)
    names = ["prologue", "S_dP", "elementwise", "dV_dK", "dS_dts", "barrier", "dpos", "total", "kind", "lookups"]
    rows = {}
    for i in range(grid):
        x, sl = i & 7, i >> 3
        bh, j = (sl // per_seq) * 8 + x, sl % per_seq
        if bh >= BH:
            continue
        rows.setdefault(("K" if j % 2 == 0 else "V", j >> 1), []).append(st[i])
    for key in sorted(rows):
        a = np.stack(rows[key])  # [wgs, 4 waves, 8]
        print(f"{key[0]} kt={key[1]:2d} " + " ".join(
            f"{n}={a[:, :, c].mean():8.0f}" for c, n in enumerate(names) if n != "kind"))


if __name__ == "__main__":
    main()
