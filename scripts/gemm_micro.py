"""Micro-benchmark of the STU projection kernels (row-panel GEMMs and weight gradients)
at the C2 / C3 shapes, timed by the library's live event timing.

    python scripts/gemm_micro.py --shape c2 --iters 50
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib  # noqa: E402

SHAPES = {"c2": (128, 211, 200, 50), "c3": (32, 2059, 2048, 256)}  # B, N, L, D (h=1, d=D)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--wgrad-only", action="store_true", help="only the grouped weight gradients")
    ap.add_argument("--wgrad-rows", type=int, default=0, help="GR_OPT_WGRAD_ROWS (0 = auto)")
    ap.add_argument("--bf16", action="store_true", help="bf16 weight gradients (gr_wgrad2_bf16)")
    ap.add_argument("--bf16-panels", action="store_true", help="bf16 projection GEMMs (*_bf16)")
    ap.add_argument("--panel-vec", type=int, default=1, help="GR_OPT_PANEL_VEC")
    ap.add_argument("--with-wgrad", action="store_true", help="also the per-matrix gr_wgrad calls")
    args = ap.parse_args()
    _lib.set_option("WGRAD_ROWS", args.wgrad_rows)  # before the workspace queries
    _lib.set_option("PANEL_VEC", args.panel_vec)
    sfx = "_bf16" if args.bf16_panels else ""
    B, N, L, D = SHAPES[args.shape]
    hv = D
    n_out = 4 * D
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    cap = B * N
    rows = B * L
    offsets = torch.arange(0, B + 1, device=dev, dtype=torch.int64) * L
    x = torch.randn(cap, D, device=dev, generator=g)
    w_uvqk = torch.randn(D, n_out, device=dev, generator=g) * 0.02
    w_o = torch.randn(D, hv, device=dev, generator=g) * 0.1
    b_o = torch.randn(D, device=dev, generator=g) * 0.1
    x_stats = torch.empty(cap, 2, device=dev)
    h_pre = torch.empty(cap, n_out, device=dev)
    uvqk = torch.empty(cap, n_out, device=dev)
    attn = torch.randn(cap, hv, device=dev, generator=g)
    attn_stats = torch.empty(cap, 2, device=dev)
    o_in = torch.empty(cap, hv, device=dev)
    y = torch.empty(cap, D, device=dev)
    dy = torch.randn(cap, D, device=dev, generator=g)
    d_uvqk = torch.randn(cap, n_out, device=dev, generator=g)
    d_attn = torch.empty(cap, hv, device=dev)
    dx = torch.empty(cap, D, device=dev)
    seed_off = torch.zeros(1, dtype=torch.int64, device=dev)
    dWo = torch.empty(D, hv, device=dev)
    dbo = torch.empty(D, device=dev)
    dWu = torch.empty(D, n_out, device=dev)
    L_ = _lib.lib()
    ws1 = L_.gr_wgrad_workspace_size(cap, D, hv)
    ws2 = L_.gr_wgrad_workspace_size(cap, D, n_out)
    ws3 = L_.gr_wgrad2_workspace_size(cap, D, n_out, D, hv)
    ws = torch.empty(max(ws1, ws2, ws3, 4), dtype=torch.uint8, device=dev)
    st = _lib.stream_handle()
    P = lambda t: t.data_ptr()  # noqa: E731

    def run_w():
        _lib.call("gr_wgrad2_bf16" if args.bf16 else "gr_wgrad2", P(x), D, P(x_stats), P(d_uvqk), n_out, D, n_out, P(dWu), None,
                  P(dy), D, None, P(o_in), hv, D, hv, P(dWo), P(dbo), P(offsets), B, cap,
                  P(ws), ws.numel(), st)

    def run():
        if args.wgrad_only:
            return run_w()
        _lib.call("hstu_ln_uvqk_fwd" + sfx, P(x), D, P(offsets), B, cap, D, P(w_uvqk), n_out, 1e-6, 1,
                  P(x_stats), P(h_pre), P(uvqk), n_out, st)
        _lib.call("hstu_gate_o_fwd" + sfx, P(uvqk), n_out, P(attn), hv, P(offsets), B, cap, hv, D,
                  P(w_o), P(b_o), P(x), D, 1e-6, 0.2, 7, P(seed_off), P(attn_stats), P(o_in),
                  P(y), D, st)
        _lib.call("hstu_gate_o_bwd" + sfx, P(dy), D, P(offsets), B, cap, hv, D, P(w_o), P(uvqk),
                  n_out, P(attn), hv, P(attn_stats), P(h_pre), n_out, 0.2, 7, P(seed_off),
                  P(d_uvqk), n_out, P(d_attn), hv, st)
        if args.with_wgrad:
            _lib.call("gr_wgrad", P(dy), D, None, P(o_in), hv, P(offsets), B, cap, D, hv, P(dWo),
                      P(dbo), P(ws), ws.numel(), st)
            _lib.call("gr_wgrad", P(x), D, P(x_stats), P(d_uvqk), n_out, P(offsets), B, cap, D,
                      n_out, P(dWu), None, P(ws), ws.numel(), st)
        _lib.call("hstu_ln_uvqk_bwd" + sfx, P(d_uvqk), n_out, P(offsets), B, cap, D, n_out, P(w_uvqk),
                  P(x), D, P(x_stats), P(dy), D, P(dx), D, st)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    for _ in range(args.iters):
        torch.cuda._sleep(2_000_000)
        run()
    torch.cuda.synchronize()
    _lib.timing_enable(False)
    names = ("ln_uvqk_fwd", "gate_o_fwd", "gate_o_bwd", "ln_uvqk_bwd", "wgrad_partial",
             "wgrad_reduce")
    kt = _lib.kernel_times(names)
    f4 = 4
    bytes_ = {
        "ln_uvqk_fwd": rows * (D + 2 * n_out + 2) * f4,
        "gate_o_fwd": rows * (hv + hv + D + 2 + hv + D) * f4,
        "gate_o_bwd": rows * (D + hv + hv + 2 + hv + hv + hv) * f4,
        "ln_uvqk_bwd": rows * (n_out + D + 2 + D + D) * f4,
        "wgrad_partial": rows * (D + hv + D + n_out + 2) * f4 / 2,
    }
    res = {}
    for n, (tot, c) in kt.items():
        if not c:
            continue
        avg = tot / c
        res[n] = {"avg_us": round(avg * 1e3, 2), "launches_per_iter": c // args.iters}
        if n in bytes_:
            res[n]["GBps"] = round(bytes_[n] / (avg * 1e-3) / 1e9, 1)
    print(json.dumps({"shape": args.shape, "rows": rows, "bf16_panels": args.bf16_panels,
                      "panel_vec": args.panel_vec, "kernels": res}))


if __name__ == "__main__":
    main()
