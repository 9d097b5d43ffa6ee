"""Micro-benchmark of the encoder's grouped weight gradients (gr_wgrad_multi) at C2: 4
layers x (_uvqk 50 x 200 over LN(x), _o 50 x 50 over dy + bias), B=128, L=200.
GR_HSTU_LIB selects a variant build (scripts/build_variant.sh).

    python scripts/wgrad_micro.py --iters 50 [--opt WGRAD_STREAM=0]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--len", type=int, default=200)
    ap.add_argument("--dim", type=int, default=50)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    for o in args.opt:
        k, v = o.split("=")
        _lib.set_option(k, int(v))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    B, Lq, D = args.batch, args.len, args.dim
    n_out = 4 * D
    cap = B * (Lq + 11)
    offs = (torch.arange(B + 1, dtype=torch.int64) * Lq).to(dev)
    keep, desc = [], []
    for _ in range(args.layers):
        x = torch.randn(cap, D, device=dev, generator=g)
        st = torch.stack([x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-6)], 1).contiguous()
        dh = torch.randn(cap, n_out, device=dev, generator=g)
        dy = torch.randn(cap, D, device=dev, generator=g)
        oin = torch.randn(cap, D, device=dev, generator=g)
        cu = torch.empty(D, n_out, device=dev)
        co = torch.empty(D, D, device=dev)
        cb = torch.empty(D, device=dev)
        keep += [x, st, dh, dy, oin, cu, co, cb]
        desc.append([x.data_ptr(), D, st.data_ptr(), dh.data_ptr(), n_out, D, n_out, cu.data_ptr(), 0])
        desc.append([dy.data_ptr(), D, 0, oin.data_ptr(), D, D, D, co.data_ptr(), cb.data_ptr()])
    d = np.ascontiguousarray(np.array(desc, dtype=np.int64))
    L = _lib.lib()
    ws_n = L.gr_wgrad_multi_workspace_size(d.ctypes.data, len(desc), cap)
    ws = torch.empty(max(ws_n, 4), dtype=torch.uint8, device=dev)

    def run():
        _lib.call("gr_wgrad_multi", d.ctypes.data, len(desc), offs.data_ptr(), B, cap, 0,
                  ws.data_ptr(), ws_n, _lib.stream_handle())
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    for _ in range(args.iters):
        run()
    torch.cuda.synchronize()
    _lib.timing_enable(False)
    kt = _lib.kernel_times()
    out = {n: round(t / c * 1e3, 2) for n, (t, c) in kt.items() if c}
    rows = B * Lq
    gb = args.layers * rows * (2 * D + n_out + D + 2) * 4 / 1e9
    out["tag"] = args.tag
    out["operand_GB"] = round(gb, 4)
    out["partial_TBps"] = round(gb / (out.get("wgrad_partial", 1e9) * 1e-6) / 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
