"""normalization="softmax_rel_bias" against "rel_bias" at the C2 (ml-1m) encoder shape:
forward + backward of the HSTU encoder (B = 128, N = 211, D = 50, 4 blocks, fp32), and the
library's per-kernel times of the softmax path.

    python scripts/softmax_micro.py --iters 20
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib  # noqa: E402
from mygenerativerecommenders_amd.hstu import HSTU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    B, N0, out_len, D, blocks = 128, 200, 11, 50, 4
    N = N0 + out_len
    g = torch.Generator().manual_seed(0)
    lengths = torch.randint(N0 // 2, N0 + 1, (B,), generator=g).cuda()
    x = torch.randn(B, N, D, generator=g).cuda()
    ts = (10**9 + torch.cumsum(torch.randint(1, 100000, (B, N), generator=g), 1)).cuda()
    res = {"B": B, "N": N, "D": D, "blocks": blocks}
    for norm in ("rel_bias", "softmax_rel_bias"):
        torch.manual_seed(1)
        enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
                   item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
                   attention_dim=D, normalization=norm, linear_config="uvqk",
                   linear_activation="silu", linear_dropout_rate=0.2,
                   attn_dropout_rate=0.0).cuda().train()
        xg = x.clone().requires_grad_(True)

        def step():
            y, _ = enc(lengths, xg, None, {"timestamps": ts})
            y.sum().backward()

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            step()
        e1.record()
        torch.cuda.synchronize()
        res[norm + "_fwd_bwd_ms"] = e0.elapsed_time(e1) / args.iters
        if norm == "softmax_rel_bias":
            _lib.timing_enable(True)
            _lib.kernel_times()
            for _ in range(args.iters):
                step()
            torch.cuda.synchronize()
            kt = _lib.kernel_times(("softmax_attn_fwd", "softmax_attn_bwd", "ln_uvqk_fwd",
                                    "gate_o_fwd", "gate_o_bwd", "ln_uvqk_bwd", "wgrad_partial",
                                    "wgrad_reduce", "rel_bias_fwd", "rel_bias_bwd"))
            _lib.timing_enable(False)
            res["softmax_per_step_device_ms"] = {k: v[0] / args.iters for k, v in kt.items() if v[1]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
