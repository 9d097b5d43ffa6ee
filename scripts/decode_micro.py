"""Cached-decoding step (HSTU.forward with delta_x_offsets / cache) at the C2 (ml-1m) and
C3-width (ml-20m-like) shapes: wall time per step against the full no-grad forward of the
same batch, the library's per-kernel times, and hstu_decode_attn's achieved HBM rate
from its algorithmic bytes (per delta row and head: the cached keys 0..p and their
values, 4 (p + 1) (dqk + dv) bytes, plus 8 (p + 1) timestamp bytes with the bias).

    python scripts/decode_micro.py --shape c2 --iters 50
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mygenerativerecommenders_amd import _lib  # noqa: E402
from mygenerativerecommenders_amd.hstu import HSTU  # noqa: E402

SHAPES = {  # B, N0, out_len, D (= dqk = dv), blocks
    "c2": (128, 200, 11, 50, 4),
    "c3": (32, 2048, 11, 256, 8),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    B, N0, out_len, D, blocks = SHAPES[args.shape]
    N = N0 + out_len
    dev = "cuda"
    torch.manual_seed(0)
    enc = HSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D, item_embedding_dim=D,
               num_blocks=blocks, num_heads=1, linear_dim=D, attention_dim=D,
               normalization="rel_bias", linear_config="uvqk", linear_activation="silu",
               linear_dropout_rate=0.2, attn_dropout_rate=0.0).to(dev).eval()
    g = torch.Generator().manual_seed(1)
    lengths = torch.full((B,), N0, dtype=torch.int64)  # every sequence at max length
    x = torch.randn(B, N, D, generator=g)
    ts = 10**9 + torch.cumsum(torch.randint(1, 100000, (B, N), generator=g), 1)
    lengths, x, ts = lengths.to(dev), x.to(dev), ts.to(dev)
    pay = {"timestamps": ts}
    with torch.no_grad():
        _, states = enc(lengths, x, None, pay, return_cache_states=True)
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), lengths.cumsum(0)])
    pos = lengths - 1  # re-encode each sequence's last item
    delta = (offsets[:-1] + pos, pos)

    def step():
        enc(lengths, x, None, pay, delta_x_offsets=delta, cache=states)

    def full():
        enc(lengths, x, None, pay)

    res = {"shape": args.shape, "B": B, "N": N, "D": D, "blocks": blocks}
    with torch.no_grad():
        for name, fn in (("decode_step", step), ("full_forward", full)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name + "_ms"] = e0.elapsed_time(e1) / args.iters
        _lib.timing_enable(True)
        _lib.kernel_times()
        for _ in range(args.iters):
            step()
        kt = _lib.kernel_times(("decode_attn", "decode_scatter", "rows_copy", "ln_uvqk_fwd",
                                "gate_o_fwd", "dense_to_jagged", "jagged_to_padded", "cumsum"))
        _lib.timing_enable(False)
    per_step = {k: v[0] / args.iters for k, v in kt.items() if v[1]}
    res["per_step_device_ms"] = per_step
    attn_ms = kt["decode_attn"][0] / (args.iters * blocks)  # per call: chunk + reduce launches
    p = pos.float().cpu()
    bytes_launch = float(((p + 1) * (2 * D * 4 + 8)).sum() + B * (2 * D * 4))
    res["per_step_device_ms_total"] = sum(per_step.values())
    res["decode_attn"] = {"avg_call_ms": attn_ms, "launches_per_call": kt["decode_attn"][1] / (args.iters * blocks), "algorithmic_bytes": bytes_launch,
                          "achieved_GBs": bytes_launch / attn_ms / 1e6,
                          "frac_of_hbm": bytes_launch / attn_ms / 1e6 / HBM_PEAK_GBS}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
