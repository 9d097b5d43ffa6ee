"""times the reference's own HSTU module (CPU fallback ops, no
fbgemm) and the oracle's reference-order restatement side by side in THIS container,
same inputs, same thread count, train mode, fwd + bwd.  The restatement qualifies as
bench.py's CPU proxy when it lands within +-20 % of the reference.

Run here (the reference exists only in the build container):
    python scripts/cpu_proxy_check.py --batch 128 > profiles/r2_cpu_proxy_check.json
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF_SRC = "/root/reference/src"


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def timeit(fn, warmup=2, iters=5):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    sys.path.insert(0, REF_SRC)
    import logging
    logging.disable(logging.CRITICAL)
    from generative_recommenders_pl.models.sequential_encoders.hstu import HSTU as RefHSTU

    import bench
    from oracle import hstu_oracle as O

    B, N0, out_len, D, blocks = args.batch, 200, 11, 50, args.blocks
    N = N0 + out_len
    torch.manual_seed(0)
    ref = RefHSTU(max_sequence_len=N0, max_output_len=out_len, embedding_dim=D,
                  item_embedding_dim=D, num_blocks=blocks, num_heads=1, linear_dim=D,
                  attention_dim=D, normalization="rel_bias", linear_config="uvqk",
                  linear_activation="silu", linear_dropout_rate=0.2,
                  attn_dropout_rate=0.0).train()
    lengths, x, ts, _, dy = bench.make_batch(B, N0, out_len, D, 123, "cpu")

    def ref_step():
        xr = x.clone().requires_grad_(True)
        y, _ = ref(past_lengths=lengths, user_embeddings=xr, valid_mask=None,
                   past_payloads={"timestamps": ts})
        (y * dy).sum().backward()

    st = {k: v.detach().clone().requires_grad_(True) for k, v in ref.state_dict().items()
          if k != "_attn_mask"}
    layers = [O.layer_params_from_state(st, i) for i in range(blocks)]
    cfg = O.HSTUConfig(N=N, D=D, H=1, dqk=D, dv=D)

    def proxy_step():
        xr = x.clone().requires_grad_(True)
        y = O.hstu_forward_reference_order(lengths, xr, ts, cfg, layers, 0.2, True)
        (y * dy).sum().backward()

    # same numbers in eval mode (no dropout) before timing
    ref.eval()
    with torch.no_grad():
        y_ref, _ = ref(past_lengths=lengths, user_embeddings=x, valid_mask=None,
                       past_payloads={"timestamps": ts})
        y_px = O.hstu_forward_reference_order(lengths, x, ts, cfg,
                                              [{k: v.detach() for k, v in l.items()} for l in layers])
    max_err = float((y_ref - y_px).abs().max())
    ref.train()
    t_ref, s_ref = timeit(ref_step, iters=args.iters)
    t_px, s_px = timeit(proxy_step, iters=args.iters)
    print(json.dumps({
        "what": "reference HSTU (CPU fallback ops) vs oracle hstu_forward_reference_order, "
                "fwd+bwd, train mode (dropout 0.2)",
        "config": {"B": B, "N0": N0, "N": N, "D": D, "blocks": blocks},
        "threads": torch.get_num_threads(), "cpu_model": cpu_model(),
        "eval_forward_max_abs_diff": max_err,
        "reference_s_per_iter": t_ref, "reference_seq_per_s": B / t_ref,
        "proxy_s_per_iter": t_px, "proxy_seq_per_s": B / t_px,
        "proxy_over_reference": (B / t_px) / (B / t_ref),
        "samples_s": {"reference": s_ref, "proxy": s_px},
    }))


if __name__ == "__main__":
    main()
