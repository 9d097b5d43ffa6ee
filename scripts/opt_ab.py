"""Optimizer-step A/B on one box, interleaved: the C2 encoder step (fp32, B = 128, AdamW)
and the C3 bf16 step (Muon + AdamW) with AdamW as optim.FlatAdamW or torch's fused
AdamW, and Muon's Newton-Schulz combines as gr_bf16_scale_add or the torch ops.
    python scripts/opt_ab.py [--steps 20] [--rounds 2]
One JSON line per run."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mygenerativerecommenders_amd import muon  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--c3-steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for rnd in range(args.rounds):
        for adamw in ("flat", "torch"):
            bench.ADAMW = adamw
            r = bench.encoder_leg(128, 200, 11, 50, 4, 1, args.steps, 5, dev, 1, 1000)
            print(json.dumps({"round": rnd, "leg": "c2", "adamw": adamw, "seq_per_s": r["value"],
                              "ms_per_step": r["ms_per_step"]}), flush=True)
        for adamw, fused in (("flat", True), ("torch", True), ("torch", False)):
            bench.ADAMW = adamw
            muon.FUSED_COMBINE = fused
            r = bench.encoder_leg(32, 2048, 11, 256, 8, 1, args.c3_steps, 2, dev, 1, 3000,
                                  muon=True, bf16=True)
            print(json.dumps({"round": rnd, "leg": "c3_bf16", "adamw": adamw, "muon_fused": fused,
                              "seq_per_s": r["value"], "ms_per_step": r["ms_per_step"]}), flush=True)
        muon.FUSED_COMBINE = True


if __name__ == "__main__":
    main()
