"""C3 bf16 leg A/B: the encoder training step at ml-20m width (B=32, N=2048, d=256,
8 blocks, Muon + AdamW) in bf16 mode with the bf16-activation layout (ops.A16) on and off.
    python scripts/c3_ab.py [--steps 5] [--only a16|f32act]
Prints one JSON line per mode: ms per step and the per-kernel device time per step."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mygenerativerecommenders_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    from mygenerativerecommenders_amd import _lib
    modes = [("a16", True, 1), ("a16_vec2", True, 2), ("f32act", False, 1)]
    for name, a16, pv in modes:
        if args.only and args.only != name:
            continue
        ops.A16 = a16
        _lib.set_option("PANEL_VEC", pv)
        r = bench.encoder_leg(32, 2048, 11, 256, 8, 1, args.steps, 2, dev, 1, 3000,
                              instrument=True, muon=True, bf16=True)
        kps = {k: round(v, 4) for k, v in sorted(r["kernel_per_step_ms"].items(), key=lambda kv: -kv[1])}
        print(json.dumps({"mode": name, "seq_per_s": r["value"], "ms_per_step": r["ms_per_step"],
                          "device_ms_per_step": round(sum(kps.values()), 3), "kernels": kps}), flush=True)


if __name__ == "__main__":
    main()
