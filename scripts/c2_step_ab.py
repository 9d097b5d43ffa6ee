"""The C2 encoder training step (fp32, B = 128, 4 blocks, AdamW; captured graphs) once:
ms per step and the per-kernel device time per step (live events, an eager re-run).
Used with scripts/ab_micro.sh to A/B prebuilt libraries.   python scripts/c2_step_ab.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

r = bench.encoder_leg(128, 200, 11, 50, 4, 1, 50, 10, torch.device("cuda", 0), 1, 1000, instrument=True)
k = {n: round(v * 1000, 1) for n, v in r["kernel_per_step_ms"].items() if n.startswith("wgrad")}
print(json.dumps({"ms_per_step": r["ms_per_step"], "seq_per_s": r["value"], "wgrad_us": k}))
