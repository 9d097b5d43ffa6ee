"""Summarises one scripts/profile_round.sh run into profiles/.

    python scripts/pmc_summary.py gpurun_out/<tag> <tag>

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per kernel (and launch grid): avg duration, FETCH_SIZE,
                                    WRITE_SIZE and corrected HBM bytes per launch
  profiles/pmc_latest.json          same content; bench.py reads it to fill roofline.traffic

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KB and come from separate --pmc passes; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Kernel names are mapped to the names the library's live timing uses (gr_timing_query).
    python scripts/pmc_summary.py gpurun_out/<tag> <tag> --no-latest   leaves pmc_latest.json
(for profiles of other legs than the headline).
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_MAP = [
    (r"bucket_map_kernel", "bucket_map"),
    # attention launches carrying a layer boundary (ABI 14): the last template flag = OP2
    (r"attn_fwd_bnd_kernel<[^(]*true>", "attn_fwd_bnd"),
    (r"attn_fwd_bnd_kernel<[^(]*false>", "attn_fwd_bnd1"),
    (r"attn_bwd_dq_bnd_kernel<[^(]*true>", "attn_bwd_dq_bnd"),
    (r"attn_bwd_dq_bnd_kernel<[^(]*false>", "attn_bwd_dq_bnd1"),
    (r"wgrad_stream_kernel", "wgrad_partial"),
    (r"ws_reduce_kernel", "wgrad_reduce"),
    (r"rowwave2_kernel<.*RwGateOBwd", "boundary_bwd"),
    (r"rowwave2_kernel", "boundary_fwd"),
    (r"mips_small_select_kernel", "mips_small"),
    (r"current_embeddings_kernel", "current_embeddings"),
    (r"attn_bwd_bf16w_k_kernel|attn_bwd_bf16w_vp_kernel|attn_bwd_bf16_dkv_kernel", "attn_bwd_dkv"),
    (r"attn_bwd_bf16w_dq_kernel|attn_bwd_bf16_dq_kernel", "attn_bwd_dq"),
    (r"attn_fwd_bf16w_kernel|attn_fwd_bf16_kernel", "attn_fwd"),
    (r"attn_bf16w_convert", "attn_bf16_copies"),
    (r"wgrad_partial_(wide|bf16)_kernel", "wgrad_partial"),
    (r"attn_fwd_kernel", "attn_fwd"),
    (r"attn_bwd_fused_kernel", "attn_bwd"),
    (r"attn_bwd_dkv_kernel", "attn_bwd_dkv"),
    (r"attn_bwd_dq_kernel|attn_bwd_dq_ds_kernel", "attn_bwd_dq"),
    (r"bias_grad_reduce_kernel", "attn_bias_reduce"),
    (r"(Op|Rw)LnUvqkBwd", "ln_uvqk_bwd"),
    (r"(Op|Rw)LnUvqk", "ln_uvqk_fwd"),
    (r"(Op|Rw)GateOBwd", "gate_o_bwd"),
    (r"(Op|Rw)GateO", "gate_o_fwd"),
    (r"wgrad_partial_kernel", "wgrad_partial"),
    (r"wgrad_reduce_kernel", "wgrad_reduce"),
    (r"mips_pack_kernel", "mips_pack"),
    (r"mips_select_kernel|mips_scoreall_kernel", "mips_select"),
    (r"mips_filter_merge_kernel", "mips_merge"),
    (r"mips_filter_kernel<[^>]*true>", "mips_sample"),
    (r"mips_filter_kernel<[^>]*false>", "mips_filter"),
    (r"mips_tau_kernel", "mips_tau"),
    # the exact path's merge: gated on the filter path's flag (C4), timed as mips_merge_fallback
    (r"mips_merge_kernel", "mips_merge_fallback"),
    (r"cumsum_kernel", "cumsum"),
    (r"encoder_prologue_kernel", "encoder_prologue"),
    (r"weight_image_kernel", "weight_images"),
    (r"bf16_scale_add", "bf16_scale_add"),
    (r"adamw_kernel", "adamw"),
    (r"dense_to_jagged_kernel", "dense_to_jagged"),
    (r"jagged_to_padded_kernel", "jagged_to_padded"),
]


def short_name(full: str):
    for pat, name in _MAP:
        if re.search(pat, full):
            # bf16-operand kernels get their own entries (same timing names, same grids)
            return name + "_bf16" if re.search(r"bf16|wide_kernel<true>", full) else name
    return None


def _counters(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        n = short_name(r["Kernel_Name"])
        if n is None:
            continue
        acc[(n, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return acc


def _durations(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = short_name(r["Kernel_Name"])
        if n is None:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc[(n, grid)].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return acc


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = _counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = _counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    dur = _durations(os.path.join(src, "trace", "run_kernel_trace.csv"))
    per_grid = {}
    for key in sorted(set(fetch) | set(write) | set(dur)):
        f = fetch.get(key, [])
        w = write.get(key, [])
        d = dur.get(key, [])
        fa = sum(f) / len(f) if f else None
        wa = sum(w) / len(w) if w else None
        per_grid[f"{key[0]}@grid{key[1]}"] = {
            "kernel": key[0], "grid": key[1], "launches_traced": len(d),
            "avg_ms": sum(d) / len(d) if d else None,
            "median_ms": sorted(d)[len(d) // 2] if d else None,
            "min_ms": min(d) if d else None,
            "fetch_kb": fa, "write_kb": wa,
            "hbm_bytes_per_launch": (2 * fa + wa) * 1024 if fa is not None and wa is not None else None,
        }
    # per kernel name: the grid with the most launches (the training-step shape)
    kernels = {}
    for ent in per_grid.values():
        cur = kernels.get(ent["kernel"])
        if cur is None or ent["launches_traced"] > cur["launches_traced"]:
            kernels[ent["kernel"]] = ent
    out = {"source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                     "separate passes; hbm = (2*FETCH+WRITE) KB*1024, gfx950 FETCH correction)",
           "kernels": kernels, "per_grid": per_grid}
    for name in (f"{tag}_pmc.json",) + (() if "--no-latest" in sys.argv else ("pmc_latest.json",)):
        with open(os.path.join(prof, name), "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
    for k, e in sorted(kernels.items()):
        hb = e["hbm_bytes_per_launch"]
        print(f"{k:18s} grid={e['grid']:>9d} avg_ms={e['avg_ms'] or 0:8.4f} "
              f"median_ms={e['median_ms'] or 0:8.4f} "
              f"hbm_MB={(hb or 0) / 1e6:9.3f}")


if __name__ == "__main__":
    main()
