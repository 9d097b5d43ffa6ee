"""Splits the C4 leg's dispatches in a bench.py kernel trace into its phases and writes
per-phase medians (profiles/<tag>_c4_phases.json).  bench.py's C4 leg (D = 50) runs, in
order: 3 warm-up batches, 1 side-stream batch, 1 graph check, the graph-replay timing
(3 + S), the eager timing (3 + S) and the instrumented pass (S batches, each behind a GPU
hold) whose live event times the bench line reports (S = --retrieval-steps).
    python scripts/c4_phases.py gpurun_out/<tag> <tag> [S]"""
import csv
import json
import statistics
import sys

src, tag = sys.argv[1], sys.argv[2]
S = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rows = list(csv.DictReader(open(f"{src}/trace/run_kernel_trace.csv")))
ev = sorted((int(r["Start_Timestamp"]), r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in rows)
# the D = 50 leg's kernels: filter KC = 2 (mips_filter_kernel<1, 2, 8, ...>); its merges
# are the filter-merge dispatches that follow a KC = 2 filter pass
seq, last_kc2 = [], False
for _, name, d in ev:
    if "mips_filter_kernel<1, 2, 8, false>" in name:
        seq.append({"filter": d})
        last_kc2 = True
    elif "mips_filter_kernel<1, 8, 8, false>" in name:
        last_kc2 = False
    elif "mips_filter_merge_kernel" in name and last_kc2 and seq and "merge" not in seq[-1]:
        seq[-1]["merge"] = d
phases = [("warm-up", 3), ("side stream", 1), ("graph check", 1), ("graph timing", 3 + S),
          ("eager timing", 3 + S), ("instrumented (the line's per-kernel times)", S)]
out, i = {"source": f"{src}/trace/run_kernel_trace.csv", "batches": len(seq), "phases": []}, 0
for name, n in phases:
    part = seq[i:i + n]
    i += n
    if not part:
        continue
    out["phases"].append({"phase": name, "batches": len(part),
                          "filter_median_us": round(statistics.median(b["filter"] for b in part) / 1e3, 2),
                          "merge_median_us": round(statistics.median(b.get("merge", 0) for b in part) / 1e3, 2)})
json.dump(out, open(f"profiles/{tag}_c4_phases.json", "w"), indent=1)
print(json.dumps(out, indent=1))
