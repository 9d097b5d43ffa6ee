"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace (graph replay or
eager): python scripts/gaps.py <kernel_trace.csv> [--last N]
Prints the total busy / idle time over the last N dispatches and the largest gaps by
(previous kernel -> next kernel)."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=2000)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ev = ev[-a.last:]
short = lambda n: n.split("(")[0].replace("void ", "").replace("gr::", "")[:60]  # noqa: E731
busy = sum(e - s for s, e, _ in ev)
span = ev[-1][1] - ev[0][0]
gaps = collections.defaultdict(lambda: [0, 0])
for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
    g = s1 - e0
    k = (short(n0), short(n1))
    gaps[k][0] += g
    gaps[k][1] += 1
print(f"dispatches {len(ev)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us  idle {(span-busy)/1e3:.1f} us")
for k, (g, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:25]:
    print(f"{g/1e3:9.1f} us  {c:5d} x  avg {g/c/1e3:6.2f}  {k[0]} -> {k[1]}")
