"""Per-call kernel timeline from a rocprofv3 kernel_trace.csv (calls separated by >1 ms gaps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
groups, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - cur[-1][1] > 1_000_000:
        groups.append(cur)
        cur = [e]
    else:
        cur.append(e)
groups.append(cur)
for g in groups[-2:]:
    t0 = g[0][0]
    print(f"--- call: span {(g[-1][1] - t0) / 1e3:.1f} us, kernels {len(g)}, busy {sum(e[1] - e[0] for e in g) / 1e3:.1f} us")
    for s, e, n in g:
        print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  {n[:70]}")
