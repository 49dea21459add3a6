"""Kernel timeline of bench.py's timed loop from a rocprofv3 kernel_trace.csv: the longest run of
back-to-back launches (gaps < 200 us), printed for its last two steps, plus the idle time between
consecutive kernels summed per step."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
groups, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - cur[-1][1] > 200_000:
        groups.append(cur)
        cur = [e]
    else:
        cur.append(e)
groups.append(cur)
g = max(groups, key=len)
t0 = g[0][0]
span = (g[-1][1] - t0) / 1e3
busy = sum(e[1] - e[0] for e in g) / 1e3
print(f"longest run: {len(g)} kernels, span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us")
n_score = sum(1 for e in g if "score" in e[2])
print(f"scoring launches in it: {n_score}; idle per step {(span - busy) / max(1, n_score):.1f} us")
tail = g[-2 * max(1, len(g) // max(1, n_score)):]
prev = None
for s, e, n in tail:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"  gap {gap:6.1f} us  dur {(e - s) / 1e3:7.1f} us  {n[:80]}")
    prev = e
