"""Kernel / host-API timeline of the last call of a workload from rocprofv3 --kernel-trace --hip-trace CSVs:
    python3 scripts/loc_timeline.py kernel_trace.csv hip_api_trace.csv [first-kernel marker, default k_loc_pos2]"""
import csv, sys
kr = list(csv.DictReader(open(sys.argv[1])))
ar = list(csv.DictReader(open(sys.argv[2])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50]) for r in kr)
# last call = kernels after the last k_loc_pos2
marker = sys.argv[3] if len(sys.argv) > 3 else "k_loc_pos2"
idx = [i for i, k in enumerate(ks) if marker in k[2]]
a = idx[-1]
b = len(ks)
g = ks[a:b]
t0, t1 = g[0][0], g[-1][1]
busy = sum(e - s for s, e, n in g)
print(f"last call: {len(g)} kernels, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
from collections import defaultdict
d = defaultdict(lambda: [0, 0])
for s, e, n in g:
    d[n][0] += 1; d[n][1] += e - s
for n, (c, t) in sorted(d.items(), key=lambda x: -x[1][1]):
    print(f"  {n:50s} {c:4d} x  {t / 1e3:8.1f} us")
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in ar)
api = [x for x in api if t0 - 3_000_000 <= x[0] <= t1]
da = defaultdict(lambda: [0, 0])
for s, e, n in api:
    da[n][0] += 1; da[n][1] += e - s
print("host API in [span - 3 ms, span end]:")
for n, (c, t) in sorted(da.items(), key=lambda x: -x[1][1])[:10]:
    print(f"  {n:40s} {c:5d} x {t / 1e3:9.1f} us")
# gaps between consecutive kernels > 20 us
gaps = [(g[i + 1][0] - g[i][1], g[i][2], g[i + 1][2]) for i in range(len(g) - 1)]
gaps.sort(reverse=True)
print("largest kernel gaps:")
for gp, x, y in gaps[:12]:
    print(f"  {gp / 1e3:8.1f} us  after {x} -> {y}")
