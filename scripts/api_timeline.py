"""Host-API + kernel timeline of the last pnp_ransac call from rocprofv3 --kernel-trace --hip-trace
CSVs (argv[1] = kernel_trace.csv, argv[2] = hip_api_trace.csv): where the wall time goes between
kernels (launch, copies, synchronisation)."""
import csv
import sys

kr = list(csv.DictReader(open(sys.argv[1])))
ar = list(csv.DictReader(open(sys.argv[2])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]) for r in kr)
ev += sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"]) for r in ar)
ev.sort()
# split by >1 ms idle gaps of kernels
ks = sorted(e for e in ev if e[2].startswith("K"))
groups, cur = [], [ks[0]]
for e in ks[1:]:
    if e[0] - cur[-1][1] > 1_000_000:
        groups.append(cur)
        cur = [e]
    else:
        cur.append(e)
groups.append(cur)
g = groups[-2]
t0, t1 = g[0][0] - 150_000, g[-1][1] + 60_000
print(f"kernels {len(g)}, span {(g[-1][1] - g[0][0]) / 1e3:.1f} us, busy {sum(e[1] - e[0] for e in g) / 1e3:.1f} us")
for s, e, n in ev:
    if t0 <= s <= t1:
        print(f"  +{(s - g[0][0]) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  {n}")
