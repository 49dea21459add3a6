"""Summarise gpurun_out/pmc_valu (scripts/pmc_valu.sh): per scoring kernel, the mean of each
counter over its launches, the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall) and VALU issue
per SIMD-cycle."""
import collections
import csv
import glob
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else glob.glob("gpurun_out/pmc_valu/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter -> sum
dur = {}
for r in rows:
    if "score" not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])
    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    if "End_Timestamp" in r and r.get("Start_Timestamp"):
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (k, d), c in per.items():
    for n, v in c.items():
        agg[k][n].append(v)
    if (k, d) in dur:
        agg[k]["wall_s"].append(dur[(k, d)])
for k, c in agg.items():
    m = {n: statistics.mean(v) for n, v in c.items()}
    print(k)
    for n in sorted(m):
        print(f"  {n:24s} {m[n]:.4g}")
    if "GRBM_GUI_ACTIVE" in m and m.get("wall_s"):
        clk = m["GRBM_GUI_ACTIVE"] / 8 / m["wall_s"]
        print(f"  effective clock          {clk / 1e9:.3f} GHz")
        if "SQ_INSTS_VALU" in m:
            simd_cycles = 1024 * m["GRBM_GUI_ACTIVE"] / 8
            print(f"  VALU wave-instr / SIMD-cycle {m['SQ_INSTS_VALU'] / simd_cycles:.3f} (2-cycle issue: 0.5 max)")
