#!/bin/bash
# r05: the EPnP-5 path's kernel trace and PMC passes (scripts/gpu_r04_epnp_pmc.sh), summarised into
# gpurun_out/r05prof/epnp_pmc.json (copied to profiles/r05 afterwards), plus the kernel stats of the
# 20k-hypothesis timing script
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r04_epnp_pmc.sh || exit 1
O=gpurun_out/r05prof
mkdir -p $O
python3 scripts/summarize_epnp_pmc.py r05 $O/epnp_pmc.json || exit 1
f=$(find gpurun_out/epmc/kt -name "*kernel_stats.csv" | head -1)
cp "$f" $O/epnp5_prof_kernel_stats.csv
cp gpurun_out/epmc/kt.log $O/epnp5_prof.txt
python3 - "$f" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("  %-50s calls %5s avg_us %9.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
