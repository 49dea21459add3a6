#!/bin/bash
# kernel trace of the EPnP-5 timing script (which kernels of the three-launch solve take the time)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/ep && mkdir -p gpurun_out/ep
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ep/kt -o run --output-format csv -- \
    python3 scripts/epnp5_prof.py 20000 3 > gpurun_out/ep/log 2>&1 || { tail -5 gpurun_out/ep/log; exit 1; }
f=$(find gpurun_out/ep/kt -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("  %-50s calls %5s avg_us %9.1f max_us %9.1f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
f=$(find gpurun_out/ep/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
# the last ms-to-best call's kernels (epnp5/philox): every kernel from the last k_cvepnp5_a on
last = max(i for i, r in enumerate(rows) if "k_cvepnp5_a" in r["Kernel_Name"])
t0 = int(rows[last]["Start_Timestamp"])
for r in rows[last:last + 16]:
    print("  %-40s start %8.1f us  dur %8.1f us" % (r["Kernel_Name"][:40], (int(r["Start_Timestamp"]) - t0) / 1e3,
                                                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
