#!/bin/bash
# Kernel averages of the C2 bench step (rocprofv3 --kernel-trace --stats), top 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/ks && mkdir -p gpurun_out/ks
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-extras --no-cpu --no-ms-to-best > gpurun_out/ks/log 2>&1 || exit $?
f=$(find gpurun_out/ks -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('  %-60s calls %5s avg_us %9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
