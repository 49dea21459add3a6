#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3prof
timeout -k 10 120 python3 scripts/c3_prof.py 2>&1 | grep wall
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o run --output-format csv -- \
    python3 scripts/c3_prof.py > gpurun_out/c3prof/log 2>&1 || exit $?
f=$(find gpurun_out/c3prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('  %-60s calls %5s avg_us %9.1f tot_ms %7.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
"
