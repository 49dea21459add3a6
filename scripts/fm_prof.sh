#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fmprof
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fmprof -o run --output-format csv -- \
    python3 scripts/fm_prof.py > gpurun_out/fmprof/log 2>&1 || exit $?
f=$(find gpurun_out/fmprof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('  %-60s calls %5s avg_us %9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
