#!/bin/bash
# rocprofv3 kernel-trace summary of the C2 scoring path for the variants given (default 23 30)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/mxprof
for v in ${VARIANTS:-23 30}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mxprof/v$v -o run --output-format csv -- \
      python3 scripts/mx_prof.py $v 10 > gpurun_out/mxprof/v$v.log 2>&1 || exit $?
  tail -1 gpurun_out/mxprof/v$v.log
  f=$(find gpurun_out/mxprof/v$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('  %-60s calls %5s avg_us %8.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
done
