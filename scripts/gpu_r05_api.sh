#!/bin/bash
# r05: host API + kernel timeline of the ms-to-best call (scripts/api_timeline.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/api && mkdir -p gpurun_out/api
for m in "epnp5 opencv" "p3p philox"; do
  d=gpurun_out/api/${m// /_}
  timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -d $d -o run --output-format csv -- \
      python3 scripts/trace_ms_to_best.py $m > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  tail -2 $d.log
  python3 scripts/api_timeline.py $(find $d -name "*kernel_trace.csv" | head -1) $(find $d -name "*hip_api_trace.csv" | head -1) | tee $d.timeline
done
