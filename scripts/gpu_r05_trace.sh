#!/bin/bash
# r05: kernel timeline of the reference-mode ms-to-best call (EPnP-5, OpenCV sampler) and of P3P
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/tr && mkdir -p gpurun_out/tr
for m in "epnp5 opencv" "p3p philox"; do
  d=gpurun_out/tr/${m// /_}
  timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
      python3 scripts/trace_ms_to_best.py $m > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  tail -2 $d.log
  python3 scripts/timeline.py $(find $d -name "*kernel_trace.csv" | head -1) | tee $d.timeline
done
