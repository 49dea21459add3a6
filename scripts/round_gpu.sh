#!/bin/bash
# Round pass on one GPU box: parity tests + smoke + bench, then the rocprof kernel-trace
# summary and the PMC passes (FETCH_SIZE, WRITE_SIZE, VALU issue, waits) of the same bench
# command, summarised into profiles/ (TAG, default r03).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
PMC=1 bash scripts/gpu_profile.sh || exit $?
python3 scripts/summarize_profiles.py "${TAG:-r03}" > gpurun_out/summary.log 2>&1; tail -8 gpurun_out/summary.log
