#!/bin/bash
# Round pass on one GPU box: parity tests + smoke + bench, then the rocprof kernel-trace
# summary and the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the same bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
PMC=1 bash scripts/gpu_profile.sh || exit $?
python3 scripts/summarize_profiles.py "${TAG:-r01}" > gpurun_out/summary.log 2>&1; tail -4 gpurun_out/summary.log
