#!/bin/bash
# r05 pass: GPU suite + smoke + bench line, then the rocprofv3 kernel trace and PMC passes of the
# bench command (summarised on the host: scripts/summarize_profiles.py r05) and the EPnP-5 trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
TAG=r05 PMC=1 bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_epnp_trace.sh
