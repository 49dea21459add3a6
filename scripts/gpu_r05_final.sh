#!/bin/bash
# r05 pass: GPU suite + smoke + bench line, then the rocprofv3 kernel trace and PMC passes of the
# bench command (summarised on the host: scripts/summarize_profiles.py r05), the EPnP-5 trace and
# the EPnP-5 kernel trace + PMC passes (gpurun_out/r05prof)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
TAG=r05 PMC=1 bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_epnp_trace.sh || exit $?
bash scripts/gpu_r05_epnp_pmc.sh
