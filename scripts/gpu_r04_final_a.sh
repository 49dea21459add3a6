#!/bin/bash
# r04 final pass, part A: GPU suite + smoke + bench line, then the rocprofv3 kernel trace and the
# PMC passes of the bench command (summarised afterwards on the host: summarize_profiles.py r04)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
TAG=r04 PMC=1 bash scripts/gpu_profile.sh
