#!/bin/bash
# r06: kernel traces + PMC passes of the location search, the K sweep and the reference-mode EPnP-5
# solve (scripts/gpu_secondary_profile.sh with WORKLOADS), summarised into profiles/pmc_secondary.json
# on the host by scripts/summarize_secondary.py r06
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WORKLOADS="${WORKLOADS:-loc ksweep epnp}" bash scripts/gpu_secondary_profile.sh
