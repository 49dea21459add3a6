#!/bin/bash
# r05 EPnP-5: the minimal-solver and direct/round-trip tests, then the timing (fixed 20k budget and
# reference-mode ms-to-best) and a kernel trace of the same script
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_epnp5.py tests/test_rvec.py tests/test_shims.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/r05_epnp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05_epnp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 3 || exit $?
bash scripts/gpu_epnp_trace.sh
