#!/bin/bash
# r04 EPnP-5: the minimal-solver tests on the three-launch form, then its timing against the
# one-kernel form (RSAC_EPNP5_SPLIT=0): fixed budget and the reference-mode ms-to-best
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_epnp5.py tests/test_shims.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/r04_epnp_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r04_epnp_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== split (three launches)"; timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 3 || exit $?
echo "== one kernel"; RSAC_EPNP5_SPLIT=0 timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 2
rc=$?; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_epnp_trace.sh
