#!/bin/bash
# r04 EPnP-5 (latency form): the EPnP-5 tests, the timing script and the kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_epnp5.py tests/test_shims.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/r04_epnp_tests.log 2>&1
rc=$?; tail -22 gpurun_out/r04_epnp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 3 || exit $?
bash scripts/gpu_epnp_trace.sh
