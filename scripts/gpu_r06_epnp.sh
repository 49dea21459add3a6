#!/bin/bash
# r06: the OpenCV-sequence EPnP-5 (k_cvepnp5_*) and everything that runs it, on the GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_epnp5.py tests/test_rvec.py tests/test_direct.py tests/test_shims.py \
    -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r06_epnp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/r06_epnp_tests.log
exit $rc
