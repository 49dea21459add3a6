#!/bin/bash
# r06: EPnP-5 tests on the six-lane SVD, then the kernel trace of the EPnP-5 timing script
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/svd
timeout -k 10 400 python -u -m pytest tests/test_epnp5.py tests/test_shims.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/svd/tests.log 2>&1 || { tail -30 gpurun_out/svd/tests.log; exit 1; }
tail -2 gpurun_out/svd/tests.log
bash scripts/gpu_epnp_trace.sh > gpurun_out/svd/trace.log 2>&1 || { tail -5 gpurun_out/svd/trace.log; exit 1; }
grep -E "hyps|ms-to-best" gpurun_out/ep/log
