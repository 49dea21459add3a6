#!/bin/bash
# r06: the refit's wave-0 solve step (bit-exact tests), then phase stamps of the refit and of the
# EPnP-5 SVD sweeps (RSAC_TRACE build in /tmp) on the C2 ms-to-best call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lm
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_direct.py tests/test_epnp.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/lm/tests.log 2>&1 || { tail -20 gpurun_out/lm/tests.log; exit 1; }
tail -2 gpurun_out/lm/tests.log
bash scripts/trace_build.sh scripts/trace_refit.py > gpurun_out/lm/trace_refit.log 2>&1 || { tail -5 gpurun_out/lm/trace_refit.log; exit 1; }
export RSAC_LIB_PATH=/tmp/rsac_trace/code-reproduction-ransac_amd/rsac/librsac.so
timeout -k 10 120 python3 scripts/trace_ms_to_best.py p3p philox > gpurun_out/lm/trace_p3p.log 2>&1 || { tail -5 gpurun_out/lm/trace_p3p.log; exit 1; }
timeout -k 10 120 python3 scripts/trace_ms_to_best.py epnp5 opencv \
    > gpurun_out/lm/trace_epnp.log 2>&1 || { tail -5 gpurun_out/lm/trace_epnp.log; exit 1; }
grep "^call" gpurun_out/lm/trace_p3p.log | tail -3
