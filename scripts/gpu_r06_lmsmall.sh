#!/bin/bash
# r06: the LM's cost-only pass for steps below the step criterion: refit / LO tests, then an
# interleaved A/B against the previous build (ms-to-best P3P / reference mode, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lms
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_rvec.py tests/test_epnp.py -m gpu -x -q -k "lo or LO or local or refit or refine or lm" \
    --timeout 120 --timeout-method thread > gpurun_out/lms/tests.log 2>&1 || { tail -30 gpurun_out/lms/tests.log; exit 1; }
tail -2 gpurun_out/lms/tests.log
timeout -k 10 600 python3 scripts/ms_ab.py build/ab/librsac_old.so build/ab/librsac_new.so --rounds 3 --calls 20 --c5 \
    > gpurun_out/lms/ab.log 2>&1 || { tail -10 gpurun_out/lms/ab.log; exit 1; }
tail -4 gpurun_out/lms/ab.log
