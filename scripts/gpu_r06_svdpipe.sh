#!/bin/bash
# r06: the SVD's norm sums pipelined into the next step: EPnP-5 tests, then an interleaved A/B
# against the previous build (ms-to-best in the reference mode, the 20k fixed-budget rate)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sp
timeout -k 10 400 python -u -m pytest tests/test_epnp5.py tests/test_cv_epnp.py tests/test_shims.py tests/test_direct.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/sp/tests.log 2>&1 || { tail -30 gpurun_out/sp/tests.log; exit 1; }
tail -2 gpurun_out/sp/tests.log
timeout -k 10 600 python3 scripts/ms_ab.py build/ab/librsac_old.so build/ab/librsac_new.so --rounds 3 --calls 20 --hyps 20000 \
    > gpurun_out/sp/ab.log 2>&1 || { tail -10 gpurun_out/sp/ab.log; exit 1; }
tail -4 gpurun_out/sp/ab.log
