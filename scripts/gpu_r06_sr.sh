#!/bin/bash
# r06: small rounds of long problems on the MFMA scorer: the GPU suite, then an interleaved A/B
# against the previous build (ms-to-best P3P / reference mode, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sr/tests.log 2>&1 \
    || { tail -30 gpurun_out/sr/tests.log; exit 1; }
tail -2 gpurun_out/sr/tests.log
timeout -k 10 600 python3 scripts/ms_ab.py build/ab/librsac_old.so build/ab/librsac_new.so --rounds 3 --calls 20 --c5 \
    > gpurun_out/sr/ab.log 2>&1 || { tail -10 gpurun_out/sr/ab.log; exit 1; }
tail -4 gpurun_out/sr/ab.log
