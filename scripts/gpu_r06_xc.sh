#!/bin/bash
# r06: the sc path centring on the fly (no stored XC/YC/ZC): the GPU suite, then an interleaved
# A/B against the previous build on C2 and C3 (scripts/mf_ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/xc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/xc/tests.log 2>&1 \
    || { tail -30 gpurun_out/xc/tests.log; exit 1; }
tail -2 gpurun_out/xc/tests.log
timeout -k 10 600 python3 scripts/mf_ab.py build/ab/librsac_old.so build/ab/librsac_new.so --rounds 3 --c3 30 \
    > gpurun_out/xc/ab.log 2>&1 || { tail -10 gpurun_out/xc/ab.log; exit 1; }
tail -8 gpurun_out/xc/ab.log
