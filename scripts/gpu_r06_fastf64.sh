#!/bin/bash
# r06: the range-proven fast f64 root / division cores (RSAC_FAST_F64) -- the EPnP-5 / rvec / shim
# GPU tests on the fast build, then an interleaved ms-to-best + EPnP-5 rate A/B against the base build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RSAC_LIB_PATH=$PWD/build/ab/librsac_fast.so timeout -k 10 600 python -u -m pytest tests/test_epnp5.py tests/test_cv_epnp.py \
  tests/test_rvec.py tests/test_direct.py tests/test_shims.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_fast.log 2>&1
rc=$?; tail -3 gpurun_out/t_fast.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/ms_ab.py build/ab/librsac_base.so build/ab/librsac_fast.so --rounds 3 --hyps 20000 \
  > gpurun_out/ab_fast.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_fast.txt; exit $rc
