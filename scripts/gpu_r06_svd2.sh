#!/bin/bash
# r06: 12 x 12 SVD lanes m-major (lane = 10 m + g: fewer LDS bank conflicts) and the register
# JacobiSVD's skip test by the fast root: EPnP / rvec / shim GPU tests on the combined build, then
# an interleaved ms-to-best / EPnP-5 rate A/B of base2 / mm / fs / both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RSAC_LIB_PATH=$PWD/build/ab/librsac_both.so timeout -k 10 600 python -u -m pytest tests/test_epnp5.py tests/test_cv_epnp.py \
  tests/test_rvec.py tests/test_direct.py tests/test_shims.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_svd2.log 2>&1
rc=$?; tail -3 gpurun_out/t_svd2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_base2.so build/ab/librsac_mm.so build/ab/librsac_fs.so \
  build/ab/librsac_both.so --rounds 3 --hyps 20000 > gpurun_out/ab_svd2.txt 2>&1
rc=$?; tail -5 gpurun_out/ab_svd2.txt; exit $rc
