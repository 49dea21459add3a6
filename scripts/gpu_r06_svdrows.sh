#!/bin/bash
# r06: 12 x 12 JacobiSVD with the norms formed from the loaded rows (wrows) and the skip test's root
# by the fast core (wrowsfs): EPnP / rvec / shim GPU tests on wrowsfs, then ms-to-best A/B vs head
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RSAC_LIB_PATH=$PWD/build/ab/librsac_wrowsfs.so timeout -k 10 600 python -u -m pytest tests/test_epnp5.py tests/test_cv_epnp.py \
  tests/test_rvec.py tests/test_direct.py tests/test_shims.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_wrows.log 2>&1
rc=$?; tail -3 gpurun_out/t_wrows.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_head.so build/ab/librsac_wrows.so build/ab/librsac_wrowsfs.so \
  --rounds 4 --hyps 20000 > gpurun_out/ab_svdrows.txt 2>&1
rc=$?; tail -5 gpurun_out/ab_svdrows.txt; exit $rc
