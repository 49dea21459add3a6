#!/bin/bash
# r06: the whole GPU suite on the tree's build (fast f64 rotation cores, anti-diagonal device
# JacobiSVD, SVD sums from their first product), then an interleaved ms-to-best / EPnP-5 rate A/B:
# ieee (r06 start) / cyc (fast rotation cores only) / anti (+ anti-diagonal 6 x 5 / 3 x 3 SVD) /
# antip0 (+ sums from the first product); then C3 with the register-held batch setup
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_ieee.so build/ab/librsac_cyc.so build/ab/librsac_anti.so \
  build/ab/librsac_antip0.so --rounds 3 --hyps 20000 > gpurun_out/ab_antidiag.txt 2>&1
rc=$?; tail -6 gpurun_out/ab_antidiag.txt; [ $rc -eq 0 ] || exit $rc
# C3 (configs[2]) with the batch setup's points held in registers between its passes (setup8) or
# re-read (setup0)
timeout -k 10 900 python -u scripts/mf_ab.py build/ab/librsac_setup0.so build/ab/librsac_setup8.so --rounds 4 \
  --calls 10 --steps 30 --c3 40 > gpurun_out/ab_setup.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_setup.txt; exit $rc
