#!/bin/bash
# r06: the LM step's solve (Cholesky roots / reciprocals, Cayley reciprocal, step-test roots) by the
# fast f64 cores with an IEEE redo outside their range: the whole GPU suite on the tree's build,
# then the ms-to-best (P3P, reference mode) + C5 A/B against the build before it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_lmbase.so build/ab/librsac_lmfast.so \
  --rounds 4 --c5 > gpurun_out/ab_lmfast.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_lmfast.txt; exit $rc
