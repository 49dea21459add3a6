#!/bin/bash
# r06: one problem's speculative scan replay + RANSAC mask done by the LM refit launch (no separate
# k_scan_mask): the whole GPU suite on the tree's build, then the ms-to-best A/B against the build
# before it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_pre.so build/ab/librsac_scanrefit.so \
  --rounds 4 > gpurun_out/ab_scanrefit.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_scanrefit.txt; exit $rc
