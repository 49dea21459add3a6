#!/bin/bash
# r06: one problem's set-up fused into the first EPnP-5 solve launch (k_cvepnp5_a_setup): the whole
# GPU suite on the tree's build, then the ms-to-best / EPnP-5 rate A/B against the build before it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_prefuse.so build/ab/librsac_fused.so \
  --rounds 4 --hyps 20000 > gpurun_out/ab_fuse.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_fuse.txt; exit $rc
