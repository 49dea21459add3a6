#!/bin/bash
# r06: one P3P problem's set-up fused with its first round's 4-lane solve (k_pnp_setup_solve4), the
# round's records built by the scaled-form scorer: the whole GPU suite on the tree's build, then the
# ms-to-best A/B against the build before it (pre = the fast-f64 LM tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ms_ab.py build/ab/librsac_pre.so build/ab/librsac_p3pfuse.so \
  --rounds 4 > gpurun_out/ab_p3pfuse.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_p3pfuse.txt; exit $rc
