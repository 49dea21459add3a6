#!/bin/bash
# r05 batch: the GPU suite on the tree, the probes, then interleaved A/B of the build/ab variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_batch_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r05_batch_tests.log; [ $rc -eq 0 ] || exit $rc
[ -n "$PROBE" ] && { bash scripts/gpu_r05_jprobe.sh || exit 1; }
timeout -k 10 500 python3 scripts/ms_ab.py "$@" --rounds 3 --calls 15 --hyps 20000
