#!/bin/bash
# GPU tests only: the named test files first (fail fast), then the whole -m gpu suite.
# Usage: bash scripts/gpu_tests.sh [first test paths...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_first.log 2>&1
  rc=$?; echo "first rc=$rc"; tail -25 gpurun_out/pytest_first.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
exit $rc
