#!/bin/bash
# r05 quick pass: the named GPU tests, then the EPnP-5 / ms-to-best timing script
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_quick_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r05_quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 5
