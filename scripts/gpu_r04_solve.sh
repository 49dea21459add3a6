#!/bin/bash
# r04 solve work: the whole -m gpu suite on the tree's library, then the solve probe (k_pnp_solve
# average on C2 and C3 per build, scripts/gpu_solve_probe.sh) for the builds named.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r04_solve_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_solve_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_solve_probe.sh "$@"
rc=$?; [ $rc -eq 0 ] || exit $rc
# the reference's default minimal solver (EPnP-5) against P3P, fixed budget, C2 problem
timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 3
