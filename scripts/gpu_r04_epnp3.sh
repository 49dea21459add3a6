#!/bin/bash
# r04 EPnP-5 round 3: the whole GPU suite, then the timing script and the kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r04_epnp3_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_epnp3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 3 || exit $?
bash scripts/gpu_epnp_trace.sh
