#!/bin/bash
# r05 EPnP-5 iteration: the EPnP GPU tests, the timing script, the ms-to-best kernel timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_epnp5.py tests/test_epnp.py tests/test_direct.py tests/test_rvec.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r05_ep_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r05_ep_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/epnp5_prof.py 20000 5 || exit 1
rm -rf gpurun_out/tr && mkdir -p gpurun_out/tr
d=gpurun_out/tr/epnp5_opencv
timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 scripts/trace_ms_to_best.py epnp5 opencv > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/timeline.py $(find $d -name "*kernel_trace.csv" | head -1) | tail -9
