#!/bin/bash
# r06: EPnP-5 tests, kernel timings, the SVD's per-phase cycle probe (RSAC_TRACE build in /tmp),
# then the K-sweep / EPnP-5 PMC passes (summarised on the host by scripts/summarize_secondary.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ep2
timeout -k 10 400 python -u -m pytest tests/test_epnp5.py tests/test_shims.py tests/test_direct.py tests/test_cv_epnp.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ep2/tests.log 2>&1 || { tail -30 gpurun_out/ep2/tests.log; exit 1; }
tail -2 gpurun_out/ep2/tests.log
bash scripts/gpu_epnp_trace.sh > gpurun_out/ep2/trace.log 2>&1 || { tail -5 gpurun_out/ep2/trace.log; exit 1; }
grep -E "hyps|ms-to-best" gpurun_out/ep/log
bash scripts/trace_build.sh scripts/trace_refit.py > gpurun_out/ep2/trace_refit.log 2>&1 || { tail -5 gpurun_out/ep2/trace_refit.log; exit 1; }
RSAC_LIB_PATH=/tmp/rsac_trace/code-reproduction-ransac_amd/rsac/librsac.so timeout -k 10 120 \
    python3 scripts/trace_ms_to_best.py epnp5 opencv > gpurun_out/ep2/trace_epnp.log 2>&1 || { tail -5 gpurun_out/ep2/trace_epnp.log; exit 1; }
grep "svd lane0" gpurun_out/ep2/trace_epnp.log | tail -3
WORKLOADS="ksweep epnp" bash scripts/gpu_secondary_profile.sh > gpurun_out/ep2/sec.log 2>&1 || { tail -5 gpurun_out/ep2/sec.log; exit 1; }
echo done
