#!/bin/bash
# r06: phase cycles of the EPnP-5 stage-3 kernel and of the SVD (RSAC_TRACE build in /tmp)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ct
bash scripts/trace_build.sh scripts/trace_refit.py > gpurun_out/ct/build.log 2>&1 || { tail -5 gpurun_out/ct/build.log; exit 1; }
RSAC_LIB_PATH=/tmp/rsac_trace/code-reproduction-ransac_amd/rsac/librsac.so timeout -k 10 120 \
    python3 scripts/trace_ms_to_best.py epnp5 opencv > gpurun_out/ct/trace_epnp.log 2>&1 || { tail -5 gpurun_out/ct/trace_epnp.log; exit 1; }
grep "epnp c\|svd lane0" gpurun_out/ct/trace_epnp.log | tail -6
