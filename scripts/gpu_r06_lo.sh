#!/bin/bash
# r06: the LO recount with one packed atomic per block: LO / refit GPU tests, then an interleaved
# A/B against the previous build (ms-to-best P3P / reference mode, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lo
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_parallel_gloo.py -m gpu -x -q -k "lo or LO or local or refit or refine" \
    --timeout 120 --timeout-method thread > gpurun_out/lo/tests.log 2>&1 || { tail -30 gpurun_out/lo/tests.log; exit 1; }
tail -2 gpurun_out/lo/tests.log
timeout -k 10 600 python3 scripts/ms_ab.py build/ab/librsac_old.so build/ab/librsac_new.so --rounds 3 --calls 20 --c5 \
    > gpurun_out/lo/ab.log 2>&1 || { tail -10 gpurun_out/lo/ab.log; exit 1; }
tail -4 gpurun_out/lo/ab.log
bash scripts/gpu_r06_refit_probe.sh > gpurun_out/lo/rp.log 2>&1 || { tail -5 gpurun_out/lo/rp.log; exit 1; }
cat gpurun_out/lo/rp.log | grep -v "^W\|^E" | tail -10
