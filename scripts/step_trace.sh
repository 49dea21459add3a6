#!/bin/bash
# Kernel trace of the C2 bench loop (20 steps) + the per-step timeline of its timed region.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/st && mkdir -p gpurun_out/st
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/st -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-extras --no-cpu --no-ms-to-best ${BENCH_ARGS} > gpurun_out/st/log 2>&1 || exit $?
f=$(find gpurun_out/st -name "*kernel_trace.csv" | head -1)
python3 scripts/step_timeline.py "$f" | tee gpurun_out/st/timeline.txt
