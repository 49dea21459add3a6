#!/bin/bash
# r06 A/B: the long-round P3P solve on 2 lanes per hypothesis (RSAC_SOLVE_LANES=2) against 1:
# parity tests on the 2-lane form, then interleaved bench steps (C2, 100k hypotheses)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
RSAC_SOLVE_LANES=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "baseline or solve or hypotheses or batched" \
    --timeout 120 --timeout-method thread > gpurun_out/s2/tests.log 2>&1 || { tail -30 gpurun_out/s2/tests.log; exit 1; }
tail -2 gpurun_out/s2/tests.log
for r in 1 2 3; do
  for L in 1 2; do
    RSAC_SOLVE_LANES=$L timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --no-ms-to-best --no-extras \
        > gpurun_out/s2/b_${L}_${r}.log 2>&1 || { tail -5 gpurun_out/s2/b_${L}_${r}.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], d['kernels_ms'])" gpurun_out/s2/b_${L}_${r}.log L=$L
  done
done
