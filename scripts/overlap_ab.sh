#!/bin/bash
# A/B: RSAC_SOLVE_OVERLAP (second half's solve on a side stream beside the first half's
# scoring) vs the single solve + score.  GPU tests with the knob on, then alternating benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RSAC_SOLVE_OVERLAP=1 timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_overlap.log 2>&1 || { tail -30 gpurun_out/pytest_overlap.log; exit 1; }
tail -2 gpurun_out/pytest_overlap.log
for i in 1 2 3; do
  for ov in 0 1; do
    RSAC_SOLVE_OVERLAP=$ov timeout -k 10 200 python bench.py --steps 50 --warmup 5 > gpurun_out/ab_.json 2> gpurun_out/ab_err.log || exit 1
    python3 - "$ov" <<'PY'
import json,sys
l=[x for x in open('gpurun_out/ab_.json') if x.startswith('{')][-1]
d=json.loads(l); print('overlap',sys.argv[1],'value %.4g ms/step %.4f kernels %s'%(d['value'],d['ms_per_step'],d['kernels_ms']))
PY
  done
done
