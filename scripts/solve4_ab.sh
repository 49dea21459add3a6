#!/bin/bash
# A/B: the four-lane P3P solve on the big C2 round (RSAC_SOLVE4_MAX) vs one lane per hypothesis
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 4096 200000 4096 200000; do
    RSAC_SOLVE4_MAX=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu --no-ms-to-best \
        2>/dev/null | tail -1 > gpurun_out/s4_$v.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/s4_$v.json')); print($v, d['ms_per_step'], d['kernels_ms'])"
done
