#!/bin/bash
# MFMA scoring variant 60: pre-filter parity tests, then an interleaved timing A/B against 49 and
# the no-recount timing variant 61.  Any failure ends the script (no further GPU work).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "(prefilter and (score_variant0 or 49 or 70 or 71 or 73)) or mixed_scales" > gpurun_out/mf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/mf_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u - > gpurun_out/mf_tune.log 2>&1 <<'PY'
import statistics, sys
sys.path.insert(0, "code-reproduction-ransac_amd")
import torch, rsac
from rsac import _lib as L, synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda(); p2 = torch.from_numpy(pr["points2d"]).cuda()
res = {v: [] for v in (49, 64, 68, 70, 71, 72, 73)}
for rnd in range(6):
    for v in res:
        L.check(L.lib().rsac_set_score_variant(v))
        key, model, info = rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, return_info=True)
        if rnd: res[v].append(info.score_ms)
        if rnd == 1: print(v, "key", key >> 32, key & 0xffffffff)
for v in res:
    print(v, "score_ms median", round(statistics.median(res[v]), 4), "min", round(min(res[v]), 4))
PY
rc=$?; echo "tune rc=$rc"; tail -8 gpurun_out/mf_tune.log
exit $rc
