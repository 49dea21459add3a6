#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
RSAC_DBG_MF=1 timeout -k 10 60 python -u - > gpurun_out/dbg/mf_dbg.log 2>&1 <<'PY'
import sys
sys.path.insert(0, "code-reproduction-ransac_amd")
import torch, rsac
from rsac import _lib as L, synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda(); p2 = torch.from_numpy(pr["points2d"]).cuda()
L.check(L.lib().rsac_set_score_variant(60))
for i in range(2):
    key, model, info = rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, return_info=True)
    print("score_ms", info.score_ms)
PY
echo "dbg rc=$?"; cat gpurun_out/dbg/mf_dbg.log | tail -5
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/dbg/kt -o run --output-format csv -- python3 scripts/tune_score.py 60 > gpurun_out/dbg/kt.log 2>&1
echo "kt rc=$?"; f=$(find gpurun_out/dbg/kt -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
for r in sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs']))[:6]:
    print('%-60s calls %5s avg_us %9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
