#!/bin/bash
# MFMA scorer check after a change: pre-filter parity tests of the MFMA variants, the flagged
# records of one C2 launch (RSAC_DBG_MF), an interleaved timing A/B, and a kernel trace of the
# A/B.  Any failure ends the script (no further GPU work).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${1:-49,73}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "${TESTK:-(prefilter and (score_variant0 or 49 or 70 or 71 or 73)) or mixed_scales}" > gpurun_out/mf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/mf_tests.log
[ $rc -eq 0 ] || exit $rc
RSAC_DBG_MF=1 timeout -k 10 120 python -u - > gpurun_out/mf_dbg.log 2>&1 <<'PY'
import sys
sys.path.insert(0, "code-reproduction-ransac_amd")
import torch, rsac
from rsac import synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda(); p2 = torch.from_numpy(pr["points2d"]).cuda()
key, model, info = rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, return_info=True)
print("key", key >> 32)
PY
rc=$?; echo "dbg rc=$rc"; tail -3 gpurun_out/mf_dbg.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=6 timeout -k 10 120 python3 scripts/tune_score.py $V > gpurun_out/mf_tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -6 gpurun_out/mf_tune.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/mfkt
ROUNDS=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mfkt -o run --output-format csv -- \
    python3 scripts/tune_score.py $V > gpurun_out/mfkt.log 2>&1
rc=$?; echo "kt rc=$rc"
f=$(find gpurun_out/mfkt -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('%-70s calls %5s avg_us %9.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))"
exit $rc
