#!/bin/bash
# MFMA scorer profile: kernel trace of tune_score.py over the given variants, then one PMC pass
# (issue and wait counters), summarised per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${1:-49,72,73}
rm -rf gpurun_out/mfp && mkdir -p gpurun_out/mfp
ROUNDS=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mfp/kt -o run --output-format csv -- \
    python3 scripts/tune_score.py $V > gpurun_out/mfp/kt.log 2>&1 || exit $?
f=$(find gpurun_out/mfp/kt -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('%-70s calls %5s avg_us %9.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))"
ROUNDS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
    -d gpurun_out/mfp/pmc -o run --output-format csv -- python3 scripts/tune_score.py $V \
    > gpurun_out/mfp/pmc.log 2>&1 || exit $?
python3 scripts/pmc_valu_summary.py $(find gpurun_out/mfp/pmc -name "*counter_collection.csv" | head -1)
