#!/bin/bash
# Issue-side counters of the scoring kernels (variants $1, default 48,49): one PMC pass of 8 SQ
# counters + 2 GRBM counters over scripts/tune_score.py (3 interleaved rounds), summarised per
# kernel by scripts/pmc_valu_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_valu
VARS=${1:-48,49}
ROUNDS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
    -d gpurun_out/pmc_valu -o run --output-format csv -- python3 scripts/tune_score.py $VARS \
    > gpurun_out/pmc_valu/log.txt 2>&1
rc=$?; tail -3 gpurun_out/pmc_valu/log.txt; exit $rc
