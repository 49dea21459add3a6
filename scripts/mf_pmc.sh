#!/bin/bash
# MFMA scorer PMC passes over scripts/tune_score.py (variants $1): the issue/wait counters, then
# the matrix-core counters; summarised per kernel by scripts/pmc_valu_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${1:-73}
rm -rf gpurun_out/mfpmc && mkdir -p gpurun_out/mfpmc
ROUNDS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
    -d gpurun_out/mfpmc/a -o run --output-format csv -- python3 scripts/tune_score.py $V \
    > gpurun_out/mfpmc/a.log 2>&1 || exit $?
python3 scripts/pmc_valu_summary.py $(find gpurun_out/mfpmc/a -name "*counter_collection.csv" | head -1)
ROUNDS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS \
    SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE \
    -d gpurun_out/mfpmc/b -o run --output-format csv -- python3 scripts/tune_score.py $V \
    > gpurun_out/mfpmc/b.log 2>&1 || exit $?
python3 scripts/pmc_valu_summary.py $(find gpurun_out/mfpmc/b -name "*counter_collection.csv" | head -1)
