#!/bin/bash
# PMC passes over the scoring kernel (one rocprofv3 --pmc invocation per counter group,
# kernel-trace only, as the MI355X guide prescribes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
V=${V:-0}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d gpurun_out/pmc/g$i -o run --output-format csv -- \
      python3 scripts/tune_score.py $V > gpurun_out/pmc/g$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
