#!/bin/bash
# Per-config rocprofv3 passes for the secondary rooflines: for each of
# C2 (solve), C3, C4, C5 a kernel trace and separate --pmc passes (VALU issue side, FETCH_SIZE,
# WRITE_SIZE), each its own run, never combined with other tracing domains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/sec
mkdir -p $P
for w in ${WORKLOADS:-c2 c3 c4 c5}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $P/$w/kt -o run --output-format csv -- \
      python3 scripts/workload_prof.py $w 6 > $P/$w.kt.log 2>&1
  rc=$?; echo "$w kernel-trace rc=$rc"; tail -1 $P/$w.kt.log; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
      -d $P/$w/valu -o run --output-format csv -- python3 scripts/workload_prof.py $w 4 > $P/$w.valu.log 2>&1
  rc=$?; echo "$w pmc valu rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $P/$w/fetch -o run --output-format csv -- \
      python3 scripts/workload_prof.py $w 4 > $P/$w.fetch.log 2>&1
  rc=$?; echo "$w pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $P/$w/write -o run --output-format csv -- \
      python3 scripts/workload_prof.py $w 4 > $P/$w.write.log 2>&1
  rc=$?; echo "$w pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find $P -name "*.csv" | head -40
