#!/bin/bash
# rocprofv3 kernel-trace summary of the bench command (same command as the
# bench line); PMC passes are separate invocations (never combined with
# tracing domains other than --kernel-trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r03}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu --no-ms-to-best --no-extras > gpurun_out/prof/bench_under_rocprof.log 2>&1
rc=$?; echo "rocprof kernel-trace rc=$rc"; tail -2 gpurun_out/prof/bench_under_rocprof.log
[ $rc -eq 0 ] || exit $rc
# C3 (BASELINE configs[2]) alone: where a 1024-problem batched call spends its time
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/c3 -o run --output-format csv -- \
    python3 scripts/c3_prof.py > gpurun_out/prof/c3_under_rocprof.log 2>&1
rc=$?; echo "rocprof C3 kernel-trace rc=$rc"; tail -1 gpurun_out/prof/c3_under_rocprof.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ms-to-best --no-extras > gpurun_out/prof/pmc_fetch.log 2>&1
  rc=$?; echo "rocprof pmc FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ms-to-best --no-extras > gpurun_out/prof/pmc_write.log 2>&1
  rc=$?; echo "rocprof pmc WRITE_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
  # issue side of the same command: VALU / SALU instructions, wave-cycle split, clock
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
      -d gpurun_out/prof/pmc_valu -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ms-to-best --no-extras > gpurun_out/prof/pmc_valu.log 2>&1
  rc=$?; echo "rocprof pmc VALU rc=$rc"; [ $rc -eq 0 ] || exit $rc
  # where the waves wait: parked (s_waitcnt / barrier) vs issue stalls, and the LDS side
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS \
      SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES \
      -d gpurun_out/prof/pmc_wait -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ms-to-best --no-extras > gpurun_out/prof/pmc_wait.log 2>&1
  rc=$?; echo "rocprof pmc wait rc=$rc"; [ $rc -eq 0 ] || exit $rc
  # VALU issue per quad-cycle: one or two VALU issued, MFMA co-execution
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_VALU_MFMA_COEXEC_CYCLES \
      SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS GRBM_GUI_ACTIVE \
      -d gpurun_out/prof/pmc_issue -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ms-to-best --no-extras > gpurun_out/prof/pmc_issue.log 2>&1
  rc=$?; echo "rocprof pmc issue rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
find gpurun_out/prof -name "*.csv" | head -20
