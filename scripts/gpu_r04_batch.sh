#!/bin/bash
# r04 batch: block scan + 8-lane fundamental solve tests, C4 timing, the scorer's in-kernel clock.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "fixed_budget or fundamental or c4 or scan" > gpurun_out/r04_scan.log 2>&1
rc=$?; tail -22 gpurun_out/r04_scan.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/workload_prof.py c4 5 || exit $?
timeout -k 10 200 bash scripts/clock_probe.sh c2 400 > gpurun_out/r04_clock.log 2>&1
rc=$?; grep -c mfclock gpurun_out/r04_clock.log; tail -2 gpurun_out/r04_clock.log; [ $rc -eq 0 ] || exit $rc
# unit-structure A/B: waves per block for the long problem, every tile by cells
timeout -k 10 600 python3 scripts/mf_ab.py build/ab/librsac_base.so build/ab/librsac_w1c2k.so \
    build/ab/librsac_w1c4k.so build/ab/librsac_w2c2k.so build/ab/librsac_w4c2k.so --rounds 3 --calls 30 --steps 60 \
    > gpurun_out/r04_ab_units.log 2>&1
rc=$?; tail -7 gpurun_out/r04_ab_units.log; exit $rc
