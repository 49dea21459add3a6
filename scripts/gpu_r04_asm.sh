#!/bin/bash
# r04: the hand-scheduled group body (RSAC_MF_ASM=1, the tree) through the whole GPU suite, then
# an interleaved A/B against the compiler's schedule (build/ab/librsac_base.so = -DRSAC_MF_ASM=0)
# on C2 (scoring kernel, step) and C3 (per call).
#   scripts/build_ab.sh base=-DRSAC_MF_ASM=0 asm=
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r04_asm_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_asm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/mf_ab.py build/ab/librsac_base.so build/ab/librsac_asm.so --rounds 4 --calls 30 \
    --steps 60 --c3 20 > gpurun_out/r04_asm_ab.log 2>&1
rc=$?; tail -4 gpurun_out/r04_asm_ab.log; exit $rc
