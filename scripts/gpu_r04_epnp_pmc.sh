#!/bin/bash
# EPnP-5 path PMC passes (its own runs, no other tracing domain): VALU issue side and LDS of the
# three-launch solve (k_epnp5_a / k_epnp5_jacobi6 or _jacobi_b / k_epnp5_c) under scripts/epnp5_prof.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/epmc
rm -rf $P && mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o run --output-format csv -- \
    python3 scripts/epnp5_prof.py 20000 3 > $P/kt.log 2>&1 || { tail -3 $P/kt.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE \
    -d $P/valu -o run --output-format csv -- python3 scripts/epnp5_prof.py 20000 2 > $P/valu.log 2>&1 || { tail -3 $P/valu.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    -d $P/f64 -o run --output-format csv -- python3 scripts/epnp5_prof.py 20000 2 > $P/f64.log 2>&1 || { tail -3 $P/f64.log; exit 1; }
find $P -name "*.csv" | head
