#!/bin/bash
# f64 issue costs (scripts/ubench/f64_rate.hip) and the solve kernels' f64 instruction mix
# (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, one --pmc pass per workload): the inputs of the
# issue-weighted solve roofline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/f64
mkdir -p $P
timeout -k 10 120 ./build/f64_rate > $P/f64_rate.txt 2>&1; rc=$?; cat $P/f64_rate.txt; [ $rc -eq 0 ] || exit $rc
for w in c2 c3; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
      SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      -d $P/$w/mix -o run --output-format csv -- python3 scripts/workload_prof.py $w 4 > $P/$w.mix.log 2>&1
  rc=$?; echo "$w pmc f64 mix rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 \
      SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
      -d $P/$w/mix32 -o run --output-format csv -- python3 scripts/workload_prof.py $w 4 > $P/$w.mix32.log 2>&1
  rc=$?; echo "$w pmc f32 mix rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find $P -name "*.csv" | head -20
