#!/bin/bash
# r06 (fast-f64 EPnP-5): kernel traces + VALU / FETCH / WRITE passes of the reference-mode EPnP-5
# solve and the K sweep (summarised on the host by scripts/summarize_secondary.py), the per-kernel
# split of the last ms-to-best call, and the EPnP kernels' LDS wait counters (own --pmc pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WORKLOADS="epnp ksweep" bash scripts/gpu_secondary_profile.sh > gpurun_out/sec_epnp.log 2>&1 || { tail -5 gpurun_out/sec_epnp.log; exit 1; }
bash scripts/gpu_epnp_trace.sh > gpurun_out/epnp_trace.txt 2>&1 || { tail -5 gpurun_out/epnp_trace.txt; exit 1; }
cat gpurun_out/epnp_trace.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/sec/epnp/lds -o run --output-format csv -- \
    python3 scripts/workload_prof.py epnp 4 > gpurun_out/sec/epnp.lds.log 2>&1
rc=$?; echo "epnp pmc lds rc=$rc"; exit $rc
