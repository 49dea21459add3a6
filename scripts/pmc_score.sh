#!/bin/bash
# PMC passes over the scoring kernel (one rocprofv3 --pmc invocation per counter group,
# kernel-trace only, as the MI355X guide prescribes).  VARIANTS = scoring variants to compare.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for V in ${VARIANTS:-23}; do
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F32 SQ_ACTIVE_INST_SCA" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_MFMA" \
           "SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc/v$V/g$i -o run --output-format csv -- \
      python3 scripts/mx_prof.py $V 4 > gpurun_out/pmc/v$V.g$i.log 2>&1
  rc=$?; echo "variant $V pmc group $i rc=$rc"; [ $rc -eq 0 ] || tail -3 gpurun_out/pmc/v$V.g$i.log
done
V=$V python3 - <<'PY'
import csv, glob, collections, os
V = os.environ["V"]
tot = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/pmc/v{V}/g*/run_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_pnp_score" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        tot[c].append(v)
print("variant", V)
for c, v in sorted(tot.items()):
    v = sorted(v)
    print(f"  {c:28s} median per launch {v[len(v)//2]:.4g}  (n={len(v)})")
PY
done
