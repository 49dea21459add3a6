#!/bin/bash
# PMC passes over the scoring kernel (one rocprofv3 --pmc invocation per counter group,
# kernel-trace only, as the MI355X guide prescribes).  V = scoring variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
V=${V:-1}
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F32" \
           "SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" \
           "SQ_WAVES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d gpurun_out/pmc/g$i -o run --output-format csv -- \
      python3 scripts/tune_score.py $V > gpurun_out/pmc/g$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc/g*/run_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_pnp_score" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        tot[c].append(v)
for c, v in sorted(tot.items()):
    v = sorted(v)
    print(f"{c:28s} median per launch {v[len(v)//2]:.4g}  (n={len(v)})")
PY
