#!/bin/bash
# r05: where the C3 scorer (k_pnp_score_mf<2>) and the C2 scorer spend their wave cycles, and the
# C2 scorer's write traffic.  Every --pmc pass a run of its own.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/c3pmc
rm -rf $P && mkdir -p $P
for w in c3 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $P/$w/kt -o run --output-format csv -- \
      python3 scripts/workload_prof.py $w 6 > $P/$w.kt.log 2>&1 || { tail -3 $P/$w.kt.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
      -d $P/$w/sq -o run --output-format csv -- python3 scripts/workload_prof.py $w 3 > $P/$w.sq.log 2>&1 \
      || { tail -3 $P/$w.sq.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_INSTS_SALU SQ_INSTS_SMEM -d $P/$w/mem -o run --output-format csv -- python3 scripts/workload_prof.py $w 3 \
      > $P/$w.mem.log 2>&1 || { tail -3 $P/$w.mem.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/$w/write -o run --output-format csv -- \
      python3 scripts/workload_prof.py $w 3 > $P/$w.write.log 2>&1 || { tail -3 $P/$w.write.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/$w/fetch -o run --output-format csv -- \
      python3 scripts/workload_prof.py $w 3 > $P/$w.fetch.log 2>&1 || { tail -3 $P/$w.fetch.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, statistics, collections
for w in ("c3", "c2"):
    kt = glob.glob(f"gpurun_out/c3pmc/{w}/kt/**/*kernel_stats.csv", recursive=True)
    for r in sorted(csv.DictReader(open(kt[0])), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
        print(w, "%-40s calls %4s avg_us %8.1f" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
    for pas in ("sq", "mem", "write", "fetch"):
        f = glob.glob(f"gpurun_out/c3pmc/{w}/{pas}/**/*counter_collection.csv", recursive=True)
        if not f:
            print(w, pas, "no csv"); continue
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f[0])):
            if "k_pnp_score_mf" not in r["Kernel_Name"]:
                continue
            acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        per = collections.defaultdict(list)
        for (d, c), v in acc.items():
            per[c].append(sum(v))
        print(w, pas, {c: "%.4g" % statistics.median(v) for c, v in sorted(per.items())})
PY
