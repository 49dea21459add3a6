#!/bin/bash
# r05: k_pnp_solve's WRITE_SIZE and time at C2 per record layout (scripts/ubench/jacobi_probe.py
# novalid / pack12 against the tree): does the write traffic follow the bytes written or the lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/wp && mkdir -p gpurun_out/wp
for v in base novalid pack12; do
  d=gpurun_out/wp/w_$v
  RSAC_LIB_PATH=$PWD/build/ab/librsac_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $d -o run --output-format csv -- \
      python3 scripts/workload_prof.py c2 3 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
  RSAC_LIB_PATH=$PWD/build/ab/librsac_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/kt -o run --output-format csv -- \
      python3 scripts/workload_prof.py c2 6 > $d.kt.log 2>&1 || { tail -3 $d.kt.log; exit 1; }
  python3 - $v $(find $d -name "*counter_collection.csv" | head -1) $(find $d/kt -name "*kernel_stats.csv" | head -1) <<'PY'
import csv, sys, statistics, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[2])):
    if "k_pnp_solve(" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
t = [float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[3])) if r["Name"].startswith("rsac::k_pnp_solve(")]
print(sys.argv[1], "k_pnp_solve WRITE_SIZE KB median", statistics.median(acc.values()), "avg_us", t)
PY
done
