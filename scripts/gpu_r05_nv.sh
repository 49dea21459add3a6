#!/bin/bash
# r05: PnP hypothesis validity in the status byte.  The GPU suite on a build whose solves write 0 to
# the validity slot (no reader may still use it), the suite on the tree, ms-to-best / EPnP A/B
# against the previous tree, and k_pnp_solve's WRITE_SIZE and time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/nv
rm -rf $O && mkdir -p $O
RSAC_LIB_PATH=$PWD/build/ab/librsac_poison.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/poison.log 2>&1
rc=$?; echo "poison suite rc=$rc"; tail -3 $O/poison.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tree.log 2>&1
rc=$?; echo "tree suite rc=$rc"; tail -3 $O/tree.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python scripts/ms_ab.py build/ab/librsac_base.so build/ab/librsac_nv.so --rounds 3 --hyps 20000 > $O/ab.log 2>&1 || exit $?
tail -3 $O/ab.log
for v in base nv; do
  d=$O/w_$v
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
