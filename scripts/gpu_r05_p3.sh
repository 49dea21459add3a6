#!/bin/bash
# r05: fused P3P arithmetic -- GPU suite on the tree, ms-to-best A/B and k_pnp_solve's time at C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/p3
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/ms_ab.py build/ab/librsac_p3a.so build/ab/librsac_p3b.so --rounds 4 > $O/ab.log 2>&1 || exit $?
tail -3 $O/ab.log
for v in p3a p3b; do
  d=$O/kt_$v
  RSAC_LIB_PATH=$PWD/build/ab/librsac_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 scripts/workload_prof.py c2 10 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
  python3 - $v $(find $d -name "*kernel_stats.csv" | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if r["Name"].startswith(("rsac::k_pnp_solve(", "void rsac::k_pnp_score_mf")):
        print(sys.argv[1], r["Name"][:40], "calls", r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
done
