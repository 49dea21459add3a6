#!/bin/bash
# Solve-kernel probes (timing only): the k_pnp_solve average on C2 and C3 for each build given
# (build/ab/librsac_<name>.so, RSAC_LIB_PATH), one rocprofv3 kernel trace per build and workload.
#   scripts/build_ab.sh base= nofm=-DRSAC_PROBE_NOFM ...; scripts/gpu_solve_probe.sh base nofm ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/sp
rm -rf $P && mkdir -p $P
for round in 1 2; do
  for name in "$@"; do
    for w in c2 c3; do
      d=$P/$name.$w.$round
      RSAC_LIB_PATH=$PWD/build/ab/librsac_$name.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run \
          --output-format csv -- python3 scripts/workload_prof.py $w 8 > $d.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
      f=$(find $d -name "*kernel_stats.csv" | head -1)
      python3 - "$f" "$name" "$w" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = {r["Name"].split("(")[0].replace("rsac::", "").replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in rows}
print(sys.argv[2], sys.argv[3], " ".join(f"{k}={v:.1f}" for k, v in sorted(out.items(), key=lambda kv: -kv[1])[:4]), flush=True)
EOF
    done
  done
done
