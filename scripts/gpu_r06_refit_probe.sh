#!/bin/bash
# r06: where the LM refit's time goes, by doubling one part at a time (probe builds from
# scripts/build_ab.sh after `git apply scripts/ubench/refit_probes_r06.patch`: base, the point pass twice,
# the wave/block sums twice, the solve step twice),
# k_pnp_refine's mean duration from rocprofv3 kernel traces, two interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
for r in 1 2; do
  for v in base pts sums solve; do
    RSAC_LIB_PATH=$PWD/build/ab/librsac_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rp/${v}_$r \
        -o run --output-format csv -- python3 scripts/refit_probe_run.py 40 > gpurun_out/rp/${v}_$r.log 2>&1 \
        || { tail -5 gpurun_out/rp/${v}_$r.log; exit 1; }
    f=$(find gpurun_out/rp/${v}_$r -name "*kernel_stats.csv" | head -1)
    python3 -c "import csv,sys; [print(sys.argv[2], r['Calls'], round(float(r['AverageNs'])/1e3,2)) for r in csv.DictReader(open(sys.argv[1])) if 'k_pnp_refine' in r['Name']]" $f $v
  done
done
