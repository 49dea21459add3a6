#!/bin/bash
# r06: interleaved kernel-time A/B of two library builds on the EPnP-5 timing script
# (k_cvepnp5_* mean durations from rocprofv3 kernel traces): bash scripts/gpu_r06_kab.sh old new
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kab
for r in 1 2 3; do
  for v in "$@"; do
    RSAC_LIB_PATH=$PWD/build/ab/librsac_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kab/${v}_$r \
        -o run --output-format csv -- python3 scripts/epnp5_prof.py 20000 3 > gpurun_out/kab/${v}_$r.log 2>&1 \
        || { tail -5 gpurun_out/kab/${v}_$r.log; exit 1; }
    f=$(find gpurun_out/kab/${v}_$r -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,sys
d={r['Name'].split('(')[0].replace('rsac::',''):float(r['AverageNs'])/1e3 for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], ' '.join(f'{k} {d[k]:.1f}' for k in ('k_cvepnp5_a','k_cvepnp5_svd','k_cvepnp5_c') if k in d))" $f $v
  done
done
