#!/bin/bash
# k_pnp_score_mw timing experiments (77 static units, 78 no count atomics, 79 both) at unit sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "2048 512 -1" "2048 2048 0" "1024 512 -1" "4096 1024 -1" "512 512 0"; do
  set -- $cfg
  RSAC_MW_BIG=$1 RSAC_MW_SMALL=$2 RSAC_MW_TAIL=$3 ROUNDS=4 timeout -k 10 60 python3 scripts/tune_score.py ${V:-73,74,77} > gpurun_out/mwx.log 2>&1 || exit 1
  echo "big $1 small $2 tail $3:"; grep variant gpurun_out/mwx.log
done
