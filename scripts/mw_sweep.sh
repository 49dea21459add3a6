#!/bin/bash
# k_pnp_score_mw unit-size sweep (RSAC_MW_BIG / RSAC_MW_SMALL / RSAC_MW_TAIL), one process each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "2048 512 -1" "10240 512 0" "1024 256 -1" "4096 1024 -1" "512 512 0" "2048 2048 0"; do
  set -- $cfg
  RSAC_MW_BIG=$1 RSAC_MW_SMALL=$2 RSAC_MW_TAIL=$3 RSAC_DBG_MF=1 ROUNDS=4 timeout -k 10 60 python3 scripts/tune_score.py 74 > gpurun_out/mws.log 2>&1 || exit 1
  echo "big $1 small $2 tail $3: $(tail -1 gpurun_out/mws.log) | $(grep 'rsac mw' gpurun_out/mws.log | tail -1)"
done
