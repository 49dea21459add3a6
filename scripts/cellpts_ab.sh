#!/bin/bash
# C2 step of the default scorer against the tail cell size (RSAC_MF_CELL_PTS) and the number of
# tail tiles (RSAC_SC_CELL_TILES), one process per setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "2048 768" "1024 768" "4096 768" "1024 1536" "512 768" "2048 1536"; do
  set -- $cfg
  RSAC_MF_CELL_PTS=$1 RSAC_SC_CELL_TILES=$2 ROUNDS=6 timeout -k 10 90 python3 -u scripts/step_variant_ab.py 98 2>&1 | grep variant | sed "s/^/cell $1 tiles $2: /" || exit 1
done
