#!/bin/bash
# C2 step time of the default scorer against RSAC_SC_CELL_TILES (tiles of the queue's tail run
# by cells), one process per setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CELLS:-128 384 768 1536}; do
  RSAC_SC_CELL_TILES=$c ROUNDS=6 timeout -k 10 90 python3 scripts/step_variant_ab.py ${V:-89} 2>/dev/null | grep variant | sed "s/^/cells $c: /" || exit 1
done
