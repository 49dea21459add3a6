#!/bin/bash
# k_pnp_score_mf cell-tile sweep (RSAC_SC_CELL_TILES), one process each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in 1 256 768 1536 3125; do
  RSAC_SC_CELL_TILES=$c ROUNDS=5 timeout -k 10 60 python3 scripts/tune_score.py ${V:-73} 2>/dev/null | grep variant | sed "s/^/cells $c: /" || exit 1
done
