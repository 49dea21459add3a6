#!/bin/bash
# C2 step with the best key fused into the scorer (RSAC_FUSE_KEY=1, no cells, no k_best_key
# launch) against the cells + k_best_key path, one process each, alternated
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for f in 1 0; do
    RSAC_FUSE_KEY=$f ROUNDS=6 timeout -k 10 90 python3 -u scripts/step_variant_ab.py 98 2>&1 | grep variant | sed "s/^/fuse $f: /" || exit 1
  done
done
