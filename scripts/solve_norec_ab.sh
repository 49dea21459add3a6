#!/bin/bash
# Share of the record writing (write_fmodel_mx) in the C2 solve: solve_ms with and without it
# (RSAC_DBG_SOLVE_NO_RECORDS: timing only, the scoring records go stale)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for e in "X=1" "RSAC_DBG_SOLVE_NO_RECORDS=1"; do
  env $e timeout -k 10 60 python3 - <<'PY' || exit 1
import os, statistics, sys, time
sys.path.insert(0, "code-reproduction-ransac_amd")
import torch, rsac
from rsac import synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda(); p2 = torch.from_numpy(pr["points2d"]).cuda()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, with_mask=True, device_result=True)
v = [rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, return_info=True)[2].solve_ms for _ in range(30)]
print("no_records" if "RSAC_DBG_SOLVE_NO_RECORDS" in os.environ else "records", "solve_ms", round(statistics.median(v), 4), flush=True)
PY
done
