#!/bin/bash
# One-, two- and four-lane P3P solve on the C2 round (100k hypotheses): solve_ms (HIP events) and
# the key, one process per setting (the knobs are read once)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "0 4096" "1000000 4096" "0 1000000"; do
  set -- $cfg
  RSAC_SOLVE2_MAX=$1 RSAC_SOLVE4_MAX=$2 timeout -k 10 60 python3 - <<'PY' || exit 1
import os, statistics, sys, time
sys.path.insert(0, "code-reproduction-ransac_amd")
import torch, rsac
from rsac import synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda(); p2 = torch.from_numpy(pr["points2d"]).cuda()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, with_mask=True, device_result=True)
torch.cuda.synchronize()
v = []
for i in range(30):
    key, model, info = rsac.evaluate_range(p2, p3, pr["K"], 0, 100000, 30.0, return_info=True)
    v.append(info.solve_ms)
print(f"solve2_max {os.environ['RSAC_SOLVE2_MAX']} solve4_max {os.environ['RSAC_SOLVE4_MAX']}: solve_ms median {statistics.median(v):.4f} key {key >> 32} {key & 0xffffffff} model {model[:3]}", flush=True)
PY
done
