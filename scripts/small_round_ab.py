"""ms-to-best (C2, device inputs, refine=True) for the small-round scoring instances, selected by
RSAC_SMALL_PP (read once per process): run once per value, e.g.
    for pp in 2 102 105 104; do RSAC_SMALL_PP=$pp python scripts/small_round_ab.py; done
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
p2 = torch.from_numpy(pr["points2d"]).cuda()
p3 = torch.from_numpy(pr["points3d"]).cuda()
walls, score = [], []
for i in range(230):
    torch.cuda.synchronize()
    t = time.perf_counter()
    R, t_, m = rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, refine=True)
    torch.cuda.synchronize()
    if i >= 30:
        walls.append((time.perf_counter() - t) * 1e3)
_, _, _, info = rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, refine=True, return_info=True)
print(f"RSAC_SMALL_PP={os.environ.get('RSAC_SMALL_PP', 'default')}: ms-to-best median {statistics.median(walls):.4f} "
      f"min {min(walls):.4f}; score_ms {info.score_ms:.4f} solve_ms {info.solve_ms:.4f}", flush=True)
