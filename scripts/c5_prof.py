"""Profile helper: C5 LO-RANSAC (100k correspondences, 50 % outliers), adaptive + LO + final refit."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

p5 = synth.pnp_problem(100_000, 0.5, seed=3)
q2 = torch.from_numpy(p5["points2d"]).cuda()
q3 = torch.from_numpy(p5["points3d"]).cuda()
for r in range(6):
    torch.cuda.synchronize()
    t = time.perf_counter()
    _, _, _, info = rsac.pnp_ransac(q2, q3, p5["K"], 5000, 30.0, lo=True, refine=True, return_info=True)
    torch.cuda.synchronize()
    print("wall ms %.2f iters %d rounds %d lo %d" % ((time.perf_counter() - t) * 1e3, info.iters, info.rounds,
                                                    info.lo_improvements))
