"""ms-to-best-model of pnp_ransac for each final-solve choice on the C2 problem (and a 100k-point one)."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "code-reproduction-ransac_amd"))
import rsac  # noqa: E402
from rsac import synth  # noqa: E402

for n in (10000, 100000):
    pr = synth.pnp_problem(n, 0.5, seed=0)
    g2 = torch.from_numpy(pr["points2d"]).cuda()
    g3 = torch.from_numpy(pr["points3d"]).cuda()
    for mode in (False, "lm", "epnp", "epnp+lm"):
        w = []
        for i in range(12):
            t = time.perf_counter()
            rsac.pnp_ransac(g2, g3, pr["K"], 5000, 30.0, refine=mode)
            torch.cuda.synchronize()
            if i >= 2:
                w.append((time.perf_counter() - t) * 1e3)
        print(n, mode, f"{statistics.median(w):.3f} ms", flush=True)
