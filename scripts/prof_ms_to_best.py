"""Where ms-to-best goes: pnp_ransac wall time by option (C2 problem)."""
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
p2d = torch.from_numpy(pr["points2d"]).cuda()
p3d = torch.from_numpy(pr["points3d"]).cuda()
for name, a, b, kw in [("device refine", p2d, p3d, dict(refine=True)),
                       ("device norefine", p2d, p3d, dict(refine=False)),
                       ("host refine", pr["points2d"], pr["points3d"], dict(refine=True)),
                       ("host norefine", pr["points2d"], pr["points3d"], dict(refine=False))]:
    walls = []
    for i in range(25):
        torch.cuda.synchronize()
        t = time.perf_counter()
        R, t_, m, info = rsac.pnp_ransac(a, b, pr["K"], 5000, 30.0, return_info=True, **kw)
        torch.cuda.synchronize()
        if i >= 5:
            walls.append((time.perf_counter() - t) * 1e3)
    print(f"{name}: median {statistics.median(walls):.3f} ms  iters {info.iters} rounds {info.rounds} "
          f"gpu_ms {info.gpu_ms:.3f}", flush=True)
