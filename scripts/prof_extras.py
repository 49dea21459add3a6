"""Wall-time breakdown of the secondary workloads (C3 batch, location search) for profiling."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
if which in ("both", "loc"):
    lp = synth.location_problem(seed=0)
    for i in range(4):
        t = time.perf_counter()
        rsac.location_search(lp["pos3d"], lp["pixels"], lp["locations"], 75.0)
        print("location_search ms", (time.perf_counter() - t) * 1e3, flush=True)
    for flags in [dict(refine=False), dict(adaptive=False, refine=False)]:
        t = time.perf_counter()
        rsac.location_search(lp["pos3d"], lp["pixels"], lp["locations"], 75.0, **flags)
        print("location_search", flags, "ms", (time.perf_counter() - t) * 1e3, flush=True)
if which in ("both", "c3"):
    probs = [synth.pnp_problem(2000, 0.5, seed=s) for s in range(1, 1025)]
    p2 = [p["points2d"] for p in probs]
    p3 = [p["points3d"] for p in probs]
    Ks = [p["K"] for p in probs]
    for i in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rsac.pnp_ransac_batched(p2, p3, Ks, 1024, 30.0, adaptive=False, refine=False)
        torch.cuda.synchronize()
        print("c3 ms", (time.perf_counter() - t) * 1e3, flush=True)
    t = time.perf_counter()
    a = np.concatenate(p3)
    print("concat ms", (time.perf_counter() - t) * 1e3)
