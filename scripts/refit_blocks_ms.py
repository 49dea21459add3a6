"""ms-to-best of the C2 problem (pnp_ransac, adaptive, LM refit, device inputs) with the refit's
cooperating blocks capped at 1, 2, 5 and the device limit (RSAC_DBG_REFIT_MAX_BLOCKS; the pose is
the same bits for any cap), interleaved, median wall time per call."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
ctx = rsac.context(0)
caps = [0, 1, 2, 5]
res = {c: [] for c in caps}
ref = None
for r in range(6):
    for c in caps:
        ctx.debug_set(1, c)
        for i in range(13):
            t = time.perf_counter()
            R, t_, m = rsac.pnp_ransac(ev.p2, ev.p3, pr["K"], 5000, 30.0, adaptive=True, refine=True, device=0)
            torch.cuda.synchronize()
            if i >= 3:
                res[c].append((time.perf_counter() - t) * 1e3)
        if ref is None:
            ref = (R, t_)
        assert np.array_equal(R, ref[0]) and np.array_equal(t_, ref[1])
ctx.debug_set(1, 0)
for c in caps:
    print(f"refit block cap {c or 'device'}: ms-to-best median {statistics.median(res[c]):.4f} ms")
print("refit ranges / blocks at n=10000:", ctx.refit_blocks(10000))
