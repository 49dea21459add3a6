"""Profile helper: C3 (1024 problems x 2000 points x 1024 hypotheses), one batched call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from rsac import synth  # noqa: E402

if len(sys.argv) > 1:
    L.check(L.lib().rsac_set_score_variant(int(sys.argv[1])))
probs = [synth.pnp_problem(2000, 0.5, seed=s) for s in range(1, 1025)]
off = np.zeros(1025, np.int64)
off[1:] = np.cumsum([len(p["points3d"]) for p in probs])
p2 = torch.from_numpy(np.concatenate([p["points2d"] for p in probs])).cuda()
p3 = torch.from_numpy(np.concatenate([p["points3d"] for p in probs])).cuda()
Ks = np.stack([p["K"] for p in probs])
for i in range(6):
    torch.cuda.synchronize()
    t = time.perf_counter()
    rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 1024, 30.0, adaptive=False, refine=False)
    torch.cuda.synchronize()
    print("wall ms %.3f" % ((time.perf_counter() - t) * 1e3))
