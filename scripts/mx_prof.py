"""Profile helper: C2 evaluate_range with one scoring variant (argv[1]) a few times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from rsac import synth  # noqa: E402

v = int(sys.argv[1]) if len(sys.argv) > 1 else -1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
L.check(L.lib().rsac_set_score_variant(v))
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda()
p2 = torch.from_numpy(pr["points2d"]).cuda()
for _ in range(reps):
    key, model, info = rsac.evaluate_range(p2, p3, pr["K"], 0, 100_000, 30.0, return_info=True)
print("variant", v, "key", key, "score_ms", info.score_ms)
