"""C2 adaptive calls with the LM refit (for rocprofv3 kernel traces of k_pnp_refine under probe builds
selected by RSAC_LIB_PATH): python3 scripts/refit_probe_run.py [calls]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 40
pr = synth.pnp_problem(10000, 0.5, seed=0)
g2 = torch.from_numpy(pr["points2d"]).cuda()
g3 = torch.from_numpy(pr["points3d"]).cuda()
for i in range(calls):
    rsac.pnp_ransac(g2, g3, pr["K"], 5000, 30.0, refine=True)
torch.cuda.synchronize()
