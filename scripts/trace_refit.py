"""One LM refit at C2 (run under scripts/trace_build.sh for phase stamps)."""
import torch
import rsac
from rsac import synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
g2 = torch.from_numpy(pr["points2d"]).cuda()
g3 = torch.from_numpy(pr["points3d"]).cuda()
for i in range(3):
    rsac.pnp_ransac(g2, g3, pr["K"], 5000, 30.0, refine=True)
    torch.cuda.synchronize()
