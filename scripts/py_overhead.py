"""Host-side split of one reference-mode pnp_ransac call (C2 problem, device inputs): the Python
wrapper around the C-ABI call vs the call itself, by cProfile over repeated calls."""
import cProfile
import os
import pstats
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
minimal = sys.argv[1] if len(sys.argv) > 1 else "epnp5"
sampler = sys.argv[2] if len(sys.argv) > 2 else "opencv"


def call():
    return rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, refine=True, minimal=minimal, sampler=sampler)


for _ in range(20):
    call()
torch.cuda.synchronize()
N = 300
t = time.perf_counter()
for _ in range(N):
    call()
    torch.cuda.synchronize()
print(f"{minimal}/{sampler}: {(time.perf_counter() - t) / N * 1e3:.4f} ms per call+sync", flush=True)
pr_ = cProfile.Profile()
pr_.enable()
for _ in range(N):
    call()
    torch.cuda.synchronize()
pr_.disable()
pstats.Stats(pr_).sort_stats("tottime").print_stats(14)
