"""One BASELINE workload alone, for rocprofv3 passes (kernel trace and separate --pmc passes) that
attribute every kernel to its config (scripts/gpu_secondary_profile.sh):

    python3 scripts/workload_prof.py c2|c3|c4|c5 [repeats]

c2: the bench step (rsac.evaluate_range, 100k hypotheses over the 10k-point problem: solve + score
    + key + mask); c3: pnp_ransac_batched_flat over 1024 x 2000 points, 1024 hypotheses each; c4:
    fundamental_ransac, 50k matches, 100k hypotheses, adaptive off; c5: pnp_ransac(lo=True) on the
    100k-point problem (the LO chain: k_pnp_refine with a source record + k_pnp_lo_count).
Inputs resident in HBM, as in bench.py.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "code-reproduction-ransac_amd")]
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

which = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
if which == "c2":
    pr = synth.pnp_problem(10_000, 0.5, seed=0)
    p2, p3 = torch.from_numpy(pr["points2d"]).to(dev), torch.from_numpy(pr["points3d"]).to(dev)
    run = lambda: rsac.evaluate_range(p2, p3, pr["K"], 0, 100_000, 30.0, with_mask=True, device_result=True)
elif which == "c3":
    from bench import c3_problems
    h2, h3, off, Ks = c3_problems()
    p2, p3 = torch.from_numpy(h2).to(dev), torch.from_numpy(h3).to(dev)
    run = lambda: rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 1024, 30.0, adaptive=False, refine=False)
elif which == "c4":
    p4 = synth.fundamental_problem(50_000, 0.8, seed=2)
    f1, f2 = torch.from_numpy(p4["pts1"]).to(dev), torch.from_numpy(p4["pts2"]).to(dev)
    run = lambda: rsac.fundamental_ransac(f1, f2, 1.5, max_iters=100_000, adaptive=False)
elif which == "c5":
    p5 = synth.pnp_problem(100_000, 0.5, seed=3)
    q2, q3 = torch.from_numpy(p5["points2d"]).to(dev), torch.from_numpy(p5["points3d"]).to(dev)
    run = lambda: rsac.pnp_ransac(q2, q3, p5["K"], 5000, 30.0, lo=True, refine=True)
else:
    raise SystemExit(f"unknown workload {which}")
walls = []
for i in range(reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    run()
    torch.cuda.synchronize()
    walls.append(time.perf_counter() - t)
print(which, "ms per call:", " ".join(f"{w * 1e3:.3f}" for w in walls), flush=True)
