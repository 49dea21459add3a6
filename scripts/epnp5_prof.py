"""The reference's own minimal solver (SOLVEPNP_ITERATIVE: EPnP on 5-point samples, testpro-K.py:72-75,
main_v1.py:497-502) against P3P at a fixed budget on the C2 problem, inputs in HBM:

    python3 scripts/epnp5_prof.py [hyps] [repeats]      (under rocprofv3 --kernel-trace for kernel times)

Prints each kernel's wall time per call and the solve/score split from rsac's HIP events.
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "code-reproduction-ransac_amd")]
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pr = synth.pnp_problem(10_000, 0.5, seed=0)
dev = torch.device("cuda", 0)
p2, p3 = torch.from_numpy(pr["points2d"]).to(dev), torch.from_numpy(pr["points3d"]).to(dev)
for minimal in ("p3p", "epnp5"):
    walls, sol, sco = [], [], []
    for i in range(reps + 1):
        torch.cuda.synchronize()
        t = time.perf_counter()
        R, t_, m, info = rsac.pnp_ransac(p2, p3, pr["K"], H, 30.0, adaptive=False, refine=False, minimal=minimal,
                                         return_info=True)
        torch.cuda.synchronize()
        if i:
            walls.append((time.perf_counter() - t) * 1e3)
            sol.append(info.solve_ms)
            sco.append(info.score_ms)
    print(f"{minimal}: {H} hyps, ms per call {statistics.median(walls):.3f} (solve {statistics.median(sol):.3f}, "
          f"score {statistics.median(sco):.3f}), {H / statistics.median(walls) * 1e3:.3e} hyp/s, "
          f"inliers {int(m.sum())}", flush=True)
# the reference's own call (main_v1.py:497-502: default flags, iterationsCount 5000, thr 30, conf 0.99),
# adaptive with the LM final solve, in both minimal modes: ms to the best model
for minimal, sampler in (("p3p", "philox"), ("epnp5", "opencv"), ("epnp5", "philox")):
    walls = []
    for i in range(reps + 2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, adaptive=True, refine=True, minimal=minimal,
                        sampler=sampler)  # the plain call: no stats, so no HIP timing events
        torch.cuda.synchronize()
        if i >= 2:
            walls.append((time.perf_counter() - t) * 1e3)
    R, t_, m, info = rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, adaptive=True, refine=True, minimal=minimal,
                                     sampler=sampler, return_info=True)
    print(f"ms-to-best {minimal}/{sampler}: {statistics.median(walls):.3f} ms, iterations {info.iters}, "
          f"inliers {int(m.sum())}, solve {info.solve_ms:.3f} ms, score {info.score_ms:.3f} ms", flush=True)
