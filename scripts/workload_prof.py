"""One BASELINE workload alone, for rocprofv3 passes (kernel trace and separate --pmc passes) that
attribute every kernel to its config (scripts/gpu_secondary_profile.sh):

    python3 scripts/workload_prof.py c2|c3|c4|c5|loc|ksweep|epnp [repeats]

c2: the bench step (rsac.evaluate_range, 100k hypotheses over the 10k-point problem: solve + score
    + key + mask); c3: pnp_ransac_batched_flat over 1024 x 2000 points, 1024 hypotheses each; c4:
    fundamental_ransac, 50k matches, 100k hypotheses, adaptive off; c5: pnp_ransac(lo=True) on the
    100k-point problem (the LO chain: k_pnp_refine with a source record + k_pnp_lo_count); loc:
    location_search over the 458 synthetic candidates (main_v1.py:254-297); ksweep:
    estimate_camera_orientation on testpro-K's 12 points x 27 intrinsics (testpro-K.py:39-162,
    reference mode); epnp: 20k EPnP-5 hypotheses on MWC subsets, adaptive off (k_cvepnp5_*).
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
elif which == "loc":  # find_homographies of main_v1.py:254-297 for the 458 candidates, one call
    lp = synth.location_problem(seed=0)
    run = lambda: rsac.location_search(lp["pos3d"], lp["pixels"], lp["locations"], 75.0)
elif which == "ksweep":  # estimate_camera_orientation of testpro-K.py:39-162, the reference's own mode
    run = lambda: rsac.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS,
                                                   synth.TESTPRO_K_FOCALS, synth.TESTPRO_K_SENSORS,
                                                   synth.TESTPRO_K_IMAGE)
elif which == "epnp":  # the reference mode's minimal solver at a fixed 20k budget on the C2 problem
    pr = synth.pnp_problem(10_000, 0.5, seed=0)
    p2, p3 = torch.from_numpy(pr["points2d"]).to(dev), torch.from_numpy(pr["points3d"]).to(dev)
    run = lambda: rsac.pnp_ransac(p2, p3, pr["K"], 20_000, 30.0, sampler="opencv", minimal="epnp5", adaptive=False,
                                  refine=False)
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
