"""Kernel timeline of pnp_ransac (C2 problem, adaptive, LM refit), for rocprofv3 --kernel-trace:
the calls are separated by 2 ms sleeps so the trace splits into per-call groups (scripts/timeline.py).

    python3 scripts/trace_ms_to_best.py [minimal] [sampler]      (default p3p philox)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
p2d = torch.from_numpy(pr["points2d"]).cuda()
p3d = torch.from_numpy(pr["points3d"]).cuda()
minimal = sys.argv[1] if len(sys.argv) > 1 else "p3p"
sampler = sys.argv[2] if len(sys.argv) > 2 else "philox"
for i in range(12):
    torch.cuda.synchronize()
    time.sleep(0.002)
    t = time.perf_counter()
    rsac.pnp_ransac(p2d, p3d, pr["K"], 5000, 30.0, refine=True, minimal=minimal, sampler=sampler)
    torch.cuda.synchronize()
    print(f"call {i}: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
