"""Is the bench step host-bound?  Times the enqueue of K asynchronous C2 steps (rsac.evaluate_range
with device results, as bench.py's step) against the wall time until the GPU is done, and the
per-call host time of each layer (Python wrapper vs the raw C call)."""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
H = int(os.environ.get("HYPS", "100000"))


def step():
    return rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True, device_result=True)


for _ in range(5):
    step()
torch.cuda.synchronize()
for K in (20, 100):
    t0 = time.perf_counter()
    calls = []
    for _ in range(K):
        t = time.perf_counter()
        step()
        calls.append(time.perf_counter() - t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"K={K}: enqueue {(t1 - t0) / K * 1e6:.1f} us/step (median call {statistics.median(calls) * 1e6:.1f}, "
          f"max {max(calls) * 1e6:.1f}), wall {(t2 - t0) / K * 1e6:.1f} us/step", flush=True)
