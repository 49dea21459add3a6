"""C3 with the inputs handed over as host f64 arrays (the PCIe-inclusive figure of bench.py's
c3_batched line): wall time per pnp_ransac_batched_flat call."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "code-reproduction-ransac_amd")]
import torch  # noqa: E402

import rsac  # noqa: E402
from bench import c3_problems  # noqa: E402

h2, h3, off, Ks = c3_problems()
walls = []
for i in range(8):
    torch.cuda.synchronize()
    t = time.perf_counter()
    rsac.pnp_ransac_batched_flat(h2, h3, off, Ks, 1024, 30.0, adaptive=False, refine=False)
    torch.cuda.synchronize()
    if i >= 2:
        walls.append((time.perf_counter() - t) * 1e3)
print(f"c3 host inputs: median {statistics.median(walls):.3f} ms per call ({walls})")
