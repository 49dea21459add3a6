"""C3 (BASELINE.json configs[2]) alone, for a rocprofv3 kernel trace: 1024 problems x 2000 points,
1024 hypotheses each, one pnp_ransac_batched_flat call per repeat, inputs resident in HBM.

    rocprofv3 --kernel-trace --stats -d gpurun_out/c3 -- python3 scripts/c3_prof.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "code-reproduction-ransac_amd")]
import torch  # noqa: E402

import rsac  # noqa: E402
from bench import c3_problems  # noqa: E402

h2, h3, off, Ks = c3_problems()
p2 = torch.from_numpy(h2).cuda()
p3 = torch.from_numpy(h3).cuda()
walls = []
for i in range(int(os.environ.get("C3_REPEATS", "12"))):
    torch.cuda.synchronize()
    t = time.perf_counter()
    rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 1024, 30.0, adaptive=False, refine=False)
    torch.cuda.synchronize()
    walls.append(time.perf_counter() - t)
print("c3 ms per call:", " ".join(f"{w * 1e3:.3f}" for w in walls), flush=True)
