"""Per-unit cost of the MFMA scorer: the C2 scoring launch (10k points, 100k hypotheses) with
every tile split into cells of c points (RSAC_DBG_MF_CELL_PTS), c = 256 ... 16384, kernel time by
HIP events (median of 20).  time = a * (wave iterations) + b * (units): b / a is the cost of one
unit (staging, epilogue, queue) in point-loop iterations."""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "code-reproduction-ransac_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10_000, 0.5, seed=0)
ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
H, N = 100_000, 10_000
ctx = rsac.context(0)
tiles = (H + 31) // 32
rows = []
CPS = [int(x) for x in sys.argv[1].split(',')] if len(sys.argv) > 1 else [0, 16384, 8192, 4096, 2048, 1024, 512, 256]
for cp in CPS:
    rsac.lib().rsac_debug_set(ctx.handle, 5, cp)
    for _ in range(5):
        rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, return_info=True, device=0)
    ms = [rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, return_info=True, device=0)[2].score_ms
          for _ in range(20)]
    cells = -(-N // cp) if cp else 1
    units = tiles * cells
    iters = tiles * sum(-(-(min(N, (c + 1) * cp) - c * cp) // 256) for c in range(cells)) if cp else tiles * -(-N // 256)
    rows.append((cp, units, iters, statistics.median(ms)))
    print(f"cell_pts {cp:6d}  units {units:7d}  block-iterations {iters:8d}  score_ms {statistics.median(ms):.4f}",
          flush=True)
rsac.lib().rsac_debug_set(ctx.handle, 5, 0)
if len(sys.argv) == 1:
    A = np.array([[r[2], r[1]] for r in rows[1:]], float)
    y = np.array([r[3] for r in rows[1:]])
    (a, b), *_ = np.linalg.lstsq(A, y, rcond=None)
    print(f"fit (cells only): ms = {a:.3e} * block-iterations + {b:.3e} * units; one unit = {b / a:.2f} iterations")
