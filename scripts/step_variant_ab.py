"""C2 bench step (evaluate_range with device results, warmed GPU) per scoring variant,
interleaved: ms/step over 50-step batches."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

variants = [int(v) for v in sys.argv[1].split(",")]
pr = synth.pnp_problem(10000, 0.5, seed=0)
ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
H = 100_000


def step():
    return rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True, device_result=True)


res = {v: [] for v in variants}
keys = {}
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:  # warm the clocks
    step()
torch.cuda.synchronize()
for rep in range(int(os.environ.get("ROUNDS", "8"))):
    for v in variants:
        L.check(L.lib().rsac_set_score_variant(v))
        k, _, _ = step()
        torch.cuda.synchronize()
        keys.setdefault(v, int(k.item()))
        assert keys[v] == keys[variants[0]]
        t = time.perf_counter()
        for _ in range(50):
            step()
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t) / 50 * 1e3)
L.check(L.lib().rsac_set_score_variant(-1))
for v in variants:
    m = statistics.median(res[v])
    print(f"variant {v}: {m:.4f} ms/step ({H / m / 1e-3:.4e} hyp/s), min {min(res[v]):.4f}", flush=True)
