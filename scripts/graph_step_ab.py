"""C2 bench step (evaluate_range, device results) eager vs captured into a HIP graph
(torch.cuda.CUDAGraph around the library's launches on the current stream): per-step wall time,
interleaved, and the replay's key equal to the eager key."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
H = 100_000


def step():
    return rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True, device_result=True)


k0, m0, mask0 = step()
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode="relaxed"):
    kg, mg, maskg = step()
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
assert int(kg.item()) == int(k0.item()), (int(kg.item()), int(k0.item()))
assert torch.equal(mg, m0) and torch.equal(maskg, mask0)
res = {"eager": [], "graph": []}
for rep in range(8):
    for name in res:
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            if name == "eager":
                step()
            else:
                g.replay()
        torch.cuda.synchronize()
        if rep:
            res[name].append((time.perf_counter() - t) / 20 * 1e3)
for name, v in res.items():
    print(f"{name}: {statistics.median(v):.4f} ms/step ({H / statistics.median(v) / 1e-3:.3e} hyp/s)", flush=True)
