"""C2 bench steps one after another on one context / stream, against steps alternating between
two contexts on two torch streams (independent batches pipelined: the next step's solve can start
on CUs the previous step's scoring tail has left).  Per-step wall time, interleaved, and the keys."""
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

pr = synth.pnp_problem(10000, 0.5, seed=0)
ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
H = 100_000
ctxs = [L.context(0), L.Context(0)]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]


def serial(k):
    out = None
    for _ in range(k):
        out = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True, device_result=True)
    return out


def piped(k):
    outs = [None, None]
    for i in range(k):
        j = i & 1
        with torch.cuda.stream(streams[j]):
            outs[j] = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True, device_result=True,
                                          context=ctxs[j])
    return outs[(k - 1) & 1]


def timed(fn, k=50):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = fn(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / k, int(out[0].item())


for fn in (serial, piped):
    timed(fn, 20)
res = {"serial": [], "piped": []}
for r in range(5):
    for name, fn in (("serial", serial), ("piped", piped)):
        ms, key = timed(fn)
        res[name].append(ms)
        print(name, f"{ms:.4f} ms/step key {key}", flush=True)
for name, v in res.items():
    print(f"{name}: median {statistics.median(v):.4f} ms/step ({H / statistics.median(v) * 1e3:.3e} hyp/s)")
