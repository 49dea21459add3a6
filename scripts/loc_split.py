"""Where the location search's wall time goes (main_v1.py:254-297 over the 458 synthetic
candidates): the call with OpenCV's sampler and the LS + LM refit (the reference's own), without
the refit, and with the Philox sampler (no host subset draws), median of 15 each."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import rsac  # noqa: E402
from rsac import synth  # noqa: E402

lp = synth.location_problem(seed=0)
for sampler, refine in (("opencv", True), ("opencv", False), ("philox", True), ("philox", False)):
    ws = []
    for i in range(18):
        t = time.perf_counter()
        rsac.location_search(lp["pos3d"], lp["pixels"], lp["locations"], 75.0, sampler=sampler, refine=refine)
        if i >= 3:
            ws.append((time.perf_counter() - t) * 1e3)
    print(f"sampler={sampler} refine={refine}: {statistics.median(ws):.3f} ms", flush=True)
