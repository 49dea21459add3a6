"""Wall time of testpro-K's sweep (rsac.estimate_camera_orientation, 27 Ks, reference mode) and of the
location search, median of 15 calls each."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import rsac  # noqa: E402
from rsac import synth  # noqa: E402

ws = []
for i in range(18):
    t = time.perf_counter()
    rsac.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, synth.TESTPRO_K_FOCALS,
                                     synth.TESTPRO_K_SENSORS, synth.TESTPRO_K_IMAGE)
    if i >= 3:
        ws.append((time.perf_counter() - t) * 1e3)
print(f"k sweep: {statistics.median(ws):.3f} ms", flush=True)
lp = synth.location_problem(seed=0)
ws = []
for i in range(18):
    t = time.perf_counter()
    rsac.location_search(lp["pos3d"], lp["pixels"], lp["locations"], 75.0)
    if i >= 3:
        ws.append((time.perf_counter() - t) * 1e3)
print(f"location search: {statistics.median(ws):.3f} ms", flush=True)
