"""Times the DEM march for both ray layouts (RSAC_DEM_WPR, read once per process)."""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "code-reproduction-ransac_amd"))
from rsac import dem, synth  # noqa: E402

pr = synth.dem_problem(int(sys.argv[1]) if len(sys.argv) > 1 else 4096, seed=0)
g = dem.DemGrid.from_geotransform(pr["z"], pr["gt"])
e, n = dem.wgs84_to_utm(pr["origin_lonlat"][None])[0]
origin = np.array([e, n, pr["origin_height"]])
d = torch.from_numpy(pr["dirs"]).cuda()
for nr in (64, 1024, len(d)):
    ms = []
    for i in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        h, s = dem.ray_intersect_dem(origin, d[:nr], g)
        b.record()
        torch.cuda.synchronize()
        if i:
            ms.append(a.elapsed_time(b))
    print(os.environ.get("RSAC_DEM_WPR", "auto"), nr, "rays", f"{statistics.median(ms):.3f} ms", flush=True)
