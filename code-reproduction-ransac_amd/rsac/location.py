"""Reference-shaped entry points of the camera-location search (main_v1.py:254-348, 862-866).

    from rsac.location import find_homographies, best_location
    num_matches = find_homographies(recs, camera_locations, 75.0)     # was main_v1.find_homographies
    theloci = best_location(num_matches)                              # main_v1.py:863-866

``recs`` / ``camera_locations`` are the reference's record dicts (main_v1.py:723-727, 758-759).
Plotting, CSV output and logging of the reference function are not reproduced; the numbers are.
"""
from __future__ import annotations

import numpy as np

from . import api


def find_homographies(recs, camera_locations, ransacbound: float = 75.0, grid_code_min: int = 0, **kw):
    """-> num_matches (L, 2) = (err1, err2) per location, as main_v1.py:254-297 returns it.

    Locations with grid_code < grid_code_min score (0, 0) without a RANSAC (main_v1.py:276-282).
    """
    pixels = np.array([r["pixel"] for r in recs], np.float64).reshape(-1, 2)
    pos3ds = np.array([r["pos3d"] for r in recs], np.float64).reshape(-1, 3)
    grids = np.array([cl["grid_code"] for cl in camera_locations])
    loc3ds = np.array([cl["pos3d"] for cl in camera_locations], np.float64).reshape(-1, 3)
    num_matches = np.zeros((loc3ds.shape[0], 2))
    sel = np.flatnonzero(grids >= grid_code_min)
    if sel.size:
        res = api.location_search(pos3ds, pixels, loc3ds[sel], ransacbound, **kw)
        num_matches[sel] = res.err
    return num_matches


def best_location(num_matches) -> int:
    """main_v1.py:863-866: argmin of err2 with zero scores replaced by 1e6."""
    e2 = np.array(num_matches, np.float64)[:, 1].copy()
    e2[e2 == 0] = 1000000
    return int(np.argmin(e2))
