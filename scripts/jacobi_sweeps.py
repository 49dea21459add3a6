"""How many JacobiSVD sweeps (and rotations per sweep) the EPnP-5 minimal solver's 12 x 12 cvSVD
of M^T M takes on the C2 problem's samples (the oracle's study hook; CPU only):

    python3 scripts/jacobi_sweeps.py [samples]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "code-reproduction-ransac_amd")]
import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
from rsac import synth  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
L = O.lib()
for f in (L.orc_cvq_sweep_hist, L.orc_cvq_rot_hist):
    f.argtypes, f.restype = [C.c_int, C.c_int], C.c_long
h0 = [L.orc_cvq_sweep_hist(12, k) for k in range(32)]
r0 = [L.orc_cvq_rot_hist(12, k) for k in range(32)]
pr = synth.pnp_problem(10_000, 0.5, seed=0)
soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
subs, _ = O.mwc_subsets(10_000, S, s=5)
for idx in subs:
    O.pnp_minimal_epnp5(soa, cam, idx)
h = [L.orc_cvq_sweep_hist(12, k) - h0[k] for k in range(32)]
r = [L.orc_cvq_rot_hist(12, k) - r0[k] for k in range(32)]
tot = sum(h)
print(f"{tot} decompositions of 12 x 12")
print("sweeps (incl. the last, rotation-free one; 31 = hit max_iter 30):")
for k, c in enumerate(h):
    if c:
        print(f"  {k:2d}: {c:6d} ({100 * c / tot:5.1f} %)")
print("rotations per decomposition in sweep k (of 66 pairs):")
for k, c in enumerate(r):
    if c:
        print(f"  sweep {k + 1:2d}: {c / tot:6.2f}")
