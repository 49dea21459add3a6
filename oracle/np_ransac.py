"""TEST INFRASTRUCTURE / CPU BASELINE ONLY -- the "CPU NumPy path" of BASELINE.json configs[0].

Only tests/ and bench.py's cpu_baseline leg import this module; the product path (rsac/) never
does.  It restates OpenCV's solvePnPRansac loop (ptsetreg.cpp RANSACPointSetRegistrator::run,
reached from main_v1.py:497-502 / testpro-K.py:72-75) with the per-hypothesis scoring written in
NumPy, one hypothesis at a time as OpenCV runs it, stopping at the iteration bound:

* subsets: OpenCV's MWC getSubset sequence (state ~0), drawn by the C restatement
  (pyoracle.mwc_subsets) -- the sampler is not the scoring loop being timed;
* the minimal solve: the C restatement's EPnP-5 (the default SOLVEPNP_ITERATIVE kernel of every
  reference call site) or P3P (pyoracle.pnp_minimal_epnp5 / pnp_minimal);
* computeError (projectPoints with zero distortion, calibration.cpp) in NumPy: the f32-rounded
  inputs projected in f64 with the C restatement's operation order (orc_pnp_err), rounded to f32,
  e = dx*dx + dy*dy in f32, inlier iff e <= (float)thr^2;
* the best update "count > max(maxGoodCount, modelPoints - 1)" and RANSACUpdateNumIters after it.

tests/test_oracle_golden.py checks it against orc_pnp_ransac_k (best, count, iterations, mask).
"""
from __future__ import annotations

import numpy as np

import pyoracle as O


def compute_error(R, t, cam, X, Y, Z, U, V):
    """Per-point f32 squared reprojection error of one model (orc_pnp_err, vectorised).
    X..V are the f32-rounded points as float64 (X, Y, Z) and float32 (U, V) arrays."""
    R = np.asarray(R, np.float64).reshape(9)
    x = R[0] * X + R[1] * Y
    x = x + R[2] * Z
    x = x + t[0]
    y = R[3] * X + R[4] * Y
    y = y + R[5] * Z
    y = y + t[1]
    z = R[6] * X + R[7] * Y
    z = z + R[8] * Z
    z = z + t[2]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        iz = np.where(z != 0.0, 1.0 / np.where(z != 0.0, z, 1.0), 1.0)
        x = x * iz
        y = y * iz
        pu = x * cam[0] + cam[2]
        pv = y * cam[1] + cam[3]
        dx = U - pu.astype(np.float32)
        dy = V - pv.astype(np.float32)
        return dx * dx + dy * dy


def pnp_ransac(points3d, points2d, K, thr=30.0, confidence=0.99, max_iters=1000, minimal="epnp5", rvec=True):
    """OpenCV's sequential loop with NumPy scoring -> dict(best, n_inliers, iters, R, t, mask).
    rvec: each minimal model scored as Rodrigues(Rodrigues(R)) (PnPRansacCallback's rvec model)."""
    soa = O.soa_pnp(points3d, points2d)
    cam = O.cam_from_K(K)
    n = len(soa[0])
    k = 5 if minimal == "epnp5" else 4
    X, Y, Z = (soa[0].astype(np.float64), soa[1].astype(np.float64), soa[2].astype(np.float64))
    U, V = soa[3], soa[4]
    thr2 = np.float32(O.thr2(thr))
    solve0 = O.pnp_minimal_epnp5 if k == 5 else (lambda s, c, idx: O.pnp_minimal(s, idx, c))

    def solve(s, c, idx):
        m = solve0(s, c, idx)
        return m if (m is None or not rvec) else (O.rvec_roundtrip(m[0]), m[1])

    if n == 4 or (n == 5 and k == 5):
        # solvePnPRansac's model_points == npoints branch: one solvePnP on all points (P3P for 4),
        # every index an inlier, no RANSAC (pyoracle.pnp_ransac / rsac_oracle.c pnp_direct)
        m = (O.pnp_minimal if n == 4 else (lambda s, idx, c: O.pnp_minimal_epnp5(s, c, idx)))(soa, np.arange(n), cam)
        if m is not None and rvec:
            m = (O.rvec_roundtrip(m[0]), m[1])
        if m is None:
            return dict(best=-1, n_inliers=0, iters=0, R=None, t=None, mask=np.zeros(n, bool))
        return dict(best=0, n_inliers=n, iters=0, R=m[0], t=m[1], mask=np.ones(n, bool))
    subsets, sst = O.mwc_subsets(n, max(max_iters, 1), s=k)
    niters = max(max_iters, 1)
    best, max_good, best_model = -1, 0, None
    i = 0
    while i < niters and i < len(subsets):
        if sst[i] < 0:  # the sampler gave up (getSubset failed): the loop ends
            break
        m = solve(soa, cam, subsets[i]) if sst[i] > 0 else None
        if m is not None:
            R, t = m
            c = int(np.count_nonzero(compute_error(R, t, cam, X, Y, Z, U, V) <= thr2))
            if c > max(max_good, k - 1):
                best, max_good, best_model = i, c, (np.asarray(R).reshape(3, 3).copy(), np.asarray(t).copy())
                niters = O.update_num_iters(confidence, (n - c) / n, k, niters)
        i += 1
    if best < 0:
        return dict(best=-1, n_inliers=0, iters=i, R=None, t=None, mask=np.zeros(n, bool))
    R, t = best_model
    mask = compute_error(R, t, cam, X, Y, Z, U, V) <= thr2
    return dict(best=best, n_inliers=max_good, iters=i, R=R, t=t, mask=mask)
