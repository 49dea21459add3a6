"""cv2-compatible shims: the reference's call sites become a one-line import swap.

    import rsac.cv2compat as cv2      # instead of `import cv2` for these calls

Covered calls (signatures and return tuples of the OpenCV Python binding):

* ``solvePnPRansac``   main_v1.py:497-502, testpro-K.py:72-75, testpro.py:536, test_pro.py:515
* ``findHomography``   main_v1.py:312, process.py:200, test02.py:263, testpro.py:350, test_pro.py:351
* ``Rodrigues``        main_v1.py:895, testpro-K.py:84, 136, 169
* ``projectPoints``    testpro-K.py:33 (compute_reprojection_error)
* ``solvePnPRefineLM`` main_v1.py:508-509, testpro-K.py:122-125

Only zero distortion is supported: every reference call passes
``np.zeros((4, 1))`` (main_v1.py:472, testpro-K.py:42); other values raise.
"""
from __future__ import annotations

import numpy as np

from . import api

RANSAC = 8
LMEDS = 4
SOLVEPNP_ITERATIVE = 0
SOLVEPNP_EPNP = 1
SOLVEPNP_P3P = 2
SOLVEPNP_AP3P = 5


class error(Exception):
    """Stands in for cv2.error (bad shapes, too few points)."""


def _check_dist(distCoeffs):
    if distCoeffs is None:
        return
    d = np.asarray(distCoeffs, np.float64)
    if d.size and np.any(d != 0):
        raise NotImplementedError("rsac supports zero distortion only (as every reference call site uses)")


def Rodrigues(src, dst=None, jacobian=None):
    """(3,1) vector <-> (3,3) matrix; returns (dst, None) (no Jacobian)."""
    return api.rodrigues(src), None


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0, confidence=0.99,
                   inliers=None, flags=SOLVEPNP_ITERATIVE):
    """-> (retval, rvec (3,1), tvec (3,1), inliers (M,1) int32 or None).

    OpenCV's structure (solvepnp.cpp solvePnPRansac): the MWC subset sequence of
    RANSACPointSetRegistrator; the minimal kernel by flags -- SOLVEPNP_P3P / AP3P (and any
    4-point input): P3P on 4-point samples (the benchmark kernel; no reference call passes it);
    otherwise (the default SOLVEPNP_ITERATIVE, EPNP, ...): EPnP on 5-point samples, with
    model_points = 5 in RANSACUpdateNumIters.  Final pose on the RANSAC inliers: EPnP for
    P3P / AP3P / EPNP (OpenCV re-solves P3P's inliers with EPnP); otherwise LM started from
    the best minimal model (SOLVEPNP_ITERATIVE's final solvePnP).  The inlier list is the
    RANSAC-phase mask, as OpenCV returns it.  Each minimal model is scored through
    Rodrigues(Rodrigues(R)), as PnPRansacCallback keeps it as an rvec (RSAC_F_RVEC_ROUNDTRIP).

    useExtrinsicGuess (testpro-K.py:73 passes False): as in solvePnPRansac, the guess never reaches
    the minimal solves (solvePnPGeneric drops it for the EPnP / P3P kernels) nor the
    count == model_points branch; with SOLVEPNP_ITERATIVE the final solve on the inliers starts
    from (rvec, tvec) instead of the RANSAC model, and both must then be given (OpenCV asserts).
    """
    _check_dist(distCoeffs)
    guess = bool(useExtrinsicGuess)
    if guess and (rvec is None or tvec is None):
        raise error("useExtrinsicGuess=True needs rvec and tvec")
    P3 = np.asarray(objectPoints, np.float64).reshape(-1, 3)
    P2 = np.asarray(imagePoints, np.float64).reshape(-1, 2)
    if P3.shape[0] != P2.shape[0]:
        raise error("objectPoints and imagePoints differ in length")
    if P3.shape[0] < 4:
        raise error("solvePnPRansac needs at least 4 points")
    # model_points: 4 for P3P / AP3P and for 4 points, 5 otherwise; when it equals the point count
    # (4 points, or 5 under the other flags) the engine takes OpenCV's direct branch: one solvePnP
    # on all points, every index an inlier, no final solve
    p3p = flags in (SOLVEPNP_P3P, SOLVEPNP_AP3P) or P3.shape[0] == 4
    refine = "epnp" if flags in (SOLVEPNP_P3P, SOLVEPNP_AP3P, SOLVEPNP_EPNP) else "lm"
    direct = P3.shape[0] == (4 if p3p else 5)  # solvePnPRansac's model_points == npoints branch
    from_guess = guess and refine == "lm" and not direct
    R, t, mask = api.pnp_ransac(P2, P3, cameraMatrix, int(iterationsCount), float(reprojectionError),
                                confidence=float(confidence), sampler="opencv", adaptive=True,
                                refine=False if from_guess else refine, minimal="p3p" if p3p else "epnp5",
                                rvec=True)
    if R is None:
        return False, (np.zeros((3, 1)) if rvec is None else rvec), (np.zeros((3, 1)) if tvec is None else tvec), None
    if from_guess:  # the final SOLVEPNP_ITERATIVE solve on the inliers, from the caller's pose
        R0 = api.rodrigues(np.asarray(rvec, np.float64).reshape(3))
        R, t = api.refine_pose_device(P2, P3, cameraMatrix, R0, np.asarray(tvec, np.float64).reshape(3),
                                      mask=np.asarray(mask))
    idx = np.flatnonzero(mask).astype(np.int32).reshape(-1, 1)
    return True, api.rodrigues(R).reshape(3, 1), t.reshape(3, 1), idx


def findHomography(srcPoints, dstPoints, method=0, ransacReprojThreshold=3.0, mask=None, maxIters=2000,
                   confidence=0.995):
    """-> (H (3,3) or None, mask (N,1) uint8)."""
    s = np.asarray(srcPoints, np.float64).reshape(-1, 2)
    d = np.asarray(dstPoints, np.float64).reshape(-1, 2)
    if s.shape[0] != d.shape[0]:
        raise error("srcPoints and dstPoints differ in length")
    if s.shape[0] < 4:
        raise error("findHomography needs at least 4 point correspondences")
    if method not in (0, RANSAC):
        raise NotImplementedError("only method=0 and cv2.RANSAC are provided")
    if method == 0 and s.shape[0] > 4:
        # all points, no RANSAC: runKernel's least-squares DLT, then the LM polish (npoints > 4)
        H = api.homography_fit(s, d)
        return H, (np.ones if H is not None else np.zeros)((s.shape[0], 1), np.uint8)
    # RANSAC; 4 points (either method) take findHomography's `method == 0 || npoints == 4` branch
    # inside the engine: runKernel on the 4 points, mask all ones, no LM
    H, m = api.homography_ransac(s, d, float(ransacReprojThreshold), max_iters=int(maxIters),
                                 confidence=float(confidence))
    return H, np.asarray(m, np.uint8).reshape(-1, 1)


def projectPoints(objectPoints, rvec, tvec, cameraMatrix, distCoeffs, imagePoints=None, jacobian=None,
                  aspectRatio=0):
    """(N,3) -> ((N,1,2) pixels, None): zero distortion, float64 as cv2 returns for f64 input; the
    projection runs on the GPU (rsac_pnp_reprojection_errors, testpro-K.py:33)."""
    _check_dist(distCoeffs)
    X = np.asarray(objectPoints, np.float64).reshape(-1, 3)
    r = np.asarray(rvec, np.float64).reshape(-1)
    R = api.rodrigues(r) if r.size == 3 else r.reshape(3, 3)
    t = np.asarray(tvec, np.float64).reshape(3)
    # the pixel argument only feeds the error, which projectPoints does not return
    _, proj = api.reprojection_errors(X, np.zeros((X.shape[0], 2)), cameraMatrix, R, t, return_projection=True)
    return proj.reshape(-1, 1, 2), None


def solvePnPRefineLM(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec, tvec, criteria=None):
    """LM refinement of (rvec, tvec) on the given correspondences -> (rvec, tvec), on the GPU
    (rsac_pnp_refine_lm: the bits of the host refit rsac_pnp_refine)."""
    _check_dist(distCoeffs)
    P3 = np.asarray(objectPoints, np.float64).reshape(-1, 3)
    P2 = np.asarray(imagePoints, np.float64).reshape(-1, 2)
    if P3.shape[0] != P2.shape[0]:
        raise error("objectPoints and imagePoints differ in length")
    if P3.shape[0] < 3:
        raise error("solvePnPRefineLM needs at least 3 points")
    R0 = api.rodrigues(np.asarray(rvec, np.float64).reshape(3))
    t0 = np.asarray(tvec, np.float64).reshape(3)
    R, t = api.refine_pose_device(P2, P3, cameraMatrix, R0, t0)
    return api.rodrigues(R).reshape(3, 1), t.reshape(3, 1)
