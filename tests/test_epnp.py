"""EPnP on the inliers: the non-minimal final solve cv2.solvePnPRansac runs
when its minimal solver is P3P (cv2.solvePnPRansac with flags=SOLVEPNP_P3P).

OpenCV is not installed, so the algorithm is pinned to its restatement (oracle/rsac_oracle.c
orc_pnp_epnp, the steps of OpenCV's epnp.cpp with this project's numerics) -- "parity unpinned"
against OpenCV itself -- and to ground truth: on inlier sets it must land on the true pose as
closely as LM does.  Bar: bit-identical R, t to the restatement (host C-ABI rsac_pnp_epnp here;
the device pass of pnp_ransac(refine="epnp") under the gpu marker).
"""
import numpy as np
import pytest

import pyoracle as O
import rsac
from rsac import synth


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def _rms(R, t, pr, m):
    P = pr["points3d"][m].astype(np.float32).astype(np.float64)
    x = (P @ R.T + t) @ pr["K"].T
    return np.sqrt(np.mean(np.sum((x[:, :2] / x[:, 2:] - pr["points2d"][m]) ** 2, 1)))


@pytest.mark.parametrize("n,outl,seed", [(4, 0.0, 1), (5, 0.0, 2), (6, 0.0, 3), (40, 0.3, 4), (3000, 0.5, 5),
                                         (20000, 0.6, 6)])
def test_host_epnp_bit_exact_vs_restatement(n, outl, seed):
    pr = synth.pnp_problem(n, outl, seed=seed)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    m = pr["inlier"].astype(np.uint8)
    Ro, to = O.pnp_epnp(soa, m, cam)
    R, t = rsac.epnp_pose(pr["points2d"], pr["points3d"], pr["K"], mask=m)
    assert Ro is not None and R is not None
    assert _bits_equal(R, Ro) and _bits_equal(t, to)
    # all points (mask None) = mask of ones
    R1, t1 = rsac.epnp_pose(pr["points2d"][m > 0], pr["points3d"][m > 0], pr["K"])
    if m.sum() >= 4:
        Ro1, to1 = O.pnp_epnp(O.soa_pnp(pr["points3d"][m > 0], pr["points2d"][m > 0]), np.ones(int(m.sum()), np.uint8),
                              cam)
        assert _bits_equal(R1, Ro1) and _bits_equal(t1, to1)


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_epnp_accuracy_on_inliers(seed):
    pr = synth.pnp_problem(5000, 0.5, seed=seed, noise_px=1.0)
    m = pr["inlier"]
    R, t = rsac.epnp_pose(pr["points2d"], pr["points3d"], pr["K"], mask=m)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and np.linalg.det(R) > 0
    # as good as the truth on its own inliers (least squares in the image, up to EPnP's algebraic cost)
    assert _rms(R, t, pr, m) <= 1.02 * _rms(pr["R"], pr["t"], pr, m)
    C, C0 = -R.T @ t, -pr["R"].T @ pr["t"]
    assert np.linalg.norm(C - C0) < 1.0  # camera centre (UTM metres, f32-rounded inputs)
    # LM from the EPnP pose only polishes it
    R2, t2 = rsac.refine_pose(pr["points2d"], pr["points3d"], pr["K"], R, t, mask=m)
    assert _rms(R2, t2, pr, m) <= _rms(R, t, pr, m) + 1e-9


def test_epnp_degenerate_inputs():
    pr = synth.pnp_problem(200, 0.0, seed=10)
    P = pr["points3d"].copy()
    P[:, 2] = P[0, 2]  # a plane: EPnP's 4-control-point frame degenerates -> no model, as OpenCV's needs its planar branch
    R, t = rsac.epnp_pose(pr["points2d"], P, pr["K"])
    Ro, to = O.pnp_epnp(O.soa_pnp(P, pr["points2d"]), np.ones(200, np.uint8), O.cam_from_K(pr["K"]))
    assert (R is None) == (Ro is None)
    m = np.zeros(200, np.uint8)
    m[:3] = 1  # < 4 inliers
    assert rsac.epnp_pose(pr["points2d"], pr["points3d"], pr["K"], mask=m) == (None, None)
    assert O.pnp_epnp(O.soa_pnp(pr["points3d"], pr["points2d"]), m, O.cam_from_K(pr["K"])) == (None, None)


# --------------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("n,outl,seed", [(4000, 0.5, 21), (12000, 0.7, 22), (300, 0.3, 23)])
def test_gpu_ransac_epnp_final_solve(n, outl, seed):
    pr = synth.pnp_problem(n, outl, seed=seed)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000, 0x5EED)
    m8 = ref["mask"].astype(np.uint8)
    Ro, to = O.pnp_epnp(soa, m8, cam)
    R, t, m = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine="epnp")
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, Ro) and _bits_equal(t, to)  # k_pnp_epnp = the restatement, bit for bit
    R2, t2, _ = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine="epnp+lm")
    Rl, tl, _ = O.pnp_refine(soa, m8, cam, Ro, to)
    assert _bits_equal(R2, Rl) and _bits_equal(t2, tl)


@pytest.mark.gpu
def test_gpu_batched_epnp_and_cv2_flags():
    probs = [synth.pnp_problem(n, 0.4, seed=140 + i) for i, n in enumerate([60, 3000, 900])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 2000, 30.0, refine="epnp")
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 2000, 0x5EED)
        Ro, to = O.pnp_epnp(O.soa_pnp(p["points3d"], p["points2d"]), ref["mask"].astype(np.uint8),
                            O.cam_from_K(p["K"]))
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, Ro) and _bits_equal(t, to)
    # cv2.solvePnPRansac(..., flags=SOLVEPNP_P3P): the EPnP final solve
    from rsac import cv2compat as rcv
    p = probs[1]
    ok, rvec, tvec, inl = rcv.solvePnPRansac(p["points3d"], p["points2d"], p["K"], np.zeros((4, 1)),
                                             iterationsCount=2000, reprojectionError=30.0, flags=rcv.SOLVEPNP_P3P)
    R, t, m = rsac.pnp_ransac(p["points2d"], p["points3d"], p["K"], 2000, 30.0, refine="epnp", sampler="opencv")
    assert ok and _bits_equal(rcv.Rodrigues(rvec)[0], rsac.rodrigues(rsac.rodrigues(R))) and _bits_equal(tvec.ravel(), t)
