"""The drop-in shims of rsac.cv2compat at the reference's own call sites, and the K sweep.

Call sites: cv2.findHomography main_v1.py:312 (process.py:200, test02.py:263),
cv2.projectPoints in compute_reprojection_error testpro-K.py:32-36, cv2.solvePnPRefineLM
main_v1.py:508-509 / testpro-K.py:122-125, cv2.Rodrigues main_v1.py:895 / testpro-K.py:84, and
estimate_camera_orientation testpro-K.py:39-125 (row a8).  INTEGRATION.md promises that these
become a one-line import swap; these tests call the shims with the reference's argument shapes
and check the return shapes and values against the oracle (oracle/) and the reference's fixtures.
"""
import json
import os

import numpy as np
import pytest

import pyoracle as O
import rsac
import rsac.cv2compat as rcv
from rsac import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden", "debuglog_homography.json")


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def _rodrigues_cases():
    rng = np.random.default_rng(5)
    vecs = []
    for k in range(100):
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        if k < 20:
            ang = 10.0 ** rng.uniform(-12, -2)  # near 0
        elif k < 40:
            ang = np.pi - 10.0 ** rng.uniform(-9, -2)  # near pi
        elif k < 45:
            ang = np.pi
        else:
            ang = rng.uniform(0, np.pi)
        vecs.append(axis * ang)
    vecs.append(np.zeros(3))
    return np.array(vecs)


def test_rodrigues_shim_matches_oracle():
    """cv2.Rodrigues (main_v1.py:895): the shim's (3,3) and (3,1) results equal the oracle's bitwise
    on 100 vectors, angles near 0 and near pi included; the round trip returns the rotation."""
    for r in _rodrigues_cases():
        R, jac = rcv.Rodrigues(r.reshape(3, 1))
        assert jac is None and R.shape == (3, 3)
        assert _bits_equal(R, O.rodrigues_v2m(r))
        v, _ = rcv.Rodrigues(R)
        assert v.shape == (3, 1)
        assert _bits_equal(v.reshape(3), O.rodrigues_m2v(R))
        R2, _ = rcv.Rodrigues(v)
        if v.any():
            np.testing.assert_allclose(R2, R, atol=1e-4)  # near pi the vector loses ~sin(theta) of precision (OpenCV alike)
        else:  # OpenCV's matrix -> vector returns 0 when sin(theta) < 1e-5 (calibration.cpp): so does the shim
            assert np.linalg.norm(r) < 2e-5 and np.array_equal(R2, np.eye(3))
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)


@pytest.mark.gpu
def test_find_homography_shim_reproduces_debuglog_masks():
    """main_v1.py:312 through the shim: H, mask = findHomography(pos2, pixels, cv2.RANSAC, thr); the
    (N, 1) uint8 masks equal the 24 masks OpenCV logged in the reference's debug.log."""
    d = json.load(open(GOLD))
    n = 0
    for b in d["blocks"]:
        if not b["complete"]:
            continue
        M = np.array(b["M"])
        pp2 = np.array(b["pp2"])
        hs = np.c_[pp2, np.ones(len(pp2))] @ M.T
        src = hs[:, :2] / hs[:, 2:3]
        H, mask = rcv.findHomography(src, np.array(b["p1"], np.float64), rcv.RANSAC, d["threshold"])
        assert H.shape == (3, 3) and mask.shape == (len(src), 1) and mask.dtype == np.uint8
        np.testing.assert_array_equal(mask[:, 0], np.array(b["mask"], np.uint8))
        n += 1
    assert n == 24


@pytest.mark.gpu
def test_project_points_and_reprojection_error_match_f64_formula():
    """testpro-K.py:32-36: projectPoints (shim) and compute_reprojection_error (rsac) on the GPU equal
    the oracle's f64 formula bit for bit (f64 inputs, no CV_32F rounding), on the 12 testpro-K
    points and on a 50k-point scene (device tensors too)."""
    import torch
    K = synth.testpro_k_candidates()[10]
    pr = synth.pnp_problem(12, 0.0, seed=3, K=K)
    q = synth.pnp_problem(50_000, 0.3, seed=4)
    for P3, P2, K_, R, t in [(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, K, pr["R"], pr["t"]),
                             (q["points3d"], q["points2d"], q["K"], q["R"], q["t"])]:
        rvec = rsac.rodrigues(R).reshape(3, 1)
        Rp = O.rodrigues_v2m(O.rodrigues_m2v(R))  # projectPoints rotates by Rodrigues(rvec)
        e_ref, p_ref = O.reproj_errors(P3, P2, K_, Rp, t, projections=True)
        proj, jac = rcv.projectPoints(P3, rvec, t.reshape(3, 1), K_, np.zeros((4, 1)))
        assert jac is None and proj.shape == (len(P3), 1, 2)
        assert _bits_equal(proj.reshape(-1, 2), p_ref)
        err = rsac.compute_reprojection_error(P3, P2, K_, np.zeros((4, 1)), rvec, t.reshape(3, 1))
        assert _bits_equal(err, e_ref)
        # numpy's own expression of the reference on the oracle's projections
        np.testing.assert_array_equal(err, np.linalg.norm(P2 - p_ref, axis=1))
        d3 = torch.from_numpy(np.asarray(P3, np.float64)).cuda()
        d2 = torch.from_numpy(np.asarray(P2, np.float64)).cuda()
        ed = rsac.reprojection_errors(d3, d2, K_, Rp, t)
        assert ed.is_cuda and _bits_equal(ed.cpu().numpy(), e_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,outl,seed", [(12, 0.0, 1), (800, 0.4, 2), (20000, 0.5, 3)])
def test_solve_pnp_refine_lm_shim_matches_oracle(n, outl, seed):
    """main_v1.py:508-509 through the shim: solvePnPRefineLM(pos3d[inl], pixels[inl], K, dist, rvec,
    tvec) on the GPU equals the oracle's LM (orc_pnp_refine) on the same subset, bit for bit."""
    pr = synth.pnp_problem(n, outl, seed=seed)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 2000, 0x5EED)
    inl = np.flatnonzero(ref["mask"])
    rvec = rsac.rodrigues(ref["R"]).reshape(3, 1)
    r2, t2 = rcv.solvePnPRefineLM(pr["points3d"][inl], pr["points2d"][inl], pr["K"], np.zeros((4, 1)), rvec,
                                  ref["t"].reshape(3, 1))
    assert r2.shape == (3, 1) and t2.shape == (3, 1)
    sub = O.soa_pnp(pr["points3d"][inl], pr["points2d"][inl])
    Ro, to, _ = O.pnp_refine(sub, np.ones(len(inl), np.uint8), O.cam_from_K(pr["K"]), rsac.rodrigues(rvec), ref["t"])
    assert _bits_equal(rsac.rodrigues(r2), rsac.rodrigues(rsac.rodrigues(Ro)))
    assert _bits_equal(t2.reshape(3), to)
    # the host twin gives the same bits
    Rh, th = rsac.refine_pose(pr["points2d"][inl], pr["points3d"][inl], pr["K"], rsac.rodrigues(rvec), ref["t"])
    assert _bits_equal(Rh, Ro) and _bits_equal(th, to)


@pytest.mark.gpu
def test_solve_pnp_ransac_shim_shapes_and_gate():
    """main_v1.py:497-506: the shim's (retval, rvec, tvec, inliers) shapes, and the reference's
    own `len(inliers) < 6` gate works on its output unchanged."""
    pr = synth.pnp_problem(3000, 0.5, seed=8)
    ok, rvec, tvec, inl = rcv.solvePnPRansac(pr["points3d"], pr["points2d"], pr["K"], np.zeros((4, 1)),
                                             iterationsCount=5000, reprojectionError=30.0, confidence=0.99)
    assert ok and rvec.shape == (3, 1) and tvec.shape == (3, 1) and inl.dtype == np.int32 and inl.shape[1] == 1
    assert len(inl) >= 6
    # the default flags (SOLVEPNP_ITERATIVE): OpenCV's MWC sequence of 5-point EPnP samples
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000, 0x5EED, sampler="opencv",
                       minimal="epnp5")
    np.testing.assert_array_equal(inl[:, 0], np.flatnonzero(ref["mask"]))
    P3 = np.tile(np.array([[739000.0, 2888500.0, 700.0]]), (50, 1))
    ok, _, _, inl = rcv.solvePnPRansac(P3, np.tile([[100.0, 200.0]], (50, 1)), pr["K"], np.zeros((4, 1)))
    assert not ok and inl is None
    with pytest.raises(rcv.error):
        rcv.solvePnPRansac(P3[:3], np.zeros((3, 2)), pr["K"], np.zeros((4, 1)))


@pytest.mark.gpu
@pytest.mark.parametrize("sampler,minimal", [("opencv", "epnp5"), ("philox", "p3p"), ("opencv", "p3p")])
def test_estimate_camera_orientation_matches_restatement(sampler, minimal):
    """testpro-K.py:39-125 on its own data (12 points, 27 intrinsics): the chosen K, every K's gate,
    mean inlier error (bitwise: the oracle restates the device's summation order) and pose, and the
    refined (rvec, tvec) equal the oracle's composition of the same steps.  The first case is the
    reference's own mode (testpro-K.py:72-75 passes no flags: EPnP on 5-point MWC samples + the LM
    final solve), which is also the function's default; the others run the P3P benchmark kernel."""
    kw = {} if (sampler, minimal) == ("opencv", "epnp5") else dict(sampler=sampler, minimal=minimal)
    res = rsac.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, synth.TESTPRO_K_FOCALS,
                                           synth.TESTPRO_K_SENSORS, synth.TESTPRO_K_IMAGE, synth.TESTPRO_K_ORIGIN,
                                           return_info=True, **kw)
    Ks = synth.testpro_k_candidates()
    np.testing.assert_array_equal(res.K, np.stack(Ks))
    ref = O.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, Ks, sampler=sampler,
                                        minimal=minimal)
    assert res.best == ref["best"]
    for k, row in enumerate(ref["rows"]):
        if row is None:
            assert not res.ok[k]
            continue
        assert res.n_inliers[k] == row["n_inliers"]
        np.testing.assert_array_equal(res.masks[k], row["mask"])
        assert _bits_equal(res.tvec_initial[k], row["t"])
        if np.isnan(row["mean"]):
            assert not res.ok[k] and np.isnan(res.mean_error[k])
        else:
            assert res.ok[k] and _bits_equal(res.mean_error[k], row["mean"])
            # numpy's mean of the reference's error vector, to rounding
            Rp = O.rodrigues_v2m(O.rodrigues_m2v(row["R"]))
            e = O.reproj_errors(synth.TESTPRO_K_POS3D[row["mask"]], synth.TESTPRO_K_PIXELS[row["mask"]], Ks[k], Rp,
                                row["t"])
            np.testing.assert_allclose(res.mean_error[k], np.mean(e), rtol=1e-13)
    assert res.best >= 0
    assert _bits_equal(rsac.rodrigues(res.rvec), rsac.rodrigues(rsac.rodrigues(ref["R"])))
    assert _bits_equal(res.tvec.reshape(3), ref["t"])
    # reported, not asserted: test_pro.py:801-802 hard-codes fx=2529, fy=1365 (f=150 mm, 127x178
    # film), the reference sweep's pick under OpenCV's EPnP kernel
    f, (sw, sh) = res.focal_sensor[res.best]
    print(f"K sweep ({sampler}, {minimal}): chose f={f} mm, {sw}x{sh} mm (fx={res.K[res.best][0, 0]:.1f}); "
          f"test_pro.py:801 hint f=150 mm 127x178 -> {'same' if (f, sw, sh) == (150, 127, 178) else 'different'}")
    # the ranking by distance to the known origin (testpro-K.py:103) is sorted
    d = [r[0] for r in res.ranking]
    assert d == sorted(d) and len(d) == int(res.ok.sum())
    # the plain call returns the reference's (rvec, tvec)
    rv, tv = rsac.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, synth.TESTPRO_K_FOCALS,
                                              synth.TESTPRO_K_SENSORS, synth.TESTPRO_K_IMAGE, **kw)
    assert _bits_equal(rv, res.rvec) and _bits_equal(tv, res.tvec)


@pytest.mark.gpu
def test_estimate_camera_orientation_all_fail():
    """Every K fails the gate (6 points, so at most 6 inliers is allowed only with a perfect fit;
    here a degenerate set): (None, None) as the reference's early return (testpro-K.py:99-101)."""
    P3 = np.tile(np.array([[739000.0, 2888500.0, 700.0]]), (8, 1))
    P2 = np.tile(np.array([[100.0, 200.0]]), (8, 1))
    rv, tv = rsac.estimate_camera_orientation(P3, P2, [90, 100], [(102, 127)], (2142, 1620))
    assert rv is None and tv is None


def test_estimate_camera_orientation_rejects_gate_below_three():
    """a gate below 3 would let a winner through that solvePnPRefineLM cannot refine;
    it is rejected before any device work (the C-ABI rejects it too: rsac_pnp_orientation_sweep)."""
    with pytest.raises(ValueError, match="min_inliers"):
        rsac.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, [150], [(127, 178)],
                                         synth.TESTPRO_K_IMAGE, min_inliers=2)


def test_solve_pnp_ransac_shim_guess_needs_rvec_tvec():
    """cv2.solvePnPRansac asserts rvec / tvec are given when useExtrinsicGuess is set (testpro-K.py:73
    passes the flag, False); the shim raises before any device work."""
    with pytest.raises(rcv.error):
        rcv.solvePnPRansac(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, synth.testpro_k_candidates()[10],
                           np.zeros((4, 1)), useExtrinsicGuess=True, iterationsCount=100, reprojectionError=30.0)


@pytest.mark.gpu
def test_solve_pnp_ransac_shim_extrinsic_guess():
    """useExtrinsicGuess=True with SOLVEPNP_ITERATIVE: the RANSAC phase is unchanged (same inliers),
    and the final solve on those inliers starts from the caller's (rvec, tvec) -- the LM from that
    start on the RANSAC-phase mask (the oracle's refit), not from the minimal model."""
    pr = synth.pnp_problem(1500, 0.4, seed=61)
    K = pr["K"]
    ok0, rv0, tv0, in0 = rcv.solvePnPRansac(pr["points3d"], pr["points2d"], K, np.zeros((4, 1)), iterationsCount=800,
                                            reprojectionError=30.0)
    rv_g = rv0 + np.array([[2e-3], [-1e-3], [1e-3]])
    tv_g = tv0 + np.array([[5.0], [-3.0], [2.0]])
    ok, rv, tv, inl = rcv.solvePnPRansac(pr["points3d"], pr["points2d"], K, np.zeros((4, 1)), rvec=rv_g.copy(),
                                         tvec=tv_g.copy(), useExtrinsicGuess=True, iterationsCount=800,
                                         reprojectionError=30.0)
    assert ok0 and ok
    np.testing.assert_array_equal(inl, in0)
    mask = np.zeros(len(pr["points3d"]), np.uint8)
    mask[inl.ravel()] = 1
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(K)
    Rl, tl, _ = O.pnp_refine(soa, mask, cam, O.rodrigues_v2m(rv_g.ravel()).reshape(9), tv_g.ravel())
    assert _bits_equal(tv.ravel(), tl)
    assert _bits_equal(rcv.Rodrigues(rv)[0], rsac.rodrigues(rsac.rodrigues(Rl)))
