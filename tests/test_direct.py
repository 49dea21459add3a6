"""OpenCV's `count == model_points` branches ([OpenCV 4.x, unvendored] solvepnp.cpp solvePnPRansac,
fundam.cpp findHomography), reached from main_v1.py:497-502, testpro-K.py:72-75 and main_v1.py:312.

solvePnPRansac: model_points is 4 for SOLVEPNP_P3P / AP3P and for npoints == 4 (kernel P3P), 5
otherwise (kernel EPnP).  When it equals the point count -- 4 points under any flags, 5 points under
the default flags -- no RANSAC runs: one solvePnP with that kernel on all points in input order,
every index an inlier, no final solve (no LM, no EPnP refit).  findHomography: 4 points (RANSAC or
method 0) -> runKernel on the 4 points, mask all ones, no LM.

The oracle restates both (rsac_oracle.c pnp_direct / orc_hom_ransac); the CPU tests pin it to its
own minimal solvers, the GPU tests compare the engine (rsac_pnp_ransac / _batched / _first_round /
orientation sweep, rsac_homography_ransac / _batched, the location search, the cv2 shims) with it
bit for bit.
"""
import numpy as np
import pytest

import np_ransac
import pyoracle as O
from rsac import synth


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def _pts(n, outl=0.0, seed=0):
    return synth.pnp_problem(n, outl, seed=seed)


# ---------------------------------------------------------------------------------------------
# oracle (CPU)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("sampler", ["philox", "opencv"])
@pytest.mark.parametrize("minimal", ["p3p", "epnp5"])
def test_oracle_four_points_is_one_p3p_solve(sampler, minimal):
    """4 points: P3P on (0, 1, 2, 3) whatever the flags, every index an inlier, no iterations."""
    pr = _pts(4, seed=11)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    ref = O.pnp_minimal(soa, np.arange(4), cam)
    assert ref is not None
    # OpenCV's sampler turns the Rodrigues round trip on: the pose is Rodrigues(rvec)
    Rexp = O.rvec_roundtrip(ref[0]) if sampler == "opencv" else ref[0]
    for fn in (O.pnp_ransac, O.pnp_ransac_seq):
        r = fn(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, 0x5EED, sampler=sampler, minimal=minimal)
        assert (r["best"], r["n_inliers"], r["iters"]) == (0, 4, 0)
        assert r["mask"].all()
        assert _bits_equal(r["R"], Rexp) and _bits_equal(r["t"], ref[1])


def test_oracle_five_points_default_flags_is_one_epnp_solve():
    pr = _pts(5, seed=12)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    ref = O.pnp_minimal_epnp5(soa, cam, np.arange(5))
    assert ref is not None
    r = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, sampler="opencv", minimal="epnp5")
    assert (r["best"], r["n_inliers"], r["iters"]) == (0, 5, 0) and r["mask"].all()
    Rexp = O.rvec_roundtrip(ref[0])  # OpenCV's sampler: the pose as Rodrigues(rvec)
    assert _bits_equal(r["R"], Rexp) and _bits_equal(r["t"], ref[1])
    npr = np_ransac.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, minimal="epnp5")
    assert (npr["best"], npr["n_inliers"], npr["iters"]) == (0, 5, 0)
    assert _bits_equal(npr["R"], Rexp) and _bits_equal(npr["t"], ref[1])
    raw = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, sampler="opencv", minimal="epnp5",
                       rvec=False)
    assert _bits_equal(raw["R"], ref[0])


def test_oracle_five_points_p3p_flags_run_ransac():
    """SOLVEPNP_P3P with 5 points: model_points 4 != 5, so RANSAC runs (OpenCV's loop)."""
    pr = _pts(5, seed=13)
    r = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, sampler="opencv", minimal="p3p")
    assert r["iters"] > 0


def test_oracle_direct_failure_is_no_model():
    """A degenerate 4-point set (all at one 3D point): solvePnP fails -> retval False, no inliers."""
    pr = _pts(4, seed=14)
    p3 = np.repeat(pr["points3d"][:1], 4, axis=0)
    r = O.pnp_ransac(p3, pr["points2d"], pr["K"], 30.0, 0.99, 500)
    assert (r["best"], r["n_inliers"]) == (-1, 0) and not r["mask"].any()


def test_oracle_homography_four_points_is_runkernel():
    hp = synth.homography_problem(4, 0.0, seed=5)
    soa = O.soa_hom(hp["src"], hp["dst"])
    ref = O.hom_minimal(soa, np.arange(4))
    r = O.hom_ransac(hp["src"], hp["dst"], 3.0, refine=True)
    assert (r["best"], r["n_inliers"], r["iters"]) == (0, 4, 0) and r["mask"].all()
    assert r["H_refined"] is None  # no LM for 4 points
    assert _bits_equal(r["H"], ref)


def test_oracle_sweep_direct_has_no_final_solve():
    """testpro-K.py's sweep on 5 points: every K's solvePnPRansac takes the direct branch (5 inliers),
    so the reference's `len(inliers) < 6` gate rejects every K; with the gate at 5 the rows are the
    raw direct poses (no LM final solve)."""
    pr = _pts(5, seed=15)
    Ks = synth.testpro_k_candidates()[:3]
    out = O.estimate_camera_orientation(pr["points3d"], pr["points2d"], Ks)
    assert out["best"] == -1
    out5 = O.estimate_camera_orientation(pr["points3d"], pr["points2d"], Ks, min_inliers=5)
    soa = O.soa_pnp(pr["points3d"], pr["points2d"])
    for k, K in enumerate(Ks):
        ref = O.pnp_minimal_epnp5(soa, O.cam_from_K(K), np.arange(5))
        row = out5["rows"][k]
        if ref is None:
            assert row is None
        else:
            assert _bits_equal(row["R"], O.rvec_roundtrip(ref[0])) and _bits_equal(row["t"], ref[1])


# ---------------------------------------------------------------------------------------------
# GPU vs oracle
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["philox", "opencv"])
@pytest.mark.parametrize("minimal", ["p3p", "epnp5"])
@pytest.mark.parametrize("refine", [False, "lm", "epnp"])
def test_gpu_pnp_four_points_direct(sampler, minimal, refine):
    import rsac
    pr = _pts(4, seed=21)
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 500, 30.0, sampler=sampler,
                                    minimal=minimal, refine=refine, return_info=True)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, sampler=sampler, minimal=minimal)
    assert ref["best"] == 0 and R is not None
    assert (info.best_hyp, info.n_inliers, info.iters) == (0, 4, 0)
    assert m.all()
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])  # no final solve


@pytest.mark.gpu
@pytest.mark.parametrize("minimal", ["p3p", "epnp5"])
def test_gpu_pnp_five_points(minimal):
    """5 points: direct EPnP under the default kernel, RANSAC under P3P; both equal the oracle."""
    import rsac
    pr = _pts(5, 0.0, seed=22)
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 500, 30.0, sampler="opencv",
                                    minimal=minimal, refine=False, return_info=True)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500, sampler="opencv", minimal=minimal)
    assert (info.best_hyp, info.n_inliers, info.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    assert (info.iters == 0) == (minimal == "epnp5")


@pytest.mark.gpu
def test_gpu_pnp_direct_device_tensors_and_failure():
    import torch
    import rsac
    pr = _pts(4, seed=23)
    p2 = torch.tensor(pr["points2d"], device="cuda")
    p3 = torch.tensor(pr["points3d"], device="cuda")
    R, t, m = rsac.pnp_ransac(p2, p3, pr["K"], 500, 30.0, refine="lm")
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500)
    assert m.is_cuda and bool(m.all())
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    bad = np.repeat(pr["points3d"][:1], 4, axis=0)
    R, t, m = rsac.pnp_ransac(pr["points2d"], bad, pr["K"], 500, 30.0)
    assert R is None and not m.any()
    R, t, m = rsac.pnp_ransac(torch.tensor(pr["points2d"], device="cuda"), torch.tensor(bad, device="cuda"),
                              pr["K"], 500, 30.0)
    assert R is None and not bool(m.any())


@pytest.mark.gpu
@pytest.mark.parametrize("minimal,sampler", [("p3p", "philox"), ("epnp5", "opencv")])
def test_gpu_pnp_batched_mixed_direct_and_ransac(minimal, sampler):
    """A ragged batch with 4- and 5-point problems among RANSAC ones: each problem equals its own
    oracle call (the direct ones without their final LM)."""
    import rsac
    probs = [_pts(n, o, seed=30 + i) for i, (n, o) in enumerate([(4, 0.0), (300, 0.5), (5, 0.0), (40, 0.3),
                                                                 (4, 0.0)])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 700, 30.0, sampler=sampler, minimal=minimal, refine=False)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 700, sampler=sampler, minimal=minimal)
        assert (R is None) == (ref["best"] < 0)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        if R is not None:
            assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    # with the LM final solve: the RANSAC problems refit, the direct ones stay raw
    out_lm = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                     [p["K"] for p in probs], 700, 30.0, sampler=sampler, minimal=minimal,
                                     refine=True)
    for i in (0, 2, 4):
        if minimal == "p3p" and i == 2:
            continue
        assert _bits_equal(out_lm[i][0], out[i][0]) and _bits_equal(out_lm[i][1], out[i][1])
        assert out_lm[i][3] == len(probs[i]["points3d"])


@pytest.mark.gpu
def test_gpu_first_round_direct_is_done():
    import rsac
    pr = _pts(4, seed=24)
    done, R, t, m, scan, info = rsac.pnp_ransac_first_round(pr["points2d"], pr["points3d"], pr["K"], 500, 30.0)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 500)
    assert done and m.all() and scan.best == 0
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


@pytest.mark.gpu
def test_gpu_cv2_shim_direct():
    import rsac
    import rsac.cv2compat as cv2
    pr = _pts(5, seed=25)
    ok, rvec, tvec, inl = cv2.solvePnPRansac(pr["points3d"], pr["points2d"], pr["K"], np.zeros((4, 1)),
                                             iterationsCount=5000, reprojectionError=30.0, confidence=0.99)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    ref = O.pnp_minimal_epnp5(soa, cam, np.arange(5))
    assert ok and inl.shape == (5, 1) and np.array_equal(inl.ravel(), np.arange(5))
    # the shim's models go through the Rodrigues round trip (OpenCV keeps them as rvecs)
    assert _bits_equal(rvec, rsac.rodrigues(O.rvec_roundtrip(ref[0]))) and _bits_equal(tvec.ravel(), ref[1])
    ok4, rvec4, tvec4, inl4 = cv2.solvePnPRansac(pr["points3d"][:4], pr["points2d"][:4], pr["K"], None,
                                                 flags=cv2.SOLVEPNP_EPNP)
    ref4 = O.pnp_minimal(soa, np.arange(4), cam)
    assert ok4 and np.array_equal(inl4.ravel(), np.arange(4))
    assert _bits_equal(rvec4, rsac.rodrigues(O.rvec_roundtrip(ref4[0]))) and _bits_equal(tvec4.ravel(), ref4[1])
    bad = np.repeat(pr["points3d"][:1], 4, axis=0)
    okb, _, _, inlb = cv2.solvePnPRansac(bad, pr["points2d"][:4], pr["K"], None)
    assert not okb and inlb is None


@pytest.mark.gpu
def test_gpu_homography_four_points_direct():
    import rsac
    import rsac.cv2compat as cv2
    hp = synth.homography_problem(4, 0.0, seed=6)
    soa = O.soa_hom(hp["src"], hp["dst"])
    ref = O.hom_minimal(soa, np.arange(4))
    H, m, info = rsac.homography_ransac(hp["src"], hp["dst"], 3.0, return_info=True)
    assert _bits_equal(H, ref) and m.all() and (info.best_hyp, info.n_inliers) == (0, 4)
    for method in (0, cv2.RANSAC):
        Hc, mc = cv2.findHomography(hp["src"], hp["dst"], method, 3.0)
        assert _bits_equal(Hc, ref) and mc.shape == (4, 1) and mc.all()
    # batched: 4-point problems among RANSAC ones
    probs = [synth.homography_problem(n, 0.3, seed=40 + i) for i, n in enumerate([4, 200, 4, 60])]
    out = rsac.homography_ransac_batched([p["src"] for p in probs], [p["dst"] for p in probs], 4.0, refine=False)
    for p, (Hb, mb, ni) in zip(probs, out):
        r = O.hom_ransac(p["src"], p["dst"], 4.0, refine=False)
        assert ni == r["n_inliers"] and np.array_equal(mb, r["mask"])
        assert _bits_equal(Hb, r["H"])


@pytest.mark.gpu
def test_gpu_location_search_four_noted_features():
    """main_v1.py:312 on a scene with 4 noted features: every location's findHomography takes the
    4-point branch; H, mask (all ones) and err1/err2 equal the restatement's."""
    import rsac
    pr = synth.location_problem(n_features=6, n_outliers=0, n_unnoted=2, seed=7, n_locations=40)
    res = rsac.location_search(pr["pos3d"], pr["pixels"], pr["locations"], 75.0)
    assert res.n_good == 4
    for l, loc in enumerate(pr["locations"]):
        r = O.find_homography(pr["pixels"], pr["pos3d"], loc, 75.0)
        assert res.ok[l] == (r["M"] is not None)
        np.testing.assert_array_equal(res.mask[l], r["mask"])
        if r["M"] is not None:
            assert r["mask"].all()
            assert _bits_equal(res.H[l], r["H"])
            np.testing.assert_allclose(res.err[l], [r["err1"], r["err2"]], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_gpu_orientation_sweep_direct():
    """The K sweep on 5 points (reference mode): every K takes the direct EPnP branch with 5
    inliers, so the reference's gate (< 6) rejects all; with the gate at 5 the per-K poses are the
    raw direct ones and the chosen K equals the restatement's."""
    import rsac
    pr = _pts(5, seed=26)
    fl, ss, img = [100.0, 150.0], [(127.0, 178.0), (178.0, 127.0)], (2142, 1620)
    rv, tv = rsac.estimate_camera_orientation(pr["points3d"], pr["points2d"], fl, ss, img)
    assert rv is None and tv is None
    res = rsac.estimate_camera_orientation(pr["points3d"], pr["points2d"], fl, ss, img, min_inliers=5,
                                           return_info=True)
    Ks, _ = rsac.intrinsics_grid(fl, ss, img)
    ref = O.estimate_camera_orientation(pr["points3d"], pr["points2d"], Ks, min_inliers=5)
    assert res.best == ref["best"]
    for k in range(len(Ks)):
        row = ref["rows"][k]
        assert res.ok[k] == (row is not None)
        if row is not None:
            assert _bits_equal(res.rvec_initial[k], rsac.rodrigues(row["R"]).ravel())
            assert res.n_inliers[k] == 5
