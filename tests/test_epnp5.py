"""The OpenCV-default minimal solver: cv2.solvePnPRansac with flags=SOLVEPNP_ITERATIVE samples
5 points (model_points = 5) and solves each sample with solvePnP(SOLVEPNP_EPNP) (OpenCV
solvepnp.cpp, PnPRansacCallback::runKernel with ransac_kernel_method = SOLVEPNP_EPNP);
RANSACUpdateNumIters runs with model_points 5.  This is the kernel every reference call site runs
(main_v1.py:497-502, testpro-K.py:72-75 pass no `flags`), and the default of
rsac.estimate_camera_orientation and of rsac.cv2compat.solvePnPRansac.

Oracle: orc_pnp_minimal_epnp5 (oracle/rsac_oracle.c) = orc_cv_epnp (oracle/cv_epnp.c), OpenCV's
operation sequence restated from its 4.x sources (undistortPoints' f32 round trip, epnp.cpp,
lapack.cpp's JacobiSVD; OpenCV itself is not installed, so against OpenCV the bits are "parity
unpinned" -- see tests/test_cv_epnp.py and profiles/r06/epnp_variants.md for why the sequence
matters).  Bar: bit-identical models, counts, winner, mask and iteration count between the GPU
solve (k_cvepnp5_a / k_cvepnp5_svd / k_cvepnp5_c), the host twin (rsac_pnp_epnp_minimal, the
same source) and the oracle.
"""
import numpy as np
import pytest

import pyoracle as O
import rsac
from rsac import synth


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def _mwc5(n, H):
    """OpenCV's getSubset sequence of 5-point samples (one MWC state from ~0)."""
    import ctypes as C
    st = C.c_uint64(2**64 - 1)
    subs = np.zeros((H, 5), np.int32)
    sst = np.zeros(H, np.int8)
    O.lib().orc_mwc_subsets(C.byref(st), n, 5, H, None, None, None, None, subs.reshape(-1), sst)
    return subs, sst


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_minimal_epnp5_host_twin_equals_oracle(seed):
    """The library's host twin of the three kernels (rsac.epnp_minimal: rsac_cvepnp.h, the 12 x 12
    JacobiSVD serially) on every MWC sample returns the oracle's bits."""
    pr = synth.pnp_problem(500, 0.3, seed=seed)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    subs, _ = _mwc5(500, 200)
    for idx in subs:
        ro = O.pnp_minimal_epnp5(soa, cam, idx)
        R, t = rsac.epnp_minimal(pr["points2d"][idx], pr["points3d"][idx], pr["K"])
        assert ro is not None
        assert _bits_equal(R, ro[0]) and _bits_equal(t, ro[1])


def test_minimal_epnp5_recovers_the_pose_from_clean_samples():
    pr = synth.pnp_problem(200, 0.0, seed=11, noise_px=0.0)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    C0 = -pr["R"].T @ pr["t"]
    subs, _ = _mwc5(200, 32)
    errs = []
    for idx in subs:
        ro = O.pnp_minimal_epnp5(soa, cam, idx)
        assert ro is not None
        R, t = ro
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-9)
        errs.append(np.linalg.norm(-R.T @ t - C0))
    # f32-rounded UTM inputs: camera centres within a few metres at 300-1500 m depth
    assert np.median(errs) < 5.0


def test_oracle_ransac_epnp5_finds_the_inliers():
    pr = synth.pnp_problem(400, 0.4, seed=12)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 1000, 0x5EED, sampler="opencv",
                       minimal="epnp5")
    assert ref["best"] >= 0
    truth = pr["inlier"]
    assert (ref["mask"] & truth).sum() >= 0.95 * truth.sum()
    # RANSACUpdateNumIters with model_points 5 bounds the run
    w = ref["n_inliers"] / 400
    assert ref["iters"] <= max(rsac.update_num_iters(0.99, 1 - w, 5, 1000), ref["best"] + 1)


# --------------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("n,outl,seed,H", [(300, 0.3, 31, 1024), (2000, 0.5, 32, 1024), (300, 0.4, 33, 6000),
                                           (400, 0.5, 34, 2048), (400, 0.5, 34, 2049)])
def test_gpu_epnp5_hypotheses_bit_exact(n, outl, seed, H):
    """Every hypothesis (Philox 5-subsets, then explicit MWC 5-subsets): status, count, model
    (k_cvepnp5_a / _svd / _c against the oracle's orc_cv_epnp).  Rounds of H <= 2048 run one-wave
    blocks, larger ones 4-wave blocks: both launch shapes and the boundary between them."""
    pr = synth.pnp_problem(n, outl, seed=seed)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    st, cn, md = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, H, 30.0, seed=77,
                                 minimal="epnp5")
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 77, H, models=True, minimal="epnp5")
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cn, oc)
    ok = st > 0
    assert ok.sum() > 0.9 * H
    assert _bits_equal(md[ok, :12], om[ok, :12])
    subs, sst = _mwc5(n, H)
    st, cn, md = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, H, 30.0, subsets=subs,
                                 minimal="epnp5")
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 0, H, subsets=subs, sub_status=sst, models=True,
                                   minimal="epnp5")
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cn, oc)
    ok = st > 0
    assert _bits_equal(md[ok, :12], om[ok, :12])


@pytest.mark.gpu
@pytest.mark.parametrize("H", [500, 4096])
def test_gpu_epnp5_degenerate_samples_bit_exact(H):
    """Half the points on the plane z = 700 m: a sample of five of them leaves M^T M with exact
    zero rows, so cvSVD's JacobiSVD fills those directions from RNG(0x12345678)
    (k_cvepnp5_svd's in-memory branch, cvq_fill_rows; the oracle counts the fills): status, count
    and model of every hypothesis against the oracle, both launch shapes."""
    pr = synth.pnp_problem(300, 0.3, seed=5)
    P3 = pr["points3d"].copy()
    P3[::2, 2] = 700.0
    soa, cam = O.soa_pnp(P3, pr["points2d"]), O.cam_from_K(pr["K"])
    subs, sst = _mwc5(300, H)
    f0 = O.lib().orc_cvq_fill_events(12)
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 0, H, subsets=subs, sub_status=sst, models=True,
                                   minimal="epnp5", rvec=True)
    assert O.lib().orc_cvq_fill_events(12) > f0
    st, cn, md = rsac.hypotheses("pnp", P3, pr["points2d"], pr["K"], 0, H, 30.0, subsets=subs, minimal="epnp5",
                                 rvec=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cn, oc)
    ok = st > 0
    assert _bits_equal(md[ok, :12], om[ok, :12])


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["opencv", "philox"])
@pytest.mark.parametrize("n,outl,seed", [(600, 0.4, 41), (3000, 0.6, 42)])
def test_gpu_epnp5_ransac_matches_oracle(sampler, n, outl, seed):
    """The adaptive loop with model_points 5: winner, count, iterations, mask and pose."""
    pr = synth.pnp_problem(n, outl, seed=seed)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 2000, 0x5EED, sampler=sampler,
                       minimal="epnp5")
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, sampler=sampler,
                                    refine=False, minimal="epnp5", return_info=True)
    assert info.best_hyp == ref["best"] and info.n_inliers == ref["n_inliers"]
    assert info.iters == ref["iters"]
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


@pytest.mark.gpu
def test_gpu_epnp5_batched_matches_per_problem_oracle():
    probs = [synth.pnp_problem(nn, 0.4, seed=150 + i) for i, nn in enumerate([80, 1500, 700])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 1500, 30.0, sampler="opencv", refine=False,
                                  minimal="epnp5")
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 1500, 0x5EED, sampler="opencv",
                           minimal="epnp5")
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["opencv", "philox"])
def test_gpu_epnp5_batched_long_rounds(sampler):
    """A batch whose later rounds exceed 2048 hypotheses in all (confidence 1: every round runs to
    the budget; 3 problems x 1024 in round 3), so the long-round launch shape (a grid row per
    problem) runs beside the short one: every problem against the oracle's own loop."""
    probs = [synth.pnp_problem(nn, 0.5, seed=170 + i) for i, nn in enumerate([300, 900, 2000])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 2000, 30.0, confidence=1.0, sampler=sampler,
                                  refine=False, minimal="epnp5")
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 1.0, 2000, 0x5EED, sampler=sampler,
                           minimal="epnp5")
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


@pytest.mark.gpu
def test_gpu_cv2_default_flags_use_epnp5():
    """cv2compat.solvePnPRansac(flags=SOLVEPNP_ITERATIVE): MWC 5-point samples, EPnP kernel, the
    RANSAC-phase inliers of the oracle's run, LM from the winner on them."""
    from rsac import cv2compat as rcv
    pr = synth.pnp_problem(1200, 0.5, seed=51)
    ok, rvec, tvec, inl = rcv.solvePnPRansac(pr["points3d"], pr["points2d"], pr["K"], np.zeros((4, 1)),
                                             iterationsCount=1500, reprojectionError=30.0)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 1500, 0x5EED, sampler="opencv",
                       minimal="epnp5")
    assert ok
    np.testing.assert_array_equal(inl.ravel(), np.flatnonzero(ref["mask"]))
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    Rl, tl, _ = O.pnp_refine(soa, ref["mask"].astype(np.uint8), cam, ref["R"].reshape(9), ref["t"])
    assert _bits_equal(tvec.ravel(), tl)
    assert _bits_equal(rcv.Rodrigues(rvec)[0], rsac.rodrigues(rsac.rodrigues(Rl)))
    # 4 points (4 inliers): OpenCV switches to P3P (model_points 4), which needs all 4 to agree
    i4 = np.flatnonzero(pr["inlier"])[:4]
    ok4, _, _, inl4 = rcv.solvePnPRansac(pr["points3d"][i4], pr["points2d"][i4], pr["K"], None,
                                         iterationsCount=50, reprojectionError=30.0)
    assert ok4 and len(inl4) == 4


