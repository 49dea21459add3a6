"""OpenCV's operation sequence for the reference's PnP minimal solver (CPU tests).

Every reference PnP call (main_v1.py:497-502, testpro-K.py:72-75, testpro.py:536-541,
test_pro.py:515-520) runs cv2.solvePnPRansac with the default flags: 5-point subsets, each solved
by solvePnP(SOLVEPNP_EPNP), the model kept as (rvec, tvec).  The oracle restates that sequence
from the OpenCV 4.x sources (oracle/cv_epnp.c; [OpenCV 4.x, unvendored]: solvepnp.cpp,
undistort.dispatch.cpp, epnp.cpp, lapack.cpp, calibration.cpp) and the library runs the same
steps (rsac_cvepnp.h).  OpenCV is not installed here, so against OpenCV itself the bits are
"parity unpinned"; profiles/r06/epnp_variants.md measures why the sequence matters: on the
reference's own 12 points the RANSAC decision of most intrinsics depends on the last bits of the
minimal solver.
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

import pyoracle as O
import rsac
from rsac import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def test_hypot_is_libm_hypot():
    """JacobiSVDImpl_'s rotation calls hypot(p, beta); both sides restate glibc 2.35's hypot
    (e_hypot.c, Borges' non-FMA kernel).  This host's libm gives the same bits on every pair whose
    operands are >= 2^-509 (JacobiSVD's rotations stay far above; below, glibc's tiny-operand path
    differs from the restatement in ~1e-5 of random pairs), across 120 binades."""
    libm = C.CDLL("libm.so.6")
    libm.hypot.argtypes = [C.c_double, C.c_double]
    libm.hypot.restype = C.c_double
    rng = np.random.default_rng(0)
    xs = rng.standard_normal((100_000, 2)) * np.exp(rng.uniform(-40, 40, (100_000, 2)))
    xs[::5, 1] = xs[::5, 0] * (1 + rng.uniform(-1e-3, 1e-3, 20_000))  # nearly equal operands
    L = O.lib()
    bad = sum(L.cvq_hypot(a, b) != libm.hypot(a, b) for a, b in xs)
    assert bad == 0
    assert L.cvq_hypot(3.0, 4.0) == 5.0 and L.cvq_hypot(0.0, -2.5) == 2.5
    assert math.isinf(L.cvq_hypot(float("inf"), float("nan")))


def test_jacobi_svd_decomposes_and_sorts():
    """cvq_jacobi_svd (lapack.cpp JacobiSVDImpl_): At (n x m) -> normalised rows U^T, W descending,
    Vt with A = U diag(W) Vt."""
    rng = np.random.default_rng(1)
    for m, n in ((6, 4), (6, 3), (6, 5), (12, 12), (3, 3)):
        A = rng.standard_normal((m, n))
        At = np.ascontiguousarray(A.T).copy()
        W = np.zeros(n)
        Vt = np.zeros((n, n))
        O.lib().cvq_jacobi_svd(At.reshape(-1), m, W, Vt.ctypes.data, n, m, n, n)
        assert np.all(np.diff(W) <= 0)
        np.testing.assert_allclose(At.T @ np.diag(W) @ Vt, A, atol=1e-12)
        np.testing.assert_allclose(At @ At.T, np.eye(n), atol=1e-12)


def test_solve_and_invert_match_numpy():
    rng = np.random.default_rng(2)
    for k in (3, 4, 5):
        A = rng.standard_normal((6, k))
        b = rng.standard_normal(6)
        x = np.zeros(k)
        O.lib().cvq_solve6(np.ascontiguousarray(A).reshape(-1), k, b, x)
        np.testing.assert_allclose(x, np.linalg.lstsq(A, b, rcond=None)[0], rtol=1e-10, atol=1e-12)
    S = rng.standard_normal((3, 3))
    X = np.zeros(9)
    O.lib().cvq_invert3(np.ascontiguousarray(S).reshape(-1), X)
    np.testing.assert_allclose(X.reshape(3, 3), np.linalg.inv(S), rtol=1e-10, atol=1e-12)


def test_cv_epnp_recovers_clean_poses():
    pr = synth.pnp_problem(200, 0.0, seed=11, noise_px=0.0)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    C0 = -pr["R"].T @ pr["t"]
    subs, _ = O.mwc_subsets(200, 40, s=5)
    errs = []
    for idx in subs:
        R, t = O.pnp_minimal_epnp5(soa, cam, idx)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-9) and np.linalg.det(R) > 0
        errs.append(np.linalg.norm(-R.T @ t - C0))
    assert np.median(errs) < 2.0  # f32-rounded UTM inputs (0.25 m ulp), 300-1500 m depth


def test_host_twin_equals_oracle_on_degenerate_samples():
    """Planar and collinear samples drive JacobiSVD into its zero-singular-value branch (the
    RNG(0x12345678) fill); the host twin (the kernels' source) keeps the oracle's bits there too."""
    K = synth.main_v1_K()
    base = np.array([739000.0, 2888500.0, 700.0])
    cases = [
        np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0], [2, 1, 0]], float),      # planar
        np.array([[0, 0, 0], [1, 1, 1], [2, 2, 2], [3, 3, 3], [4, 4, 4]], float),      # collinear
        np.array([[0, 0, 0], [0, 0, 0], [5, 1, 2], [1, 7, 3], [2, 2, 9]], float),      # duplicate point
    ]
    px = np.array([[100, 200], [300, 210], [120, 400], [310, 420], [500, 430]], float)
    f0 = [O.lib().orc_cvq_fill_events(n) for n in (3, 12)]
    for P in cases:
        P3 = P * 30.0 + base
        R, t = rsac.epnp_minimal(px, P3, K)
        Ro, to = O.pnp_minimal_epnp5(O.soa_pnp(P3, px), O.cam_from_K(K), [0, 1, 2, 3, 4])
        assert _bits_equal(R, Ro) and _bits_equal(t, to)
    # the planar and collinear samples reach the fill branch of the 3 x 3 and of the 12 x 12 SVD
    assert O.lib().orc_cvq_fill_events(3) > f0[0] and O.lib().orc_cvq_fill_events(12) > f0[1]


def test_rodrigues_is_cvrodrigues2():
    """cvRodrigues2 both ways (JacobiSVD orthogonalisation, c I + c1 r r^T + s [r]x): the library and
    the oracle give the same bits, and the values are Rodrigues' formula to ~1e-15."""
    rng = np.random.default_rng(4)
    for _ in range(300):
        r = rng.standard_normal(3)
        r *= rng.uniform(1e-3, 3.1) / np.linalg.norm(r)
        R = rsac.rodrigues(r)
        Ro = O.rodrigues_v2m(r)
        assert _bits_equal(R, Ro)
        th = np.linalg.norm(r)
        k = r / th
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        np.testing.assert_allclose(R, np.eye(3) + math.sin(th) * Kx + (1 - math.cos(th)) * Kx @ Kx, atol=2e-15)
        back = rsac.rodrigues(R).ravel()
        assert _bits_equal(back, O.rodrigues_m2v(R))
        np.testing.assert_allclose(back, r, atol=1e-13)
    # the model computeError scores: Rodrigues(Rodrigues(R)), host == oracle
    R = rsac.rodrigues(rng.standard_normal(3))
    assert _bits_equal(rsac.rodrigues(rsac.rodrigues(R)), O.rvec_roundtrip(R))


def test_decision_study_table_is_current():
    """profiles/r06/epnp_variants.json (scripts/epnp_variants.py) was produced by this oracle: the
    per-K RANSAC decisions it records for main_v1's K and for testpro-K's f = 150 mm 127 x 178 mm
    recompute identically under all three restatements."""
    with open(os.path.join(ROOT, "profiles", "r06", "epnp_variants.json")) as f:
        study = json.load(f)
    cases = {c["K"]: c for c in study["c1"]["cases"]}
    Ks = list(synth.testpro_k_candidates())
    for name, K in (("main_v1", synth.main_v1_K()), ("f150 127x178", Ks[10])):
        for seq in ("cv", "rr", "rr_unfused"):
            with O.sequence(seq):
                r = O.pnp_ransac(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, K, 30.0, 0.99, 5000, 0x5EED,
                                 sampler="opencv", minimal="epnp5")
            rec = cases[name][seq]
            assert (r["best"], r["iters"], np.flatnonzero(r["mask"]).tolist()) == (rec["best"], rec["iters"],
                                                                                  rec["inliers"])


@pytest.mark.parametrize("seq", ["rr", "rr_unfused"])
def test_other_restatements_still_solve(seq):
    """The round-4/5 restatement (kept for the study) still recovers clean poses in both builds."""
    pr = synth.pnp_problem(200, 0.0, seed=12, noise_px=0.0)
    soa, cam = O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])
    C0 = -pr["R"].T @ pr["t"]
    subs, _ = O.mwc_subsets(200, 16, s=5)
    with O.sequence(seq):
        errs = [np.linalg.norm(-R.T @ t - C0) for R, t in (O.pnp_minimal_epnp5(soa, cam, idx) for idx in subs)]
    assert np.median(errs) < 2.0
