"""The C ABI (include/rsac.h) without a GPU: the library loads, exports every
declared entry point, and fails cleanly (no crash, no CPU fallback) when no
HIP device is visible."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from rsac import _lib as L

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "rsac.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"RSAC_EXPORT[^;(]*?\b(rsac_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ["rsac_create", "rsac_destroy", "rsac_pnp_ransac", "rsac_pnp_ransac_batched", "rsac_homography_ransac",
              "rsac_homography_ransac_batched", "rsac_score_poses", "rsac_pnp_evaluate_range", "rsac_pnp_mask",
              "rsac_pnp_hypotheses", "rsac_homography_hypotheses", "rsac_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_ctypes_table_matches_header():
    assert sorted(n for n, _, _ in L.SIGNATURES) == declared_symbols()


def test_abi_version():
    assert L.lib().rsac_abi_version() == L.ABI_VERSION


def test_host_only_helpers():
    import rsac
    R = rsac.rodrigues([0.0, 0.0, np.pi / 2])
    np.testing.assert_allclose(R, [[0, -1, 0], [1, 0, 0], [0, 0, 1]], atol=1e-12)
    assert rsac.update_num_iters(0.99, 0.5, 4, 5000) == 71


# 9000 / 70000 / 300000: 9 / 64 / 64 ranges of the block-compacted order (the last one's ranges
# exceed one LDS tile on the GPU); masked: every third point dropped, so ranges compact unevenly
@pytest.mark.parametrize("n,masked", [(500, False), (4097, True), (9000, False), (9000, True), (70000, True),
                                      (300000, True)])
def test_host_refine_matches_oracle(n, masked):
    import pyoracle as O
    import rsac
    from rsac import synth
    pr = synth.pnp_problem(n, 0.0, seed=5, noise_px=0.5)
    R0 = synth.random_rotation(np.random.default_rng(9)) * 0 + pr["R"]
    t0 = pr["t"] + np.array([0.5, -0.3, 0.2])
    mask = np.ones(n, np.uint8)
    if masked:
        mask[np.random.default_rng(n).random(n) < 0.33] = 0
    R, t = rsac.refine_pose(pr["points2d"], pr["points3d"], pr["K"], R0, t0, mask=mask if masked else None)
    soa = O.soa_pnp(pr["points3d"], pr["points2d"])
    Ro, to, _ = O.pnp_refine(soa, mask, O.cam_from_K(pr["K"]), R0, t0)
    # same arithmetic and summation order (the GPU kernel's) on both sides: bit-identical
    np.testing.assert_array_equal(R, Ro)
    np.testing.assert_array_equal(t, to)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)


def test_create_without_device_fails_cleanly():
    if L.lib().rsac_device_count() > 0:
        pytest.skip("a HIP device is visible")
    h = C.c_void_p()
    code = L.lib().rsac_create(0, C.byref(h))
    assert code == L.ENODEV
    assert b"device" in L.lib().rsac_last_error()
    import rsac
    with pytest.raises(rsac.RsacError):
        rsac.pnp_ransac(np.zeros((10, 2)), np.zeros((10, 3)), np.eye(3))


def test_host_homography_refit_matches_oracle_bitwise():
    """findHomography's refit (runKernel DLT on the inliers + OpenCV's LMSolver, 10 iterations) is
    host C++ in librsac; it must equal the restatement bit for bit (same IEEE operation order)."""
    import json
    import os

    import pyoracle as O
    import rsac
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "debuglog_homography.json")))
    for b in [b for b in d["blocks"] if b["complete"]]:
        M = np.array(b["M"])
        pp2 = np.array(b["pp2"])
        hs = np.c_[pp2, np.ones(len(pp2))] @ M.T
        src, dst = hs[:, :2] / hs[:, 2:3], np.array(b["p1"], np.float64)
        mask = np.array(b["mask"], np.uint8)
        H = rsac.homography_fit(src, dst, mask)
        Ho = O.hom_refine(O.soa_hom(src, dst), mask, np.eye(3))
        np.testing.assert_array_equal(H, Ho)


def _lm_blocks(n):  # rsac_math.h lm_blocks (= oracle/rsac_oracle.c lm_blocks)
    return 1 if n <= 4096 else min(64, -(-n // 1024))


def _lm_chunk(n):  # rsac_math.h lm_chunk
    nb = _lm_blocks(n)
    return -(-n // nb)


def test_refit_ranges_fit_one_tile_up_to_262144_points():
    # k_pnp_refine stages a range's masked points once per refit when the range has at most
    # kLmStage = 4096 indices: that holds for every n <= kLmMaxBlocks * kLmStage = 262144, and
    # the tile-by-tile path is taken only above it.  Every range is non-empty.
    for n in list(range(1, 70000, 7)) + list(range(262000, 262145)):
        nb, c = _lm_blocks(n), _lm_chunk(n)
        assert c <= 4096, n
        assert (nb - 1) * c < n <= nb * c, n
    assert _lm_chunk(262145) == 4097
    assert (_lm_blocks(4097), _lm_chunk(4097)) == (5, 820)
    assert (_lm_blocks(65536), _lm_chunk(65536)) == (64, 1024)
    assert (_lm_blocks(65537), _lm_chunk(65537)) == (64, 1025)
