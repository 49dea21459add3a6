"""GPU parity: librsac.so (HIP, gfx950) against the CPU restatement (oracle/).

Bar (DESIGN.md "Parity"): per-hypothesis status and inlier counts, the models
themselves (bitwise, float64) and the RANSAC-phase masks are identical to the
oracle for the same seed; refined R, t agree within 1e-4.  Every case is checked
exhaustively against the oracle, including the BASELINE.json sizes: C2 (10k points,
all 100k hypotheses, and the bench step's own key / model / mask) and C3 (1024
problems x 2000 points x 1024 hypotheses, every problem).
"""
import json
import os

import numpy as np
import pytest

import pyoracle as O
import rsac
from rsac import _lib as L
from rsac import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "debuglog_homography.json")


def _bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def _pnp_case(n, outl, seed):
    pr = synth.pnp_problem(n, outl, seed=seed)
    return pr, O.soa_pnp(pr["points3d"], pr["points2d"]), O.cam_from_K(pr["K"])


@pytest.mark.parametrize("n,outl,seed,H", [(4, 0.0, 1, 256), (5, 0.2, 2, 256), (12, 0.3, 3, 512),
                                           (100, 0.5, 4, 1000), (256, 0.5, 8, 300), (257, 0.5, 8, 300),
                                           (1000, 0.5, 5, 700), (2999, 0.6, 6, 333)])
def test_pnp_hypotheses_bit_exact_philox(n, outl, seed, H):
    pr, soa, cam = _pnp_case(n, outl, seed)
    st, cnt, mdl = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 17, H, 30.0, seed=seed)
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, seed, H, hyp0=17, models=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cnt, oc)
    assert _bits_equal(mdl[:, :12], om[:, :12])
    # the solves leave the validity slot to the status byte; the host probe output fills it in
    np.testing.assert_array_equal(mdl[:, 12], (st > 0).astype(np.float64))


def test_pnp_hypotheses_bit_exact_opencv_subsets():
    pr, soa, cam = _pnp_case(500, 0.5, 7)
    subs, sst = O.mwc_subsets(500, 800)
    st, cnt, mdl = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, 800, 30.0, subsets=subs)
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 0, 800, subsets=subs, sub_status=sst, models=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cnt, oc)
    assert _bits_equal(mdl[:, :12], om[:, :12])


@pytest.mark.parametrize("ki", [0, 7, 13, 16, 19, 26])
def test_testpro_k_points_bit_exact(ki):
    K = synth.testpro_k_candidates()[ki]
    soa = O.soa_pnp(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS)
    cam = O.cam_from_K(K)
    st, cnt, mdl = rsac.hypotheses("pnp", synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, K, 0, 2048, 30.0)
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 0x5EED, 2048, models=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cnt, oc)
    assert _bits_equal(mdl[:, :12], om[:, :12])


def _debuglog():
    d = json.load(open(GOLD))
    out = []
    for b in d["blocks"]:
        if not b["complete"]:
            continue
        M = np.array(b["M"])
        pp2 = np.array(b["pp2"])
        hs = np.c_[pp2, np.ones(len(pp2))] @ M.T
        out.append((hs[:, :2] / hs[:, 2:3], np.array(b["p1"], np.float64), np.array(b["mask"], bool)))
    return out, d["threshold"]


def test_homography_hypotheses_bit_exact_debuglog():
    blocks, thr = _debuglog()
    for src, dst, _ in blocks:
        soa = O.soa_hom(src, dst)
        subs, sst = O.mwc_subsets(12, 300, hom=soa)
        st, cnt, mdl = rsac.hypotheses("homography", src, dst, None, 0, 300, thr, subsets=subs)
        oc, os_, om = O.hom_hypotheses(soa, thr, 0, 300, subsets=subs, sub_status=sst, models=True)
        np.testing.assert_array_equal(st, os_)
        np.testing.assert_array_equal(cnt, oc)
        assert _bits_equal(mdl[:, :9], om[:, :9])


def test_homography_ransac_reproduces_reference_masks():
    """The GPU path reproduces the masks OpenCV recorded in the reference's debug.log."""
    blocks, thr = _debuglog()
    for src, dst, mref in blocks:
        H, m = rsac.homography_ransac(src, dst, thr, max_iters=2000, confidence=0.995, sampler="opencv")
        assert H is not None
        np.testing.assert_array_equal(m, mref)


def test_homography_batched_location_search_equals_singles():
    blocks, thr = _debuglog()
    srcs = [b[0] for b in blocks]
    dsts = [b[1] for b in blocks]
    batched = rsac.homography_ransac_batched(srcs, dsts, thr)
    for (src, dst, mref), (Hb, mb, nb) in zip(blocks, batched):
        np.testing.assert_array_equal(mb, mref)
        Hs, ms = rsac.homography_ransac(src, dst, thr)
        np.testing.assert_allclose(Hb, Hs, rtol=0, atol=0)


@pytest.mark.parametrize("seed", [11, 12])
def test_homography_philox_bit_exact(seed):
    pr = synth.homography_problem(3000, 0.4, seed=seed)
    soa = O.soa_hom(pr["src"], pr["dst"])
    st, cnt, mdl = rsac.hypotheses("homography", pr["src"], pr["dst"], None, 5, 900, 4.0, seed=seed)
    oc, os_, om = O.hom_hypotheses(soa, 4.0, seed, 900, hyp0=5, models=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cnt, oc)
    assert _bits_equal(mdl[:, :9], om[:, :9])


@pytest.mark.parametrize("sampler", ["philox", "opencv"])
def test_pnp_ransac_end_to_end_vs_oracle(sampler):
    pr, soa, cam = _pnp_case(4000, 0.5, 21)
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, sampler=sampler,
                                    refine=False, return_info=True)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000, 0x5EED, sampler=sampler)
    assert info.best_hyp == ref["best"]
    assert info.n_inliers == ref["n_inliers"]
    assert info.iters == ref["iters"]
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    # refined pose: LM on the same inliers from the same start
    R2, t2, m2 = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, sampler=sampler, refine=True)
    Ro, to, _ = O.pnp_refine(soa, ref["mask"].astype(np.uint8), cam, ref["R"], ref["t"])
    np.testing.assert_array_equal(m2, ref["mask"])
    # the GPU refit (k_pnp_refine) uses the restatement's arithmetic and summation order
    assert _bits_equal(R2, Ro) and _bits_equal(t2, to)
    assert np.abs(R2 - pr["R"]).max() < 5e-3  # ground truth, through f32-rounded UTM inputs


def test_pnp_ransac_non_adaptive_equals_adaptive_prefix():
    pr, soa, cam = _pnp_case(3000, 0.5, 22)
    _, _, m1, i1 = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 3000, 30.0, adaptive=True,
                                   refine=False, return_info=True)
    _, _, m2, i2 = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 3000, 30.0, adaptive=False,
                                   refine=False, return_info=True)
    assert i1.best_hyp == i2.best_hyp and i1.iters == i2.iters
    assert i2.hyps_scored == 3000
    np.testing.assert_array_equal(m1, m2)


def test_pnp_batched_ragged_equals_singles():
    probs = [synth.pnp_problem(n, 0.4, seed=30 + i) for i, n in enumerate([4, 9, 64, 65, 700, 2049])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 2000, 30.0, refine=False)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 2000, 0x5EED)
        if ref["best"] < 0:
            assert R is None
            continue
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


@pytest.mark.parametrize("adaptive", [True, False])
def test_pnp_batched_mixed_scales_equals_oracle(adaptive):
    # one batch, problems inside and outside the MFMA scorer's f16 operand range (centred
    # coordinates above 2^15 or below 1/64 run the form-1 path of k_pnp_score_mf); non-adaptive:
    # one 1500-hypothesis round (the MFMA kernel, not the small-round instance)
    base = [synth.pnp_problem(n, 0.4, seed=70 + i) for i, n in enumerate([3000, 1500, 2500, 800])]
    scales = [1.0, 1e3, 1e-5, 1.0]
    probs = []
    for p, sc in zip(base, scales):
        q = dict(p)
        q["points3d"] = p["points3d"] * sc
        probs.append(q)
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 1500, 30.0, refine=False, adaptive=adaptive)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 1500, 0x5EED)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


def test_pnp_batched_long_problem_cells_equals_oracle():
    # a batch with a problem longer than one inline-recount unit (16 384 points): every tile of
    # the batch then runs by cells, and the short problem's cells past its end are skipped.  90 %
    # outliers keep the adaptive bound above the budget, so the rounds grow past the small-round
    # instance (16 tiles) into the MFMA scorer
    base = [synth.pnp_problem(n, 0.9, seed=90 + i) for i, n in enumerate([20000, 3000])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in base], [p["points3d"] for p in base],
                                  [p["K"] for p in base], 2048, 30.0, refine=False)
    for p, (R, t, m, ni) in zip(base, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 2048, 0x5EED)
        assert ref["iters"] == 2048
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


def test_pnp_batched_many_long_problems_by_cells():
    # a large batch of problems longer than one inline-recount unit (16 384 points):
    # 48 x 20 000 points, so every tile runs by cells on the 4-wave scorer; no segment bound, no
    # launch split, every problem's winner equals a one-problem call's, a few the oracle's
    probs = [synth.pnp_problem(20000, 0.6, seed=700 + i) for i in range(48)]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 512, 30.0, refine=False, adaptive=False)
    for i in (0, 23, 47):
        p = probs[i]
        R, t, m, ni = out[i]
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 512, 0x5EED)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    for i in range(0, 48, 6):
        R1, t1, m1 = rsac.pnp_ransac(probs[i]["points2d"], probs[i]["points3d"], probs[i]["K"], 512, 30.0,
                                     refine=False, adaptive=False)
        np.testing.assert_array_equal(m1, out[i][2])
        assert _bits_equal(R1, out[i][0]) and _bits_equal(t1, out[i][1])


def test_k_sweep_batched():
    """testpro-K.py:58-75 as one batched call over the 27 intrinsics."""
    Ks = synth.testpro_k_candidates()
    out = rsac.pnp_ransac_batched([synth.TESTPRO_K_PIXELS] * 27, [synth.TESTPRO_K_POS3D] * 27, Ks, 5000, 30.0,
                                  refine=False)
    for K, (R, t, m, ni) in zip(Ks, out):
        ref = O.pnp_ransac(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, K, 30.0, 0.99, 5000, 0x5EED)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])


@pytest.mark.parametrize("refine", [False, True])
def test_device_inputs_match_host_inputs(refine):
    # device f64 inputs of one P3P problem take the set-up into the first solve launch
    # (k_pnp_setup_solve4, the round's records built by the scorer, r06); host inputs do not
    import torch
    pr, soa, cam = _pnp_case(5000, 0.5, 40)
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, refine=refine,
                                    return_info=True)
    p2 = torch.from_numpy(pr["points2d"]).cuda()
    p3 = torch.from_numpy(pr["points3d"]).cuda()
    Rd, td, md, infod = rsac.pnp_ransac(p2, p3, pr["K"], 2000, 30.0, refine=refine, return_info=True)
    assert md.is_cuda
    np.testing.assert_array_equal(md.cpu().numpy(), m)
    assert _bits_equal(Rd, R) and _bits_equal(td, t)
    assert (infod.best_hyp, infod.iters, infod.n_inliers) == (info.best_hyp, info.iters, info.n_inliers)


def test_batched_large_host_inputs_match_device_inputs():
    # a host f64 batch of 320 000 points (converted on the host pool in chunks, one copy,
    # rsac_api.hip stage_points): the same winners, counts and masks as the same batch handed
    # over as device tensors (converted on the device by k_pnp_setup_b)
    import torch
    probs = [synth.pnp_problem(2000, 0.5, seed=500 + s) for s in range(160)]
    off = np.zeros(161, np.int64)
    off[1:] = np.cumsum([len(p["points3d"]) for p in probs])
    h2 = np.concatenate([p["points2d"] for p in probs])
    h3 = np.concatenate([p["points3d"] for p in probs])
    Ks = np.stack([p["K"] for p in probs])
    Rh, th, okh, nh, mh = rsac.pnp_ransac_batched_flat(h2, h3, off, Ks, 256, 30.0, adaptive=False, refine=False)
    Rd, td, okd, nd, md = rsac.pnp_ransac_batched_flat(torch.from_numpy(h2).cuda(), torch.from_numpy(h3).cuda(),
                                                       off, Ks, 256, 30.0, adaptive=False, refine=False)
    np.testing.assert_array_equal(okh, okd)
    np.testing.assert_array_equal(nh, nd)
    np.testing.assert_array_equal(np.asarray(mh), md.cpu().numpy())
    assert _bits_equal(Rh, Rd) and _bits_equal(th, td)
    for i in (0, 79, 159):  # and the oracle on a few problems
        ref = O.pnp_ransac(probs[i]["points3d"], probs[i]["points2d"], probs[i]["K"], 30.0, 0.99, 256, 0x5EED)
        assert nh[i] == ref["n_inliers"]
        assert _bits_equal(Rh[i], ref["R"]) and _bits_equal(th[i], ref["t"])


def test_score_poses_vs_oracle_counts():
    pr, soa, cam = _pnp_case(7000, 0.5, 41)
    rng = np.random.default_rng(0)
    poses = []
    for k in range(40):
        R = pr["R"] if k % 2 == 0 else synth.random_rotation(rng)
        t = pr["t"] + rng.normal(size=3) * (0.0 if k == 0 else 0.5)
        poses.append(np.concatenate([R.reshape(9), t]))
    poses = np.array(poses)
    cnt = rsac.score_poses(pr["points2d"], pr["points3d"], pr["K"], poses, 30.0)
    ref = [O.pnp_count(p[:9].reshape(3, 3), p[9:], soa, cam, 30.0) for p in poses]
    np.testing.assert_array_equal(cnt, ref)


def test_baseline_c2_exhaustive_and_bench_step():
    """BASELINE.json configs[1] exactly as bench.py runs it: synth.pnp_problem(10000, 0.5, seed=0),
    Philox seed 0x5EED, hypotheses [0, 100 000).  Every hypothesis' status and count equals the
    oracle's, and the bench step itself (evaluate_range on device tensors, device_result=True)
    returns the oracle's best key, model and RANSAC-phase mask."""
    import torch
    from rsac import parallel as par
    pr, soa, cam = _pnp_case(10000, 0.5, 0)
    H = 100_000
    st, cnt, mdl = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, H, 30.0)
    oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 0x5EED, H, models=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cnt, oc)
    assert _bits_equal(mdl[:, :12], om[:, :12])
    okey = par.best_key_of(oc, os_, 0)
    ocnt, obest = par.unpack_key(okey)
    oc_best, omask = O.pnp_count(om[obest, :9].reshape(3, 3), om[obest, 9:12], soa, cam, 30.0, mask=True)
    assert oc_best == ocnt == int(omask.sum())
    # the bench step (bench.py step(): device tensors in, nothing waits for the host)
    ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
    key_t, model_t, mask_t = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True,
                                                 device_result=True)
    torch.cuda.synchronize()
    assert int(key_t.item()) == okey
    assert _bits_equal(model_t.cpu().numpy(), om[obest, :12])
    np.testing.assert_array_equal(mask_t.cpu().numpy(), omask)
    assert (omask == pr["inlier"]).mean() > 0.99
    # the same step as two shards (ranks 0 and 1 of a world of 2): the all-reduced key is the
    # oracle's, and the winner re-derived from it on the losing shard is the oracle's model
    k0, _ = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H // 2, 30.0, device_result=True)
    k1, _ = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], H // 2, H // 2, 30.0, device_result=True)
    kmax = torch.maximum(k0, k1)
    assert int(kmax.item()) == okey
    wm, wmask = rsac.winner(ev.p2, ev.p3, pr["K"], kmax, 30.0)
    assert _bits_equal(wm.cpu().numpy(), om[obest, :12])
    np.testing.assert_array_equal(wmask.cpu().numpy(), omask)


def test_baseline_c3_batched_every_problem():
    """BASELINE.json configs[2] on one GPU, as bench.py's c3 line runs it: 1024 problems x 2000
    points (synth seeds 1..1024), 1024 hypotheses each, one pnp_ransac_batched_flat call with
    inputs in HBM, adaptive off, no refit.  Every problem's status, inlier count, R, t (bitwise)
    and RANSAC-phase mask equal the oracle's sequential loop."""
    import torch
    probs = [synth.pnp_problem(2000, 0.5, seed=s) for s in range(1, 1025)]
    off = np.zeros(1025, np.int64)
    off[1:] = np.cumsum([len(p["points3d"]) for p in probs])
    p2 = torch.from_numpy(np.concatenate([p["points2d"] for p in probs])).cuda()
    p3 = torch.from_numpy(np.concatenate([p["points3d"] for p in probs])).cuda()
    Ks = np.stack([p["K"] for p in probs])
    R, t, ok, ninl, mask = rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 1024, 30.0, adaptive=False, refine=False)
    mask = mask.cpu().numpy()
    for i, p in enumerate(probs):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 1024, 0x5EED)
        assert ok[i] == (ref["best"] >= 0), i
        assert ninl[i] == ref["n_inliers"], i
        np.testing.assert_array_equal(mask[off[i]:off[i + 1]], ref["mask"], err_msg=str(i))
        assert _bits_equal(R[i], ref["R"]) and _bits_equal(t[i], ref["t"]), i


def test_degenerate_inputs():
    # all points identical -> every minimal solve fails -> no model, mask all False
    P3 = np.tile(np.array([[739000.0, 2888500.0, 700.0]]), (50, 1))
    P2 = np.tile(np.array([[100.0, 200.0]]), (50, 1))
    R, t, m = rsac.pnp_ransac(P2, P3, synth.main_v1_K(), 500, 30.0)
    assert R is None and not m.any()
    with pytest.raises(rsac.RsacError):
        rsac.pnp_ransac(P2[:3], P3[:3], synth.main_v1_K(), 500, 30.0)
    # collinear homography input: checkSubset rejects every subset
    s = np.c_[np.arange(20.0), 2 * np.arange(20.0)]
    H, m = rsac.homography_ransac(s, s * 3, 3.0)
    assert H is None and not m.any()


# ---------------------------------------------------------------------------------------------
# float32 pre-filter: must never change a decision (DESIGN.md "Scoring").  Both scoring forms are
# checked: the MFMA kernel (k_pnp_score_mf, rounds above 16 tiles of 32 hypotheses) and the
# scaled-form small-round instance (k_pnp_score_sc, rounds of at most 16 tiles).
# ---------------------------------------------------------------------------------------------
@pytest.fixture(params=["small_round", "mfma"])
def score_path(request):
    return request.param


def _pose_batch(poses, path):
    """The poses as scored: as given (16 or fewer: the small-round instance) or repeated to 1024
    poses (32 tiles: the MFMA kernel); returns (batch, index of each given pose's first copy)."""
    poses = np.asarray(poses, np.float64)
    if path == "small_round":
        assert len(poses) <= 16 * 32
        return poses, np.arange(len(poses))
    reps = -(-1024 // len(poses))
    return np.tile(poses, (reps, 1))[:1024], np.arange(len(poses))


# 40 000 hypotheses = 1250 tiles: more than one per resident block, so the launch has
# whole-problem units (counts stored) besides the cells of the queue's tail (counts added)
@pytest.mark.parametrize("n,seed,H", [(10000, 0, 40000), (4097, 3, 20000), (777, 9, 20000), (3000, 5, 500)])
def test_f32_prefilter_equals_exact_kernel(n, seed, H):
    pr, soa, cam = _pnp_case(n, 0.5, seed)
    st_f, c_f, _ = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, H, 30.0)
    st_e, c_e, _ = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, H, 30.0, exact_only=True)
    np.testing.assert_array_equal(st_f, st_e)
    np.testing.assert_array_equal(c_f, c_e)


def test_f32_prefilter_long_problem():
    # 100k points x 50k hypotheses: problems above 16 384 points run every tile by cells (a wave
    # lists at most 64 flagged iterations per unit); counts must still equal the exact kernel's
    pr = synth.pnp_problem(100_000, 0.5, seed=11)
    st_f, c_f, _ = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, 50_000, 30.0)
    st_e, c_e, _ = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, 50_000, 30.0, exact_only=True)
    np.testing.assert_array_equal(st_f, st_e)
    np.testing.assert_array_equal(c_f, c_e)


def test_short_problems_beside_a_long_one_equal_oracle():
    # a batch of many short problems next to one long one -- every tile runs by
    # cells, and most cells of the short problems' tiles lie past their ends and are skipped
    # without a unit barrier; the unit index slot must not be rewritten while another wave of
    # the block still reads it (double-buffered unit_s)
    probs = [synth.pnp_problem(300 + 7 * i, 0.5, seed=200 + i) for i in range(40)]
    probs.insert(17, synth.pnp_problem(20000, 0.5, seed=199))
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 1024, 30.0, adaptive=False, refine=False)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 1024, 0x5EED)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


def test_large_batch_of_long_problems_equals_oracle():
    # 64 problems of 17 000 points (each longer than one inline-recount unit,
    # so every tile runs by cells) in one non-adaptive launch of 512 hypotheses each; the round
    # used to be split by a record-list bound that the inline recount never needs
    probs = [synth.pnp_problem(17000, 0.5, seed=300 + i) for i in range(64)]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 512, 30.0, adaptive=False, refine=False)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 512, 0x5EED)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


def _boundary_case(seed, n=6000, thr=30.0):
    """Pixels placed at distance ~thr from the exact projection of the true pose, so that e ~ T to
    within float32 rounding: every pair lands in (or next to) the pre-filter's undecided band."""
    pr = synth.pnp_problem(n, 0.0, seed=seed, noise_px=0.0)
    soa = O.soa_pnp(pr["points3d"], pr["points2d"])
    cam = O.cam_from_K(pr["K"])
    R, t = pr["R"], pr["t"]
    X = np.stack(soa[:3], axis=1).astype(np.float64)
    pc = X @ R.T + t
    iz = 1.0 / pc[:, 2]
    pu = (pc[:, 0] * iz) * cam[0] + cam[2]
    pv = (pc[:, 1] * iz) * cam[1] + cam[3]
    rng = np.random.default_rng(seed)
    ang = rng.uniform(0, 2 * np.pi, n)
    rad = thr * (1.0 + rng.choice([-1, 1], n) * rng.choice([0.0, 1e-8, 3e-8, 1e-7, 1e-6, 1e-5, 1e-3], n))
    px = np.stack([pu + rad * np.cos(ang), pv + rad * np.sin(ang)], axis=1)
    return pr["points3d"], px, pr["K"], np.concatenate([R.reshape(9), t])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_f32_prefilter_threshold_boundary(seed, score_path):
    P3, P2, K, pose = _boundary_case(seed)
    soa = O.soa_pnp(P3, P2)
    cam = O.cam_from_K(K)
    rng = np.random.default_rng(seed)
    poses = [pose]
    for _ in range(15):  # small perturbations of the pose keep most pairs near the boundary
        p = pose.copy()
        p[9:] += rng.normal(size=3) * 1e-3
        poses.append(p)
    poses = np.array(poses)
    batch, first = _pose_batch(poses, score_path)
    fast = rsac.score_poses(P2, P3, K, batch, 30.0)
    exact = rsac.score_poses(P2, P3, K, batch, 30.0, exact_only=True)
    ref = [O.pnp_count(p[:9].reshape(3, 3), p[9:], soa, cam, 30.0) for p in poses]
    np.testing.assert_array_equal(exact, np.resize(ref, len(batch)))
    np.testing.assert_array_equal(fast, np.resize(ref, len(batch)))
    assert 0 < ref[0] < len(P3)  # the construction really straddles the threshold


def test_f32_prefilter_nonfinite_and_huge_coordinates(score_path):
    # NaN / inf coordinates (the exact test: an outlier) and a scene scaled by 1e15 (beyond the
    # range where the f32 evaluation is safe: every pair goes to the exact recount)
    pr = synth.pnp_problem(3000, 0.3, seed=45)
    P3, P2 = pr["points3d"].copy(), pr["points2d"].copy()
    rng = np.random.default_rng(3)
    bad = rng.choice(len(P3), 40, replace=False)
    P3[bad[:10], 0] = np.nan
    P3[bad[10:20], 2] = np.inf
    P2[bad[20:30], 0] = -np.inf
    P2[bad[30:], 1] = np.nan
    R, t = pr["R"], pr["t"]
    poses = np.array([np.concatenate([R.reshape(9), t])] +
                     [np.concatenate([R.reshape(9), t + rng.normal(size=3) * 0.05]) for _ in range(5)])
    cam = O.cam_from_K(pr["K"])
    batch, _ = _pose_batch(poses, score_path)
    fast = rsac.score_poses(P2, P3, pr["K"], batch, 30.0)
    ref = [O.pnp_count(p[:9].reshape(3, 3), p[9:], O.soa_pnp(P3, P2), cam, 30.0) for p in poses]
    np.testing.assert_array_equal(fast, np.resize(ref, len(batch)))
    assert ref[0] > 1000
    s = 1e15
    P3h = pr["points3d"] * s
    poses_h = poses.copy()
    poses_h[:, 9:] *= s
    batch, _ = _pose_batch(poses_h, score_path)
    fast = rsac.score_poses(pr["points2d"], P3h, pr["K"], batch, 30.0)
    ref = [O.pnp_count(p[:9].reshape(3, 3), p[9:], O.soa_pnp(P3h, pr["points2d"]), cam, 30.0) for p in poses_h]
    np.testing.assert_array_equal(fast, np.resize(ref, len(batch)))


def test_f32_prefilter_poses_past_the_f32_range(score_path):
    """Poses whose translation leaves the range the f32 / f16 record can hold (degenerate EPnP-5
    samples produce |t| ~ 1e37 .. 1e93, r06): the record falls back to "every pair undecided" with
    finite zero operands, so the fast count never reads a NaN (the pads of a 300-point problem once
    counted as inliers: 320 > n); counts equal the oracle's exact ones, for ragged problem sizes."""
    for n in (300, 2000):
        pr = synth.pnp_problem(n, 0.3, seed=46)
        R, t = pr["R"], pr["t"]
        rng = np.random.default_rng(4)
        poses = [np.concatenate([R.reshape(9), t])]
        for s in (1e20, 1e30, 1e36, 1e37, 3e38, 1e40, 1e93, 1e300):
            d = rng.normal(size=3)
            poses.append(np.concatenate([R.reshape(9), t + d / np.linalg.norm(d) * s]))
            poses.append(np.concatenate([R.reshape(9), -t * s / np.linalg.norm(t)]))
        poses = np.array(poses)
        cam = O.cam_from_K(pr["K"])
        batch, _ = _pose_batch(poses, score_path)
        fast = rsac.score_poses(pr["points2d"], pr["points3d"], pr["K"], batch, 30.0)
        ref = [O.pnp_count(p[:9].reshape(3, 3), p[9:], O.soa_pnp(pr["points3d"], pr["points2d"]), cam, 30.0)
               for p in poses]
        np.testing.assert_array_equal(fast, np.resize(ref, len(batch)))
        assert ref[0] > 0.6 * n and max(ref[1:]) <= n


def test_f32_prefilter_points_behind_and_on_camera_plane(score_path):
    pr = synth.pnp_problem(3000, 0.3, seed=44)
    R, t = pr["R"], pr["t"]
    C = -R.T @ t
    rng = np.random.default_rng(1)
    # points on the camera plane (z_cam = 0), behind the camera, and right at the centre
    extra_c = np.concatenate([np.c_[rng.normal(size=(200, 2)) * 50, np.zeros(200)],
                              np.c_[rng.normal(size=(200, 2)) * 50, -rng.uniform(1, 500, 200)],
                              np.zeros((3, 3))])
    extra_w = (extra_c - t) @ R
    P3 = np.concatenate([pr["points3d"], extra_w, C[None, :]])
    P2 = np.concatenate([pr["points2d"], rng.uniform(0, 2000, size=(len(extra_w) + 1, 2))])
    soa = O.soa_pnp(P3, P2)
    cam = O.cam_from_K(pr["K"])
    poses = np.array([np.concatenate([R.reshape(9), t])] +
                     [np.concatenate([synth.random_rotation(rng).reshape(9), t + rng.normal(size=3)]) for _ in range(7)])
    batch, _ = _pose_batch(poses, score_path)
    fast = rsac.score_poses(P2, P3, pr["K"], batch, 30.0)
    ref = [O.pnp_count(p[:9].reshape(3, 3), p[9:], soa, cam, 30.0) for p in poses]
    np.testing.assert_array_equal(fast, np.resize(ref, len(batch)))


# ---------------------------------------------------------------------------------------------
# multi-GPU driver on one rank (the gloo tests in test_parallel_gloo.py cover world_size 2)
# ---------------------------------------------------------------------------------------------
def test_parallel_driver_single_rank_equals_pnp_ransac():
    from rsac import parallel as par
    pr = synth.pnp_problem(3000, 0.6, seed=12)
    ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
    ada = par.sharded_ransac(ev, 5000, 0.99, round_size=512)
    R, t, mask, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=False,
                                       return_info=True)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000)
    assert (ada.best, ada.n_inliers, ada.iters) == (info.best_hyp, info.n_inliers, info.iters)
    assert (ada.best, ada.n_inliers, ada.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(ada.model[:9].reshape(3, 3), ref["R"])
    np.testing.assert_array_equal(ev.mask(ada.model), ref["mask"])
    fixed = par.sharded_best(ev, 20000)
    st, cn = ev.hypotheses(0, 20000)
    assert par.pack_key(fixed.n_inliers, fixed.best) == par.best_key_of(cn, st, 0)


# ---------------------------------------------------------------------------------------------
# camera-location search (main_v1.py:254-348, 419, 862-866)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed,thr", [(0, 75.0), (1, 120.0), (2, 75.0)])
def test_location_search_matches_restatement(seed, thr):
    pr = synth.location_problem(seed=seed)
    res = rsac.location_search(pr["pos3d"], pr["pixels"], pr["locations"], thr)
    assert res.n_good == int(np.count_nonzero(np.any(pr["pixels"] != 0, axis=1)))
    ref = [O.find_homography(pr["pixels"], pr["pos3d"], loc, thr) for loc in pr["locations"]]
    for l, r in enumerate(ref):
        assert res.ok[l] == (r["M"] is not None)
        np.testing.assert_array_equal(res.mask[l], r["mask"])
        if r["M"] is not None:
            np.testing.assert_array_equal(res.H[l], r["H"])  # RANSAC + host refit are bit-exact
    err = np.array([[r["err1"], r["err2"]] for r in ref])
    np.testing.assert_allclose(res.err, err, rtol=1e-9, atol=1e-9)
    assert res.best == O.best_location(err)


def test_location_search_reference_shaped_driver():
    from rsac.location import best_location, find_homographies
    pr = synth.location_problem(seed=3, n_locations=60)
    recs = [{"pixel": p, "pos3d": q, "symbol": str(i)} for i, (p, q) in enumerate(zip(pr["pixels"], pr["pos3d"]))]
    grid = np.arange(60) % 7 - 1  # grid_code -1 locations are skipped (main_v1.py:276-282)
    locs = [{"grid_code": g, "pos3d": q} for g, q in zip(grid, pr["locations"])]
    nm = find_homographies(recs, locs, 75.0)
    assert np.all(nm[grid < 0] == 0)
    for l in np.flatnonzero(grid >= 0)[:10]:
        r = O.find_homography(pr["pixels"], pr["pos3d"], pr["locations"][l], 75.0)
        np.testing.assert_allclose(nm[l], [r["err1"], r["err2"]], rtol=1e-9)
    assert best_location(nm) == O.best_location(nm)


def test_location_search_debuglog_masks():
    """Each debug.log findHomography call as a one-location search: pos3d = (1, sy, sx) makes pos2 =
    src exactly, so the search must reproduce the logged RANSAC masks (thr 120)."""
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "debuglog_homography.json")))
    for b in [b for b in d["blocks"] if b["complete"]]:
        M = np.array(b["M"])
        pp2 = np.array(b["pp2"])
        hs = np.c_[pp2, np.ones(len(pp2))] @ M.T
        src = hs[:, :2] / hs[:, 2:3]
        pos3d = np.c_[np.ones(len(src)), src[:, 1], src[:, 0]]
        res = rsac.location_search(pos3d, np.array(b["p1"]), np.zeros((1, 3)), d["threshold"])
        np.testing.assert_array_equal(res.mask[0], np.array(b["mask"], bool))


def test_location_search_too_few_noted_features():
    pr = synth.location_problem(seed=4)
    px = pr["pixels"].copy()
    px[3:] = 0
    with pytest.raises(rsac.RsacError):
        rsac.location_search(pr["pos3d"], px, pr["locations"][:5], 75.0)


@pytest.mark.parametrize("sampler", ["philox", "opencv"])
def test_many_rounds_equal_sequential_loop(sampler):
    """Adaptive runs over many rounds (first round 64, doubling) must give the sequential loop's
    best, count and iteration count: every round's scoring launch starts a fresh work queue and
    the OpenCV MWC state carries over between rounds."""
    from rsac import _lib as L
    pr = synth.pnp_problem(1500, 0.85, seed=77)
    ctx = L.context(0)
    L.check(L.lib().rsac_set_round_size(ctx.handle, 64))
    try:
        R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 3000, 30.0, sampler=sampler,
                                        refine=False, return_info=True)
    finally:
        L.check(L.lib().rsac_set_round_size(ctx.handle, 4096))
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 3000, 0x5EED, sampler=sampler)
    assert info.rounds > 3
    assert (info.best_hyp, info.n_inliers, info.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(m, ref["mask"])


def test_batched_flat_device_inputs_equal_lists():
    import torch
    probs = [synth.pnp_problem(n, 0.5, seed=90 + i) for i, n in enumerate([300, 2000, 40, 1200])]
    lists = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                    [p["K"] for p in probs], 600, 30.0, adaptive=False, refine=False)
    off = np.r_[0, np.cumsum([len(p["points3d"]) for p in probs])]
    p2 = torch.from_numpy(np.concatenate([p["points2d"] for p in probs])).cuda()
    p3 = torch.from_numpy(np.concatenate([p["points3d"] for p in probs])).cuda()
    R, t, ok, ninl, mask = rsac.pnp_ransac_batched_flat(p2, p3, off, np.stack([p["K"] for p in probs]), 600, 30.0,
                                                        adaptive=False, refine=False)
    assert mask.is_cuda
    mask = mask.cpu().numpy()
    for i, (Rl, tl, ml, nl) in enumerate(lists):
        assert ok[i] == (Rl is not None) and ninl[i] == nl
        np.testing.assert_array_equal(R[i], Rl)
        np.testing.assert_array_equal(t[i], tl)
        np.testing.assert_array_equal(mask[off[i]:off[i + 1]], ml)


def test_batched_refit_bit_exact_per_problem():
    probs = [synth.pnp_problem(n, 0.4, seed=120 + i) for i, n in enumerate([50, 3000, 700, 12000])]
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 2000, 30.0, refine=True)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 2000, 0x5EED)
        soa = O.soa_pnp(p["points3d"], p["points2d"])
        Ro, to, _ = O.pnp_refine(soa, ref["mask"].astype(np.uint8), O.cam_from_K(p["K"]), ref["R"], ref["t"])
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, Ro) and _bits_equal(t, to)


@pytest.mark.parametrize("outl,refine", [(0.85, True), (0.85, False), (0.93, True)])
def test_speculative_first_round_falls_back(outl, refine):
    # the first round (256 hypotheses) cannot end these scans: the device's speculative finish is
    # discarded and the loop resumes at round 2; results equal the restatement's
    pr = synth.pnp_problem(3000, outl, seed=int(outl * 100))
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=refine,
                                    return_info=True)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000, 0x5EED)
    assert info.rounds > 1
    assert (info.best_hyp, info.n_inliers, info.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(m, ref["mask"])
    if refine:
        soa = O.soa_pnp(pr["points3d"], pr["points2d"])
        ref["R"], ref["t"], _ = O.pnp_refine(soa, ref["mask"].astype(np.uint8), O.cam_from_K(pr["K"]), ref["R"],
                                             ref["t"])
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


def _refit_case(n, outl, seed=77):
    pr = synth.pnp_problem(n, outl, seed=seed)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 2000, 0x5EED)
    soa = O.soa_pnp(pr["points3d"], pr["points2d"])
    Ro, to, _ = O.pnp_refine(soa, ref["mask"].astype(np.uint8), O.cam_from_K(pr["K"]), ref["R"], ref["t"])
    return pr, ref, Ro, to


@pytest.mark.parametrize("n,outl", [(4096, 0.3), (4097, 0.6), (65536, 0.5), (65537, 0.5), (300000, 0.5)])
def test_refit_block_ranges_bit_exact(n, outl):
    # one range at 4096 points, 5 ranges of 820 indices at 4097; 65536: 64 ranges of exactly
    # 1024 (the block count saturates), 65537: 64 ranges of 1025 (still one tile each);
    # 300000 points: 64 ranges of 4688 indices, each more than one LDS tile, so every pass
    # re-stages its tiles (k_pnp_refine tile path)
    pr, ref, Ro, to = _refit_case(n, outl)
    ranges, _ = rsac.context().refit_blocks(n)
    assert ranges == (1 if n <= 4096 else min(64, -(-n // 1024)))
    R, t, m = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, refine=True)
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, Ro) and _bits_equal(t, to)


@pytest.mark.parametrize("cap", [1, 3, 7])
@pytest.mark.parametrize("n", [20000, 65537, 300000])
def test_refit_fewer_blocks_than_ranges_bit_exact(n, cap):
    # a device that cannot hold lm_blocks(n) blocks at once: G = cap blocks walk the ranges
    # x, x + G, ... each (staged once when their indices fit one tile, else tile by tile);
    # the summation order, and so the pose, is unchanged
    ctx = rsac.context()
    pr, ref, Ro, to = _refit_case(n, 0.5)
    try:
        ctx.debug_set(L.DBG_REFIT_MAX_BLOCKS, cap)
        ranges, blocks = ctx.refit_blocks(n)
        assert blocks == min(cap, ranges)
        R, t, m = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, refine=True)
        R2, t2, _, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=False,
                                          lo=True, return_info=True)
    finally:
        ctx.debug_set(L.DBG_REFIT_MAX_BLOCKS, 0)
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, Ro) and _bits_equal(t, to)
    lo = O.pnp_ransac_lo(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000)
    assert info.lo_improvements == lo["lo_improvements"]
    assert _bits_equal(R2, lo["R"]) and _bits_equal(t2, lo["t"])


def test_refit_missing_block_recovers_with_one_block():
    # one block of the refit's stride is never launched (test hook), as when other work holds the
    # CUs: the others stop waiting after ~1 s, the failure is detected after the call's
    # synchronisation and the call is redone with one block per refit -- the same pose, bit for
    # bit; the context keeps its multi-block limit afterwards
    ctx = rsac.context()
    pr, ref, Ro, to = _refit_case(20000, 0.5)
    before = ctx.refit_blocks(20000)
    try:
        ctx.debug_set(L.DBG_REFIT_DROP_BLOCK, 1)
        R, t, m = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, refine=True)
        np.testing.assert_array_equal(m, ref["mask"])
        assert _bits_equal(R, Ro) and _bits_equal(t, to)
        R2, t2, _, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=False,
                                          lo=True, return_info=True)
    finally:
        ctx.debug_set(L.DBG_REFIT_DROP_BLOCK, 0)
    assert ctx.refit_blocks(20000) == before
    lo = O.pnp_ransac_lo(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000)
    assert info.lo_improvements == lo["lo_improvements"]
    assert _bits_equal(R2, lo["R"]) and _bits_equal(t2, lo["t"])
    R, t, m = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, refine=True)
    assert _bits_equal(R, Ro) and _bits_equal(t, to)


_COOP_CHILD = """
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import rsac
from rsac import synth
for n in (20000, 65537):
    pr = synth.pnp_problem(n, 0.5, seed=77)
    R, t, m = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 2000, 30.0, refine=True)
    print(np.asarray(R, np.float64).tobytes().hex(), np.asarray(t, np.float64).tobytes().hex())
"""


def test_refit_cooperative_launch_bit_exact():
    # RSAC_REFIT_COOP=1 (read when a context first refits, hence a child process): the multi-block
    # refit goes through hipLaunchCooperativeKernel; the pose is the oracle's, bit for bit
    import subprocess
    import sys
    pkg = os.path.dirname(os.path.dirname(rsac.__file__))
    out = subprocess.run([sys.executable, "-c", _COOP_CHILD, pkg], env=dict(os.environ, RSAC_REFIT_COOP="1"),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = out.stdout.split("\n")
    for n, line in zip((20000, 65537), lines):
        _, _, Ro, to = _refit_case(n, 0.5)
        rh, th = line.split()
        assert rh == np.asarray(Ro, np.float64).tobytes().hex() and th == np.asarray(to, np.float64).tobytes().hex()


# ---------------------------------------------------------------------------------------------
# LO-RANSAC (BASELINE.json configs[4])
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,outl,seed", [(3000, 0.8, 5), (20000, 0.7, 5), (5000, 0.5, 9), (100000, 0.5, 3)])
def test_lo_ransac_matches_restatement(n, outl, seed):
    pr = synth.pnp_problem(n, outl, seed=seed)
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=False, lo=True,
                                    return_info=True)
    ref = O.pnp_ransac_lo(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000)
    assert (info.best_hyp, info.n_inliers, info.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    assert info.lo_improvements == ref["lo_improvements"]
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    np.testing.assert_array_equal(m, ref["mask"])


def test_parallel_driver_lo_single_rank_equals_pnp_ransac_lo():
    from rsac import parallel as par
    pr = synth.pnp_problem(8000, 0.75, seed=31)
    ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
    res = par.sharded_ransac(ev, 5000, 0.99, round_size=333, lo=True)
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=False, lo=True,
                                    return_info=True)
    assert (res.best, res.n_inliers, res.iters) == (info.best_hyp, info.n_inliers, info.iters)
    assert _bits_equal(res.model[:9].reshape(3, 3), R) and _bits_equal(res.model[9:], t)


# ---------------------------------------------------------------------------------------------
# fundamental matrix (BASELINE.json configs[3]): bit-exact against the restatement
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,outl,H", [(8, 0.0, 64), (60, 0.5, 700), (3000, 0.8, 1500), (20000, 0.8, 600)])
def test_fundamental_hypotheses_bit_exact(n, outl, H):
    pr = synth.fundamental_problem(n, outl, seed=n)
    soa = O.soa_hom(pr["pts1"], pr["pts2"])
    st, cnt, mdl = rsac.hypotheses("fundamental", pr["pts1"], pr["pts2"], None, 11, H, 1.5, seed=7)
    oc, os_, om = O.fm_hypotheses(soa, 1.5, 7, H, hyp0=11, models=True)
    np.testing.assert_array_equal(st, os_)
    np.testing.assert_array_equal(cnt, oc)
    assert _bits_equal(mdl[:, :9], om[:, :9])


@pytest.mark.parametrize("n,outl,thr", [(20000, 0.8, 1.5), (5000, 0.3, 0.4), (5000, 0.5, 6.0), (3001, 0.8, 60.0)])
def test_fundamental_f32_prefilter_equals_exact_kernel(n, outl, thr):
    # the f32 Sampson pre-filter (k_fm_score_f32) must never change a decision: counts equal the
    # all-f64 kernel's, and the thresholds put many pairs inside the pre-filter's band
    pr = synth.fundamental_problem(n, outl, seed=n + 5)
    st_f, c_f, _ = rsac.hypotheses("fundamental", pr["pts1"], pr["pts2"], None, 0, 3000, thr, seed=3)
    st_e, c_e, _ = rsac.hypotheses("fundamental", pr["pts1"], pr["pts2"], None, 0, 3000, thr, seed=3,
                                   exact_only=True)
    np.testing.assert_array_equal(st_f, st_e)
    np.testing.assert_array_equal(c_f, c_e)
    assert c_e.max() > 0


@pytest.mark.parametrize("n,outl", [(5000, 0.5), (50000, 0.8)])
def test_fundamental_ransac_matches_restatement(n, outl):
    pr = synth.fundamental_problem(n, outl, seed=2)
    F, m, info = rsac.fundamental_ransac(pr["pts1"], pr["pts2"], 1.5, max_iters=3000, return_info=True)
    ref = O.fm_ransac(pr["pts1"], pr["pts2"], 1.5, 0.99, 3000)
    assert (info.best_hyp, info.n_inliers, info.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    assert _bits_equal(F, ref["F"])
    np.testing.assert_array_equal(m, ref["mask"])


# ---------------------------------------------------------------------------------------------
# asynchronous device-result path (bench step) and the on-device winner re-derivation
# ---------------------------------------------------------------------------------------------
def test_async_evaluate_range_and_winner_match_sync():
    import torch
    pr = synth.pnp_problem(6000, 0.5, seed=61)
    p2 = torch.from_numpy(pr["points2d"]).cuda()
    p3 = torch.from_numpy(pr["points3d"]).cuda()
    # back-to-back async calls with different thresholds / ranges on one context: the pinned
    # staging buffers must not be overwritten before their copies ran
    outs = [rsac.evaluate_range(p2, p3, pr["K"], b, 3000, thr, with_mask=True, device_result=True)
            for b, thr in [(0, 30.0), (3000, 12.0), (6000, 30.0), (9000, 50.0)]]
    torch.cuda.synchronize()
    for (key_t, model_t, mask_t), (b, thr) in zip(outs, [(0, 30.0), (3000, 12.0), (6000, 30.0), (9000, 50.0)]):
        key, model, mask = rsac.evaluate_range(pr["points2d"], pr["points3d"], pr["K"], b, 3000, thr, with_mask=True)
        assert int(key_t.item()) == key
        assert _bits_equal(model_t.cpu().numpy(), model)
        np.testing.assert_array_equal(mask_t.cpu().numpy(), mask)
        # the winner re-derived from the key alone (what a losing rank does)
        wm, wmask = rsac.winner(p2, p3, pr["K"], key_t, thr)
        assert _bits_equal(wm.cpu().numpy(), model)
        np.testing.assert_array_equal(wmask.cpu().numpy(), mask)


def test_winner_of_empty_key_is_zero():
    import torch
    pr = synth.pnp_problem(500, 0.5, seed=62)
    p2 = torch.from_numpy(pr["points2d"]).cuda()
    p3 = torch.from_numpy(pr["points3d"]).cuda()
    wm, wmask = rsac.winner(p2, p3, pr["K"], torch.zeros(1, dtype=torch.int64, device="cuda"), 30.0)
    assert not wm.cpu().numpy().any() and not wmask.cpu().numpy().any()


# ---------------------------------------------------------------------------------------------
# the multi-GPU round's device path: {status, count} rows written by the kernels and the
# device-listed scan (rsac_pnp_hypothesis_rows, rsac_scan_device)
# ---------------------------------------------------------------------------------------------
def test_hypothesis_rows_equal_hypotheses():
    import torch
    pr = synth.pnp_problem(5000, 0.5, seed=64)
    p2 = torch.from_numpy(pr["points2d"]).cuda()
    p3 = torch.from_numpy(pr["points3d"]).cuda()
    rows = torch.full((3000, 2), -7, dtype=torch.int32, device="cuda")
    rsac.api.hypothesis_rows(p2, p3, pr["K"], 123, 2500, 30.0, rows)
    st, cn, _ = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 123, 2500, 30.0)
    r = rows.cpu().numpy()
    np.testing.assert_array_equal(r[:2500, 0], st)
    np.testing.assert_array_equal(r[:2500, 1], cn)
    assert (r[2500:] == -7).all()


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_scan_device_equals_host_scan(seed):
    """rsac_scan_device (records listed on the device, bound applied on the host) consumes rows as
    the host scan does: random counts / statuses (zeros, a sampler failure), rounds of random
    length, stop_on_improve with raised counts in between (LO), and runs of more improvements
    than the record list holds (the exact host fallback)."""
    import torch
    rng = np.random.default_rng(seed)
    H = 6000
    counts = rng.integers(0, 3000, H).astype(np.int32)
    if seed == 3:
        counts[:200] = np.arange(200) * 10  # 199 improvements in a row
    status = rng.choice(np.array([0, 1], np.int8), H, p=[0.1, 0.9])
    if seed == 1:
        status[4500] = -1
    rows = torch.from_numpy(np.stack([status.astype(np.int32), counts], axis=1)).cuda()
    for lo in (False, True):
        a = rsac.Scan(H, 5000, 0.999, 4)
        b = rsac.Scan(H, 5000, 0.999, 4)
        pos = 0
        while not a.done and pos < H:
            step = int(rng.integers(1, 900))
            step = min(step, H - pos)
            if lo:
                ca = a.step_rows(rows[pos:], step, stop_on_improve=True)
                cb = b.step_rows(rows[pos:].cpu().numpy(), step, stop_on_improve=True)
                assert (ca, a.improved) == (cb, b.improved)
                if a.improved:
                    raised = a.max_good + int(rng.integers(0, 3))
                    a.raise_count(raised)
                    b.raise_count(raised)
                pos += ca
            else:
                a.step_rows(rows[pos:], step)
                b.step_rows(rows[pos:].cpu().numpy(), step)
                pos += step
            assert (a.best, a.max_good, a.iters, a.niters, a.done) == (b.best, b.max_good, b.iters, b.niters, b.done)


def test_fast_f64_cores_equal_ieee_operators():
    # rsac_math.h dsqrt_fast / ddiv_fast and the Jacobi rotation's fast form (rsac_cvepnp.h), the
    # compiler's IEEE sequences without their scaling wrappers, against the IEEE operators on the
    # device: 4M random operand sets inside the ranges their callers prove, plus the range ends
    ctx = rsac.context(0)
    ctx.debug_set(7, 1 << 22)  # RSAC_DBG_F64_SELFTEST
    assert ctx.debug_get(7) == 0


def _spec_counters():
    import ctypes as C
    ctx = rsac.context(0)
    f, r = C.c_int64(0), C.c_int64(0)
    rsac.lib().rsac_debug_get(ctx.handle, 3, C.byref(f))  # RSAC_DBG_SPEC_FINISHES
    rsac.lib().rsac_debug_get(ctx.handle, 4, C.byref(r))  # RSAC_DBG_SPEC_REDOS
    return f.value, r.value


@pytest.mark.parametrize("sampler,minimal", [("opencv", "p3p"), ("opencv", "epnp5"), ("philox", "p3p")])
def test_speculative_first_round_overflow_restarts_the_sampler(sampler, minimal):
    """when the host's replay of a speculative first round finds more
    improvements than the device records, the scan restarts at hypothesis 0 -- and so must
    OpenCV's MWC sampler (a resumed state would redraw hypotheses 0.. from positions 256.. of its
    sequence).  RSAC_DBG_SPEC_OVERFLOW forces that branch on a run that needs later rounds; the
    result must still be the oracle's sequential loop."""
    pr = synth.pnp_problem(1500, 0.8, seed=91)
    ctx = rsac.context(0)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 3000, 0x5EED, sampler=sampler,
                       minimal=minimal)
    assert ref["iters"] > 256  # the run goes past the speculative first round
    f0, r0 = _spec_counters()
    ctx.debug_set(6, 1)  # RSAC_DBG_SPEC_OVERFLOW
    try:
        R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 3000, 30.0, sampler=sampler,
                                        minimal=minimal, refine=False, return_info=True)
    finally:
        ctx.debug_set(6, 0)
    f1, r1 = _spec_counters()
    assert f1 - f0 == 1 and r1 - r0 == 1  # the speculative finish ran and was redone
    assert info.best_hyp == ref["best"] and info.n_inliers == ref["n_inliers"] and info.iters == ref["iters"]
    np.testing.assert_array_equal(m, ref["mask"])
    assert np.array_equal(R, ref["R"]) and np.array_equal(t, ref["t"])


@pytest.mark.parametrize("sampler,minimal", [("philox", "p3p"), ("opencv", "p3p"), ("opencv", "epnp5")])
def test_fixed_budget_device_pick_batched(sampler, minimal):
    """adaptive off: k_scan_records picks every problem's winner on the device and the masks are
    enqueued behind it (no host round trip).  A ragged batch with a problem that has no model
    (all points equal) and one of 4 points: every result equals the oracle's sequential loop, the
    speculative finish is taken once per call and never redone."""
    probs = [synth.pnp_problem(n, 0.4, seed=170 + i) for i, n in enumerate([900, 50, 2600, 4, 300])]
    dead = dict(probs[1])
    dead["points3d"] = np.tile(probs[1]["points3d"][:1], (50, 1))
    probs[1] = dead
    f0, r0 = _spec_counters()
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 700, 30.0, adaptive=False, refine=False, sampler=sampler,
                                  minimal=minimal)
    f1, r1 = _spec_counters()
    assert (f1 - f0, r1 - r0) == (1, 0)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 700, 0x5EED, sampler=sampler,
                           minimal=minimal)
        assert (R is None) == (ref["best"] < 0)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        if R is not None:
            assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
    # the same batch with the LM refit enqueued behind the device's pick: the refined poses are
    # the oracle's refit of its own winners
    out2 = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                   [p["K"] for p in probs], 700, 30.0, adaptive=False, refine=True, sampler=sampler,
                                   minimal=minimal)
    assert _spec_counters()[1] == r0
    for p, (R, t, m, ni) in zip(probs, out2):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 700, 0x5EED, sampler=sampler,
                           minimal=minimal)
        if ref["best"] < 0:
            assert R is None
            continue
        if len(p["points3d"]) == 4:  # solvePnPRansac's count == model_points branch: no final solve
            assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"]) and m.all()
            continue
        soa, cam = O.soa_pnp(p["points3d"], p["points2d"]), O.cam_from_K(p["K"])
        Rl, tl, _ = O.pnp_refine(soa, ref["mask"].astype(np.uint8), cam, ref["R"].reshape(9), ref["t"])
        assert _bits_equal(R, Rl) and _bits_equal(t, tl)


def test_two_contexts_on_two_streams_equal_serial():
    """bench.py's pipelined steps: evaluate_range calls alternating between two contexts on two
    torch streams (running concurrently) give every step the serial call's key, model and mask."""
    import torch
    from rsac import parallel as par
    pr, soa, cam = _pnp_case(10000, 0.5, 0)
    ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
    H = 40_000
    k0, m0, mk0 = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], 0, H, 30.0, with_mask=True, device_result=True)
    torch.cuda.synchronize()
    ctxs = [rsac.context(0), rsac.Context(0)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    outs = []
    for i in range(8):
        j = i & 1
        with torch.cuda.stream(streams[j]):
            base = (i // 2) * 1000  # different ranges in flight at once
            outs.append((base,) + rsac.evaluate_range(ev.p2, ev.p3, pr["K"], base, H, 30.0, with_mask=True,
                                                      device_result=True, context=ctxs[j]))
    torch.cuda.synchronize()
    for base, k, m, mk in outs:
        kr, mr, mkr = rsac.evaluate_range(ev.p2, ev.p3, pr["K"], base, H, 30.0, with_mask=True, device_result=True)
        torch.cuda.synchronize()
        assert int(k.item()) == int(kr.item())
        assert _bits_equal(m.cpu().numpy(), mr.cpu().numpy())
        np.testing.assert_array_equal(mk.cpu().numpy(), mkr.cpu().numpy())
    assert int(outs[0][1].item()) == int(k0.item())


@pytest.mark.parametrize("n,outl,seed,lo", [(3000, 0.5, 41, False), (4000, 0.8, 42, False), (4000, 0.8, 43, True),
                                            (3000, 0.4, 44, True)])
def test_first_round_mode_equals_pnp_ransac(n, outl, seed, lo):
    """rsac_pnp_ransac_first_round (the sharded loop's redundant round 1): when
    the 256-hypothesis round ends the scan it is pnp_ransac bit for bit; otherwise its scan state
    is the sequential scan of hypotheses [0, 256) and the best model so far, and the sharded loop
    continued from it (one rank) ends where pnp_ransac does."""
    from rsac import parallel as par
    pr = synth.pnp_problem(n, outl, seed=seed)
    done, R, t, mask, scan, finfo = rsac.pnp_ransac_first_round(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0,
                                                         refine=False, lo=lo)
    Rf, tf, mf, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, refine=False, lo=lo,
                                       return_info=True)
    if done:
        assert (scan.best, scan.max_good, scan.iters) == (info.best_hyp, info.n_inliers, info.iters)
        assert finfo.lo_improvements == info.lo_improvements
        assert _bits_equal(R, Rf) and _bits_equal(t, tf)
        np.testing.assert_array_equal(mask, mf)
    else:
        assert scan.iters == par.FIRST_ROUND and info.iters > par.FIRST_ROUND
        assert mask is None
        if not lo:  # the scan of the round's rows, replayed on the host
            st, cn, _ = rsac.hypotheses("pnp", pr["points3d"], pr["points2d"], pr["K"], 0, par.FIRST_ROUND, 30.0)
            ref = rsac.Scan(5000, n, 0.99, 4).step(cn, st)
            assert (scan.best, scan.max_good, scan.niters) == (ref.best, ref.max_good, ref.niters)
            m = np.concatenate([R.reshape(9), t])
            ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
            assert _bits_equal(m, ev.model(scan.best))
    # the sharded loop (one rank) goes on from the exported state to pnp_ransac's result
    ev = par.PnPShard(pr["points2d"], pr["points3d"], pr["K"], 30.0, device=0)
    res = par.sharded_ransac(ev, 5000, 0.99, round_size=1024, lo=lo)
    assert (res.best, res.n_inliers, res.iters) == (info.best_hyp, info.n_inliers, info.iters)
    assert res.lo_improvements == info.lo_improvements
    assert _bits_equal(res.model[:9].reshape(3, 3), Rf) and _bits_equal(res.model[9:], tf)


@pytest.mark.parametrize("refine,adaptive", [(False, False), (True, True)])
def test_batched_rows_on_device_equal_flat_outputs(refine, adaptive):
    """rsac_pnp_ransac_batched_rows (the C3 problem-shard rows, written on the device) carries
    exactly pnp_ransac_batched_flat's (ok, n_inliers, R, t), and parallel.pnp_batched_rows hands
    the device tensor to the all-gather (one rank here)."""
    import torch
    from rsac import parallel as par
    probs = [synth.pnp_problem(n, o, seed=s) for s, (n, o) in enumerate([(500, 0.4), (64, 0.9), (2000, 0.5),
                                                                          (6, 0.0), (1200, 0.7)])]
    off = np.zeros(len(probs) + 1, np.int64)
    off[1:] = np.cumsum([len(p["points3d"]) for p in probs])
    p2 = torch.from_numpy(np.concatenate([p["points2d"] for p in probs])).cuda()
    p3 = torch.from_numpy(np.concatenate([p["points3d"] for p in probs])).cuda()
    Ks = np.stack([p["K"] for p in probs])
    R, t, ok, ninl, mask = rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 700, 30.0, adaptive=adaptive, refine=refine)
    rows, mask2 = rsac.pnp_ransac_batched_rows(p2, p3, off, Ks, 700, 30.0, adaptive=adaptive, refine=refine)
    assert rows.is_cuda and rows.shape == (len(probs), 14)
    h = rows.cpu().numpy()
    np.testing.assert_array_equal(h[:, 0], ok.astype(np.float64))
    np.testing.assert_array_equal(h[:, 1], np.where(ok, ninl, 0))
    assert _bits_equal(h[ok, 2:11], R.reshape(-1, 9)[ok]) and _bits_equal(h[ok, 11:14], t[ok])
    assert not h[~ok, 2:].any()
    np.testing.assert_array_equal(mask2.cpu().numpy(), mask.cpu().numpy())
    g = par.sharded_batched(par.pnp_batched_rows(p2, p3, off, Ks, 700, 30.0, adaptive=adaptive, refine=refine),
                            len(probs))
    assert _bits_equal(g.cpu().numpy(), h)


@pytest.mark.parametrize("sampler", ["philox", "opencv"])
def test_fixed_budget_long_round_block_scan(sampler):
    """Rounds of >= 8192 hypotheses replay their scan in one 1024-thread block per problem
    (k_scan_records_blk, C4's 100k round): a ragged batch (a dead problem, a 4-point one, a 97 %
    outlier one with many improvements) over 9000 hypotheses equals the oracle's sequential loop,
    the device's pick is never redone."""
    probs = [synth.pnp_problem(n, o, seed=190 + i) for i, (n, o) in
             enumerate([(1200, 0.6), (40, 0.4), (3000, 0.97), (4, 0.0), (700, 0.85)])]
    dead = dict(probs[1])
    dead["points3d"] = np.tile(probs[1]["points3d"][:1], (40, 1))
    probs[1] = dead
    f0, r0 = _spec_counters()
    out = rsac.pnp_ransac_batched([p["points2d"] for p in probs], [p["points3d"] for p in probs],
                                  [p["K"] for p in probs], 9000, 30.0, adaptive=False, refine=False, sampler=sampler)
    f1, r1 = _spec_counters()
    assert (f1 - f0, r1 - r0) == (1, 0)
    for p, (R, t, m, ni) in zip(probs, out):
        ref = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, 9000, 0x5EED, sampler=sampler)
        assert (R is None) == (ref["best"] < 0)
        assert ni == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        if R is not None:
            assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])


def test_fundamental_fixed_budget_long_round():
    """C4's shape at test size: adaptive off, 12000 hypotheses in one round (block scan), bit-exact
    against the restatement's scan."""
    pr = synth.fundamental_problem(20000, 0.8, seed=4)
    F, m, info = rsac.fundamental_ransac(pr["pts1"], pr["pts2"], 1.5, max_iters=12000, adaptive=False,
                                         return_info=True)
    ref = O.fm_ransac(pr["pts1"], pr["pts2"], 1.5, 0.99, 12000)
    assert (info.best_hyp, info.n_inliers) == (ref["best"], ref["n_inliers"])
    assert _bits_equal(F, ref["F"])
    np.testing.assert_array_equal(m, ref["mask"])


@pytest.mark.parametrize("minimal,outl", [("p3p", 0.8), ("epnp5", 0.7), ("epnp5", 0.85)])
def test_speculative_first_round_opencv_sampler(minimal, outl):
    """OpenCV's sampler also takes the speculative first round (r05): when the round ends the scan
    the device's finish stands; when it does not, the loop resumes with the MWC state the first
    round left (LoopOut::rngs).  Both equal the restatement's sequential loop."""
    pr = synth.pnp_problem(3000, outl, seed=int(outl * 100) + 7)
    f0, _ = _spec_counters()
    R, t, m, info = rsac.pnp_ransac(pr["points2d"], pr["points3d"], pr["K"], 5000, 30.0, sampler="opencv",
                                    minimal=minimal, refine=False, return_info=True)
    ref = O.pnp_ransac(pr["points3d"], pr["points2d"], pr["K"], 30.0, 0.99, 5000, sampler="opencv", minimal=minimal)
    assert _spec_counters()[0] == f0 + 1
    assert (info.best_hyp, info.n_inliers, info.iters) == (ref["best"], ref["n_inliers"], ref["iters"])
    np.testing.assert_array_equal(m, ref["mask"])
    assert _bits_equal(R, ref["R"]) and _bits_equal(t, ref["t"])
