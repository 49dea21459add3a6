"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU restatement (oracle/rsac_oracle.c).

Only tests/, bench.py's ``cpu_baseline`` leg and ``__graft_entry__.smoke()`` may
import this module, and only as the checker or the timed CPU baseline.  The
product package (code-reproduction-ransac_amd/rsac) never imports it.

Inputs follow OpenCV's conversion in cv2.solvePnPRansac / cv2.findHomography
(main_v1.py:497, main_v1.py:312): float64 arrays are rounded to float32 and
stored structure-of-arrays.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_LIB_UNFUSED = os.path.join(_HERE, "liboracle_unfused.so")
_libs = {}
# The PnP restatement in use (oracle/rsac_oracle.c orc_set_sequence):
#   "cv"         OpenCV's operation sequence for the EPnP-5 minimal solver and the Rodrigues round
#                trip (oracle/cv_epnp.c) -- the default, the one the GPU reproduces;
#   "rr"         the round-4/5 restatement (round-robin Jacobi EPnP with fused steps, polar Rodrigues);
#   "rr_unfused" the same built with every explicit fma as a rounded product + a rounded sum.
# The last two exist for the decision-change study (tests/test_cv_epnp.py, scripts/epnp_variants.py).
SEQUENCES = ("cv", "rr", "rr_unfused")
_sequence = "cv"


class sequence:
    """Context manager: ``with pyoracle.sequence("rr"): ...`` runs the PnP oracle in another
    restatement (not thread-safe: the study runs one variant at a time)."""

    def __init__(self, name):
        if name not in SEQUENCES:
            raise ValueError(f"unknown sequence {name!r}")
        self.name = name

    def __enter__(self):
        global _sequence
        self.prev, _sequence = _sequence, self.name
        return self

    def __exit__(self, *exc):
        global _sequence
        _sequence = self.prev
        return False

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    key = _LIB_UNFUSED if _sequence == "rr_unfused" else _LIB_PATH
    L = _libs.get(key)
    if L is None:
        srcs = [os.path.join(_HERE, f) for f in ("rsac_oracle.c", "cv_epnp.c")]
        if not os.path.exists(key) or os.path.getmtime(key) < max(os.path.getmtime(f) for f in srcs):
            build()
        L = _libs[key] = _load(key)
    L.orc_set_sequence(0 if _sequence == "cv" else 1)
    return L


def _load(path):
    L = C.CDLL(path)
    L.orc_set_sequence.argtypes = [C.c_int]
    L.orc_set_sequence.restype = None
    L.orc_cv_epnp.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_void_p, C.c_int, _f64p, _f64p, _f64p]
    L.orc_cv_epnp.restype = C.c_int
    L.orc_cvq_fill_events.argtypes = [C.c_int]
    L.orc_cvq_fill_events.restype = C.c_long
    L.cvq_hypot.argtypes = [C.c_double, C.c_double]
    L.cvq_hypot.restype = C.c_double
    L.cvq_jacobi_svd.argtypes = [_f64p, C.c_int, _f64p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]
    L.cvq_jacobi_svd.restype = None
    L.cvq_svd3.argtypes = [_f64p, _f64p, _f64p, _f64p]
    L.cvq_svd3.restype = None
    L.cvq_invert3.argtypes = [_f64p, _f64p]
    L.cvq_invert3.restype = None
    L.cvq_solve6.argtypes = [_f64p, C.c_int, _f64p, _f64p]
    L.cvq_solve6.restype = None
    L.orc_mwc_next.argtypes = [C.POINTER(C.c_uint64)]
    L.orc_mwc_next.restype = C.c_uint32
    L.orc_mwc_uniform.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int]
    L.orc_mwc_uniform.restype = C.c_int
    L.orc_philox4x32_10.argtypes = [_u32p, _u32p, _u32p]
    L.orc_philox4x32_10.restype = None
    L.orc_philox_subset.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_int, C.c_int, _i32p]
    L.orc_philox_subset.restype = C.c_int
    L.orc_update_num_iters.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int]
    L.orc_update_num_iters.restype = C.c_int
    L.orc_scan.argtypes = [_i32p, _i8p, C.c_int64, C.c_int, C.c_int, C.c_double, C.c_int,
                           C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    L.orc_scan.restype = C.c_int64
    L.orc_pnp_err.argtypes = [_f64p, _f64p, _f64p] + [C.c_float] * 5
    L.orc_pnp_err.restype = C.c_float
    L.orc_thr2.argtypes = [C.c_double]
    L.orc_thr2.restype = C.c_float
    L.orc_reproj_errors.argtypes = [_f64p, _f64p, _f64p, _f64p, _f64p, C.c_int, C.c_void_p, C.c_void_p]
    L.orc_reproj_errors.restype = None
    L.orc_reproj_mean_sum.argtypes = [_f64p, _f64p, _f64p, _f64p, _f64p, _u8p, C.c_int, C.POINTER(C.c_int)]
    L.orc_reproj_mean_sum.restype = C.c_double
    L.orc_pnp_count.argtypes = [_f64p, _f64p, _f64p, _f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, C.c_float,
                                C.c_void_p]
    L.orc_pnp_count.restype = C.c_int32
    L.orc_p3p.argtypes = [_f64p, _f64p, _f64p, _f64p]
    L.orc_p3p.restype = C.c_int
    L.orc_pnp_minimal.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _i32p, _f64p, _f64p, _f64p]
    L.orc_pnp_minimal.restype = C.c_int
    L.orc_hom_check_subset.argtypes = [_f32p, _f32p, _f32p, _f32p, _i32p]
    L.orc_hom_check_subset.restype = C.c_int
    L.orc_hom_minimal.argtypes = [_f32p, _f32p, _f32p, _f32p, _i32p, _f64p]
    L.orc_hom_minimal.restype = C.c_int
    L.orc_hom_err.argtypes = [_f64p] + [C.c_float] * 4
    L.orc_hom_err.restype = C.c_float
    L.orc_hom_count.argtypes = [_f64p, _f32p, _f32p, _f32p, _f32p, C.c_int, C.c_float, C.c_void_p]
    L.orc_hom_count.restype = C.c_int32
    L.orc_mwc_subsets.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, _i32p, _i8p]
    L.orc_mwc_subsets.restype = None
    L.orc_pnp_hypotheses.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_float, C.c_uint64,
                                     C.c_uint32, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, _i32p, _i8p,
                                     C.c_void_p]
    L.orc_pnp_hypotheses.restype = None
    L.orc_pnp_hypotheses_k.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_float, C.c_uint64,
                                       C.c_uint32, C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, _i32p, _i8p,
                                       C.c_void_p, C.c_int]
    L.orc_pnp_hypotheses_k.restype = None
    L.orc_pnp_minimal_epnp5.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _i32p, _f64p, _f64p, _f64p]
    L.orc_pnp_minimal_epnp5.restype = C.c_int
    L.orc_hom_hypotheses.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_float, C.c_uint64, C.c_uint32,
                                     C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, _i32p, _i8p, C.c_void_p]
    L.orc_hom_hypotheses.restype = None
    L.orc_rodrigues_v2m.argtypes = [_f64p, _f64p]
    L.orc_rodrigues_v2m.restype = None
    L.orc_rodrigues_m2v.argtypes = [_f64p, _f64p]
    L.orc_rodrigues_m2v.restype = None
    L.orc_pnp_refine.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _u8p, C.c_int, _f64p, _f64p, _f64p, C.c_int]
    L.orc_pnp_refine.restype = C.c_int
    L.orc_pnp_epnp.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _u8p, C.c_int, _f64p, _f64p, _f64p]
    L.orc_pnp_epnp.restype = C.c_int
    L.orc_hom_refine.argtypes = [_f32p, _f32p, _f32p, _f32p, _u8p, C.c_int, _f64p]
    L.orc_hom_refine.restype = C.c_int
    L.orc_pnp_ransac.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                 C.c_int, C.c_uint64, C.c_int, _f64p, _f64p, _u8p, C.POINTER(C.c_int32),
                                 C.POINTER(C.c_int64)]
    L.orc_pnp_ransac.restype = C.c_int64
    L.orc_pnp_ransac_k.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                   C.c_int, C.c_uint64, C.c_int, C.c_int, _f64p, _f64p, _u8p, C.POINTER(C.c_int32),
                                   C.POINTER(C.c_int64), C.c_int]
    L.orc_pnp_ransac_k.restype = C.c_int64
    L.orc_pnp_ransac_seq.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                     C.c_int, C.c_uint64, _f64p, _f64p, _u8p, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int64)]
    L.orc_pnp_ransac_seq.restype = C.c_int64
    L.orc_pnp_ransac_seq_k.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                       C.c_int, C.c_uint64, C.c_int, C.c_int, _f64p, _f64p, _u8p,
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int]
    L.orc_rvec_roundtrip.argtypes = [_f64p]
    L.orc_rvec_roundtrip.restype = None
    L.orc_rd_acos.argtypes = [C.c_double]
    L.orc_rd_acos.restype = C.c_double
    L.orc_rd_sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.orc_rd_sincos.restype = None
    L.orc_pnp_ransac_seq_k.restype = C.c_int64
    L.orc_pnp_hypotheses_mt.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_float, C.c_uint64,
                                        C.c_int64, C.c_int64, _i32p, _i8p, C.c_int]
    L.orc_pnp_hypotheses_mt.restype = None
    L.orc_pnp_ransac_lo.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                    C.c_int, C.c_uint64, _f64p, _f64p, _u8p, C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
    L.orc_pnp_ransac_lo.restype = C.c_int64
    L.orc_pnp_ransac_lo_seq.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                    C.c_int, C.c_uint64, _f64p, _f64p, _u8p, C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
    L.orc_pnp_ransac_lo_seq.restype = C.c_int64
    L.orc_pnp_local_opt.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_float, _f64p, _f64p,
                                    C.c_int32, C.POINTER(C.c_int32)]
    L.orc_pnp_local_opt.restype = C.c_int32
    L.orc_hom_ransac.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_double, C.c_double, C.c_int,
                                 C.c_uint64, C.c_int, _f64p, _u8p, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    L.orc_hom_ransac.restype = C.c_int64
    L.orc_fm_minimal8.argtypes = [_f32p, _f32p, _f32p, _f32p, _f64p]
    L.orc_fm_minimal8.restype = C.c_int
    L.orc_fm_count.argtypes = [_f64p, _f32p, _f32p, _f32p, _f32p, C.c_int, C.c_float, C.c_void_p]
    L.orc_fm_count.restype = C.c_int32
    L.orc_fm_hypotheses.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_float, C.c_uint64, C.c_int64,
                                    C.c_int64, _i32p, _i8p, C.c_void_p]
    L.orc_fm_hypotheses.restype = None
    L.orc_fm_hypotheses_mt.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_float, C.c_uint64, C.c_int64,
                                       C.c_int64, _i32p, _i8p, C.c_int]
    L.orc_fm_hypotheses_mt.restype = None
    L.orc_pnp_ransac_lo_mt.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, _f64p, C.c_double, C.c_double,
                                       C.c_int, C.c_uint64, _f64p, _f64p, _u8p, C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_int]
    L.orc_pnp_ransac_lo_mt.restype = C.c_int64
    L.orc_fm_ransac.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_double, C.c_double, C.c_int, C.c_uint64,
                                _f64p, _u8p, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    L.orc_fm_ransac.restype = C.c_int64
    return L


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ----------------------------------------------------------------------------------------------
# data conversion (OpenCV: objectPoints / imagePoints -> CV_32F)
# ----------------------------------------------------------------------------------------------
def soa_pnp(points3d, points2d):
    P = np.asarray(points3d, np.float64).reshape(-1, 3).astype(np.float32)
    p = np.asarray(points2d, np.float64).reshape(-1, 2).astype(np.float32)
    return tuple(np.ascontiguousarray(P[:, k]) for k in range(3)) + tuple(np.ascontiguousarray(p[:, k]) for k in range(2))


def soa_hom(src, dst):
    s = np.asarray(src, np.float64).reshape(-1, 2).astype(np.float32)
    d = np.asarray(dst, np.float64).reshape(-1, 2).astype(np.float32)
    return (np.ascontiguousarray(s[:, 0]), np.ascontiguousarray(s[:, 1]),
            np.ascontiguousarray(d[:, 0]), np.ascontiguousarray(d[:, 1]))


def cam_from_K(K):
    K = np.asarray(K, np.float64).reshape(3, 3)
    return np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], np.float64)


# ----------------------------------------------------------------------------------------------
# samplers / scan
# ----------------------------------------------------------------------------------------------
def philox(ctr, key):
    out = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(np.asarray(ctr, np.uint32), np.asarray(key, np.uint32), out)
    return out


def philox_subset(seed, problem, hyp, n, s=4):
    idx = np.zeros(s, np.int32)
    r = lib().orc_philox_subset(seed, problem, hyp, n, s, idx)
    return None if r < 0 else idx


def mwc_sequence(k, state=(1 << 64) - 1):
    st = C.c_uint64(state)
    return np.array([lib().orc_mwc_next(C.byref(st)) for _ in range(k)], np.uint64)


def mwc_subsets(n, H, s=4, hom=None, state=(1 << 64) - 1):
    """Subsets of OpenCV getSubset() for H consecutive RANSAC iterations."""
    st = C.c_uint64(state)
    out = np.zeros((H, s), np.int32)
    status = np.zeros(H, np.int8)
    if hom is not None:
        sx, sy, dx, dy = hom
        lib().orc_mwc_subsets(C.byref(st), n, s, H, _ptr(sx), _ptr(sy), _ptr(dx), _ptr(dy), out, status)
    else:
        lib().orc_mwc_subsets(C.byref(st), n, s, H, None, None, None, None, out, status)
    return out, status


def update_num_iters(p, ep, s, max_iters):
    return lib().orc_update_num_iters(p, ep, s, max_iters)


def scan(counts, status, n, s, confidence, max_iters):
    counts = np.ascontiguousarray(counts, np.int32)
    status = np.ascontiguousarray(status, np.int8)
    good = C.c_int32(0)
    iters = C.c_int64(0)
    best = lib().orc_scan(counts, status, len(counts), n, s, confidence, max_iters, C.byref(good), C.byref(iters))
    return int(best), int(good.value), int(iters.value)


def thr2(thr):
    return lib().orc_thr2(float(thr))


# ----------------------------------------------------------------------------------------------
# PnP
# ----------------------------------------------------------------------------------------------
def pnp_minimal(soa, idx, cam):
    R = np.zeros(9)
    t = np.zeros(3)
    ok = lib().orc_pnp_minimal(*soa, np.ascontiguousarray(idx, np.int32), cam, R, t)
    return (R.reshape(3, 3), t) if ok else None


def p3p(bearings, world):
    Rs = np.zeros(36)
    ts = np.zeros(12)
    k = lib().orc_p3p(np.ascontiguousarray(bearings, np.float64).reshape(9),
                      np.ascontiguousarray(world, np.float64).reshape(9), Rs, ts)
    return [(Rs[9 * i:9 * i + 9].reshape(3, 3).copy(), ts[3 * i:3 * i + 3].copy()) for i in range(k)]


def pnp_count(R, t, soa, cam, thr, mask=False):
    n = len(soa[0])
    m = np.zeros(n, np.uint8) if mask else None
    c = lib().orc_pnp_count(np.ascontiguousarray(R, np.float64).reshape(9), np.ascontiguousarray(t, np.float64),
                            cam, *soa, n, thr2(thr), _ptr(m))
    return (c, m.astype(bool)) if mask else c


def pnp_hypotheses(soa, cam, thr, seed, H, hyp0=0, problem=0, subsets=None, sub_status=None, models=False,
                   minimal="p3p", rvec=None):
    """minimal: "p3p" (4-point samples, SOLVEPNP_P3P) or "epnp5" (5-point samples, EPnP: the
    default SOLVEPNP_ITERATIVE kernel of solvePnPRansac); subsets H x 4 or H x 5.  rvec: every
    model's R -> Rodrigues(Rodrigues(R)) before it is counted (RSAC_F_RVEC_ROUNDTRIP); default on
    exactly when subsets are given (as rsac.hypotheses)."""
    if rvec is None:
        rvec = subsets is not None
    n = len(soa[0])
    k = 5 if minimal == "epnp5" else 4
    counts = np.zeros(H, np.int32)
    status = np.zeros(H, np.int8)
    mdl = np.zeros((H, 16)) if models else None
    subs = None if subsets is None else np.ascontiguousarray(subsets, np.int32)
    sst = None if sub_status is None else np.ascontiguousarray(sub_status, np.int8)
    lib().orc_pnp_hypotheses_k(*soa, n, cam, thr2(thr), seed, problem, hyp0, H, k, _ptr(subs), _ptr(sst), counts,
                               status, _ptr(mdl), int(bool(rvec)))
    return (counts, status, mdl) if models else (counts, status)


def pnp_ransac(points3d, points2d, K, thr=30.0, confidence=0.99, max_iters=5000, seed=0x5EED, sampler="philox",
               minimal="p3p", rvec=None):
    """orc_pnp_ransac_k: OpenCV's loop; 4 points (5 under minimal="epnp5") take solvePnPRansac's
    count == model_points branch instead (one minimal solve on all points, every index an inlier,
    best 0, iters 0).  rvec (default: sampler == "opencv", as rsac.pnp_ransac): the minimal
    models' Rodrigues round trip."""
    rvec = sampler == "opencv" if rvec is None else rvec
    soa = soa_pnp(points3d, points2d)
    n = len(soa[0])
    cam = cam_from_K(K)
    R = np.zeros(9)
    t = np.zeros(3)
    mask = np.zeros(n, np.uint8)
    good = C.c_int32(0)
    iters = C.c_int64(0)
    best = lib().orc_pnp_ransac_k(*soa, n, cam, thr, confidence, max_iters, seed, 1 if sampler == "opencv" else 0,
                                  5 if minimal == "epnp5" else 4, R, t, mask, C.byref(good), C.byref(iters),
                                  int(bool(rvec)))
    return dict(best=int(best), R=R.reshape(3, 3), t=t, mask=mask.astype(bool), n_inliers=int(good.value),
                iters=int(iters.value))


def rvec_roundtrip(R):
    """Rodrigues(Rodrigues(R)) in the deterministic restatement (orc_rvec_roundtrip)."""
    R = np.ascontiguousarray(R, np.float64).reshape(9).copy()
    lib().orc_rvec_roundtrip(R)
    return R.reshape(3, 3)


def rd_acos(x):
    return lib().orc_rd_acos(float(x))


def rd_sincos(th):
    s, c = C.c_double(0), C.c_double(0)
    lib().orc_rd_sincos(float(th), C.byref(s), C.byref(c))
    return s.value, c.value


def pnp_minimal_epnp5(soa, cam, idx):
    """EPnP on the 5 sampled points (orc_pnp_minimal_epnp5) -> (R, t) or None."""
    R, t = np.zeros(9), np.zeros(3)
    ok = lib().orc_pnp_minimal_epnp5(*soa, np.ascontiguousarray(idx, np.int32), cam, R, t)
    return (R.reshape(3, 3), t) if ok else None


def pnp_ransac_seq(points3d, points2d, K, thr=30.0, confidence=0.99, max_iters=5000, seed=0x5EED,
                   sampler="philox", minimal="p3p", rvec=None):
    """OpenCV's loop one hypothesis at a time, stopping at the iteration bound (orc_pnp_ransac_seq_k;
    sampler "opencv" draws each iteration's MWC subset as OpenCV does, minimal "epnp5" = the default
    SOLVEPNP_ITERATIVE kernel); rvec as pnp_ransac."""
    rvec = sampler == "opencv" if rvec is None else rvec
    soa = soa_pnp(points3d, points2d)
    n = len(soa[0])
    R, t = np.zeros(9), np.zeros(3)
    mask = np.zeros(n, np.uint8)
    good = C.c_int32(0)
    iters = C.c_int64(0)
    best = lib().orc_pnp_ransac_seq_k(*soa, n, cam_from_K(K), thr, confidence, max_iters, seed,
                                      1 if sampler == "opencv" else 0, 5 if minimal == "epnp5" else 4, R, t, mask,
                                      C.byref(good), C.byref(iters), int(bool(rvec)))
    return dict(best=int(best), R=R.reshape(3, 3), t=t, mask=mask.astype(bool), n_inliers=int(good.value),
                iters=int(iters.value))


def pnp_hypotheses_mt(soa, cam, thr, seed, H, hyp0=0, threads=1):
    """pnp_hypotheses on `threads` OpenMP threads (orc_pnp_hypotheses_mt)."""
    counts = np.zeros(H, np.int32)
    status = np.zeros(H, np.int8)
    lib().orc_pnp_hypotheses_mt(*soa, len(soa[0]), cam, thr2(thr), seed, hyp0, H, counts, status, int(threads))
    return counts, status


def pnp_ransac_lo(points3d, points2d, K, thr=30.0, confidence=0.99, max_iters=5000, seed=0x5EED, lazy=False,
                  threads=0):
    """LO-RANSAC restatement (orc_pnp_ransac_lo): local optimisation at every new best.  lazy=True
    evaluates each hypothesis when the scan reaches it and stops at the bound (orc_pnp_ransac_lo_seq:
    OpenCV's loop shape, the C5 CPU leg); threads > 0 evaluates rounds of hypotheses over that many
    OpenMP threads and scans them in order (orc_pnp_ransac_lo_mt); the results are the same."""
    soa = soa_pnp(points3d, points2d)
    n = len(soa[0])
    cam = cam_from_K(K)
    R = np.zeros(9)
    t = np.zeros(3)
    mask = np.zeros(n, np.uint8)
    good = C.c_int32(0)
    iters = C.c_int64(0)
    nlo = C.c_int32(0)
    if threads > 0:
        best = lib().orc_pnp_ransac_lo_mt(*soa, n, cam, thr, confidence, max_iters, seed, R, t, mask, C.byref(good),
                                          C.byref(iters), C.byref(nlo), int(threads))
    else:
        fn = lib().orc_pnp_ransac_lo_seq if lazy else lib().orc_pnp_ransac_lo
        best = fn(*soa, n, cam, thr, confidence, max_iters, seed, R, t, mask, C.byref(good), C.byref(iters),
                  C.byref(nlo))
    return dict(best=int(best), R=R.reshape(3, 3), t=t, mask=mask.astype(bool), n_inliers=int(good.value),
                iters=int(iters.value), lo_improvements=int(nlo.value))


def reproj_errors(points3d, points2d, K, R, t, projections=False):
    """compute_reprojection_error (testpro-K.py:32-36): f64 projectPoints + per-point L2 norm."""
    p3 = np.ascontiguousarray(np.asarray(points3d, np.float64).reshape(-1, 3))
    p2 = np.ascontiguousarray(np.asarray(points2d, np.float64).reshape(-1, 2))
    n = p3.shape[0]
    err = np.zeros(n)
    proj = np.zeros((n, 2)) if projections else None
    lib().orc_reproj_errors(np.ascontiguousarray(R, np.float64).reshape(9), np.ascontiguousarray(t, np.float64),
                            cam_from_K(K), p3, p2, n, _ptr(proj), _ptr(err))
    return (err, proj) if projections else err


def reproj_mean(points3d, points2d, K, R, t, mask):
    """Mean inlier error in the GPU's summation order -> (mean, count)."""
    p3 = np.ascontiguousarray(np.asarray(points3d, np.float64).reshape(-1, 3))
    p2 = np.ascontiguousarray(np.asarray(points2d, np.float64).reshape(-1, 2))
    c = C.c_int(0)
    s = lib().orc_reproj_mean_sum(np.ascontiguousarray(R, np.float64).reshape(9), np.ascontiguousarray(t, np.float64),
                                  cam_from_K(K), p3, p2, np.ascontiguousarray(mask, np.uint8), p3.shape[0],
                                  C.byref(c))
    return s / c.value if c.value else float("nan"), int(c.value)


def estimate_camera_orientation(pos3d, pixels, Ks, thr=30.0, confidence=0.99, max_iters=5000, seed=0x5EED,
                                sampler="opencv", min_inliers=6, minimal="epnp5", rvec=None, threads=None):
    """testpro-K.py:39-125 restated on the oracle's pieces: per K the RANSAC (pnp_ransac) + the LM
    final solve on its inliers (solvePnPRansac's SOLVEPNP_ITERATIVE final solvePnP), the gate,
    the mean inlier error through the pose's Rodrigues vector, the first strict minimum, then
    the LM refit (solvePnPRefineLM) of the winner on its inlier subset.  The defaults are the
    reference's own mode (testpro-K.py:72-75 passes no flags: SOLVEPNP_ITERATIVE = EPnP on 5-point
    MWC samples, model_points 5); minimal="p3p" / sampler="philox" is the benchmark kernel.  rvec
    (default: sampler == "opencv"): the minimal models' Rodrigues round trip."""
    rvec = sampler == "opencv" if rvec is None else bool(rvec)
    P3 = np.asarray(pos3d, np.float64).reshape(-1, 3)
    P2 = np.asarray(pixels, np.float64).reshape(-1, 2)
    soa = soa_pnp(P3, P2)
    rows = []
    best, best_err = -1, float("inf")
    # the per-K RANSACs are independent (ctypes drops the GIL): run them on a thread pool, then
    # select in the reference's loop order
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=threads or min(len(Ks), os.cpu_count() or 1, 16)) as ex:
        runs = list(ex.map(lambda K: pnp_ransac(P3, P2, K, thr, confidence, max_iters, seed, sampler=sampler,
                                                minimal=minimal, rvec=rvec), Ks))
    # solvePnPRansac's count == model_points branch (4 points; 5 under EPnP-5) has no final solve
    direct = P3.shape[0] == 4 or (P3.shape[0] == 5 and minimal == "epnp5")
    for k, K in enumerate(Ks):
        r = runs[k]
        if r["best"] < 0:
            rows.append(None)
            continue
        if direct:
            R, t = r["R"], r["t"]
        else:
            R, t, _ = pnp_refine(soa, r["mask"].astype(np.uint8), cam_from_K(K), r["R"], r["t"])
        row = dict(R=R, t=t, mask=r["mask"], n_inliers=r["n_inliers"])
        rows.append(row)
        if r["n_inliers"] < min_inliers:
            row["mean"] = float("nan")
            continue
        Rp = rodrigues_v2m(rodrigues_m2v(R))
        row["mean"], _ = reproj_mean(P3, P2, K, Rp, t, r["mask"])
        if row["mean"] < best_err:
            best_err, best = row["mean"], k
    if best < 0:
        return dict(best=-1, rows=rows, R=None, t=None)
    w = rows[best]
    sub3, sub2 = P3[w["mask"]], P2[w["mask"]]
    Rp = rodrigues_v2m(rodrigues_m2v(w["R"]))
    Rr, tr, _ = pnp_refine(soa_pnp(sub3, sub2), np.ones(len(sub3), np.uint8), cam_from_K(Ks[best]), Rp, w["t"])
    return dict(best=best, rows=rows, R=Rr, t=tr)


def pnp_local_opt(soa, cam, thr, R, t, count):
    """One LO-RANSAC local optimisation -> (R, t, count, steps)."""
    R = np.ascontiguousarray(R, np.float64).reshape(9).copy()
    t = np.ascontiguousarray(t, np.float64).copy()
    steps = C.c_int32(0)
    c = lib().orc_pnp_local_opt(*soa, len(soa[0]), cam, thr2(thr), R, t, int(count), C.byref(steps))
    return R.reshape(3, 3), t, int(c), int(steps.value)


def pnp_refine(soa, mask, cam, R, t, max_iter=20):
    R = np.ascontiguousarray(R, np.float64).reshape(9).copy()
    t = np.ascontiguousarray(t, np.float64).copy()
    it = lib().orc_pnp_refine(*soa, np.ascontiguousarray(mask, np.uint8), len(soa[0]), cam, R, t, max_iter)
    return R.reshape(3, 3), t, it


def pnp_epnp(soa, mask, cam):
    """EPnP on the masked points -> (R, t) or (None, None)."""
    R, t = np.zeros(9), np.zeros(3)
    ok = lib().orc_pnp_epnp(*soa, np.ascontiguousarray(mask, np.uint8), len(soa[0]), cam, R, t)
    return (R.reshape(3, 3), t) if ok else (None, None)


# ----------------------------------------------------------------------------------------------
# homography
# ----------------------------------------------------------------------------------------------
def hom_check_subset(soa, idx):
    return bool(lib().orc_hom_check_subset(*soa, np.ascontiguousarray(idx, np.int32)))


def hom_minimal(soa, idx):
    H = np.zeros(9)
    ok = lib().orc_hom_minimal(*soa, np.ascontiguousarray(idx, np.int32), H)
    return H.reshape(3, 3) if ok else None


def hom_count(H, soa, thr, mask=False):
    n = len(soa[0])
    m = np.zeros(n, np.uint8) if mask else None
    c = lib().orc_hom_count(np.ascontiguousarray(H, np.float64).reshape(9), *soa, n, thr2(thr), _ptr(m))
    return (c, m.astype(bool)) if mask else c


def hom_hypotheses(soa, thr, seed, H, hyp0=0, problem=0, subsets=None, sub_status=None, models=False):
    n = len(soa[0])
    counts = np.zeros(H, np.int32)
    status = np.zeros(H, np.int8)
    mdl = np.zeros((H, 16)) if models else None
    subs = None if subsets is None else np.ascontiguousarray(subsets, np.int32)
    sst = None if sub_status is None else np.ascontiguousarray(sub_status, np.int8)
    lib().orc_hom_hypotheses(*soa, n, thr2(thr), seed, problem, hyp0, H, _ptr(subs), _ptr(sst), counts, status,
                             _ptr(mdl))
    return (counts, status, mdl) if models else (counts, status)


def hom_ransac(src, dst, thr, confidence=0.995, max_iters=2000, seed=0x5EED, sampler="opencv", refine=True):
    """cv2.findHomography(src, dst, cv2.RANSAC, thr) restated (main_v1.py:312)."""
    soa = soa_hom(src, dst)
    n = len(soa[0])
    Hm = np.zeros(9)
    mask = np.zeros(n, np.uint8)
    good = C.c_int32(0)
    iters = C.c_int64(0)
    best = lib().orc_hom_ransac(*soa, n, thr, confidence, max_iters, seed, 1 if sampler == "opencv" else 0, Hm,
                                mask, C.byref(good), C.byref(iters))
    Href = None
    if best >= 0 and refine and n > 4:
        Href = Hm.copy()
        lib().orc_hom_refine(*soa, mask, n, Href)
        Href = Href.reshape(3, 3)
    return dict(best=int(best), H=Hm.reshape(3, 3), H_refined=Href, mask=mask.astype(bool),
                n_inliers=int(good.value), iters=int(iters.value))


def hom_refine(soa, mask, H):
    Hc = np.ascontiguousarray(H, np.float64).reshape(9).copy()
    lib().orc_hom_refine(*soa, np.ascontiguousarray(mask, np.uint8), len(soa[0]), Hc)
    return Hc.reshape(3, 3)


def rodrigues_v2m(r):
    R = np.zeros(9)
    lib().orc_rodrigues_v2m(np.ascontiguousarray(r, np.float64).reshape(3), R)
    return R.reshape(3, 3)


def rodrigues_m2v(R):
    r = np.zeros(3)
    lib().orc_rodrigues_m2v(np.ascontiguousarray(R, np.float64).reshape(9), r)
    return r


# ----------------------------------------------------------------------------------------------
# camera-location search (main_v1.py:254-348, 419, 862-866), numpy restatement, literal loops
# ----------------------------------------------------------------------------------------------
def location_pos2(pos3ds, camera_location):
    """main_v1.py:301-308: pos2 and the `good` (noted-pixel) flags are computed per feature."""
    pos2 = np.zeros((len(pos3ds), 2))
    for i in range(len(pos3ds)):
        p = pos3ds[i, :] - camera_location
        p = np.array([p[2], p[1], p[0]])
        p = p / p[2]
        pos2[i, :] = p[0:2]
    return pos2


def location_errors(pos2_good, pixels_good, M, mask, ransacbound):
    """main_v1.py:332-348 + 419: err1, err2 of one location given M = inv(H) and the RANSAC mask."""
    err1 = 0.0
    err2 = 0.0
    mask = np.asarray(mask).reshape(-1).astype(np.uint8)
    for i in range(pos2_good.shape[0]):
        p1 = pixels_good[i, :]
        pp = np.array([pos2_good[i, 0], pos2_good[i, 1], 1.0])
        pp2 = np.matmul(np.linalg.inv(M), pp)
        pp2 = pp2 / pp2[2]
        P1 = np.array([p1[0], p1[1], 1.0])
        PP2 = np.matmul(M, P1)
        PP2 = PP2 / PP2[2]
        P2 = pos2_good[i, :]
        if mask[i] == 1:
            err1 += np.linalg.norm(p1 - pp2[0:2])
            err2 += np.linalg.norm(P2 - PP2[0:2])
    err2 += np.sum(1 - mask) * ransacbound
    return err1, err2


def find_homography(pixels, pos3ds, camera_location, ransacbound):
    """main_v1.py:300-348, 419 with cv2.findHomography restated (hom_ransac, OpenCV sampler + refit).

    -> dict(M, err1, err2, mask, H); no model -> err (0, 0), which the driver maps to 1e6 (the
    reference itself would raise at np.linalg.inv(None))."""
    pixels = np.asarray(pixels, np.float64)
    good = (pixels[:, 0] != 0) | (pixels[:, 1] != 0)
    pos2 = location_pos2(np.asarray(pos3ds, np.float64), np.asarray(camera_location, np.float64))
    res = hom_ransac(pos2[good], pixels[good], ransacbound, 0.995, 2000, sampler="opencv", refine=True)
    if res["best"] < 0:
        return dict(M=None, H=None, err1=0.0, err2=0.0, mask=res["mask"])
    H = res["H_refined"] if res["H_refined"] is not None else res["H"]
    M = np.linalg.inv(H)
    e1, e2 = location_errors(pos2[good], pixels[good], M, res["mask"], ransacbound)
    return dict(M=M, H=H, err1=e1, err2=e2, mask=res["mask"])


def best_location(num_matches):
    """main_v1.py:863-866"""
    e2 = np.array(num_matches, np.float64)[:, 1].copy()
    e2[e2 == 0] = 1000000
    return int(np.argmin(e2))


# ----------------------------------------------------------------------------------------------
# fundamental matrix (BASELINE.json configs[3]; semantics defined by the restatement)
# ----------------------------------------------------------------------------------------------
def fm_minimal(soa, idx):
    F = np.zeros(9)
    sub = [np.ascontiguousarray(a[np.asarray(idx)], np.float32) for a in soa]
    ok = lib().orc_fm_minimal8(*sub, F)
    return bool(ok), F.reshape(3, 3)


def fm_count(F, soa, thr, mask=False):
    m = np.zeros(len(soa[0]), np.uint8) if mask else None
    c = lib().orc_fm_count(np.ascontiguousarray(F, np.float64).reshape(9), *soa, len(soa[0]), thr2(thr), _ptr(m))
    return (int(c), m.astype(bool)) if mask else int(c)


def fm_hypotheses(soa, thr, seed, H, hyp0=0, models=False):
    n = len(soa[0])
    counts = np.zeros(H, np.int32)
    status = np.zeros(H, np.int8)
    mdl = np.zeros((H, 16)) if models else None
    lib().orc_fm_hypotheses(*soa, n, thr2(thr), seed, hyp0, H, counts, status, _ptr(mdl))
    return (counts, status, mdl) if models else (counts, status)


def fm_hypotheses_mt(soa, thr, seed, H, hyp0=0, threads=1):
    """fm_hypotheses over `threads` OpenMP threads (orc_fm_hypotheses_mt)."""
    counts = np.zeros(H, np.int32)
    status = np.zeros(H, np.int8)
    lib().orc_fm_hypotheses_mt(*soa, len(soa[0]), thr2(thr), seed, hyp0, H, counts, status, int(threads))
    return counts, status


def fm_ransac(pts1, pts2, thr=1.5, confidence=0.99, max_iters=100000, seed=0x5EED):
    soa = soa_hom(pts1, pts2)
    n = len(soa[0])
    F = np.zeros(9)
    mask = np.zeros(n, np.uint8)
    good = C.c_int32(0)
    iters = C.c_int64(0)
    best = lib().orc_fm_ransac(*soa, n, thr, confidence, max_iters, seed, F, mask, C.byref(good), C.byref(iters))
    return dict(best=int(best), F=F.reshape(3, 3), mask=mask.astype(bool), n_inliers=int(good.value),
                iters=int(iters.value))

