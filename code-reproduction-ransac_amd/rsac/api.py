"""Python entry points over the C ABI (librsac.so).

``pnp_ransac(points2D, points3D, K, n_iters, reproj_thresh) -> (R, t, inlier_mask)``
is the north-star entry point: it replaces the RANSAC loop that
``cv2.solvePnPRansac`` runs for the reference (main_v1.py:497-502,
testpro-K.py:72-75, testpro.py:536-541, test_pro.py:515-520).
``homography_ransac`` replaces ``cv2.findHomography(..., cv2.RANSAC, thr)``
(main_v1.py:312, process.py:200).  The batched forms replace the Python loops
around those calls (main_v1.py:274-284, testpro-K.py:58-75).

Inputs may be numpy arrays (host, float64 as the reference holds them) or
torch tensors on the GPU (float64 AoS, used in place).  Results for GPU
inputs keep the mask on the GPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


class _In:
    """Marshalled input: pointer + whether it is on the device + keepalive."""

    def __init__(self, a, cols: int):
        self.device = False
        self.torch = False
        if _is_torch(a):
            import torch
            self.torch = True
            if a.dtype == torch.float64 and a.dim() == 2 and a.shape[1] == cols and a.is_contiguous():
                t = a  # already the (n, cols) float64 layout: no view or copy (the common GPU call)
            else:
                t = a.reshape(-1, cols).to(torch.float64).contiguous()
            self.device = t.is_cuda
            if not self.device:
                t = t.numpy()
            self.keep = t
            self.n = t.shape[0]
            self.ptr = t.data_ptr() if self.device else t.ctypes.data
            self.dev_index = a.device.index if self.device else None
        else:
            arr = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, cols))
            self.keep = arr
            self.n = arr.shape[0]
            self.ptr = arr.ctypes.data
            self.dev_index = None


def _stream_of(inp: _In):
    if inp.device:
        import torch
        # torch's raw getter returns the handle without building a Stream object (0.06 against
        # 1.7 us per call, scripts/py_overhead.py); the public form where a build lacks it
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            return C.c_void_p(raw(inp.dev_index))
        return C.c_void_p(torch.cuda.current_stream(inp.keep.device).cuda_stream)
    return C.c_void_p(0)


def _device_of(inp: _In, device):
    if device is not None:
        return int(device)
    if inp.dev_index is not None:
        return int(inp.dev_index)
    return 0


def _flags(adaptive, refine, sampler, exact_only=False, minimal="p3p", rvec=None):
    f = 0
    # rvec (PnP): each minimal model's rotation through Rodrigues(Rodrigues(R)) before it is scored,
    # as OpenCV's PnPRansacCallback keeps the model as (rvec, tvec) (main_v1.py:497, testpro-K.py:72);
    # default: on with OpenCV's sampler (the reference's own mode), off for Philox
    if (sampler == "opencv") if rvec is None else rvec:
        f |= L.F_RVEC_ROUNDTRIP
    # minimal: "p3p" (4-point samples, SOLVEPNP_P3P: this project's benchmark kernel, north_star's)
    # or "epnp5" (5-point samples solved by EPnP: solvePnPRansac's default SOLVEPNP_ITERATIVE
    # kernel, model_points 5 -- what the reference's calls run, main_v1.py:497, testpro-K.py:72)
    if minimal == "epnp5":
        f |= L.F_MINIMAL_EPNP5
    elif minimal != "p3p":
        raise ValueError(f"minimal must be 'p3p' or 'epnp5', got {minimal!r}")
    if adaptive:
        f |= L.F_ADAPTIVE
    # refine: True / "lm" -> LM from the minimal model; "epnp" -> EPnP on the inliers (solvePnPRansac
    # with SOLVEPNP_P3P); "epnp+lm" -> EPnP, then LM from it
    if refine is True or refine == "lm":
        f |= L.F_REFINE
    elif refine == "epnp":
        f |= L.F_EPNP
    elif refine == "epnp+lm":
        f |= L.F_EPNP | L.F_REFINE
    elif refine not in (False, None):
        raise ValueError(f"refine must be True/False, 'lm', 'epnp' or 'epnp+lm', got {refine!r}")
    if sampler == "opencv":
        f |= L.F_SAMPLER_OPENCV
    elif sampler != "philox":
        raise ValueError(f"sampler must be 'philox' or 'opencv', got {sampler!r}")
    if exact_only:
        f |= L.F_EXACT_ONLY
    return f


def _mask_buffer(inp: _In, n: int):
    if inp.device:
        import torch
        # bool storage is one byte holding 0 / 1: the ABI's uint8 mask, no reinterpreting view after
        m = torch.empty(max(n, 1), dtype=torch.bool, device=inp.keep.device)
        return m, m.data_ptr(), L.F_DEVICE_OUT
    m = np.zeros(max(n, 1), np.uint8)
    return m, m.ctypes.data, 0


def _finish_mask(m, n):
    # uint8 0/1 -> bool without a copy (torch: reinterpret the bytes, unless already bool)
    if _is_torch(m):
        import torch
        m = m if m.shape[0] == n else m[:n]
        return m if m.dtype == torch.bool else m.view(dtype=torch.bool)
    return m[:n].view(np.bool_)


@dataclass
class RansacInfo:
    ok: bool
    n_inliers: int
    best_hyp: int
    iters: int
    hyps_scored: int
    rounds: int
    gpu_ms: float
    solve_ms: float
    score_ms: float
    lo_improvements: int = 0


def _info(code, st: L.Stats) -> RansacInfo:
    return RansacInfo(ok=code == L.OK, n_inliers=st.n_inliers, best_hyp=st.best_hyp, iters=st.iters,
                      hyps_scored=st.hyps_scored, rounds=st.rounds, gpu_ms=st.gpu_ms, solve_ms=st.solve_ms,
                      score_ms=st.score_ms, lo_improvements=st.lo_improvements)


def _K9(K) -> np.ndarray:
    K = np.ascontiguousarray(np.asarray(K, dtype=np.float64).reshape(3, 3))
    return K.reshape(9).copy()


def pnp_ransac(points2D, points3D, K, n_iters: int = 5000, reproj_thresh: float = 30.0, *,
               confidence: float = 0.99, seed: int = 0x5EED, sampler: str = "philox", adaptive: bool = True,
               refine: bool = True, device=None, return_info: bool = False, exact_only: bool = False,
               lo: bool = False, minimal: str = "p3p", rvec=None):
    """RANSAC PnP on the GPU: (points2D, points3D, K, n_iters, reproj_thresh) -> (R, t, inlier_mask).

    Defaults follow the reference call (iterationsCount=5000, reprojectionError=30,
    confidence=0.99; main_v1.py:497-502).  ``R`` is 3x3, ``t`` (3,) with
    x_cam = R X + t; ``inlier_mask`` is the RANSAC-phase mask (OpenCV's
    convention).  On failure R and t are None and the mask is all False.
    lo=True runs LO-RANSAC (local optimisation at every new best; BASELINE.json C5).
    minimal="epnp5" samples 5 points and solves them with EPnP (OpenCV's default
    SOLVEPNP_ITERATIVE kernel; RANSACUpdateNumIters with model_points 5).
    rvec (default: sampler == "opencv"): score each minimal model as Rodrigues(Rodrigues(R)), the
    rotation OpenCV's computeError projects with.  4 points (5 under minimal="epnp5") take
    solvePnPRansac's count == model_points branch: one minimal solve on all points, every index
    an inlier, no final solve.
    """
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    if p3.n != p2.n:
        raise ValueError(f"points3D ({p3.n}) and points2D ({p2.n}) differ in length")
    if p3.device != p2.device:
        raise ValueError("points3D and points2D must both be host arrays or both GPU tensors")
    n = p3.n
    ctx = L.context(_device_of(p3, device))
    flags = _flags(adaptive, refine, sampler, exact_only, minimal, rvec) | (L.F_LO if lo else 0)
    if p3.device:
        flags |= L.F_DEVICE_IN
    K9 = _K9(K)
    R = np.zeros(9)
    t = np.zeros(3)
    mask, mptr, mflag = _mask_buffer(p3, n)
    flags |= mflag
    st = L.Stats()
    with ctx.lock:
        code = L.check(L.lib().rsac_pnp_ransac(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), n,
                                               K9.ctypes.data, int(n_iters), float(reproj_thresh),
                                               float(confidence), int(seed) & (2**64 - 1), flags, R.ctypes.data,
                                               t.ctypes.data, C.c_void_p(mptr),
                                               C.byref(st) if return_info else None, _stream_of(p3)))
    m = _finish_mask(mask, n)
    out = (R.reshape(3, 3), t, m) if code == L.OK else (None, None, m)
    return out + (_info(code, st),) if return_info else out


def pnp_ransac_first_round(points2D, points3D, K, n_iters: int = 5000, reproj_thresh: float = 30.0, *,
                           confidence: float = 0.99, seed: int = 0x5EED, refine: bool = True, lo: bool = False,
                           device=None):
    """The multi-GPU adaptive loop's first round (rsac_pnp_ransac_first_round):
    pnp_ransac (Philox, adaptive) capped at its first 256-hypothesis round, run redundantly on
    every rank with no collective.  Returns (done, R, t, mask, scan, info) where scan is the Scan
    after the round and info the RansacInfo: done=True -> (R, t, mask) is pnp_ransac's result (R
    None: no model); done=False -> the scan goes on from scan.iters and (R, t) is the best model
    so far (mask None)."""
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    if p3.n != p2.n:
        raise ValueError(f"points3D ({p3.n}) and points2D ({p2.n}) differ in length")
    if p3.device != p2.device:
        raise ValueError("points3D and points2D must both be host arrays or both GPU tensors")
    n = p3.n
    ctx = L.context(_device_of(p3, device))
    flags = _flags(True, refine, "philox") | (L.F_LO if lo else 0) | (L.F_DEVICE_IN if p3.device else 0)
    R, t = np.zeros(9), np.zeros(3)
    mask, mptr, mflag = _mask_buffer(p3, n)
    flags |= mflag
    scan = Scan(n_iters, n, confidence, 4)
    st = L.Stats()
    with ctx.lock:
        code = L.check(L.lib().rsac_pnp_ransac_first_round(
            ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), n, _K9(K).ctypes.data, int(n_iters),
            float(reproj_thresh), float(confidence), int(seed) & (2**64 - 1), flags, R.ctypes.data, t.ctypes.data,
            C.c_void_p(mptr), C.byref(scan.st), C.byref(st), _stream_of(p3)))
    info = _info(code, st)
    if code == L.MORE:
        has = scan.best >= 0
        return False, (R.reshape(3, 3) if has else None), (t if has else None), None, scan, info
    m = _finish_mask(mask, n)
    return True, (R.reshape(3, 3) if code == L.OK else None), (t if code == L.OK else None), m, scan, info


def homography_ransac(src, dst, reproj_thresh: float = 3.0, *, max_iters: int = 2000, confidence: float = 0.995,
                      seed: int = 0x5EED, sampler: str = "opencv", adaptive: bool = True, refine: bool = True,
                      device=None, return_info: bool = False):
    """RANSAC homography src -> dst on the GPU: -> (H, mask).

    Mirrors cv2.findHomography(src, dst, cv2.RANSAC, thr) (main_v1.py:312):
    OpenCV's MWC subset sequence by default (sampler="opencv"), f32 error,
    RANSAC-phase mask, then a least-squares + LM polish of H on the inliers.
    """
    s = _In(src, 2)
    d = _In(dst, 2)
    if s.n != d.n:
        raise ValueError("src and dst differ in length")
    n = s.n
    ctx = L.context(_device_of(s, device))
    flags = _flags(adaptive, refine, sampler)
    if s.device:
        flags |= L.F_DEVICE_IN
    H = np.zeros(9)
    mask, mptr, mflag = _mask_buffer(s, n)
    flags |= mflag
    st = L.Stats()
    with ctx.lock:
        code = L.check(L.lib().rsac_homography_ransac(ctx.handle, C.c_void_p(s.ptr), C.c_void_p(d.ptr), n,
                                                      int(max_iters), float(reproj_thresh), float(confidence),
                                                      int(seed) & (2**64 - 1), flags, H.ctypes.data,
                                                      C.c_void_p(mptr), C.byref(st), _stream_of(s)))
    m = _finish_mask(mask, n)
    out = (H.reshape(3, 3), m) if code == L.OK else (None, m)
    return out + (_info(code, st),) if return_info else out


def fundamental_ransac(pts1, pts2, reproj_thresh: float = 1.5, *, max_iters: int = 100_000,
                       confidence: float = 0.99, seed: int = 0x5EED, adaptive: bool = True, device=None,
                       return_info: bool = False, exact_only: bool = False):
    """Fundamental matrix RANSAC (BASELINE.json configs[3]): 8-point samples, Sampson test.

    pts1, pts2 (N,2) with x2^T F x1 = 0.  Returns (F (3,3) unit Frobenius norm or None, mask).
    """
    a = _In(pts1, 2)
    b = _In(pts2, 2)
    if a.n != b.n:
        raise ValueError("pts1 and pts2 differ in length")
    ctx = L.context(_device_of(a, device))
    flags = _flags(adaptive, False, "philox", exact_only) | (L.F_DEVICE_IN if a.device else 0)
    mask, mptr, mflag = _mask_buffer(a, a.n)
    flags |= mflag
    F = np.zeros(9)
    st = L.Stats()
    with ctx.lock:
        code = L.check(L.lib().rsac_fundamental_ransac(ctx.handle, C.c_void_p(a.ptr), C.c_void_p(b.ptr), a.n,
                                                       int(max_iters), float(reproj_thresh), float(confidence),
                                                       int(seed) & (2**64 - 1), flags, F.ctypes.data,
                                                       C.c_void_p(mptr), C.byref(st), _stream_of(a)))
    m = _finish_mask(mask, a.n)
    out = (F.reshape(3, 3) if code == L.OK else None, m)
    return out + (_info(code, st),) if return_info else out


def _concat(parts, cols):
    arrs = [np.asarray(p, dtype=np.float64).reshape(-1, cols) for p in parts]
    off = np.zeros(len(arrs) + 1, np.int64)
    off[1:] = np.cumsum([a.shape[0] for a in arrs])
    return np.ascontiguousarray(np.concatenate(arrs, axis=0) if arrs else np.zeros((0, cols))), off


def pnp_ransac_batched(points2D_list, points3D_list, K_list, n_iters: int = 5000, reproj_thresh: float = 30.0, *,
                       confidence: float = 0.99, seed: int = 0x5EED, sampler: str = "philox", adaptive: bool = True,
                       refine: bool = True, device: int = 0, minimal: str = "p3p", rvec=None):
    """P independent PnP problems in one call (K sweep of testpro-K.py:58-75, C3 of BASELINE.json).

    Returns a list of (R, t, mask, n_inliers) per problem (R, t None on failure).
    """
    p3, off = _concat(points3D_list, 3)
    p2, off2 = _concat(points2D_list, 2)
    if not np.array_equal(off, off2):
        raise ValueError("per-problem 3D/2D point counts differ")
    P = len(off) - 1
    Ks = np.ascontiguousarray(np.stack([np.asarray(k, np.float64).reshape(9) for k in K_list]))
    if Ks.shape[0] != P:
        raise ValueError("one K per problem required")
    if P and np.diff(off).min() < 4:
        raise ValueError("every problem needs >= 4 correspondences")
    ctx = L.context(device)
    flags = _flags(adaptive, refine, sampler, minimal=minimal, rvec=rvec)
    R = np.zeros((P, 9))
    t = np.zeros((P, 3))
    status = np.zeros(P, np.int32)
    ninl = np.zeros(P, np.int32)
    mask = np.zeros(max(int(off[-1]), 1), np.uint8)
    with ctx.lock:
        L.check(L.lib().rsac_pnp_ransac_batched(ctx.handle, p3.ctypes.data, p2.ctypes.data, off.ctypes.data, P,
                                                Ks.ctypes.data, int(n_iters), float(reproj_thresh), float(confidence),
                                                int(seed) & (2**64 - 1), flags, R.ctypes.data, t.ctypes.data,
                                                status.ctypes.data, ninl.ctypes.data, mask.ctypes.data, None))
    out = []
    for p in range(P):
        m = mask[off[p]:off[p + 1]].astype(bool)
        ok = status[p] == L.OK
        out.append((R[p].reshape(3, 3) if ok else None, t[p] if ok else None, m, int(ninl[p])))
    return out


def pnp_ransac_batched_flat(points2D, points3D, offsets, Ks, n_iters: int = 5000, reproj_thresh: float = 30.0, *,
                            confidence: float = 0.99, seed: int = 0x5EED, sampler: str = "philox",
                            adaptive: bool = True, refine: bool = True, device=None, minimal: str = "p3p"):
    """Batched PnP over problems already concatenated: points2D (N,2), points3D (N,3) f64 (numpy,
    or torch cuda tensors that stay on the device), offsets (P+1) int64, Ks (P,3,3).

    Returns (R (P,3,3), t (P,3), ok (P,) bool, n_inliers (P,), mask (N,) bool -- on the device
    for device inputs).  Same results as pnp_ransac_batched on the split lists.
    """
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    off = np.ascontiguousarray(np.asarray(offsets, np.int64).reshape(-1))
    P = off.size - 1
    if P < 1 or off[0] != 0 or off[-1] != p3.n or p2.n != p3.n:
        raise ValueError("offsets must run from 0 to the number of points")
    if np.diff(off).min() < 4:
        raise ValueError("every problem needs >= 4 correspondences")
    Kf = np.ascontiguousarray(np.asarray(Ks, np.float64).reshape(P, 9))
    ctx = L.context(_device_of(p3, device))
    flags = _flags(adaptive, refine, sampler, minimal=minimal) | (L.F_DEVICE_IN if p3.device else 0)
    mask, mptr, mflag = _mask_buffer(p3, p3.n)
    flags |= mflag
    R = np.zeros((P, 9))
    t = np.zeros((P, 3))
    status = np.zeros(P, np.int32)
    ninl = np.zeros(P, np.int32)
    with ctx.lock:
        L.check(L.lib().rsac_pnp_ransac_batched(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), off.ctypes.data, P,
                                                Kf.ctypes.data, int(n_iters), float(reproj_thresh), float(confidence),
                                                int(seed) & (2**64 - 1), flags, R.ctypes.data, t.ctypes.data,
                                                status.ctypes.data, ninl.ctypes.data, C.c_void_p(mptr),
                                                _stream_of(p3)))
    return R.reshape(P, 3, 3), t, status == L.OK, ninl, _finish_mask(mask, p3.n)


def pnp_ransac_batched_rows(points2D, points3D, offsets, Ks, n_iters: int = 5000, reproj_thresh: float = 30.0, *,
                            confidence: float = 0.99, seed: int = 0x5EED, sampler: str = "philox",
                            adaptive: bool = True, refine: bool = True, device=None, minimal: str = "p3p"):
    """pnp_ransac_batched_flat with the results as one (P, 14) float64 tensor of rows (ok, n_inliers,
    R 9, t 3) on the device, written there by the library (rsac_pnp_ransac_batched_rows): the
    multi-GPU problem shards all-gather them with no host arrays in between.  Inputs as
    pnp_ransac_batched_flat (device tensors stay on the device) -> (rows, mask)."""
    import torch
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    off = np.ascontiguousarray(np.asarray(offsets, np.int64).reshape(-1))
    P = off.size - 1
    if P < 1 or off[0] != 0 or off[-1] != p3.n or p2.n != p3.n:
        raise ValueError("offsets must run from 0 to the number of points")
    if np.diff(off).min() < 4:
        raise ValueError("every problem needs >= 4 correspondences")
    Kf = np.ascontiguousarray(np.asarray(Ks, np.float64).reshape(P, 9))
    dev = _device_of(p3, device)
    ctx = L.context(dev)
    flags = _flags(adaptive, refine, sampler, minimal=minimal) | (L.F_DEVICE_IN if p3.device else 0)
    mask, mptr, mflag = _mask_buffer(p3, p3.n)
    flags |= mflag
    rows = torch.empty((P, 14), dtype=torch.float64, device=torch.device("cuda", dev))
    stream = _stream_of(p3) if p3.device else C.c_void_p(torch.cuda.current_stream(rows.device).cuda_stream)
    with ctx.lock:
        L.check(L.lib().rsac_pnp_ransac_batched_rows(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr),
                                                     off.ctypes.data, P, Kf.ctypes.data, int(n_iters),
                                                     float(reproj_thresh), float(confidence), int(seed) & (2**64 - 1),
                                                     flags, C.c_void_p(rows.data_ptr()), C.c_void_p(mptr), stream))
    return rows, _finish_mask(mask, p3.n)


def homography_ransac_batched(src_list, dst_list, reproj_thresh: float = 3.0, *, max_iters: int = 2000,
                              confidence: float = 0.995, seed: int = 0x5EED, sampler: str = "opencv",
                              adaptive: bool = True, refine: bool = True, device: int = 0):
    """P independent findHomography calls in one launch sequence (main_v1.py:274-284)."""
    s, off = _concat(src_list, 2)
    d, off2 = _concat(dst_list, 2)
    if not np.array_equal(off, off2):
        raise ValueError("per-problem src/dst counts differ")
    P = len(off) - 1
    if P and np.diff(off).min() < 4:
        raise ValueError("every problem needs >= 4 correspondences")
    ctx = L.context(device)
    flags = _flags(adaptive, refine, sampler)
    H = np.zeros((P, 9))
    status = np.zeros(P, np.int32)
    ninl = np.zeros(P, np.int32)
    mask = np.zeros(max(int(off[-1]), 1), np.uint8)
    with ctx.lock:
        L.check(L.lib().rsac_homography_ransac_batched(ctx.handle, s.ctypes.data, d.ctypes.data, off.ctypes.data, P,
                                                       int(max_iters), float(reproj_thresh), float(confidence),
                                                       int(seed) & (2**64 - 1), flags, H.ctypes.data,
                                                       status.ctypes.data, ninl.ctypes.data, mask.ctypes.data, None))
    out = []
    for p in range(P):
        ok = status[p] == L.OK
        out.append((H[p].reshape(3, 3) if ok else None, mask[off[p]:off[p + 1]].astype(bool), int(ninl[p])))
    return out


def score_poses(points2D, points3D, K, poses, reproj_thresh: float = 30.0, device=None, exact_only: bool = False):
    """Inlier counts of given poses ((H, 3, 4) [R | t] or (H, 12)) -- the minimal scoring slice."""
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    poses = np.asarray(poses, np.float64)
    if poses.ndim == 3:
        poses = np.concatenate([poses[:, :, :3].reshape(-1, 9), poses[:, :, 3]], axis=1)
    poses = np.ascontiguousarray(poses.reshape(-1, 12))
    ctx = L.context(_device_of(p3, device))
    flags = (L.F_DEVICE_IN if p3.device else 0) | (L.F_EXACT_ONLY if exact_only else 0)
    counts = np.zeros(poses.shape[0], np.int32)
    K9 = _K9(K)
    with ctx.lock:
        L.check(L.lib().rsac_score_poses(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n, K9.ctypes.data,
                                         poses.ctypes.data, poses.shape[0], float(reproj_thresh), flags,
                                         counts.ctypes.data, _stream_of(p3)))
    return counts


def evaluate_range(points2D, points3D, K, hyp_begin: int, n_hyps: int, reproj_thresh: float = 30.0, *,
                   seed: int = 0x5EED, device=None, return_info: bool = False, exact_only: bool = False,
                   with_mask: bool = False, device_result: bool = False, context=None):
    """Evaluate Philox hypotheses [hyp_begin, hyp_begin + n_hyps) of one problem.

    Returns (key, model12[, mask][, info]) where key = (count << 32) | (0xFFFFFFFF - best_index)
    (or -1) and mask is the best hypothesis' RANSAC-phase mask (with_mask=True; on the GPU for
    GPU inputs).  The sharded driver (rsac.parallel) all-reduces the key with MAX.

    device_result=True (GPU tensor inputs): nothing waits for the GPU; key is a 1-element int64
    tensor (raw packed key, 0 = no model) and model12 a float64 tensor, both on the device.
    context: an rsac Context of its own (default: the device's shared one) -- calls on different
    contexts and torch streams may run concurrently (each context has its own device scratch).
    """
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    if device_result and not p3.device:
        raise ValueError("device_result needs GPU tensor inputs")
    ctx = context if context is not None else L.context(_device_of(p3, device))
    flags = (L.F_DEVICE_IN if p3.device else 0) | (L.F_EXACT_ONLY if exact_only else 0)
    K9 = _K9(K)
    st = L.Stats()
    mask = mptr = None
    if with_mask:
        mask, mptr, mflag = _mask_buffer(p3, p3.n)
        flags |= mflag
    if device_result:
        import torch
        dev = p3.keep.device
        key_t = torch.empty(1, dtype=torch.int64, device=dev)  # written by the call (no fill launch)
        model_t = torch.empty(12, dtype=torch.float64, device=dev)
        with ctx.lock:
            L.check(L.lib().rsac_pnp_evaluate_range(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n,
                                                    K9.ctypes.data, int(hyp_begin), int(n_hyps),
                                                    float(reproj_thresh), int(seed) & (2**64 - 1),
                                                    flags | L.F_ASYNC,
                                                    C.cast(key_t.data_ptr(), C.POINTER(C.c_int64)),
                                                    C.c_void_p(model_t.data_ptr()),
                                                    C.c_void_p(mptr) if with_mask else None, C.byref(st),
                                                    _stream_of(p3)))
        out = (key_t, model_t)
        return out + (_finish_mask(mask, p3.n),) if with_mask else out
    key = C.c_int64(-1)
    model = np.zeros(12)
    with ctx.lock:
        code = L.check(L.lib().rsac_pnp_evaluate_range(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n,
                                                       K9.ctypes.data, int(hyp_begin), int(n_hyps),
                                                       float(reproj_thresh), int(seed) & (2**64 - 1), flags,
                                                       C.byref(key), model.ctypes.data,
                                                       C.c_void_p(mptr) if with_mask else None, C.byref(st),
                                                       _stream_of(p3)))
    out = (int(key.value), model)
    if with_mask:
        out = out + (_finish_mask(mask, p3.n),)
    if return_info:
        out = out + (_info(code, st),)
    return out


def hypothesis_rows(points2D, points3D, K, hyp_begin: int, n_hyps: int, reproj_thresh: float, rows, *,
                    seed: int = 0x5EED):
    """{status, count} int32 rows of Philox hypotheses [hyp_begin, hyp_begin + n_hyps) written into
    the device tensor ``rows`` (at least (n_hyps, 2) int32, contiguous) on the inputs' stream, without
    waiting -- the multi-GPU round's exchange format (rsac_pnp_hypothesis_rows)."""
    import torch
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    if not (p3.device and rows.is_cuda and rows.dtype == torch.int32 and rows.is_contiguous()
            and rows.shape[0] >= n_hyps and rows.shape[-1] == 2):
        raise ValueError("hypothesis_rows needs GPU tensor inputs and an (n, 2) int32 contiguous device tensor")
    ctx = L.context(_device_of(p3, None))
    with ctx.lock:
        L.check(L.lib().rsac_pnp_hypothesis_rows(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n,
                                                 _K9(K).ctypes.data, int(hyp_begin), int(n_hyps),
                                                 float(reproj_thresh), int(seed) & (2**64 - 1),
                                                 L.F_DEVICE_IN | L.F_DEVICE_OUT, C.c_void_p(rows.data_ptr()),
                                                 _stream_of(p3)))
    return rows


def winner(points2D, points3D, K, key, reproj_thresh: float = 30.0, *, seed: int = 0x5EED, with_mask: bool = True,
           context=None):
    """Re-derive the hypothesis named by a device packed key (e.g. after an all-reduce) on this
    GPU: (model12 tensor, mask tensor) without a host round trip (rsac_pnp_winner).  context: as
    evaluate_range."""
    import torch
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    if not p3.device:
        raise ValueError("winner() needs GPU tensor inputs")
    ctx = context if context is not None else L.context(_device_of(p3, None))
    dev = p3.keep.device
    model_t = torch.zeros(12, dtype=torch.float64, device=dev)
    mask_t = torch.empty(max(p3.n, 1), dtype=torch.uint8, device=dev) if with_mask else None
    K9 = _K9(K)
    with ctx.lock:
        L.check(L.lib().rsac_pnp_winner(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n, K9.ctypes.data,
                                        float(reproj_thresh), int(seed) & (2**64 - 1), C.c_void_p(key.data_ptr()),
                                        C.c_void_p(model_t.data_ptr()),
                                        C.c_void_p(mask_t.data_ptr()) if with_mask else None, _stream_of(p3)))
    return model_t, (_finish_mask(mask_t, p3.n) if with_mask else None)


def hypotheses(model: str, a, b, K=None, hyp_begin: int = 0, n_hyps: int = 1024, reproj_thresh: float = 30.0, *,
               seed: int = 0x5EED, subsets=None, device=None, exact_only: bool = False, minimal: str = "p3p",
               rvec=None):
    """Raw per-hypothesis (status, counts, models) of the GPU hot path for one problem.

    model "pnp": a = points3D (N,3), b = points2D (N,2), K required.
    model "homography": a = src (N,2), b = dst (N,2).
    model "fundamental": a = pts1 (N,2), b = pts2 (N,2).
    subsets: optional (n_hyps, 4) int32 index table replacing the Philox draw ((n_hyps, 5) for
    minimal="epnp5", PnP's 5-point EPnP kernel).  rvec: PnP models through Rodrigues(Rodrigues(R));
    the default (None) is on exactly when subsets are given, as pnp_ransac(sampler="opencv") scores
    OpenCV's MWC subsets, so the probe returns the rotations that run scores.
    """
    if rvec is None:
        rvec = subsets is not None
    pnp = model == "pnp"
    if model not in ("pnp", "homography", "fundamental"):
        raise ValueError(f"unknown model {model!r}")
    A = _In(a, 3 if pnp else 2)
    B = _In(b, 2)
    ctx = L.context(_device_of(A, device))
    flags = (L.F_DEVICE_IN if A.device else 0) | (L.F_EXACT_ONLY if exact_only else 0)
    flags |= L.F_RVEC_ROUNDTRIP if (rvec and pnp) else 0
    k = 4
    if minimal == "epnp5":
        if not pnp:
            raise ValueError("minimal='epnp5' is a PnP kernel")
        flags |= L.F_MINIMAL_EPNP5
        k = 5
    elif minimal != "p3p":
        raise ValueError(f"minimal must be 'p3p' or 'epnp5', got {minimal!r}")
    counts = np.zeros(n_hyps, np.int32)
    status = np.zeros(n_hyps, np.int8)
    models = np.zeros((n_hyps, 16))
    sub = None if subsets is None else np.ascontiguousarray(np.asarray(subsets, np.int32).reshape(n_hyps, k))
    with ctx.lock:
        if pnp:
            K9 = _K9(K)
            L.check(L.lib().rsac_pnp_hypotheses(ctx.handle, C.c_void_p(A.ptr), C.c_void_p(B.ptr), A.n, K9.ctypes.data,
                                                int(hyp_begin), int(n_hyps), float(reproj_thresh),
                                                int(seed) & (2**64 - 1), flags,
                                                None if sub is None else sub.ctypes.data, counts.ctypes.data,
                                                status.ctypes.data, models.ctypes.data, _stream_of(A)))
        elif model == "fundamental":
            L.check(L.lib().rsac_fundamental_hypotheses(ctx.handle, C.c_void_p(A.ptr), C.c_void_p(B.ptr), A.n,
                                                        int(hyp_begin), int(n_hyps), float(reproj_thresh),
                                                        int(seed) & (2**64 - 1), flags, counts.ctypes.data,
                                                        status.ctypes.data, models.ctypes.data, _stream_of(A)))
        else:
            L.check(L.lib().rsac_homography_hypotheses(ctx.handle, C.c_void_p(A.ptr), C.c_void_p(B.ptr), A.n,
                                                       int(hyp_begin), int(n_hyps), float(reproj_thresh),
                                                       int(seed) & (2**64 - 1), flags,
                                                       None if sub is None else sub.ctypes.data, counts.ctypes.data,
                                                       status.ctypes.data, models.ctypes.data, _stream_of(A)))
    return status, counts, models


def pose_mask(points2D, points3D, K, model12, reproj_thresh: float = 30.0, device=None):
    """RANSAC-test mask (and count) of one pose model (R 9 row-major, t 3)."""
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    ctx = L.context(_device_of(p3, device))
    flags = L.F_DEVICE_IN if p3.device else 0
    mask, mptr, mflag = _mask_buffer(p3, p3.n)
    flags |= mflag
    cnt = C.c_int32(0)
    K9 = _K9(K)
    m12 = np.ascontiguousarray(np.asarray(model12, np.float64).reshape(12))
    with ctx.lock:
        L.check(L.lib().rsac_pnp_mask(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n, K9.ctypes.data,
                                      m12.ctypes.data, float(reproj_thresh), flags, C.c_void_p(mptr), C.byref(cnt),
                                      _stream_of(p3)))
    return _finish_mask(mask, p3.n), int(cnt.value)


def refine_pose(points2D, points3D, K, R, t, mask=None, max_iter: int = 20):
    """LM refinement of (R, t) on host arrays (cv2.solvePnPRefineLM, main_v1.py:508) -> (R, t)."""
    P3 = np.ascontiguousarray(np.asarray(points3D, np.float64).reshape(-1, 3))
    P2 = np.ascontiguousarray(np.asarray(points2D, np.float64).reshape(-1, 2))
    Rr = np.ascontiguousarray(np.asarray(R, np.float64).reshape(9)).copy()
    tr = np.ascontiguousarray(np.asarray(t, np.float64).reshape(3)).copy()
    m = None if mask is None else np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(-1))
    K9 = _K9(K)
    L.check(L.lib().rsac_pnp_refine(P3.ctypes.data, P2.ctypes.data, P3.shape[0], K9.ctypes.data,
                                    None if m is None else m.ctypes.data, Rr.ctypes.data, tr.ctypes.data,
                                    int(max_iter)))
    return Rr.reshape(3, 3), tr


def refine_pose_device(points2D, points3D, K, R, t, mask=None, device=None):
    """cv2.solvePnPRefineLM (main_v1.py:508, testpro-K.py:122) on the GPU: LM from (R, t) over the
    (masked) correspondences -> (R, t).  Host arrays; the same bits as refine_pose (host)."""
    P3 = np.ascontiguousarray(np.asarray(points3D, np.float64).reshape(-1, 3))
    P2 = np.ascontiguousarray(np.asarray(points2D, np.float64).reshape(-1, 2))
    if P3.shape[0] != P2.shape[0]:
        raise ValueError("points3D and points2D differ in length")
    Rr = np.ascontiguousarray(np.asarray(R, np.float64).reshape(9)).copy()
    tr = np.ascontiguousarray(np.asarray(t, np.float64).reshape(3)).copy()
    m = None if mask is None else np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(-1))
    ctx = L.context(0 if device is None else int(device))
    with ctx.lock:
        L.check(L.lib().rsac_pnp_refine_lm(ctx.handle, P3.ctypes.data, P2.ctypes.data, P3.shape[0], _K9(K).ctypes.data,
                                           None if m is None else m.ctypes.data, Rr.ctypes.data, tr.ctypes.data, None))
    return Rr.reshape(3, 3), tr


def reprojection_errors(points3D, points2D, K, R, t, *, device=None, return_projection: bool = False):
    """compute_reprojection_error (testpro-K.py:32-36) on the GPU: ||pixel - projectPoints(X)||_2
    per point, f64 throughout (zero distortion).  R (3,3) or a Rodrigues vector (3,), t (3,).
    GPU tensor inputs keep the outputs on the device.  -> errors (N,) [, projections (N, 2)]."""
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    if p3.n != p2.n:
        raise ValueError("points3D and points2D differ in length")
    if p3.device != p2.device:
        raise ValueError("points3D and points2D must both be host arrays or both GPU tensors")
    r = np.asarray(R, np.float64)
    R9 = np.ascontiguousarray(rodrigues(r).reshape(9) if r.size == 3 else r.reshape(9))
    t3 = np.ascontiguousarray(np.asarray(t, np.float64).reshape(3))
    n = p3.n
    ctx = L.context(_device_of(p3, device))
    if p3.device:
        import torch
        err = torch.empty(max(n, 1), dtype=torch.float64, device=p3.keep.device)
        proj = torch.empty((max(n, 1), 2), dtype=torch.float64, device=p3.keep.device) if return_projection else None
        eptr, pptr = err.data_ptr(), (proj.data_ptr() if proj is not None else None)
        flags = L.F_DEVICE_IN
    else:
        err = np.zeros(max(n, 1))
        proj = np.zeros((max(n, 1), 2)) if return_projection else None
        eptr, pptr = err.ctypes.data, (proj.ctypes.data if proj is not None else None)
        flags = 0
    with ctx.lock:
        L.check(L.lib().rsac_pnp_reprojection_errors(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), n,
                                                     _K9(K).ctypes.data, R9.ctypes.data, t3.ctypes.data, flags,
                                                     C.c_void_p(pptr) if pptr else None, C.c_void_p(eptr),
                                                     _stream_of(p3)))
    return (err[:n], proj[:n]) if return_projection else err[:n]


def compute_reprojection_error(pos3d, pixels, K, dist_coeffs, rvec, tvec):
    """The reference's helper (testpro-K.py:32-36) with its signature: projectPoints through the
    Rodrigues vector rvec, then the per-point L2 norm -- on the GPU (reprojection_errors)."""
    if dist_coeffs is not None and np.any(np.asarray(dist_coeffs, np.float64) != 0):
        raise NotImplementedError("zero distortion only (as every reference call site uses)")
    rv = np.asarray(rvec, np.float64).reshape(-1)
    R = rodrigues(rv) if rv.size == 3 else rv.reshape(3, 3)
    e = reprojection_errors(pos3d, pixels, K, R, tvec)
    return e


@dataclass
class OrientationResult:
    """Outputs of estimate_camera_orientation (testpro-K.py:39-162), one row per intrinsic."""
    rvec: np.ndarray | None          # (3, 1) solvePnPRefineLM's rotation vector (None: every K failed)
    tvec: np.ndarray | None          # (3, 1)
    best: int                        # index of the chosen K (-1: none)
    K: np.ndarray                    # (P, 3, 3) the candidates, loop order (focal outer, sensor inner)
    mean_error: np.ndarray           # (P,) mean inlier reprojection error (NaN: failed the gate)
    ok: np.ndarray                   # (P,) passed "success and >= 6 inliers" (testpro-K.py:77)
    n_inliers: np.ndarray            # (P,)
    rvec_initial: np.ndarray         # (P, 3) solvePnPRansac's rotation vectors
    tvec_initial: np.ndarray         # (P, 3)
    masks: np.ndarray                # (P, N) RANSAC-phase inlier masks
    focal_sensor: list               # (focal length, (sensor w, sensor h)) of every K
    ranking: list                    # (distance to the known origin, mean error, K index, camera origin), sorted

    @property
    def best_K(self):
        return self.K[self.best] if self.best >= 0 else None


def intrinsics_grid(focal_lengths, sensor_sizes, image_size):
    """The candidate intrinsics of testpro-K.py:58-70, in its loop order."""
    Ks, fs = [], []
    for focal_length in focal_lengths:
        for (sensor_width, sensor_height) in sensor_sizes:
            fx = focal_length / (sensor_width / image_size[0])
            fy = focal_length / (sensor_height / image_size[1])
            Ks.append(np.array([[fx, 0, image_size[0] / 2], [0, fy, image_size[1] / 2], [0, 0, 1]], np.float64))
            fs.append((focal_length, (sensor_width, sensor_height)))
    return np.stack(Ks), fs


def estimate_camera_orientation(pos3d, pixels, focal_lengths, sensor_sizes, image_size, known_camera_origin=None, *,
                                n_iters: int = 5000, reproj_thresh: float = 30.0, confidence: float = 0.99,
                                seed: int = 0x5EED, sampler: str = "opencv", minimal: str = "epnp5", refine="lm",
                                min_inliers: int = 6, device: int = 0, return_info: bool = False, rvec=None):
    """estimate_camera_orientation of testpro-K.py:39-125 as one GPU call sequence
    (rsac_pnp_orientation_sweep): solvePnPRansac under every candidate K (one batched launch), the
    mean inlier reprojection error of each on the device, the first K with the smallest, then
    solvePnPRefineLM of its pose on its inliers.  Returns (rvec, tvec) like the reference
    ((None, None) when every K failed), or the OrientationResult with return_info=True.

    The defaults are what testpro-K.py:72-75 executes: cv2.solvePnPRansac with no `flags`, i.e.
    SOLVEPNP_ITERATIVE -- EPnP on 5-point samples drawn from OpenCV's MWC stream
    (minimal="epnp5", sampler="opencv"), then the LM final solve on the inliers (refine="lm").
    minimal="p3p" / sampler="philox" run this project's benchmark kernel instead."""
    if int(min_inliers) < 3:
        raise ValueError("min_inliers must be >= 3 (solvePnPRefineLM needs 3 inliers)")
    P3 = np.ascontiguousarray(np.asarray(pos3d, np.float64).reshape(-1, 3))
    P2 = np.ascontiguousarray(np.asarray(pixels, np.float64).reshape(-1, 2))
    if P3.shape[0] != P2.shape[0]:
        raise ValueError("pos3d and pixels differ in length")
    Ks, fs = intrinsics_grid(focal_lengths, sensor_sizes, image_size)
    P, n = Ks.shape[0], P3.shape[0]
    K9 = np.ascontiguousarray(Ks.reshape(P, 9))
    best = C.c_int32(-1)
    mean = np.zeros(P)
    models = np.zeros((P, 12))
    status = np.zeros(P, np.int32)
    ninl = np.zeros(P, np.int32)
    masks = np.zeros((P, max(n, 1)), np.uint8)
    R, t = np.zeros(9), np.zeros(3)
    ctx = L.context(device)
    with ctx.lock:
        code = L.check(L.lib().rsac_pnp_orientation_sweep(
            ctx.handle, P3.ctypes.data, P2.ctypes.data, n, K9.ctypes.data, P, int(n_iters), float(reproj_thresh),
            float(confidence), int(seed) & (2**64 - 1), _flags(True, refine, sampler, minimal=minimal, rvec=rvec), int(min_inliers),
            C.byref(best), mean.ctypes.data, models.ctypes.data, status.ctypes.data, ninl.ctypes.data,
            masks.ctypes.data, R.ctypes.data, t.ctypes.data, None))
    ok = status == L.OK
    b = int(best.value)
    rvec = rodrigues(R.reshape(3, 3)).reshape(3, 1) if code == L.OK else None
    tvec = t.reshape(3, 1).copy() if code == L.OK else None
    if not return_info:
        return rvec, tvec
    rv0 = np.stack([rodrigues(models[k, :9].reshape(3, 3)).reshape(3) for k in range(P)])
    ranking = []
    if known_camera_origin is not None:
        o = np.asarray(known_camera_origin, np.float64).reshape(3)
        for k in np.flatnonzero(ok):
            Rk = rodrigues(rv0[k])
            origin = -Rk.T @ models[k, 9:12]
            ranking.append((float(np.linalg.norm(origin - o)), float(mean[k]), int(k), origin))
        ranking.sort(key=lambda x: x[0])  # testpro-K.py:103 (stable, as Python's sort)
    return OrientationResult(rvec=rvec, tvec=tvec, best=b, K=Ks, mean_error=mean, ok=ok, n_inliers=ninl,
                             rvec_initial=rv0, tvec_initial=models[:, 9:12].copy(), masks=masks[:, :n].astype(bool),
                             focal_sensor=fs, ranking=ranking)


def epnp_pose(points2D, points3D, K, mask=None):
    """EPnP on all (or the masked) points, cv2.solvePnP(..., flags=SOLVEPNP_EPNP) -> (R, t) or
    (None, None) for < 4 points / a planar cloud.  Host arrays; the same numbers as the device pass
    of pnp_ransac(refine="epnp")."""
    P3 = np.ascontiguousarray(np.asarray(points3D, np.float64).reshape(-1, 3))
    P2 = np.ascontiguousarray(np.asarray(points2D, np.float64).reshape(-1, 2))
    m = None if mask is None else np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(-1))
    R, t = np.zeros(9), np.zeros(3)
    code = L.check(L.lib().rsac_pnp_epnp(P3.ctypes.data, P2.ctypes.data, P3.shape[0], _K9(K).ctypes.data,
                                         None if m is None else m.ctypes.data, R.ctypes.data, t.ctypes.data))
    return (R.reshape(3, 3), t) if code == L.OK else (None, None)


def epnp_minimal(points2D, points3D, K):
    """solvePnPRansac's default minimal solver on one 5-point sample, on the host: solvePnP(...,
    SOLVEPNP_EPNP) in OpenCV's operation sequence (rsac_cvepnp.h, the source the k_cvepnp5_*
    kernels run) -> (R, t).  Inputs are rounded to f32 like solvePnPRansac's CV_32F copies."""
    P3 = np.ascontiguousarray(np.asarray(points3D, np.float64).reshape(5, 3))
    P2 = np.ascontiguousarray(np.asarray(points2D, np.float64).reshape(5, 2))
    R, t = np.zeros(9), np.zeros(3)
    L.check(L.lib().rsac_pnp_epnp_minimal(P3.ctypes.data, P2.ctypes.data, _K9(K).ctypes.data, R.ctypes.data,
                                          t.ctypes.data))
    return R.reshape(3, 3), t


def homography_fit(src, dst, mask=None):
    """Least-squares normalised DLT + LM on all (or masked) points -> H (findHomography method 0)."""
    s = np.ascontiguousarray(np.asarray(src, np.float64).reshape(-1, 2))
    d = np.ascontiguousarray(np.asarray(dst, np.float64).reshape(-1, 2))
    m = None if mask is None else np.ascontiguousarray(np.asarray(mask, np.uint8).reshape(-1))
    H = np.zeros(9)
    code = L.check(L.lib().rsac_homography_fit(s.ctypes.data, d.ctypes.data, s.shape[0],
                                               None if m is None else m.ctypes.data, H.ctypes.data))
    return H.reshape(3, 3) if code == L.OK else None


def rodrigues(src):
    """cv2.Rodrigues (main_v1.py:895): (3,) vector <-> (3, 3) matrix."""
    a = np.ascontiguousarray(np.asarray(src, np.float64))
    if a.size == 3:
        R = np.zeros(9)
        L.lib().rsac_rodrigues_v2m(a.reshape(3).ctypes.data, R.ctypes.data)
        return R.reshape(3, 3)
    if a.size == 9:
        r = np.zeros(3)
        L.lib().rsac_rodrigues_m2v(a.reshape(9).ctypes.data, r.ctypes.data)
        return r.reshape(3, 1)
    raise ValueError("Rodrigues expects a 3-vector or a 3x3 matrix")


def update_num_iters(p: float, ep: float, model_points: int, max_iters: int) -> int:
    """RANSACUpdateNumIters of OpenCV, as the driver applies it after every new best model."""
    return int(L.lib().rsac_update_num_iters(float(p), float(ep), int(model_points), int(max_iters)))


@dataclass
class LocationResult:
    """Outputs of rsac.location_search, one row per candidate camera location."""
    err: np.ndarray  # (L, 2) f64: err1, err2 (num_matches of main_v1.py:273; (0, 0) = no model)
    H: np.ndarray  # (L, 3, 3) findHomography's H (main_v1.py:312; M = inv(H) at :314)
    ok: np.ndarray  # (L,) bool
    n_inliers: np.ndarray  # (L,) int32
    mask: np.ndarray  # (L, n_good) bool, RANSAC-phase
    n_good: int  # features noted on the image

    @property
    def best(self) -> int:
        """argmin of err2 with 0 -> 1e6, as main_v1.py:863-866 picks the camera location."""
        e2 = self.err[:, 1].copy()
        e2[e2 == 0] = 1000000
        return int(np.argmin(e2))


def location_search(pos3d, pixels, locations, ransacbound: float = 75.0, *, max_iters: int = 2000,
                    confidence: float = 0.995, sampler: str = "opencv", adaptive: bool = True, refine: bool = True,
                    device: int = 0) -> LocationResult:
    """The camera-location search of find_homographies (main_v1.py:254-297) in one call.

    pos3d (N,3) feature positions, pixels (N,2) (rows (0,0) = not noted on the image,
    main_v1.py:304), locations (L,3) candidate camera positions.  For every location the
    homography RANSAC of find_homography (main_v1.py:300-312) and its err1/err2 score
    (main_v1.py:332-348, 419) run on the GPU.
    """
    P3 = np.ascontiguousarray(np.asarray(pos3d, np.float64).reshape(-1, 3))
    P2 = np.ascontiguousarray(np.asarray(pixels, np.float64).reshape(-1, 2))
    LC = np.ascontiguousarray(np.asarray(locations, np.float64).reshape(-1, 3))
    if P3.shape[0] != P2.shape[0]:
        raise ValueError("pos3d and pixels differ in length")
    L_, n = LC.shape[0], P3.shape[0]
    n_good_max = int(np.count_nonzero((P2[:, 0] != 0) | (P2[:, 1] != 0)))
    err = np.zeros((L_, 2))
    H = np.zeros((L_, 9))
    st = np.zeros(L_, np.int32)
    ninl = np.zeros(L_, np.int32)
    mask = np.zeros(max(L_ * n_good_max, 1), np.uint8)
    ng = C.c_int32(0)
    ctx = L.context(device)
    with ctx.lock:
        L.check(L.lib().rsac_location_search(ctx.handle, P3.ctypes.data, P2.ctypes.data, n, LC.ctypes.data, L_,
                                             float(ransacbound), int(max_iters), float(confidence),
                                             _flags(adaptive, refine, sampler), H.ctypes.data, err.ctypes.data,
                                             st.ctypes.data, ninl.ctypes.data, mask.ctypes.data, C.byref(ng), None))
    g = int(ng.value)
    return LocationResult(err=err, H=H.reshape(L_, 3, 3), ok=st == L.OK, n_inliers=ninl,
                          mask=mask[:L_ * g].reshape(L_, g).astype(bool), n_good=g)


def local_opt(points2D, points3D, K, model12, reproj_thresh: float = 30.0, device=None):
    """One LO-RANSAC local optimisation of a pose -> (model12, inlier count, steps)."""
    p3 = _In(points3D, 3)
    p2 = _In(points2D, 2)
    ctx = L.context(_device_of(p3, device))
    m_in = np.ascontiguousarray(np.asarray(model12, np.float64).reshape(12))
    m_out = np.zeros(12)
    cnt = C.c_int32(0)
    steps = C.c_int32(0)
    K9 = _K9(K)
    with ctx.lock:
        L.check(L.lib().rsac_pnp_local_opt(ctx.handle, C.c_void_p(p3.ptr), C.c_void_p(p2.ptr), p3.n, K9.ctypes.data,
                                           m_in.ctypes.data, float(reproj_thresh),
                                           L.F_DEVICE_IN if p3.device else 0, m_out.ctypes.data, C.byref(cnt),
                                           C.byref(steps), _stream_of(p3)))
    return m_out, int(cnt.value), int(steps.value)


class Scan:
    """OpenCV's sequential best-model scan (rsac_scan of include/rsac.h) over counts produced
    elsewhere -- the multi-GPU driver feeds it each round's gathered counts."""

    def __init__(self, max_iters: int, n_points: int, confidence: float = 0.99, model_points: int = 4):
        self.st = L.ScanState()
        L.lib().rsac_scan_init(C.byref(self.st), int(max_iters))
        self.n = int(n_points)
        self.conf = float(confidence)
        self.s = int(model_points)

    def step(self, counts, status):
        c = np.ascontiguousarray(counts, np.int32)
        st = np.ascontiguousarray(status, np.int8)
        if c.shape != st.shape:
            raise ValueError("counts and status differ in length")
        L.check(L.lib().rsac_scan(C.byref(self.st), c.ctypes.data, st.ctypes.data, c.size, self.n, self.s, self.conf))
        return self

    def step_until_best(self, counts, status) -> int:
        """Scan until a new best (LO-RANSAC); returns how many entries were consumed (the
        new best is the last of them when ``improved``)."""
        c = np.ascontiguousarray(counts, np.int32)
        st = np.ascontiguousarray(status, np.int8)
        before = self.iters
        imp = C.c_int32(0)
        L.check(L.lib().rsac_scan_until_best(C.byref(self.st), c.ctypes.data, st.ctypes.data, c.size, self.n, self.s,
                                             self.conf, C.byref(imp)))
        self.improved = bool(imp.value)
        return self.iters - before

    def step_rows(self, rows, count: int, stop_on_improve: bool = False) -> int:
        """Consume the first ``count`` {status, count} rows of an (m, 2) int32 array or tensor (a
        gathered multi-GPU round).  GPU tensors are scanned on the device (rsac_scan_device: only
        the improvements come to the host).  Returns the rows consumed (``improved`` is set when
        stop_on_improve stopped at a new best)."""
        before = self.iters
        if _is_torch(rows) and rows.is_cuda:
            import torch
            r = rows[:count]
            if not r.is_contiguous() or r.dtype != torch.int32:
                r = r.to(torch.int32).contiguous()
            imp = C.c_int32(0)
            ctx = L.context(r.device.index)
            with ctx.lock:
                L.check(L.lib().rsac_scan_device(ctx.handle, C.byref(self.st), C.c_void_p(r.data_ptr()), int(count),
                                                 self.n, self.s, self.conf, 1 if stop_on_improve else 0, C.byref(imp),
                                                 C.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)))
            self.improved = bool(imp.value)
            return self.iters - before
        a = np.asarray(rows.cpu() if _is_torch(rows) else rows)[:count]
        if stop_on_improve:
            return self.step_until_best(a[:, 1], a[:, 0].astype(np.int8))
        self.step(a[:, 1], a[:, 0].astype(np.int8))
        self.improved = False
        return self.iters - before

    def raise_count(self, count: int):
        """Apply a locally optimised inlier count."""
        L.check(L.lib().rsac_scan_raise(C.byref(self.st), int(count), self.n, self.s, self.conf))

    done = property(lambda self: bool(self.st.done))
    best = property(lambda self: int(self.st.best))
    max_good = property(lambda self: int(self.st.max_good))
    iters = property(lambda self: int(self.st.iter))
    niters = property(lambda self: int(self.st.niters))

