"""ctypes binding of librsac.so (include/rsac.h).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``)
and loaded from this directory.  There is no fallback: if the HIP library is
missing or no device is visible, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# RSAC_LIB_PATH: another build of the same library (kernel A/B scripts, scripts/mf_ab.py)
LIB_PATH = os.environ.get("RSAC_LIB_PATH") or os.path.join(_HERE, "librsac.so")

# status codes / flags (include/rsac.h)
OK = 0
NO_MODEL = 1
MORE = 2  # rsac_pnp_ransac_first_round: the first round did not end the scan
EINVAL = -1
ETOOFEW = -2
EHIP = -3
ENOMEM = -4
ENODEV = -5

F_SAMPLER_OPENCV = 1 << 0
F_ADAPTIVE = 1 << 1
F_REFINE = 1 << 2
F_DEVICE_IN = 1 << 3
F_DEVICE_SOA = 1 << 4
F_DEVICE_OUT = 1 << 5
F_EXACT_ONLY = 1 << 6
F_LO = 1 << 7
F_ASYNC = 1 << 8
F_EPNP = 1 << 9
F_MINIMAL_EPNP5 = 1 << 10
F_RVEC_ROUNDTRIP = 1 << 11

DBG_REFIT_MAX_BLOCKS = 1
DBG_REFIT_DROP_BLOCK = 2
DBG_F64_SELFTEST = 7

ABI_VERSION = 2  # include/rsac.h RSAC_ABI_VERSION


class Stats(C.Structure):
    _fields_ = [("best_hyp", C.c_int64), ("iters", C.c_int64), ("hyps_scored", C.c_int64),
                ("n_inliers", C.c_int32), ("rounds", C.c_int32), ("gpu_ms", C.c_double), ("solve_ms", C.c_double),
                ("score_ms", C.c_double), ("lo_improvements", C.c_int32), ("reserved", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class ScanState(C.Structure):
    """rsac_scan_state of include/rsac.h"""
    _fields_ = [("niters", C.c_int64), ("best", C.c_int64), ("iter", C.c_int64), ("max_good", C.c_int32),
                ("done", C.c_int32)]


# (name, restype, argtypes) -- one row per declaration of include/rsac.h
_vp, _i32, _i64, _u32, _u64, _d = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
SIGNATURES = [
    ("rsac_create", C.c_int, [C.c_int, C.POINTER(_vp)]),
    ("rsac_destroy", None, [_vp]),
    ("rsac_last_error", C.c_char_p, []),
    ("rsac_abi_version", C.c_int, []),
    ("rsac_device_count", C.c_int, []),
    ("rsac_set_timing", C.c_int, [_vp, _i32]),
    ("rsac_last_stats", C.c_int, [_vp, C.POINTER(Stats)]),
    ("rsac_set_round_size", C.c_int, [_vp, _i64]),
    ("rsac_refit_blocks", C.c_int, [_vp, _i32, C.POINTER(_i32), C.POINTER(_i32)]),
    ("rsac_debug_set", C.c_int, [_vp, _i32, _i64]),
    ("rsac_debug_get", C.c_int, [_vp, _i32, _vp]),
    ("rsac_pnp_ransac", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _d, _d, _u64, _u32, _vp, _vp, _vp,
                                  C.POINTER(Stats), _vp]),
    ("rsac_pnp_ransac_batched", C.c_int, [_vp, _vp, _vp, _vp, _i32, _vp, _i32, _d, _d, _u64, _u32, _vp, _vp, _vp,
                                          _vp, _vp, _vp]),
    ("rsac_pnp_ransac_batched_rows", C.c_int, [_vp, _vp, _vp, _vp, _i32, _vp, _i32, _d, _d, _u64, _u32, _vp, _vp,
                                               _vp]),
    ("rsac_homography_ransac", C.c_int, [_vp, _vp, _vp, _i32, _i32, _d, _d, _u64, _u32, _vp, _vp,
                                         C.POINTER(Stats), _vp]),
    ("rsac_homography_ransac_batched", C.c_int, [_vp, _vp, _vp, _vp, _i32, _i32, _d, _d, _u64, _u32, _vp, _vp, _vp,
                                                 _vp, _vp]),
    ("rsac_score_poses", C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _i32, _d, _u32, _vp, _vp]),
    ("rsac_pnp_evaluate_range", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i64, _i64, _d, _u64, _u32,
                                          C.POINTER(_i64), _vp, _vp, C.POINTER(Stats), _vp]),
    ("rsac_pnp_hypotheses", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i64, _i32, _d, _u64, _u32, _vp, _vp, _vp, _vp,
                                      _vp]),
    ("rsac_homography_hypotheses", C.c_int, [_vp, _vp, _vp, _i32, _i64, _i32, _d, _u64, _u32, _vp, _vp, _vp, _vp,
                                             _vp]),
    ("rsac_pnp_mask", C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _d, _u32, _vp, C.POINTER(_i32), _vp]),
    ("rsac_pnp_epnp", C.c_int, [_vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    ("rsac_pnp_epnp_minimal", C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("rsac_pnp_refine", C.c_int, [_vp, _vp, _i32, _vp, _vp, _vp, _vp, _i32]),
    ("rsac_homography_fit", C.c_int, [_vp, _vp, _i32, _vp, _vp]),
    ("rsac_rodrigues_v2m", None, [_vp, _vp]),
    ("rsac_rodrigues_m2v", None, [_vp, _vp]),
    ("rsac_update_num_iters", C.c_int, [_d, _d, C.c_int, C.c_int]),
    ("rsac_location_search", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _d, _i32, _d, _u32, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp]),
    ("rsac_fundamental_ransac", C.c_int, [_vp, _vp, _vp, _i32, _i32, _d, _d, _u64, _u32, _vp, _vp, _vp, _vp]),
    ("rsac_fundamental_hypotheses", C.c_int, [_vp, _vp, _vp, _i32, _i64, _i32, _d, _u64, _u32, _vp, _vp, _vp, _vp]),
    ("rsac_pnp_winner", C.c_int, [_vp, _vp, _vp, _i32, _vp, _d, _u64, _vp, _vp, _vp, _vp]),
    ("rsac_utm_convert", C.c_int, [_vp, C.c_int, _vp, _i64, _i32, _i32, _u32, _vp, _vp]),
    ("rsac_dem_ray_intersect", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _i32, _d, _d, _d, _d, _i32, _i32, _d, _d,
                                         _i32, _u32, _vp, _vp, _vp]),
    ("rsac_scan_init", None, [_vp, _i32]),
    ("rsac_scan_until_best", C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _d, _vp]),
    ("rsac_scan_raise", C.c_int, [_vp, _i32, _i32, _i32, _d]),
    ("rsac_pnp_local_opt", C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _d, _u32, _vp, _vp, _vp, _vp]),
    ("rsac_scan", C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _d]),
    ("rsac_pnp_refine_lm", C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    ("rsac_pnp_reprojection_errors", C.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    ("rsac_pnp_ransac_first_round", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _d, _d, _u64, _u32, _vp, _vp, _vp,
                                              C.POINTER(ScanState), C.POINTER(Stats), _vp]),
    ("rsac_pnp_hypothesis_rows", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i64, _i32, _d, _u64, _u32, _vp, _vp]),
    ("rsac_scan_device", C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _d, _i32, _vp, _vp]),
    ("rsac_pnp_orientation_sweep", C.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _i32, _d, _d, _u64, _u32, _i32, _vp,
                                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
]

_lib = None
_lock = threading.RLock()


class RsacError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rsac error {code}: {msg}")
        self.code = code


def _share_hip_runtime_with_torch():
    """Make librsac bind to the HIP runtime torch uses, whatever the import order.

    torch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7) and loads it
    as ``libamdhip64.so`` from its lib/ directory; librsac needs
    ``libamdhip64.so.7``.  Loading torch's copy first (RTLD_GLOBAL) makes both
    resolve to ONE runtime, so torch tensors' device pointers and streams are
    valid in librsac and torch can still initialise after us.
    """
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except Exception:
        spec = None
    if spec is None or not spec.origin:
        return
    hip = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(hip):
        C.CDLL(hip, mode=C.RTLD_GLOBAL)


def lib():
    """Load librsac.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (make -C code-reproduction-ransac_amd/csrc)")
        _share_hip_runtime_with_torch()
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.rsac_abi_version() != ABI_VERSION:
            raise ImportError("librsac.so ABI version mismatch")
        _lib = L
    return _lib


def check(code):
    if code < 0:
        msg = lib().rsac_last_error()
        raise RsacError(code, msg.decode() if msg else "")
    return code


class Context:
    """One rsac_ctx (device scratch + stream) per (process, device)."""

    def __init__(self, device: int = 0):
        self.device = device
        self._h = C.c_void_p()
        check(lib().rsac_create(device, C.byref(self._h)))
        self.lock = threading.Lock()

    @property
    def handle(self):
        return self._h

    def set_timing(self, on: bool = True):
        """HIP events around every PnP call's solve and scoring launches (rsac_set_timing)"""
        check(lib().rsac_set_timing(self._h, 1 if on else 0))

    def last_stats(self) -> dict:
        """rsac_stats of the last PnP call on this context (with set_timing on)"""
        st = Stats()
        check(lib().rsac_last_stats(self._h, C.byref(st)))
        return st.as_dict()

    def set_round_size(self, n: int):
        check(lib().rsac_set_round_size(self._h, int(n)))

    def refit_blocks(self, n: int) -> tuple[int, int]:
        """(ranges of the refit's summation order, cooperating blocks on this device) for n points"""
        r, b = _i32(), _i32()
        check(lib().rsac_refit_blocks(self._h, int(n), C.byref(r), C.byref(b)))
        return r.value, b.value

    def debug_set(self, key: int, value: int):
        """test hooks of include/rsac.h (DBG_REFIT_MAX_BLOCKS, DBG_REFIT_DROP_BLOCK, DBG_MF_CELL_PTS,
        DBG_SPEC_OVERFLOW, DBG_F64_SELFTEST)"""
        check(lib().rsac_debug_set(self._h, int(key), int(value)))

    def debug_get(self, key: int) -> int:
        """read-only counters of include/rsac.h (DBG_SPEC_FINISHES, DBG_SPEC_REDOS, DBG_F64_SELFTEST)"""
        v = C.c_int64(0)
        check(lib().rsac_debug_get(self._h, int(key), C.byref(v)))
        return v.value

    def close(self):
        if self._h:
            lib().rsac_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts: dict[int, Context] = {}


def context(device: int = 0) -> Context:
    with _lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = Context(device)
            _contexts[device] = ctx
        return ctx
