"""Where a pnp_ransac call's host time goes: the Python wrapper vs the C-ABI call (C2 problem,
device tensors, adaptive, LM refit)."""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
p2d = torch.from_numpy(pr["points2d"]).cuda()
p3d = torch.from_numpy(pr["points3d"]).cuda()


def med(f, n=200):
    for _ in range(20):
        f()
    w = []
    for _ in range(n):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f()
        torch.cuda.synchronize()
        w.append((time.perf_counter() - t) * 1e6)
    return statistics.median(w)


print("wrapper total us %.1f" % med(lambda: rsac.pnp_ransac(p2d, p3d, pr["K"], 5000, 30.0, refine=True)))
ctx = L.context(0)
K9 = np.ascontiguousarray(np.asarray(pr["K"], np.float64).reshape(9))
R = np.zeros(9)
t = np.zeros(3)
mask = torch.empty(10000, dtype=torch.uint8, device="cuda")
st = L.Stats()
flags = L.F_ADAPTIVE | L.F_REFINE | L.F_DEVICE_IN | L.F_DEVICE_OUT
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
lib = L.lib()


def raw():
    lib.rsac_pnp_ransac(ctx.handle, C.c_void_p(p3d.data_ptr()), C.c_void_p(p2d.data_ptr()), 10000, K9.ctypes.data,
                        5000, 30.0, 0.99, 0x5EED, flags, R.ctypes.data, t.ctypes.data, C.c_void_p(mask.data_ptr()),
                        C.byref(st), stream)


print("raw C call us %.1f" % med(raw))
print("empty torch sync us %.1f" % med(lambda: None))
