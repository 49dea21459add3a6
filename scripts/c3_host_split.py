"""C3 (BASELINE.json configs[2]) wall time split: the Python wrapper (pnp_ransac_batched_flat)
against the raw C-ABI call with its arguments prepared once, and the GPU span of the call's
kernels (HIP events around the call on the same stream), inputs in HBM.  Median over 20 calls.

    python scripts/c3_host_split.py
"""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "code-reproduction-ransac_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from bench import c3_problems  # noqa: E402

h2, h3, off, Ks = c3_problems()
p2 = torch.from_numpy(h2).cuda()
p3 = torch.from_numpy(h3).cuda()
P = off.size - 1
N = int(off[-1])


def wrapper():
    rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 1024, 30.0, adaptive=False, refine=False)


ctx = L.context(0)
Kf = np.ascontiguousarray(np.asarray(Ks, np.float64).reshape(P, 9))
offc = np.ascontiguousarray(off.astype(np.int64))
R = np.zeros((P, 9))
t = np.zeros((P, 3))
status = np.zeros(P, np.int32)
ninl = np.zeros(P, np.int32)
wrapper()
torch.cuda.synchronize()
# the flags the wrapper uses (adaptive off, refit off, device inputs / mask)
from rsac import api  # noqa: E402
fl = api._flags(False, False, "philox") | L.F_DEVICE_IN
mbuf, mptr, mflag = api._mask_buffer(api._In(p3, 3), N)
fl |= mflag
stream = api._stream_of(api._In(p3, 3))


def raw():
    L.check(L.lib().rsac_pnp_ransac_batched(ctx.handle, C.c_void_p(p3.data_ptr()), C.c_void_p(p2.data_ptr()),
                                            offc.ctypes.data, P, Kf.ctypes.data, 1024, 30.0, 0.99, 0x5EED, fl,
                                            R.ctypes.data, t.ctypes.data, status.ctypes.data, ninl.ctypes.data,
                                            C.c_void_p(mptr), stream))


def timed(f, n=20):
    w = []
    for i in range(n + 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        if i >= 3:
            w.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(w)


s = torch.cuda.current_stream()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
gs = []
for i in range(23):
    ev0.record(s)
    raw()
    ev1.record(s)
    torch.cuda.synchronize()
    if i >= 3:
        gs.append(ev0.elapsed_time(ev1))
print(f"c3 wrapper {timed(wrapper):.4f} ms, raw C call {timed(raw):.4f} ms, "
      f"events around the raw call {statistics.median(gs):.4f} ms", flush=True)
