"""Host-side split of one reference-mode pnp_ransac call (C2 problem, device inputs): the Python
wrapper around the C-ABI call vs the call itself, by cProfile over repeated calls."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.pnp_problem(10000, 0.5, seed=0)
p2 = torch.from_numpy(pr["points2d"]).cuda()
p3 = torch.from_numpy(pr["points3d"]).cuda()
minimal = sys.argv[1] if len(sys.argv) > 1 else "epnp5"
sampler = sys.argv[2] if len(sys.argv) > 2 else "opencv"


def call():
    return rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, refine=True, minimal=minimal, sampler=sampler)


for _ in range(20):
    call()
torch.cuda.synchronize()
N = 300
t = time.perf_counter()
for _ in range(N):
    call()
    torch.cuda.synchronize()
print(f"{minimal}/{sampler}: {(time.perf_counter() - t) / N * 1e3:.4f} ms per call+sync", flush=True)
pr_ = cProfile.Profile()
pr_.enable()
for _ in range(N):
    call()
    torch.cuda.synchronize()
pr_.disable()
pstats.Stats(pr_).sort_stats("tottime").print_stats(14)

# the wrapper's torch calls one by one (us per call)
def per_call(f, n=20000):
    for _ in range(200):
        f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t) / n * 1e6


dev = p3.device
print("torch.empty u8        %.2f us" % per_call(lambda: torch.empty(10000, dtype=torch.uint8, device=dev)))
print("torch.empty bool      %.2f us" % per_call(lambda: torch.empty(10000, dtype=torch.bool, device=dev)))
m8 = torch.empty(10000, dtype=torch.uint8, device=dev)
print("view(bool)            %.2f us" % per_call(lambda: m8.view(dtype=torch.bool)))
print("current_stream        %.2f us" % per_call(lambda: torch.cuda.current_stream(dev).cuda_stream))
print("raw current stream    %.2f us" % per_call(lambda: torch._C._cuda_getCurrentRawStream(0)))
print("data_ptr              %.2f us" % per_call(lambda: p3.data_ptr()))
print("_In                   %.2f us" % per_call(lambda: rsac.api._In(p3, 3)))
print("_K9                   %.2f us" % per_call(lambda: rsac.api._K9(pr["K"])))
print("np.zeros(9)           %.2f us" % per_call(lambda: np.zeros(9)))
