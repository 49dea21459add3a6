#!/bin/bash
# fundamental-matrix parity tests + C4 timing (f32 pre-filter vs the f64 kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fundamental" --timeout 120 --timeout-method thread > gpurun_out/fm_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/fm_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u - <<'PY'
import sys, time
sys.path.insert(0, "code-reproduction-ransac_amd")
import torch, rsac
from rsac import synth
pr = synth.fundamental_problem(50000, 0.8, seed=2)
p1 = torch.from_numpy(pr["pts1"]).cuda(); p2 = torch.from_numpy(pr["pts2"]).cuda()
for ex in (False, True, False, True):
    F, m, info = rsac.fundamental_ransac(p1, p2, 1.5, max_iters=100000, adaptive=False, return_info=True, exact_only=ex) if False else (None, None, None)
    t = time.perf_counter()
    st, c, _ = rsac.hypotheses("fundamental", p1, p2, None, 0, 100000, 1.5, seed=0x5EED, exact_only=ex)
    torch.cuda.synchronize()
    print("exact_only" if ex else "f32 prefilter", "hypotheses() wall ms", round((time.perf_counter() - t) * 1e3, 2), "max count", c.max())
PY
