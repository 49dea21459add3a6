cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "prefilter and ([25- or [26- or [27- or [28- or [30- or [32-)" --timeout 120 --timeout-method thread > gpurun_out/mx_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/mx_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/tune_score.py 23,25,26,27,28,30,32 > gpurun_out/mx_tune.log 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/mx_tune.log | tail -10
RSAC_MX_STATS=1 timeout -k 10 100 python -u -c "
import sys; sys.path.insert(0,'code-reproduction-ransac_amd')
import torch, rsac
from rsac import _lib as L, synth
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr['points3d']).cuda(); p2 = torch.from_numpy(pr['points2d']).cuda()
for v in (30, 31):
    L.check(L.lib().rsac_set_score_variant(v))
    rsac.evaluate_range(p2, p3, pr['K'], 0, 100000, 30.0, return_info=True)
" 2>&1 | grep -v amdgpu.ids
