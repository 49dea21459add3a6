"""Worker of test_dist_rehearsal.py (TEST INFRASTRUCTURE): one rank of a CPU rehearsal of bench.py's
multi-GPU legs, launched by `python -m torch.distributed.run --nproc-per-node 2 ...` with gloo.

It drives the same rsac.parallel functions bench.py calls at N > 1 -- c3_problem_shards (C3:
problem chunks + one all-gather of the rows) and adaptive_shards (C5: sharded LO-RANSAC;
ms-to-best: the sharded adaptive loop) -- with evaluators backed by the CPU restatement (oracle/)
instead of the GPU kernels, and writes rank r's results to <out>/rank<r>.json.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "code-reproduction-ransac_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pyoracle as O  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

C3_PROBLEMS, C3_POINTS, C3_HYPS = 16, 500, 256
C5_POINTS = 20000


class OracleShard:
    """PnPShard's interface, computed by oracle/."""

    def __init__(self, pr, thr=30.0, seed=0x5EED):
        self.soa = O.soa_pnp(pr["points3d"], pr["points2d"])
        self.cam = O.cam_from_K(pr["K"])
        self.thr, self.seed = thr, seed
        self.n = len(self.soa[0])

    def hypotheses(self, begin, count):
        counts, status = O.pnp_hypotheses(self.soa, self.cam, self.thr, self.seed, count, hyp0=begin)
        return status, counts

    def model(self, index):
        _, _, m = O.pnp_hypotheses(self.soa, self.cam, self.thr, self.seed, 1, hyp0=index, models=True)
        return m[0, :12].copy()

    def local_opt(self, model12, count):
        R, t, c, steps = O.pnp_local_opt(self.soa, self.cam, self.thr, model12[:9], model12[9:12], count)
        return np.concatenate([R.reshape(9), t]), c, steps


def c3_run_local(probs):
    def run(begin, count):
        rows = np.zeros((count, 14))
        for i in range(count):
            p = probs[begin + i]
            r = O.pnp_ransac(p["points3d"], p["points2d"], p["K"], 30.0, 0.99, C3_HYPS)
            if r["best"] >= 0:
                rows[i] = [1, r["n_inliers"], *r["R"].reshape(9), *r["t"]]
        return rows
    return run


def main():
    out = sys.argv[1]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    try:
        probs = [synth.pnp_problem(C3_POINTS, 0.5, seed=s) for s in range(1, C3_PROBLEMS + 1)]
        rows, _ = par.c3_problem_shards(c3_run_local(probs), C3_PROBLEMS, repeats=1)
        c5 = OracleShard(synth.pnp_problem(C5_POINTS, 0.5, seed=3))
        lo, _ = par.adaptive_shards(c5, 5000, 0.99, round_size=512, lo=True, repeats=1)
        ada, _ = par.adaptive_shards(OracleShard(synth.pnp_problem(3000, 0.7, seed=12)), 5000, 0.99, round_size=256,
                                     lo=False, repeats=1)
        comm = par.comm_report(C3_PROBLEMS, 1000, samples=10)
        comm.pop("rank")
        comm.pop("allreduce_8b_us")  # timing: differs between ranks only before the max
        res = {"comm": comm, "c3": rows.cpu().numpy().tolist(),
               "c5": [lo.best, lo.n_inliers, lo.iters, lo.lo_improvements, lo.model.tolist()],
               "ada": [ada.best, ada.n_inliers, ada.iters, ada.model.tolist()]}
        json.dump(res, open(os.path.join(out, f"rank{rank}.json"), "w"))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
