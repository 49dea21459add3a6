"""A/B the scoring-kernel variants in one process (interleaved rounds, cdna guide rule 24)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import _lib as L  # noqa: E402
from rsac import synth  # noqa: E402

variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3,4,5,6".split(","))]
pr = synth.pnp_problem(10000, 0.5, seed=0)
p3 = torch.from_numpy(pr["points3d"]).cuda()
p2 = torch.from_numpy(pr["points2d"]).cuda()
H = 100_000
res = {v: [] for v in variants}
keys = {}
for rnd in range(int(os.environ.get("ROUNDS", "6"))):
    for v in variants:
        L.check(L.lib().rsac_set_score_variant(v))
        key, model, info = rsac.evaluate_range(p2, p3, pr["K"], 0, H, 30.0, return_info=True)
        keys.setdefault(v, key)
        if v not in (61, 68, 72, 78, 79):  # timing-only variants (no exact recount or no counts)
            assert key == keys[variants[0]], (v, key, keys)
        if rnd > 0:
            res[v].append(info.score_ms)
for v in variants:
    print(f"variant {v}: score_ms median {statistics.median(res[v]):.4f} min {min(res[v]):.4f}")
