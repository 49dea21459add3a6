"""Profile helper: C4 scoring (50k matches, 80 % outliers, 100k hypotheses), f32 pre-filter and f64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import synth  # noqa: E402

pr = synth.fundamental_problem(50000, 0.8, seed=2)
p1 = torch.from_numpy(pr["pts1"]).cuda()
p2 = torch.from_numpy(pr["pts2"]).cuda()
for ex in (False, True) * 3:
    rsac.hypotheses("fundamental", p1, p2, None, 0, 100000, 1.5, seed=0x5EED, exact_only=ex)
