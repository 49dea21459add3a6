"""r06 debug: the one count the MFMA scorer gets wrong on the degenerate-plane EPnP-5 scene."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("oracle", "code-reproduction-ransac_amd", "tests")]
import pyoracle as O
import rsac
from rsac import synth
from test_epnp5 import _mwc5
pr = synth.pnp_problem(300, 0.3, seed=5)
P3 = pr["points3d"].copy(); P3[::2, 2] = 700.0
soa, cam = O.soa_pnp(P3, pr["points2d"]), O.cam_from_K(pr["K"])
subs, sst = _mwc5(300, 4096)
oc, os_, om = O.pnp_hypotheses(soa, cam, 30.0, 0, 4096, subsets=subs, sub_status=sst, models=True, minimal="epnp5")
st, cn, md = rsac.hypotheses("pnp", P3, pr["points2d"], pr["K"], 0, 4096, 30.0, subsets=subs, minimal="epnp5")
st2, cn2, md2 = rsac.hypotheses("pnp", P3, pr["points2d"], pr["K"], 0, 4096, 30.0, subsets=subs, minimal="epnp5", exact_only=True)
bad = np.flatnonzero(cn != oc)
print("mismatch", bad, cn[bad], oc[bad], "exact_only", cn2[bad], "exact_only mism", np.flatnonzero(cn2 != oc))
np.set_printoptions(precision=17)
for b in bad:
    print("model", repr(md[b, :12]), "oracle", repr(om[b, :12]), "bits equal", np.array_equal(md[b, :12].view(np.uint64), om[b, :12].view(np.uint64)))
    R = md[b, :9].reshape(3, 3); t = md[b, 9:12]
    X = P3 @ R.T + t
    print("z range", X[:, 2].min(), X[:, 2].max())
