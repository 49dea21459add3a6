"""Interleaved A/B of two copies of the Python package (the same librsac.so) on ms-to-best:
    python scripts/py_ab.py PKG_ROOT_A PKG_ROOT_B [--rounds 4]
Each (round, package) runs scripts/ms_ab.py's worker in its own process with RSAC_PKG_ROOT set and
RSAC_LIB_PATH = the tree's library."""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("pkgs", nargs=2)
ap.add_argument("--rounds", type=int, default=4)
a = ap.parse_args()
lib = os.path.join(ROOT, "code-reproduction-ransac_amd", "rsac", "librsac.so")
res = {p: [] for p in a.pkgs}
for _ in range(a.rounds):
    for p in a.pkgs:
        env = dict(os.environ, RSAC_PKG_ROOT=os.path.abspath(p), RSAC_LIB_PATH=lib)
        r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "scripts", "ms_ab.py"), "--worker", "--calls", "40",
                            "--hyps", "0"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stdout, r.stderr)
            sys.exit(r.returncode)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["pkg"] = p
        print(json.dumps(d), flush=True)
        res[p].append(d)
for p, v in res.items():
    print(p, "p3p", round(statistics.median(x["p3p_philox"] for x in v), 5), "epnp5",
          round(statistics.median(x["epnp5_opencv"] for x in v), 4))
