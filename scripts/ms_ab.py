"""Interleaved A/B of librsac builds on ms-to-best (the reference-mode pnp_ransac call on the C2
problem: adaptive, LM refit), with --hyps the fixed-budget EPnP-5 solve rate, and with --c5 the
LO-RANSAC call on BASELINE configs[4] (100k correspondences).

    python scripts/ms_ab.py build/ab/librsac_a.so build/ab/librsac_b.so ... [--rounds 3]

Each (round, build) runs in its own process (RSAC_LIB_PATH selects the build), in the order
a b c a b c ..., so clock drift spreads over all builds.  Prints one JSON line per run and the
median over rounds of each run's median.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = (("epnp5", "opencv"), ("p3p", "philox"))


def worker(calls, hyps, c5=False):
    # RSAC_PKG_ROOT: another copy of the Python package (wrapper A/B runs); the library stays the tree's
    # (or RSAC_LIB_PATH's)
    sys.path[:0] = [os.environ.get("RSAC_PKG_ROOT") or os.path.join(ROOT, "code-reproduction-ransac_amd")]
    import torch
    import rsac
    from rsac import synth
    pr = synth.pnp_problem(10_000, 0.5, seed=0)
    dev = torch.device("cuda", 0)
    p2, p3 = torch.from_numpy(pr["points2d"]).to(dev), torch.from_numpy(pr["points3d"]).to(dev)
    out = {"lib": os.path.basename(os.environ.get("RSAC_LIB_PATH", ""))}
    for minimal, sampler in MODES:
        walls = []
        for i in range(calls + 5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, adaptive=True, refine=True, minimal=minimal,
                            sampler=sampler)  # the plain call: no stats, no timing events
            torch.cuda.synchronize()
            if i >= 5:
                walls.append((time.perf_counter() - t) * 1e3)
        R, t_, m, info = rsac.pnp_ransac(p2, p3, pr["K"], 5000, 30.0, adaptive=True, refine=True, minimal=minimal,
                                         sampler=sampler, return_info=True)
        out[f"{minimal}_{sampler}"] = statistics.median(walls)
        out[f"{minimal}_{sampler}_key"] = [info.iters, int(m.sum())]
    if hyps:
        walls = []
        for i in range(8):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.pnp_ransac(p2, p3, pr["K"], hyps, 30.0, adaptive=False, refine=False, minimal="epnp5")
            torch.cuda.synchronize()
            if i >= 3:
                walls.append((time.perf_counter() - t) * 1e3)
        out["epnp5_fixed_hyp_s"] = hyps / statistics.median(walls) * 1e3
    if c5:
        p5 = synth.pnp_problem(100_000, 0.5, seed=3)
        q2, q3 = torch.from_numpy(p5["points2d"]).to(dev), torch.from_numpy(p5["points3d"]).to(dev)
        walls = []
        for i in range(calls + 3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            R, t_, m = rsac.pnp_ransac(q2, q3, p5["K"], 5000, 30.0, lo=True, refine=True)
            torch.cuda.synchronize()
            if i >= 3:
                walls.append((time.perf_counter() - t) * 1e3)
        out["c5_lo"] = statistics.median(walls)
        out["c5_lo_key"] = [int(m.sum())]
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--hyps", type=int, default=0)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--c5", action="store_true")
    a = ap.parse_args()
    if a.worker:
        worker(a.calls, a.hyps, a.c5)
        return
    res = {lib: [] for lib in a.libs}
    for _ in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, RSAC_LIB_PATH=os.path.abspath(lib))
            r = subprocess.run([sys.executable, "-u", __file__, "--worker", "--calls", str(a.calls), "--hyps",
                                str(a.hyps)] + (["--c5"] if a.c5 else []), env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(r.stdout, r.stderr, flush=True)
                sys.exit(r.returncode)
            line = r.stdout.strip().splitlines()[-1]
            print(line, flush=True)
            res[lib].append(json.loads(line))
    keys = [k for k in res[a.libs[0]][0] if k != "lib" and not k.endswith("_key")]
    print("summary (median over rounds):", " ".join(keys))
    for lib, v in res.items():
        print(f"  {os.path.basename(lib):28s} " + " ".join(f"{statistics.median(x[k] for x in v):.4g}" for k in keys))


if __name__ == "__main__":
    main()
