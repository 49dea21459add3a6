"""Interleaved A/B of librsac builds on the C2 step (scoring kernel time + async step time).

    python scripts/mf_ab.py build/ab/a.so build/ab/b.so ... [--rounds 3]

Each (round, build) runs in its own process (RSAC_LIB_PATH selects the build), in the order
a b c a b c ..., so clock drift spreads over all builds.  Prints one JSON line per run and a
summary (median over rounds of each run's median).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(calls, steps, c3_calls=0):
    sys.path[:0] = [os.path.join(ROOT, "code-reproduction-ransac_amd")]
    import torch
    import rsac
    from rsac import parallel as par
    from rsac import synth
    pr = synth.pnp_problem(10_000, 0.5, seed=0)
    K = pr["K"]
    ev = par.PnPShard(pr["points2d"], pr["points3d"], K, 30.0, device=0)
    H = 100_000

    def step():
        return rsac.evaluate_range(ev.p2, ev.p3, K, 0, H, 30.0, with_mask=True, device_result=True)

    t = time.perf_counter()
    while time.perf_counter() - t < 1.0:
        step()
        torch.cuda.synchronize()
    sc, so = [], []
    for _ in range(calls):
        _, _, info = rsac.evaluate_range(ev.p2, ev.p3, K, 0, H, 30.0, return_info=True, device=0)
        sc.append(info.score_ms)
        so.append(info.solve_ms)
    torch.cuda.synchronize()
    prof = None
    L = rsac._lib.lib()
    if hasattr(L, "rsac_debug_mf_prof"):  # phase-timing build (RSAC_MF_V & 32): one call's phase sums
        import ctypes as C
        buf = (C.c_ulonglong * 8)()
        L.rsac_debug_mf_prof(buf, 1)
        rsac.evaluate_range(ev.p2, ev.p3, K, 0, H, 30.0, return_info=True, device=0)
        L.rsac_debug_mf_prof(buf, 1)
        tot = sum(buf[:5])
        prof = {n: round(buf[i] / tot, 4) for i, n in enumerate(["stage", "loop", "recount", "epilogue", "queue"])}
    t0 = time.perf_counter()
    for _ in range(steps):
        k = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    c3 = None
    if c3_calls:  # C3 (configs[2]) wall time per call, inputs in HBM
        sys.path.insert(0, ROOT)
        from bench import c3_problems
        h2, h3, off, Ks = c3_problems()
        g2, g3 = torch.from_numpy(h2).cuda(), torch.from_numpy(h3).cuda()
        walls = []
        for i in range(c3_calls + 3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = rsac.pnp_ransac_batched_flat(g2, g3, off, Ks, 1024, 30.0, adaptive=False, refine=False)
            torch.cuda.synchronize()
            if i >= 3:
                walls.append((time.perf_counter() - t) * 1e3)
        c3 = {"ms": statistics.median(walls), "ninl_sum": int(out[3].sum())}
    print(json.dumps({"lib": os.environ.get("RSAC_LIB_PATH"), "score_ms": statistics.median(sc),
                      "score_min": min(sc), "solve_ms": statistics.median(so), "step_ms": ms,
                      "key": [int(k[0].item()), c3 and c3["ninl_sum"]], "c3_ms": c3 and c3["ms"],
                      "prof": prof}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--c3", type=int, default=0, help="also time this many C3 calls per run")
    a = ap.parse_args()
    if a.worker:
        worker(a.calls, a.steps, a.c3)
        return
    res = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, RSAC_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, "-u", __file__, "--worker", "--calls", str(a.calls), "--steps",
                                  str(a.steps), "--c3", str(a.c3)], env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout, out.stderr, flush=True)
                sys.exit(out.returncode)
            line = out.stdout.strip().splitlines()[-1]
            print(line, flush=True)
            res[lib].append(json.loads(line))
    keys = {json.dumps(v[0]["key"]) for v in res.values()}
    print("summary (median over rounds): lib score_ms step_ms solve_ms [c3_ms]; keys agree:", len(keys) == 1)
    for lib, v in res.items():
        c3 = f" {statistics.median(x['c3_ms'] for x in v):.4f}" if a.c3 else ""
        print(f"  {os.path.basename(lib):24s} {statistics.median(x['score_ms'] for x in v):.4f} "
              f"{statistics.median(x['step_ms'] for x in v):.4f} {statistics.median(x['solve_ms'] for x in v):.4f}{c3}")


if __name__ == "__main__":
    main()
