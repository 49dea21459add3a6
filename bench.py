#!/usr/bin/env python3
"""bench.py -- RANSAC hypotheses/sec on BASELINE.json config 2, 1..8 MI355X.

Workload (BASELINE.json configs[1]): one synthetic PnP
problem, 10 000 2D-3D correspondences shaped like the reference's UTM scene,
50 % outliers, P3P minimal solver, reprojection threshold 30 px
(main_v1.py:497-502), 100 000 hypotheses per GPU per step, inputs resident
in HBM.  A step = sample -> P3P -> score all 10k points for every hypothesis
of this rank's shard, global best by all-reduce(MAX) of the packed key
(count << 32 | ~index) over RCCL, then the winner's RANSAC-phase mask.
Weak scaling: rank r owns hypotheses [r*H, (r+1)*H) of the same Philox stream; the
exchange is rsac.parallel's all-reduce(MAX) of one int64 key; a rank that lost re-derives
the winner's model from its index (no broadcast).

Also reported: ms-to-best-model (adaptive termination on, LM refit on, wall
time of the full rsac.pnp_ransac call), the scoring kernel's roofline, and
the CPU restatement timed on this host (oracle/, 1 thread).

Launch: python bench.py [--gpus 1 --steps 10 --warmup 3]; for N > 1 the driver
runs it under torch.distributed.run with one rank per GPU.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "code-reproduction-ransac_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsac  # noqa: E402
from rsac import parallel as par  # noqa: E402
from rsac import synth  # noqa: E402

METRIC = "RANSAC hypotheses/sec + ms-to-best-model, 10k pts 50% outliers, 1/2/4/8 GPU"
BYTES_PER_POINT = 20  # f32 X, Y, Z, u, v
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec peak
WARMUP_MIN_S = 0.25  # minimum wall time of the untimed warmup steps (clock ramp)
VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, f32 vector peak
VALU_ISSUE_PEAK = 1024 * 0.5 * 2.4e9  # wave64 VALU instructions/s: 1024 SIMDs, 2 cycles each, 2.4 GHz
FLOP_PER_PAIR = 11  # k_pnp_score_mf: the VALU test per pair (q1, q2, D, t: 5 FMAs + 1 multiply)
MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md, dense f16 matrix peak
MFMA_FLOP_PER_PAIR = 32 * 32 * 16 * 2 / 256  # one v_mfma_f32_32x32x16_f16 per 8 hypotheses x 32 points


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points", type=int, default=10_000)
    ap.add_argument("--hyps", type=int, default=100_000, help="hypotheses per GPU per step")
    ap.add_argument("--thr", type=float, default=30.0)
    ap.add_argument("--cpu-hyps", type=int, default=150_000, help="CPU baseline sample (hypotheses, 1 thread)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ms-to-best", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the C3/C4/C5, location-search and DEM-march lines")
    ap.add_argument("--backend", default="nccl", help="process-group backend (nccl = RCCL; gloo only to rehearse "
                                                       "the N>1 path on fewer GPUs than ranks)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if args.backend != "nccl":
        local = local % max(1, torch.cuda.device_count())  # rehearsal: ranks may share a GPU
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    pr = synth.pnp_problem(args.points, 0.5, seed=0)
    K = pr["K"]
    H = args.hyps
    base = rank * H
    score_ms = []
    solve_ms = []

    ev = par.PnPShard(pr["points2d"], pr["points3d"], K, args.thr, device=local)
    nccl = dist is not None and args.backend == "nccl"

    def step():
        # one pass over the batch, asynchronous end to end: solve + score + fused best key + the
        # winner's mask stay on the device; for N > 1 the key is all-reduced (RCCL, MAX) and every
        # rank re-derives the global winner's model and mask from it (rsac_pnp_winner), so no
        # step waits for the host
        key_t, model_t, mask = rsac.evaluate_range(ev.p2, ev.p3, K, base, H, args.thr, with_mask=True,
                                                   device_result=True)
        if dist is None:
            return key_t
        if nccl:
            dist.all_reduce(key_t, op=dist.ReduceOp.MAX)
        else:  # gloo rehearsal: host round trip
            kc = key_t.cpu()
            dist.all_reduce(kc, op=dist.ReduceOp.MAX)
            key_t.copy_(kc)
        rsac.winner(ev.p2, ev.p3, K, key_t, args.thr)
        return key_t

    # W untimed warmup steps, continued until at least WARMUP_MIN_S of them have run: the GPU's
    # clock ramps up under sustained load, and 10 steps after 3 warmup steps ran 13 % slower than
    # at steady state (0.367 vs 0.325 ms/step on one box); the timed region is still exactly K steps
    # (the extra count is agreed over the ranks, so every rank runs the same number of steps)
    t_w = time.perf_counter()
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    spent = time.perf_counter() - t_w
    extra = max(0, math.ceil((WARMUP_MIN_S - spent) / (spent / max(1, args.warmup))))
    if dist is not None:
        ex = torch.tensor([extra], dtype=torch.int64, device=par._comm_device(None))
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        extra = int(ex.item())
    for i in range(extra):
        step()
        if i % 16 == 15:
            torch.cuda.synchronize()  # keep the host within a few steps of the GPU
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        key_t = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        et = torch.tensor([elapsed], dtype=torch.float64, device=par._comm_device(None))
        dist.all_reduce(et, op=dist.ReduceOp.MAX)
        elapsed = float(et.item())

    cnt = int(key_t.item()) >> 32
    # kernel times of the same call, from the HIP events of a synchronous run (outside the timed loop)
    for _ in range(3):
        _, _, info = rsac.evaluate_range(ev.p2, ev.p3, K, base, H, args.thr, return_info=True, device=local)
        score_ms.append(info.score_ms)
        solve_ms.append(info.solve_ms)

    out = None
    if rank == 0:
        hyps_total = world * H * args.steps
        value = hyps_total / elapsed
        score_avg = statistics.mean(score_ms)
        solve_avg = statistics.mean(solve_ms)
        achieved = args.points * BYTES_PER_POINT * H / (score_avg * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_score_kernel.json")
        if os.path.exists(pmc):
            try:
                d = json.load(open(pmc))
                if d.get("points") == args.points and d.get("hyps") == H:
                    traffic = d.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        # the issue-side roofline of the same launch: VALU wave-instructions per second (PMC count
        # of a profiled run of this command, profiles/pmc_score_valu.json) against the wave64
        # issue peak, 1024 SIMDs x 1 instruction / 2 cycles at the 2.4 GHz peak clock; and the
        # algorithmic f32 flops (31 per pair: the 16.5 instructions, FMAs counted twice) against
        # the 157.3 TFLOP/s vector peak
        roof_valu = None
        pv = os.path.join(ROOT, "profiles", "pmc_score_valu.json")
        pairs = args.points * H
        tflops = pairs * FLOP_PER_PAIR / (score_avg * 1e-3) / 1e12
        roof_valu = {"bound": "valu", "flop_per_pair": FLOP_PER_PAIR, "achieved_tflops": tflops,
                     "peak_tflops": VALU_PEAK_TFLOPS, "frac_flops": tflops / VALU_PEAK_TFLOPS}
        if os.path.exists(pv):
            try:
                d = json.load(open(pv))
                if d.get("points") == args.points and d.get("hyps") == H:
                    ips = d["valu_instr_per_launch"] / (score_avg * 1e-3)
                    roof_valu.update({"achieved": ips / 1e9, "peak": VALU_ISSUE_PEAK / 1e9, "unit": "G wave-instr/s",
                                      "frac": ips / VALU_ISSUE_PEAK,
                                      "valu_instr_per_launch": d["valu_instr_per_launch"],
                                      "effective_clock_ghz_profiled": d.get("effective_clock_ghz")})
            except Exception:
                pass
        ms_to_best = None
        if not args.no_ms_to_best:
            walls = []
            for i in range(23):
                # the plain call (R, t, mask): no stats, so no HIP timing events either
                t = time.perf_counter()
                R, t_, m = rsac.pnp_ransac(ev.p2, ev.p3, K, 5000, args.thr, confidence=0.99, adaptive=True,
                                           refine=True, device=local)
                torch.cuda.synchronize()
                if i >= 3:
                    walls.append((time.perf_counter() - t) * 1e3)
            ms_to_best = statistics.median(walls)
        # same step with the inputs handed over as host numpy arrays (f64 AoS -> pinned -> H2D ->
        # f32 SoA conversion on the device): the PCIe-inclusive rate, never `value`
        host_ms = []
        for i in range(8):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.evaluate_range(pr["points2d"], pr["points3d"], K, base, H, args.thr, with_mask=True, device=local)
            torch.cuda.synchronize()
            if i >= 2:
                host_ms.append((time.perf_counter() - t) * 1e3)
        pcie_rate = H / (statistics.median(host_ms) * 1e-3)
        extras = {} if (args.no_extras or world > 1) else extra_workloads(local, args)
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(pr, args)
            if "dem_ray_march" in extras:
                extras["dem_ray_march"]["cpu_baseline"] = cpu_baseline_dem(args)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "hypotheses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic (rsac.synth.pnp_problem seed 0: UTM-scale points, main_v1.py K, N(0,1px) noise)",
            "config": {"workload": "C2: 10k 2D-3D correspondences, 50% outliers, P3P, thr 30 px, "
                                   f"{H} hypotheses per GPU per step, global best via RCCL all-reduce(MAX)",
                       "points": args.points, "hypotheses_per_gpu": H, "outlier_ratio": 0.5,
                       "parallelism": f"dp{world} (hypothesis shards)"},
            "ms_to_best_model": ms_to_best,
            "pcie_inclusive_hyp_s": pcie_rate,
            "best_inliers": int(cnt),
            "kernels_ms": {"pnp_solve": solve_avg, "pnp_score": score_avg},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "scoring stage (HIP events): k_pnp_score_mf (flagged windows recounted inside, variant 98) + k_best_key",
                         "algorithmic_bytes_per_launch": args.points * BYTES_PER_POINT * H},
            "roofline_valu": roof_valu,
            "roofline_mfma": {"bound": "mfma", "flop_per_pair": MFMA_FLOP_PER_PAIR,
                              "achieved": pairs * MFMA_FLOP_PER_PAIR / (score_avg * 1e-3) / 1e12,
                              "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": pairs * MFMA_FLOP_PER_PAIR / (score_avg * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS,
                              "note": "f16 matrix flops of the projection (hi/lo operands), dense peak"},
            "cpu_baseline": cpu,
            "extras": extras,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return out


def extra_workloads(local, args):
    """Secondary lines (not `value`): C3 of BASELINE.json (1024 problems x 2000 points, 1024
    hypotheses each, one batched call) and the 458-location search of main_v1.py:274/862."""
    out = {}
    probs = [synth.pnp_problem(2000, 0.5, seed=s) for s in range(1, 1025)]
    off = np.zeros(1025, np.int64)
    off[1:] = np.cumsum([len(p["points3d"]) for p in probs])
    dev = torch.device("cuda", local)
    p2 = torch.from_numpy(np.concatenate([p["points2d"] for p in probs])).to(dev)
    p3 = torch.from_numpy(np.concatenate([p["points3d"] for p in probs])).to(dev)
    Ks = np.stack([p["K"] for p in probs])

    def c3(p2_, p3_):
        walls = []
        for i in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.pnp_ransac_batched_flat(p2_, p3_, off, Ks, 1024, args.thr, adaptive=False, refine=False)
            torch.cuda.synchronize()
            if i >= 1:
                walls.append(time.perf_counter() - t)
        return statistics.median(walls)

    w = c3(p2, p3)
    wh = c3(p2.cpu().numpy(), p3.cpu().numpy())
    out["c3_batched"] = {"problems": 1024, "points": 2000, "hyps_per_problem": 1024, "ms": w * 1e3,
                         "hyp_s": 1024 * 1024 / w, "host_inputs_ms": wh * 1e3, "host_inputs_hyp_s": 1024 * 1024 / wh,
                         "note": "inputs resident in HBM (and, second figure, handed over as host f64 arrays); "
                                 "per-problem winners + RANSAC masks, adaptive off, no refit"}
    # C5 (BASELINE.json configs[4]): LO-RANSAC, 100k correspondences, adaptive, inputs in HBM
    p5 = synth.pnp_problem(100_000, 0.5, seed=3)
    q2 = torch.from_numpy(p5["points2d"]).to(dev)
    q3 = torch.from_numpy(p5["points3d"]).to(dev)
    walls = []
    for i in range(6):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _, _, _, info = rsac.pnp_ransac(q2, q3, p5["K"], 5000, args.thr, lo=True, refine=True, return_info=True,
                                        device=local)
        torch.cuda.synchronize()
        if i >= 1:
            walls.append(time.perf_counter() - t)
    out["c5_lo_ransac"] = {"points": 100_000, "outlier_ratio": 0.5, "ms_to_best": statistics.median(walls) * 1e3,
                           "iters": info.iters, "n_inliers": info.n_inliers, "lo_improvements": info.lo_improvements,
                           "note": "1 GPU; the multi-GPU form is rsac.parallel.sharded_ransac(lo=True)"}
    # C4 (BASELINE.json configs[3]): fundamental matrix, 50k matches, 80 % outliers, 100k hypotheses
    p4 = synth.fundamental_problem(50_000, 0.8, seed=2)
    f1 = torch.from_numpy(p4["pts1"]).to(dev)
    f2 = torch.from_numpy(p4["pts2"]).to(dev)
    walls = []
    for i in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _, _, info4 = rsac.fundamental_ransac(f1, f2, 1.5, max_iters=100_000, adaptive=False, return_info=True,
                                              device=local)
        torch.cuda.synchronize()
        if i >= 1:
            walls.append(time.perf_counter() - t)
    w4 = statistics.median(walls)
    out["c4_fundamental"] = {"matches": 50_000, "outlier_ratio": 0.8, "hyps": 100_000, "ms": w4 * 1e3,
                             "hyp_s": 100_000 / w4, "n_inliers": info4.n_inliers, "score_ms": info4.score_ms,
                             "solve_ms": info4.solve_ms,
                             "note": "8-point + Sampson (f64), inputs in HBM, fixed budget (adaptive off)"}
    lp = synth.location_problem(seed=0)
    walls = []
    for i in range(6):
        t = time.perf_counter()
        rsac.location_search(lp["pos3d"], lp["pixels"], lp["locations"], 75.0, device=local)
        if i >= 1:
            walls.append(time.perf_counter() - t)
    out["location_search"] = {"locations": len(lp["locations"]), "features": len(lp["pos3d"]),
                              "ms": statistics.median(walls) * 1e3,
                              "note": "find_homographies of main_v1.py:254-297 (OpenCV-sampler RANSAC + LM refit + "
                                      "err1/err2) for every candidate, one call"}
    out["dem_ray_march"] = dem_workload(local)
    # the final solve on the C2 problem's inliers: ms-to-best-model for each refit choice
    p2c = synth.pnp_problem(args.points, 0.5, seed=0)
    g2 = torch.from_numpy(p2c["points2d"]).to(dev)
    g3 = torch.from_numpy(p2c["points3d"]).to(dev)
    fin = {}
    for mode in (False, "lm", "epnp", "epnp+lm"):
        walls = []
        for i in range(12):
            t = time.perf_counter()
            rsac.pnp_ransac(g2, g3, p2c["K"], 5000, args.thr, refine=mode, device=local)
            torch.cuda.synchronize()
            if i >= 2:
                walls.append((time.perf_counter() - t) * 1e3)
        fin[str(mode).lower()] = statistics.median(walls)
    out["final_solve_ms_to_best"] = dict(fin, note="pnp_ransac wall time, adaptive, C2 problem; refine=False/lm/"
                                                    "epnp (solvePnPRansac SOLVEPNP_P3P)/epnp+lm")
    return out


def dem_workload(local, n_rays=4096):
    """pixel_to_geo's march (main_v1.py:635-684) for n_rays pixels of a synthetic 577x577 SRTM-like
    DEM (rsac.synth.dem_problem), inputs in HBM, one call; kernel time by HIP events."""
    from rsac import dem
    pr = synth.dem_problem(n_rays, seed=0)
    g = dem.DemGrid.from_geotransform(pr["z"], pr["gt"])
    e, n = dem.wgs84_to_utm(pr["origin_lonlat"][None], device=local)[0]
    origin = np.array([e, n, pr["origin_height"]])
    dev = torch.device("cuda", local)
    d = torch.from_numpy(pr["dirs"]).to(dev)
    ms = []
    for i in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        hits, st = dem.ray_intersect_dem(origin, d, g)
        b.record()
        torch.cuda.synchronize()
        if i >= 1:
            ms.append(a.elapsed_time(b))
    st = st.cpu().numpy()
    h = hits.cpu().numpy()
    w = statistics.median(ms)
    # polygon-sized call (one 1898.json object's outline): latency, a block per ray
    d64 = d[:64].contiguous()
    ms64 = []
    for i in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        dem.ray_intersect_dem(origin, d64, g)
        b.record()
        torch.cuda.synchronize()
        if i >= 1:
            ms64.append(a.elapsed_time(b))
    steps_hit = np.rint(np.linalg.norm(h[st == 0] - origin, axis=1)) + 1
    return {"rays": n_rays, "ms": w, "rays_s": n_rays / w * 1e3, "hit": int((st == 0).sum()),
            "no_hit": int((st == 1).sum()), "off_dem": int((st == 2).sum()),
            "mean_steps_of_hits": float(steps_hit.mean()) if steps_hit.size else None,
            "rays64_ms": statistics.median(ms64),
            "note": "1 m steps, <=10000 per ray, UTM->WGS84 + bilinear DEM per step (f64); inputs in HBM"}


def cpu_baseline_dem(args, n_rays=3):
    """CPU leg for the DEM march: the literal per-ray loop of oracle/dem_oracle.py (numpy scalar
    steps + scipy RegularGridInterpolator, as main_v1.py:635-656) on a few rays of the same scene."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dem_oracle as D
    pr = synth.dem_problem(n_rays, seed=0)
    gt = pr["gt"]
    e, n = D.wgs84_to_utm(*pr["origin_lonlat"])
    o = np.array([e, n, pr["origin_height"]])
    interp = D.make_interpolator(pr["z"], gt[3], gt[5], gt[0], gt[1])
    t = time.perf_counter()
    for i in range(n_rays):
        D.ray_intersect_dem(o, pr["dirs"][i], interp)
    dt = time.perf_counter() - t
    return {"value": n_rays / dt, "unit": "rays/s", "cores": 1, "kind": "port",
            "sample": f"{n_rays} rays of the dem_ray_march scene, literal Python loop, {dt:.1f} s"}


def cpu_baseline(pr, args):
    """The CPU restatement (oracle/, C, 1 thread) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import pyoracle as O
    except Exception as e:  # oracle not built
        return {"value": None, "error": str(e)}
    soa = O.soa_pnp(pr["points3d"], pr["points2d"])
    cam = O.cam_from_K(pr["K"])
    n = args.cpu_hyps
    O.pnp_hypotheses(soa, cam, args.thr, 0x5EED, 50)  # warm
    t = time.perf_counter()
    O.pnp_hypotheses(soa, cam, args.thr, 0x5EED, n)
    dt = time.perf_counter() - t
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": n / dt, "unit": "hypotheses/s", "cores": 1, "kind": "port",
            "sample": f"{n} hypotheses of the same C2 problem (10k points), oracle/rsac_oracle.c -O2, 1 thread, "
                      f"{dt:.1f} s",
            "cpu_model": model, "os_cpu_count": os.cpu_count()}


if __name__ == "__main__":
    main()
