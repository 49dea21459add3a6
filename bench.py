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

Also reported: ms-to-best-model (adaptive termination on, LM refit on, wall time of the full
rsac.pnp_ransac call), the scoring kernel's roofline (VALU issue: the binding roof, DESIGN.md
§3), the CPU restatement timed on this host (oracle/, 1 thread and OpenMP), and the other
BASELINE configs: at N = 1 in `extras` (C3, C4, C5, location search, DEM march); at N > 1 in
`multi_gpu` (C3 problem shards + all-gather, C5 sharded LO-RANSAC, sharded adaptive ms-to-best).

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
FLOP_PER_PAIR = 11  # k_pnp_score_mf: f32 flops of the VALU test per pair (q1, q2, D, t: 5 FMAs = 10 + 1 multiply)
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
    ap.add_argument("--cpu-hyps", type=int, default=100_000, help="CPU baseline sample (hypotheses, 1 thread)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0),
                    help="threads of the CPU baseline's multi-core leg (default: OMP_NUM_THREADS, else all cores)")
    ap.add_argument("--streams", type=int, default=2, help="contexts / HIP streams the steps alternate over "
                                                               "(1: one after another on one stream)")
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

    # steps are independent batches: they alternate between `--streams` rsac contexts (each its own
    # device scratch) on as many HIP streams, so step i + 1's solve starts on the CUs step i's
    # scoring tail frees (scripts/stream_pipe_ab.py: 0.262 vs 0.285 ms/step); --streams 1 is the
    # serial form, also measured below (ms_per_step_serial)
    nstreams = max(1, args.streams)
    ctxs = [rsac.context(local)] + [rsac.Context(local) for _ in range(nstreams - 1)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]

    def step(i=0, serial=False):
        # one pass over the batch, asynchronous end to end: solve + score + fused best key + the
        # winner's mask stay on the device; for N > 1 the key is all-reduced (RCCL, MAX) and every
        # rank re-derives the global winner's model and mask from it (rsac_pnp_winner), so no
        # step waits for the host
        j = 0 if serial else i % nstreams
        with torch.cuda.stream(streams[j]):
            key_t, model_t, mask = rsac.evaluate_range(ev.p2, ev.p3, K, base, H, args.thr, with_mask=True,
                                                       device_result=True, context=ctxs[j])
            if dist is None:
                return key_t
            if nccl:
                dist.all_reduce(key_t, op=dist.ReduceOp.MAX)
            else:  # gloo rehearsal: host round trip
                kc = key_t.cpu()
                dist.all_reduce(kc, op=dist.ReduceOp.MAX)
                key_t.copy_(kc)
            rsac.winner(ev.p2, ev.p3, K, key_t, args.thr, context=ctxs[j])
            return key_t

    # W untimed warmup steps, continued until at least WARMUP_MIN_S of them have run: the GPU's
    # clock ramps up under sustained load, and 10 steps after 3 warmup steps ran 13 % slower than
    # at steady state (0.367 vs 0.325 ms/step on one box); the timed region is still exactly K steps
    # (the extra count is agreed over the ranks, so every rank runs the same number of steps)
    t_w = time.perf_counter()
    for i in range(max(1, args.warmup)):
        step(i)
    torch.cuda.synchronize()
    spent = time.perf_counter() - t_w
    extra = max(0, math.ceil((WARMUP_MIN_S - spent) / (spent / max(1, args.warmup))))
    if dist is not None:
        ex = torch.tensor([extra], dtype=torch.int64, device=par._comm_device(None))
        dist.all_reduce(ex, op=dist.ReduceOp.MAX)
        extra = int(ex.item())
    for i in range(extra):
        step(i)
        if i % 16 == 15:
            torch.cuda.synchronize()  # keep the host within a few steps of the GPU

    def timed(serial):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            key_t = step(i, serial)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if dist is not None:
            et = torch.tensor([elapsed], dtype=torch.float64, device=par._comm_device(None))
            dist.all_reduce(et, op=dist.ReduceOp.MAX)
            elapsed = float(et.item())
        return elapsed, key_t

    elapsed, key_t = timed(False)
    elapsed_serial, key_serial = timed(True) if nstreams > 1 else (elapsed, key_t)
    cnt = int(key_t.item()) >> 32
    if int(key_serial.item()) != int(key_t.item()):
        raise RuntimeError("pipelined and serial steps picked different winners")
    # kernel times of the same call, from the HIP events of synchronous runs (outside the timed
    # loop): score_ms spans the scoring kernel alone (k_pnp_score_mf), solve_ms k_pnp_solve
    for _ in range(10):
        _, _, info = rsac.evaluate_range(ev.p2, ev.p3, K, base, H, args.thr, return_info=True, device=local)
        score_ms.append(info.score_ms)
        solve_ms.append(info.solve_ms)
    # N > 1: the other BASELINE configs across the ranks (collectives: every rank takes part)
    multi = multi_gpu_legs(local, args, pr) if (dist is not None and not args.no_extras) else None

    out = None
    if rank == 0:
        hyps_total = world * H * args.steps
        value = hyps_total / elapsed
        score_avg = statistics.mean(score_ms)
        solve_avg = statistics.mean(solve_ms)
        algo_gbs = args.points * BYTES_PER_POINT * H / (score_avg * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_score_kernel.json")
        if os.path.exists(pmc):
            try:
                d = json.load(open(pmc))
                if d.get("points") == args.points and d.get("hyps") == H:
                    traffic = d.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        # The binding roof of k_pnp_score_mf is VALU issue: the kernel re-reads its
        # 400 kB of point operands from L2, so HBM is far from busy.  achieved = VALU
        # wave-instructions per launch (SQ_INSTS_VALU, PMC pass of this same command,
        # profiles/pmc_score_valu.json) / the kernel's average duration measured here (HIP events
        # around the scoring kernel alone); peak = 1024 SIMDs x 1 wave64 instruction / 2 cycles at
        # 2.4 GHz.  HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE, profiles/pmc_score_kernel.json) and
        # its rate are reported beside it, and SURVEY §8d's algorithmic bytes (20 B per pair) as
        # a rate, which is not an HBM rate (it exceeds the HBM peak many times).
        pairs = args.points * H
        valu_instr = None
        pv = os.path.join(ROOT, "profiles", "pmc_score_valu.json")
        if os.path.exists(pv):
            try:
                d = json.load(open(pv))
                if d.get("points") == args.points and d.get("hyps") == H:
                    valu_instr = d["valu_instr_per_launch"]
            except Exception:
                valu_instr = None
        t_s = score_avg * 1e-3
        roofline = {"bound": "valu_issue", "kernel": "k_pnp_score_mf",
                    "span": "HIP events around the scoring kernel alone (k_pnp_score_mf; the k_best_key "
                            "reduction follows the second event), mean of 10 synchronous launches",
                    "kernel_ms": score_avg, "traffic": traffic,
                    "valu_instr_per_launch": valu_instr, "peak": VALU_ISSUE_PEAK / 1e9,
                    "unit": "G VALU wave-instructions/s"}
        if valu_instr:
            roofline.update({"achieved": valu_instr / t_s / 1e9, "frac": valu_instr / t_s / VALU_ISSUE_PEAK})
        else:
            roofline.update({"achieved": None, "frac": None, "note": "no PMC count for this workload"})
        if traffic:
            roofline.update({"hbm_gbs": traffic / t_s / 1e9, "hbm_frac": traffic / t_s / 1e9 / HBM_PEAK_GBS})
        roofline.update({"algorithmic_bytes_per_launch": args.points * BYTES_PER_POINT * H,
                         "algorithmic_gbs": algo_gbs,
                         "f32_vector_tflops": pairs * FLOP_PER_PAIR / t_s / 1e12,
                         "f32_vector_frac": pairs * FLOP_PER_PAIR / t_s / 1e12 / VALU_PEAK_TFLOPS})
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
            "ms_per_step_serial": elapsed_serial / args.steps * 1e3,
            "streams": nstreams,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic (rsac.synth.pnp_problem seed 0: UTM-scale points, main_v1.py K, N(0,1px) noise)",
            "config": {"workload": "C2: 10k 2D-3D correspondences, 50% outliers, P3P, thr 30 px, "
                                   f"{H} hypotheses per GPU per step, global best via RCCL all-reduce(MAX); "
                                   f"steps alternate over {nstreams} contexts / HIP streams",
                       "points": args.points, "hypotheses_per_gpu": H, "outlier_ratio": 0.5,
                       "parallelism": f"dp{world} (hypothesis shards)"},
            "ms_to_best_model": ms_to_best,
            "pcie_inclusive_hyp_s": pcie_rate,
            "best_inliers": int(cnt),
            "kernels_ms": {"pnp_solve": solve_avg, "pnp_score": score_avg},
            "roofline": roofline,
            "roofline_solve": sec_roofline("c2", "k_pnp_solve", solve_avg,
                                           "HIP events around the solve launch, mean of 10 synchronous launches"),
            "roofline_mfma": {"bound": "mfma", "flop_per_pair": MFMA_FLOP_PER_PAIR,
                              "achieved": pairs * MFMA_FLOP_PER_PAIR / t_s / 1e12,
                              "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": pairs * MFMA_FLOP_PER_PAIR / t_s / 1e12 / MFMA_PEAK_TFLOPS,
                              "note": "f16 matrix flops of the projection (hi/lo operands), dense peak"},
            "cpu_baseline": cpu,
            "extras": extras,
            "multi_gpu": multi,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return out


def c3_problems():
    """BASELINE.json configs[2]: 1024 problems x 2000 points (synth seeds 1..1024), concatenated."""
    probs = [synth.pnp_problem(2000, 0.5, seed=s) for s in range(1, 1025)]
    off = np.zeros(1025, np.int64)
    off[1:] = np.cumsum([len(p["points3d"]) for p in probs])
    return (np.concatenate([p["points2d"] for p in probs]), np.concatenate([p["points3d"] for p in probs]), off,
            np.stack([p["K"] for p in probs]))


def multi_gpu_legs(local, args, pr2):
    """N > 1 (every rank): the other BASELINE configs across the GPUs, each timed between barriers,
    max over ranks, median of 3 -- C3 (configs[2]: problem chunks per rank, one all-gather of the
    per-problem rows), C5 (configs[4]: sharded adaptive LO-RANSAC, per-round all-gather of the
    {status, count} rows), and ms-to-best-model of C2 through the sharded adaptive loop."""
    import torch.distributed as dist
    world = dist.get_world_size()
    dev = torch.device("cuda", local)
    sync = torch.cuda.synchronize
    out = {}
    # what the line runs on: backend, world size as the backend sees it, an 8-byte all-reduce's latency,
    # every rank's share of C3's problems and of C2's hypotheses
    out["comm"] = par.comm_report(1024, args.hyps * world, sync=sync)
    p2, p3, off, Ks = c3_problems()
    g2, g3 = torch.from_numpy(p2).to(dev), torch.from_numpy(p3).to(dev)
    run = par.pnp_batched_rows(g2, g3, off, Ks, 1024, args.thr, adaptive=False, refine=False)
    rows, w = par.c3_problem_shards(run, 1024, sync=sync, repeats=3)
    rows = rows.cpu().numpy()
    out["c3_problem_shards"] = {"problems": 1024, "points": 2000, "hyps_per_problem": 1024, "ms": w * 1e3,
                                "hyp_s": 1024 * 1024 / w, "problems_ok": int(rows[:, 0].sum()),
                                "inliers_total": int(rows[:, 1].sum()),
                                "note": f"{-(-1024 // world)} problems per rank, pnp_ransac_batched_flat on each "
                                        "rank's chunk (inputs in HBM), one all-gather of (ok, inliers, R, t) rows"}
    p5 = synth.pnp_problem(100_000, 0.5, seed=3)
    ev5 = par.PnPShard(p5["points2d"], p5["points3d"], p5["K"], args.thr, device=local)
    r5, w5 = par.adaptive_shards(ev5, 5000, 0.99, round_size=4096, lo=True, sync=sync)
    out["c5_sharded_lo"] = {"points": 100_000, "ms_to_best": w5 * 1e3, "best": r5.best, "iters": r5.iters,
                            "n_inliers": r5.n_inliers, "lo_improvements": r5.lo_improvements,
                            "note": "sharded_ransac(lo=True): round 1 (256 hypotheses, LO) redundantly on every "
                                    "rank with no collective; later rounds split over the ranks, all-gather of "
                                    "the rows (RCCL), device-listed scan, LO on every rank"}
    ev2 = par.PnPShard(pr2["points2d"], pr2["points3d"], pr2["K"], args.thr, device=local)
    r2, w2 = par.adaptive_shards(ev2, 5000, 0.99, round_size=4096, lo=False, sync=sync)
    out["ms_to_best_sharded"] = {"ms": w2 * 1e3, "best": r2.best, "iters": r2.iters, "n_inliers": r2.n_inliers,
                                 "note": "C2 problem, sharded_ransac (adaptive, no refit; round 1 redundantly on "
                                         "every rank with the device's speculative finish, no collective when it "
                                         "ends the scan), max over ranks"}
    return out


def sec_roofline(cfg, kernel, kernel_ms, span):
    """Roofline object of a secondary config's dominant kernel: VALU wave-instructions and HBM bytes
    per launch from profiles/pmc_secondary.json (scripts/gpu_secondary_profile.sh +
    scripts/summarize_secondary.py: its own --pmc passes of the same workload), divided by the
    launch's duration measured here (kernel_ms; `span` says how).  kernel_ms None: the kernel
    trace's mean duration from the same JSON.  kernel None: the config's dominant kernel (the
    largest share of the trace's kernel time)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_secondary.json")))
        ks = d["configs"][cfg]["kernels"]
        kernel = kernel or next(iter(ks))
        e = ks[kernel]
        tag = d["configs"][cfg].get("tag", d.get("tag"))
    except (OSError, KeyError, ValueError, StopIteration):
        return None
    src = "profile"
    if not kernel_ms:
        kernel_ms, src = e["mean_us"] / 1e3, "kernel trace mean (profiles/pmc_secondary.json)"
    t_s = kernel_ms * 1e-3
    r = {"bound": "valu_issue", "kernel": kernel, "kernel_ms": kernel_ms, "span": span if src == "profile" else src,
         "peak": VALU_ISSUE_PEAK / 1e9, "unit": "G VALU wave-instructions/s", "profile": tag,
         "share_of_kernel_time": e.get("share")}
    v = e.get("valu_instr_per_launch")
    if v:
        r.update({"valu_instr_per_launch": v, "achieved": v / t_s / 1e9, "frac": v / t_s / VALU_ISSUE_PEAK})
    h = e.get("hbm")
    if h:
        r.update({"traffic": h["traffic_bytes"], "hbm_gbs": h["traffic_bytes"] / t_s / 1e9,
                  "hbm_frac": h["traffic_bytes"] / t_s / 1e9 / HBM_PEAK_GBS, "write_bytes": e["write_kib"] * 1024})
    return r


def extra_workloads(local, args):
    """Secondary lines (not `value`): C3 of BASELINE.json (1024 problems x 2000 points, 1024
    hypotheses each, one batched call) and the 458-location search of main_v1.py:274/862."""
    out = {}
    h2, h3, off, Ks = c3_problems()
    dev = torch.device("cuda", local)
    p2 = torch.from_numpy(h2).to(dev)
    p3 = torch.from_numpy(h3).to(dev)

    def c3(p2_, p3_, calls=10, warm_s=0.3):
        # untimed calls for >= warm_s first: the clock ramps over the first ~20 calls
        # (scripts/c3_prof.py: 1.12 -> 0.90 ms per call), as for the main step's warmup
        t_end = time.perf_counter() + warm_s
        while True:
            rsac.pnp_ransac_batched_flat(p2_, p3_, off, Ks, 1024, args.thr, adaptive=False, refine=False)
            torch.cuda.synchronize()
            if time.perf_counter() >= t_end:
                break
        walls = []
        for i in range(calls):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.pnp_ransac_batched_flat(p2_, p3_, off, Ks, 1024, args.thr, adaptive=False, refine=False)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t)
        return statistics.median(walls)

    w = c3(p2, p3)
    wh = c3(p2.cpu().numpy(), p3.cpu().numpy())
    # the scoring kernel's span of one call (HIP events around its launch, rsac_set_timing)
    ctx = rsac.context(local)
    ctx.set_timing(True)
    rsac.pnp_ransac_batched_flat(p2, p3, off, Ks, 1024, args.thr, adaptive=False, refine=False)
    torch.cuda.synchronize()
    st3 = ctx.last_stats()
    ctx.set_timing(False)
    out["c3_batched"] = {"problems": 1024, "points": 2000, "hyps_per_problem": 1024, "ms": w * 1e3,
                         "hyp_s": 1024 * 1024 / w, "host_inputs_ms": wh * 1e3, "host_inputs_hyp_s": 1024 * 1024 / wh,
                         "score_ms": st3["score_ms"], "solve_ms": st3["solve_ms"],
                         "roofline": sec_roofline("c3", "k_pnp_score_mf<2>", st3["score_ms"],
                                                  "HIP events around the scoring launch of one call"),
                         "roofline_solve": sec_roofline("c3", "k_pnp_solve", st3["solve_ms"],
                                                        "HIP events around the solve launch of one call"),
                         "note": "inputs resident in HBM (and, second figure, handed over as host f64 arrays); "
                                 "per-problem winners + RANSAC masks, adaptive off, no refit"}
    # C5 (BASELINE.json configs[4]): LO-RANSAC, 100k correspondences, adaptive, inputs in HBM
    p5 = synth.pnp_problem(100_000, 0.5, seed=3)
    q2 = torch.from_numpy(p5["points2d"]).to(dev)
    q3 = torch.from_numpy(p5["points3d"]).to(dev)
    walls = []
    for i in range(12):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _, _, _, info = rsac.pnp_ransac(q2, q3, p5["K"], 5000, args.thr, lo=True, refine=True, return_info=True,
                                        device=local)
        torch.cuda.synchronize()
        if i >= 2:
            walls.append(time.perf_counter() - t)
    out["c5_lo_ransac"] = {"points": 100_000, "outlier_ratio": 0.5, "ms_to_best": statistics.median(walls) * 1e3,
                           "iters": info.iters, "n_inliers": info.n_inliers, "lo_improvements": info.lo_improvements,
                           "roofline_lo_chain": sec_roofline("c5", "k_pnp_refine", None, ""),
                           "note": "1 GPU; the multi-GPU form is rsac.parallel.sharded_ransac(lo=True); the LO "
                                   "chain's refits (k_pnp_refine) are latency-bound, see roofline_lo_chain"}
    # C4 (BASELINE.json configs[3]): fundamental matrix, 50k matches, 80 % outliers, 100k hypotheses
    p4 = synth.fundamental_problem(50_000, 0.8, seed=2)
    f1 = torch.from_numpy(p4["pts1"]).to(dev)
    f2 = torch.from_numpy(p4["pts2"]).to(dev)
    walls = []
    for i in range(8):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _, _, info4 = rsac.fundamental_ransac(f1, f2, 1.5, max_iters=100_000, adaptive=False, return_info=True,
                                              device=local)
        torch.cuda.synchronize()
        if i >= 2:
            walls.append(time.perf_counter() - t)
    w4 = statistics.median(walls)
    out["c4_fundamental"] = {"matches": 50_000, "outlier_ratio": 0.8, "hyps": 100_000, "ms": w4 * 1e3,
                             "hyp_s": 100_000 / w4, "n_inliers": info4.n_inliers, "score_ms": info4.score_ms,
                             "solve_ms": info4.solve_ms,
                             "roofline": sec_roofline("c4", "k_fm_score_q<8>", info4.score_ms,
                                                      "HIP events around the scoring launch (rsac_stats score_ms)"),
                             "roofline_solve": sec_roofline("c4", "k_fm_solve_g8", info4.solve_ms,
                                                            "HIP events around the solve launch (rsac_stats solve_ms)"),
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
                              "roofline": sec_roofline("loc", None, None, ""),
                              "note": "find_homographies of main_v1.py:254-297 (OpenCV-sampler RANSAC + LM refit + "
                                      "err1/err2) for every candidate, one call, host arrays; the roofline is the "
                                      "dominant kernel of the call's kernel trace (profiles/pmc_secondary.json 'loc'); "
                                      "CPU legs in cpu_baseline.location_search"}
    # the K sweep (testpro-K.py:39-162): 27 intrinsics x the 12 points, the reference's own mode
    # (EPnP-5 on MWC subsets, LM final solve), then solvePnPRefineLM of the winner; host arrays
    walls = []
    for i in range(8):
        t = time.perf_counter()
        ks = rsac.estimate_camera_orientation(synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, synth.TESTPRO_K_FOCALS,
                                              synth.TESTPRO_K_SENSORS, synth.TESTPRO_K_IMAGE, device=local,
                                              return_info=True)
        if i >= 2:
            walls.append(time.perf_counter() - t)
    fs = [(f, s) for f in synth.TESTPRO_K_FOCALS for s in synth.TESTPRO_K_SENSORS]
    out["k_sweep"] = {"intrinsics": len(fs), "points": 12, "ms": statistics.median(walls) * 1e3,
                      "pick": {"focal_mm": fs[ks.best][0], "sensor_mm": list(fs[ks.best][1])} if ks.best >= 0 else None,
                      "accepted": int(np.sum(np.asarray(ks.ok))),
                      "roofline": sec_roofline("ksweep", None, None, ""),
                      "note": "rsac.estimate_camera_orientation on testpro-K.py:198-234 (27 Ks: 9 focal lengths x "
                              "3 film cells), one call sequence: the batched RANSACs, the gate, the mean inlier "
                              "errors, the pick, the LM refit; median of 6; CPU legs in cpu_baseline.k_sweep"}
    # C3 at the per-rank loads of N = 8 / 4 / 2 / 1 GPUs (128 .. 1024 problems of 2000 points x 1024
    # hypotheses): the one-GPU curve the multi-GPU problem shards follow
    scal = {}
    for P in (128, 256, 512, 1024):
        n_pts = int(off[P])
        a2, a3 = p2[:n_pts], p3[:n_pts]
        ws = []
        for i in range(8):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.pnp_ransac_batched_flat(a2, a3, off[:P + 1], Ks[:P], 1024, args.thr, adaptive=False, refine=False)
            torch.cuda.synchronize()
            if i >= 2:
                ws.append(time.perf_counter() - t)
        w = statistics.median(ws)
        scal[str(P)] = {"ms": w * 1e3, "hyp_s": P * 1024 / w}
    out["c3_per_rank_loads"] = dict(scal, note="C3 problem shards as one GPU sees them at 8 / 4 / 2 / 1 ranks "
                                             "(128 / 256 / 512 / 1024 problems x 2000 points x 1024 hypotheses, "
                                             "one batched call, inputs in HBM, median of 6)")
    # the alternative split: every rank all 1024 problems, 1024 / N hypotheses each
    hsh = {}
    n_all = int(off[1024])
    for Hs in (128, 256, 512):
        ws = []
        for i in range(8):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rsac.pnp_ransac_batched_flat(p2[:n_all], p3[:n_all], off[:1025], Ks[:1024], Hs, args.thr, adaptive=False,
                                         refine=False)
            torch.cuda.synchronize()
            if i >= 2:
                ws.append(time.perf_counter() - t)
        w = statistics.median(ws)
        hsh[str(Hs)] = {"ms": w * 1e3, "hyp_s": 1024 * Hs / w}
    out["c3_hyp_shard_loads"] = dict(hsh, note="C3 hypothesis shards as one GPU would see them at 8 / 4 / 2 ranks "
                                             "(1024 problems x 2000 points x 128 / 256 / 512 hypotheses, one batched "
                                             "call, inputs in HBM, median of 6; the shards' winners would need one "
                                             "all-reduce per problem)")
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
                                                    "epnp (solvePnPRansac's final solve after SOLVEPNP_P3P)/epnp+lm")
    # the reference call's own mode on the C2 problem (main_v1.py:497-502: no flags = EPnP on 5-point
    # MWC samples, iterationsCount 5000, thr 30, conf 0.99, then the LM final solve): ms to the best
    # model, and the EPnP-5 minimal solver's throughput at a fixed 20k-hypothesis budget
    walls = []
    for i in range(25):
        # the plain call (R, t, mask), as the P3P leg: no stats, so no HIP timing events either
        t = time.perf_counter()
        rsac.pnp_ransac(g2, g3, p2c["K"], 5000, args.thr, sampler="opencv", minimal="epnp5", refine=True,
                        device=local)
        torch.cuda.synchronize()
        if i >= 4:
            walls.append((time.perf_counter() - t) * 1e3)
    _, _, mr, infr = rsac.pnp_ransac(g2, g3, p2c["K"], 5000, args.thr, sampler="opencv", minimal="epnp5",
                                     refine=True, return_info=True, device=local)
    walls_f, sol_f = [], []
    for i in range(13):  # the plain call timed (3 warm-up calls), the solve's HIP-event time from a stats call
        torch.cuda.synchronize()
        t = time.perf_counter()
        rsac.pnp_ransac(g2, g3, p2c["K"], 20_000, args.thr, minimal="epnp5", adaptive=False, refine=False,
                        device=local)
        torch.cuda.synchronize()
        if i >= 3:
            walls_f.append(time.perf_counter() - t)
    for i in range(3):
        _, _, _, inff = rsac.pnp_ransac(g2, g3, p2c["K"], 20_000, args.thr, minimal="epnp5", adaptive=False,
                                        refine=False, return_info=True, device=local)
        sol_f.append(inff.solve_ms)
    # the cost of OpenCV's Rodrigues round trip (RSAC_F_RVEC_ROUNDTRIP, on in the reference mode):
    # the same 20k EPnP-5 solve with and without it, HIP events around the solve launches
    rt_ms = {}
    for rv in (False, True):
        ms = []
        for i in range(5):
            _, _, _, inf_rt = rsac.pnp_ransac(g2, g3, p2c["K"], 20_000, args.thr, minimal="epnp5", adaptive=False,
                                              refine=False, rvec=rv, return_info=True, device=local)
            if i >= 1:
                ms.append(inf_rt.solve_ms)
        rt_ms[rv] = statistics.median(ms)
    out["c2_reference_mode"] = {"points": args.points, "ms_to_best": statistics.median(walls), "iters": infr.iters,
                                "n_inliers": infr.n_inliers, "epnp5_fixed_hyps": 20_000,
                                "epnp5_fixed_hyp_s": 20_000 / statistics.median(walls_f),
                                "epnp5_solve_ms": statistics.median(sol_f),
                                "epnp5_solve_ms_rvec_roundtrip": rt_ms[True], "epnp5_solve_ms_no_roundtrip": rt_ms[False],
                                "note": "cv2.solvePnPRansac defaults (EPnP-5 minimal solver on MWC subsets, LM final "
                                        "solve) on the C2 problem, inputs in HBM, median of 10; the EPnP-5 solve "
                                        "runs OpenCV's operation sequence as k_cvepnp5_a / k_cvepnp5_svd (the 12 x 12 "
                                        "JacobiSVD, six lanes per hypothesis) / k_cvepnp5_c; CPU leg in "
                                        "cpu_baseline.c2_reference_mode",
                                "roofline": sec_roofline("epnp", None, None, "")}
    # C1 (BASELINE.json configs[0], the reference plumbing): the reference call's own mode on its 12
    # testpro-K points under main_v1's K -- solvePnPRansac defaults (EPnP-5, MWC subsets, LM final
    # solve), 1000 iterations cap, thr 30; host arrays in and out, as the reference passes them
    K1 = synth.main_v1_K()
    walls = []
    for i in range(8):
        t = time.perf_counter()
        R1, t1, m1, info1 = rsac.pnp_ransac(synth.TESTPRO_K_PIXELS, synth.TESTPRO_K_POS3D, K1, 1000, 30.0,
                                            sampler="opencv", minimal="epnp5", refine=True, return_info=True,
                                            device=local)
        if i >= 1:
            walls.append(time.perf_counter() - t)
    out["c1_reference_mode"] = {"points": 12, "ms": statistics.median(walls) * 1e3, "iters": info1.iters,
                                "n_inliers": info1.n_inliers, "inliers": [int(k) for k in np.flatnonzero(m1)],
                                "note": "rsac.pnp_ransac with host arrays, sampler=opencv, minimal=epnp5, LM final "
                                        "solve (cv2.solvePnPRansac defaults), median of 7; CPU legs in "
                                        "cpu_baseline.c1"}
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


def _cpu_quota():
    """The CPU share of this process: (affinity CPUs, cgroup quota in CPUs or None)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return aff, quota


def _median_rate(fn, units, samples=5, warmup=0):
    """median over `samples` runs of units / seconds of fn(), after `warmup` untimed runs ->
    (rate, median seconds)"""
    for _ in range(warmup):
        fn()
    walls = []
    for _ in range(samples):
        t = time.perf_counter()
        fn()
        walls.append(time.perf_counter() - t)
    w = statistics.median(walls)
    return units / w, w


def cpu_baseline(pr, args):
    """The CPU restatement (oracle/, C, gcc -O3) on bounded samples of the same workloads, on this
    host: C2 on 1 thread (`value`), on the OMP_NUM_THREADS share and on every CPU of the affinity
    mask, C2 ms-to-best (OpenCV's sequential loop, stopping at the iteration bound; P3P and the
    reference's own EPnP-5 mode), C1 (BASELINE.json configs[0]: the reference plumbing, C
    restatement and the NumPy path, under main_v1's K and under testpro-K's f = 150 mm K), C3
    (problems over the threads), C4 (1 thread and the threads) and C5 (LO: OpenCV's sequential loop
    on 1 thread, and its rounds' hypotheses over the threads).  Throughput legs: median of 5
    samples; the short latency legs (C1, both ms-to-best legs): median of 21 after 3 warm-ups
    (BASELINE.md)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import np_ransac as NR
        import pyoracle as O
    except Exception as e:  # oracle not built
        return {"value": None, "error": str(e)}
    from concurrent.futures import ThreadPoolExecutor
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    threads = args.cpu_threads or env_threads or os.cpu_count() or 1
    aff, quota = _cpu_quota()
    soa = O.soa_pnp(pr["points3d"], pr["points2d"])
    cam = O.cam_from_K(pr["K"])
    n = max(1000, args.cpu_hyps // 5)
    O.pnp_hypotheses(soa, cam, args.thr, 0x5EED, 50)  # warm
    rate1, w1 = _median_rate(lambda: O.pnp_hypotheses(soa, cam, args.thr, 0x5EED, n), n)
    n_mt = 2000 * threads
    rate_mt, w_mt = _median_rate(lambda: O.pnp_hypotheses_mt(soa, cam, args.thr, 0x5EED, n_mt, threads=threads), n_mt)
    n_all = 500 * aff
    rate_all, w_all = _median_rate(lambda: O.pnp_hypotheses_mt(soa, cam, args.thr, 0x5EED, n_all, threads=aff), n_all)
    _, w_best = _median_rate(lambda: O.pnp_ransac_seq(pr["points3d"], pr["points2d"], pr["K"], args.thr, 0.99, 5000), 1,
                             samples=21, warmup=3)
    # the reference call's own mode on the same problem (EPnP-5 on MWC subsets, each model through
    # the Rodrigues round trip, main_v1.py:497-502)
    _, w_ref = _median_rate(lambda: O.pnp_ransac_seq(pr["points3d"], pr["points2d"], pr["K"], args.thr, 0.99, 5000,
                                                     sampler="opencv", minimal="epnp5"), 1, samples=21, warmup=3)
    # C1 (BASELINE.json configs[0]): the 12 testpro-K points (testpro-K.py:198-225) under main_v1's K
    # (main_v1.py:870-883), 1000 iterations, thr 30, the reference call's own mode (no flags:
    # EPnP on 5-point MWC samples, testpro-K.py:72 / main_v1.py:497)
    P3, P2, K1 = synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS, synth.main_v1_K()
    c1 = O.pnp_ransac_seq(P3, P2, K1, 30.0, 0.99, 1000, sampler="opencv", minimal="epnp5")
    _, w_c1 = _median_rate(lambda: O.pnp_ransac_seq(P3, P2, K1, 30.0, 0.99, 1000, sampler="opencv",
                                                    minimal="epnp5"), 1, samples=21, warmup=3)
    c1n = NR.pnp_ransac(P3, P2, K1, 30.0, 0.99, 1000, "epnp5")
    _, w_c1n = _median_rate(lambda: NR.pnp_ransac(P3, P2, K1, 30.0, 0.99, 1000, "epnp5"), 1, samples=21, warmup=3)
    # ... and under a K of testpro-K.py's sweep, as configs[0] words it: f = 150 mm on the 127 x 178 mm
    # cell (testpro-K.py:58-70), fx 2529.9, fy 1365.2 -- the K test_pro.py:801-802 hard-codes
    Kt = synth.testpro_k_candidates()[10]
    c1k = O.pnp_ransac_seq(P3, P2, Kt, 30.0, 0.99, 1000, sampler="opencv", minimal="epnp5")
    _, w_c1k = _median_rate(lambda: O.pnp_ransac_seq(P3, P2, Kt, 30.0, 0.99, 1000, sampler="opencv",
                                                     minimal="epnp5"), 1, samples=21, warmup=3)
    c1kn = NR.pnp_ransac(P3, P2, Kt, 30.0, 0.99, 1000, "epnp5")
    _, w_c1kn = _median_rate(lambda: NR.pnp_ransac(P3, P2, Kt, 30.0, 0.99, 1000, "epnp5"), 1, samples=21, warmup=3)
    # C3: 32 of the 1024 problems (seeds 1..32), 1024 hypotheses each, problems over the threads
    probs = [synth.pnp_problem(2000, 0.5, seed=s) for s in range(1, 33)]
    soas = [(O.soa_pnp(p["points3d"], p["points2d"]), O.cam_from_K(p["K"])) for p in probs]

    def c3_run():
        with ThreadPoolExecutor(max_workers=threads) as ex:
            list(ex.map(lambda sc: O.pnp_hypotheses(sc[0], sc[1], args.thr, 0x5EED, 1024), soas))

    rate_c3, w_c3 = _median_rate(c3_run, 32 * 1024)
    # C4: 300 fundamental-matrix hypotheses over the 50k matches, 1 thread
    p4 = synth.fundamental_problem(50_000, 0.8, seed=2)
    s4 = O.soa_hom(p4["pts1"], p4["pts2"])
    rate_c4, w_c4 = _median_rate(lambda: O.fm_hypotheses(s4, 1.5, 0x5EED, 300), 300)
    n4 = 60 * threads
    rate_c4mt, w_c4mt = _median_rate(lambda: O.fm_hypotheses_mt(s4, 1.5, 0x5EED, n4, threads=threads), n4)
    # C5: LO-RANSAC to the best model on the 100k-point problem, 1 thread, OpenCV's loop shape
    p5 = synth.pnp_problem(100_000, 0.5, seed=3)
    r5 = O.pnp_ransac_lo(p5["points3d"], p5["points2d"], p5["K"], args.thr, 0.99, 5000, lazy=True)
    _, w_c5 = _median_rate(lambda: O.pnp_ransac_lo(p5["points3d"], p5["points2d"], p5["K"], args.thr, 0.99, 5000,
                                                   lazy=True), 1)
    r5m = O.pnp_ransac_lo(p5["points3d"], p5["points2d"], p5["K"], args.thr, 0.99, 5000, threads=threads)
    _, w_c5mt = _median_rate(lambda: O.pnp_ransac_lo(p5["points3d"], p5["points2d"], p5["K"], args.thr, 0.99, 5000,
                                                     threads=threads), 1)
    # location search (main_v1.py:254-297): the reference's loop over the 458 candidates, each
    # find_homography (pos2, the C restatement's findHomography, the literal err1/err2 loop), 1 thread
    # and the candidates over the threads
    lp = synth.location_problem(seed=0)

    def loc_one(c):
        return O.find_homography(lp["pixels"], lp["pos3d"], c, 75.0)

    _, w_loc = _median_rate(lambda: [loc_one(c) for c in lp["locations"]], 1, samples=3)

    def loc_mt():
        with ThreadPoolExecutor(max_workers=threads) as ex:
            list(ex.map(loc_one, lp["locations"]))

    _, w_loc_mt = _median_rate(loc_mt, 1, samples=3)
    # the K sweep (testpro-K.py:39-162): 27 RANSACs + refits, 1 thread and the Ks over the threads
    Ks27 = synth.testpro_k_candidates()
    ks1 = O.estimate_camera_orientation(P3, P2, Ks27, threads=1)
    _, w_ks = _median_rate(lambda: O.estimate_camera_orientation(P3, P2, Ks27, threads=1), 1, samples=5)
    _, w_ks_mt = _median_rate(lambda: O.estimate_camera_orientation(P3, P2, Ks27, threads=min(threads, 27)), 1,
                              samples=5)
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = f"cgroup quota {quota:g} CPUs" if quota else "no cgroup quota"
    return {"value": rate1, "unit": "hypotheses/s", "cores": 1, "kind": "port",
            "sample": f"{n} hypotheses of the same C2 problem (10k points), oracle/rsac_oracle.c -O3, 1 thread, "
                      f"median of 5 ({w1:.2f} s each)",
            "cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "omp_num_threads_env": env_threads, "threads": threads,
            "c2_mt": {"value": rate_mt, "unit": "hypotheses/s", "cores": threads,
                      "sample": f"{n_mt} hypotheses, OpenMP over {threads} threads (OMP_NUM_THREADS share), "
                                f"median of 5 ({w_mt:.2f} s each)"},
            "c2_all_cpus": {"value": rate_all, "unit": "hypotheses/s", "cores": aff,
                            "sample": f"{n_all} hypotheses, OpenMP over all {aff} CPUs of the affinity mask "
                                      f"({share}), median of 5 ({w_all:.2f} s each)"},
            "c2_ms_to_best": {"ms": w_best * 1e3, "cores": 1,
                              "sample": "OpenCV's sequential loop (orc_pnp_ransac_seq), stops at the iteration "
                                        "bound, no refit, median of 21 after 3 warm-ups"},
            "c2_reference_mode": {"ms_to_best": w_ref * 1e3, "cores": 1,
                                  "sample": "orc_pnp_ransac_seq with EPnP-5 on MWC subsets (the reference call's "
                                            "defaults, each model through the Rodrigues round trip) on the C2 "
                                            "problem, stops at the iteration bound, no refit, median of 21 after 3 "
                                            "warm-ups"},
            "c1": {"ms_c": w_c1 * 1e3, "ms_numpy": w_c1n * 1e3, "cores": 1, "iters": c1["iters"],
                   "best": c1["best"], "n_inliers": c1["n_inliers"],
                   "inliers": [int(i) for i in np.flatnonzero(c1["mask"])],
                   "numpy_equal": bool(c1n["best"] == c1["best"] and np.array_equal(c1n["mask"], c1["mask"])),
                   "sample": "BASELINE configs[0]: 12 testpro-K points, main_v1 K, 1000 iterations cap, thr 30, "
                             "EPnP-5 on OpenCV's MWC subsets, sequential loop to the bound; C restatement "
                             "(orc_pnp_ransac_seq_k) and the NumPy path (oracle/np_ransac.py), ms per solve, "
                             "median of 21 after 3 warm-ups"},
            "c1_testpro_k": {"ms_c": w_c1k * 1e3, "ms_numpy": w_c1kn * 1e3, "cores": 1, "iters": c1k["iters"],
                             "best": c1k["best"], "n_inliers": c1k["n_inliers"],
                             "inliers": [int(i) for i in np.flatnonzero(c1k["mask"])],
                             "K": [float(Kt[0, 0]), float(Kt[1, 1]), float(Kt[0, 2]), float(Kt[1, 2])],
                             "numpy_equal": bool(c1kn["best"] == c1k["best"] and np.array_equal(c1kn["mask"],
                                                                                                c1k["mask"])),
                             "sample": "configs[0] with K from testpro-K.py (f 150 mm, 127 x 178 mm cell: the K "
                                       "test_pro.py:801-802 prints), otherwise as c1, median of 21 after 3 "
                                       "warm-ups"},
            "location_search": {"ms": w_loc * 1e3, "ms_mt": w_loc_mt * 1e3, "cores": 1, "cores_mt": threads,
                                "sample": "the 458 candidates of rsac.synth.location_problem: pyoracle.find_homography "
                                          "per candidate (main_v1.py:300-348 + 419 restated: pos2, the C findHomography "
                                          "with OpenCV's sampler + refit, the literal err1/err2 loop), 1 thread and "
                                          f"the candidates over {threads} threads, median of 3"},
            "k_sweep": {"ms": w_ks * 1e3, "ms_mt": w_ks_mt * 1e3, "cores": 1, "cores_mt": min(threads, 27),
                        "pick": int(ks1["best"]),
                        "sample": "pyoracle.estimate_camera_orientation on testpro-K.py:198-234 (27 Ks, EPnP-5 on "
                                  "MWC subsets, the oracle's LM refits), the Ks on 1 thread and over "
                                  f"{min(threads, 27)} threads, median of 5"},
            "c3": {"hyp_s": rate_c3, "cores": threads,
                   "sample": f"32 of the 1024 problems x 1024 hypotheses, problems over {threads} threads, "
                             f"median of 5 ({w_c3:.2f} s each)"},
            "c4": {"hyp_s": rate_c4, "cores": 1, "sample": f"300 hypotheses, 50k matches, median of 5 ({w_c4:.2f} s each)"},
            "c4_mt": {"hyp_s": rate_c4mt, "cores": threads,
                      "sample": f"{n4} hypotheses, 50k matches, OpenMP over {threads} threads "
                                f"(orc_fm_hypotheses_mt), median of 5 ({w_c4mt:.2f} s each)"},
            "c5": {"ms_to_best": w_c5 * 1e3, "iters": r5["iters"], "lo_improvements": r5["lo_improvements"],
                   "cores": 1, "sample": "orc_pnp_ransac_lo_seq on the 100k-point problem (each hypothesis "
                                         "evaluated when the scan reaches it, LO at every new best, stops at the "
                                         "bound), median of 5"},
            "c5_mt": {"ms_to_best": w_c5mt * 1e3, "iters": r5m["iters"], "lo_improvements": r5m["lo_improvements"],
                      "cores": threads,
                      "sample": f"orc_pnp_ransac_lo_mt: rounds of hypotheses (256 doubling to 4096) evaluated over "
                                f"{threads} OpenMP threads, each round scanned with its LO steps in order on one "
                                f"thread (OpenCV's loop is sequential: every new best moves the bound), median of "
                                f"5"}}


if __name__ == "__main__":
    main()
