"""Decision-change study of the PnP restatement (test infrastructure; CPU only).

How far is the oracle's EPnP-5 (the minimal solver of every reference PnP call: cv2.solvePnPRansac
with default flags, main_v1.py:497-502, testpro-K.py:72-75) from OpenCV's own operation sequence,
and does the difference change a RANSAC decision?  Three restatements (oracle/pyoracle.py
SEQUENCES):
  cv          OpenCV's sequence (oracle/cv_epnp.c: undistortPoints f32 round trip, raw-centroid
              control points, cvMulTransposed, one-sided Jacobi SVD, cvSolve(SVD) betas, qr_solve
              Gauss-Newton, SVD rotation; cvRodrigues2 through cvSVD)
  rr          rounds 4-5 (round-robin Jacobi, Householder betas, polar rotation, fused steps)
  rr_unfused  rr with every explicit fma as a rounded product + a rounded sum
on
  C1      the 12 testpro-K points (testpro-K.py:198-225) under its 27 intrinsics + main_v1's K:
          per-hypothesis counts over 5000 MWC subsets, and the RANSAC decision (best, iterations,
          mask) of each K;
  K sweep estimate_camera_orientation (testpro-K.py:39-162): the K each rule picks, and where
          f = 150 mm, 127 x 178 mm (test_pro.py:801-802's fx=2529, fy=1365) ranks under both;
  C2      the 10k-point problem (BASELINE configs[1]), 20k MWC 5-point subsets: per-hypothesis count
          differences, and the adaptive RANSAC decision.
Writes profiles/r06/epnp_variants.json and .md.  Usage: python scripts/epnp_variants.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "code-reproduction-ransac_amd")]
import pyoracle as O  # noqa: E402
from rsac import synth  # noqa: E402

SEQS = ("cv", "rr", "rr_unfused")
PAIRS = (("cv", "rr"), ("cv", "rr_unfused"), ("rr", "rr_unfused"))


def c1_cases():
    Ks = list(synth.testpro_k_candidates())
    names = [f"f{f} {w}x{h}" for f in synth.TESTPRO_K_FOCALS for (w, h) in synth.TESTPRO_K_SENSORS]
    return Ks + [synth.main_v1_K()], names + ["main_v1"]


def hyp_counts(P3, P2, K, H, seq):
    soa = O.soa_pnp(P3, P2)
    subs, sst = O.mwc_subsets(len(P3), H, s=5)
    with O.sequence(seq):
        counts, status = O.pnp_hypotheses(soa, O.cam_from_K(K), 30.0, 0, H, subsets=subs, sub_status=sst,
                                          minimal="epnp5", rvec=True)
    return counts, status


def ransac(P3, P2, K, seq, max_iters=5000):
    with O.sequence(seq):
        r = O.pnp_ransac(P3, P2, K, 30.0, 0.99, max_iters, 0x5EED, sampler="opencv", minimal="epnp5")
    return dict(best=r["best"], iters=r["iters"], n_inliers=r["n_inliers"],
                inliers=np.flatnonzero(r["mask"]).tolist())


def sweep(seq):
    Ks = synth.testpro_k_candidates()
    P3, P2 = synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS
    with O.sequence(seq):
        res = O.estimate_camera_orientation(P3, P2, Ks)
    names = [(f, s) for f in synth.TESTPRO_K_FOCALS for s in synth.TESTPRO_K_SENSORS]
    acc = []
    for k, row in enumerate(res["rows"]):
        if row is None or not np.isfinite(row.get("mean", np.nan)):
            continue
        with O.sequence(seq):
            Rp = O.rodrigues_v2m(O.rodrigues_m2v(row["R"]))
        origin = -Rp.T @ row["t"]
        acc.append(dict(k=k, f=names[k][0], sensor=list(names[k][1]), mean=row["mean"], n_inliers=row["n_inliers"],
                        dist=float(np.linalg.norm(origin - synth.TESTPRO_K_ORIGIN))))
    by_err = sorted(acc, key=lambda a: a["mean"])
    by_dist = sorted(acc, key=lambda a: a["dist"])
    hint = [i for i, a in enumerate(acc) if a["f"] == 150 and a["sensor"] == [127, 178]]

    def rank(order):
        for i, a in enumerate(order):
            if a["f"] == 150 and a["sensor"] == [127, 178]:
                return i + 1
        return None
    pick = names[res["best"]] if res["best"] >= 0 else None
    return dict(pick=None if pick is None else dict(f=pick[0], sensor=list(pick[1])), accepted=len(acc),
                hint_accepted=bool(hint), hint_rank_by_error=rank(by_err), hint_rank_by_distance=rank(by_dist),
                hint_mean=acc[hint[0]]["mean"] if hint else None,
                top_by_distance=[dict(f=a["f"], sensor=a["sensor"], dist=round(a["dist"], 2), mean=round(a["mean"], 3))
                                 for a in by_dist[:6]],
                top_by_error=[dict(f=a["f"], sensor=a["sensor"], mean=round(a["mean"], 3), n_inliers=a["n_inliers"])
                              for a in by_err[:6]])


def main():
    t0 = time.time()
    out = dict(sequences=SEQS)
    Ks, names = c1_cases()
    P3, P2 = synth.TESTPRO_K_POS3D, synth.TESTPRO_K_PIXELS
    # C1: per-hypothesis counts and decisions
    c1 = dict(hyp_diff={f"{a}|{b}": 0 for a, b in PAIRS}, hyps=0, decision_diff={f"{a}|{b}": [] for a, b in PAIRS},
              cases=[])
    for K, nm in zip(Ks, names):
        cnt = {s: hyp_counts(P3, P2, K, 5000, s)[0] for s in SEQS}
        dec = {s: ransac(P3, P2, K, s) for s in SEQS}
        c1["hyps"] += 5000
        for a, b in PAIRS:
            c1["hyp_diff"][f"{a}|{b}"] += int(np.count_nonzero(cnt[a] != cnt[b]))
            if dec[a] != dec[b]:
                c1["decision_diff"][f"{a}|{b}"].append(nm)
        c1["cases"].append(dict(K=nm, **{s: dec[s] for s in SEQS}))
    out["c1"] = c1
    # K sweep
    out["k_sweep"] = {s: sweep(s) for s in SEQS}
    # C2
    pr = synth.pnp_problem(10_000, 0.5, seed=0)
    cnt = {s: hyp_counts(pr["points3d"], pr["points2d"], pr["K"], 20_000, s) for s in SEQS}
    c2 = dict(hyps=20_000, hyp_diff={}, max_abs_count_diff={}, decisions={})
    for a, b in PAIRS:
        d = cnt[a][0] != cnt[b][0]
        c2["hyp_diff"][f"{a}|{b}"] = int(np.count_nonzero(d))
        c2["max_abs_count_diff"][f"{a}|{b}"] = int(np.max(np.abs(cnt[a][0] - cnt[b][0])))
    for s in SEQS:
        r = ransac(pr["points3d"], pr["points2d"], pr["K"], s)
        c2["decisions"][s] = dict(best=r["best"], iters=r["iters"], n_inliers=r["n_inliers"])
    masks = {s: ransac(pr["points3d"], pr["points2d"], pr["K"], s)["inliers"] for s in SEQS}
    c2["mask_equal"] = {f"{a}|{b}": masks[a] == masks[b] for a, b in PAIRS}
    out["c2"] = c2
    out["seconds"] = round(time.time() - t0, 1)
    os.makedirs(os.path.join(ROOT, "profiles", "r06"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r06", "epnp_variants.json"), "w") as f:
        json.dump(out, f, indent=1)
    md = ["# EPnP-5 restatements: decision changes (scripts/epnp_variants.py)", ""]
    md.append("Per-hypothesis inlier counts that differ, over MWC 5-point subsets (every model through the "
              "Rodrigues round trip):")
    md.append("")
    md.append("| pair | C1 (28 K x 5000 hyps) | C2 (20k hyps) | C2 max abs count diff |")
    md.append("|---|---|---|---|")
    for a, b in PAIRS:
        k = f"{a}|{b}"
        md.append(f"| {a} vs {b} | {c1['hyp_diff'][k]} | {c2['hyp_diff'][k]} | {c2['max_abs_count_diff'][k]} |")
    md.append("")
    md.append("RANSAC decisions (best index, iterations, inlier set) that differ:")
    md.append("")
    md.append("| pair | C1 Ks with a different decision | C2 mask equal |")
    md.append("|---|---|---|")
    for a, b in PAIRS:
        k = f"{a}|{b}"
        md.append(f"| {a} vs {b} | {len(c1['decision_diff'][k])} / 28: {', '.join(c1['decision_diff'][k]) or '-'} "
                  f"| {c2['mask_equal'][k]} |")
    md.append("")
    md.append("C2 adaptive decisions: " + "; ".join(f"{s}: best {v['best']}, iters {v['iters']}, inliers {v['n_inliers']}"
                                                   for s, v in c2["decisions"].items()))
    md.append("")
    md.append("K sweep (testpro-K.py:39-162): the pick (first smallest mean inlier error) and the rank of "
              "f = 150 mm, 127 x 178 mm (test_pro.py:801-802) under testpro-K's two orderings:")
    md.append("")
    md.append("| sequence | pick | accepted Ks | f150 127x178 accepted | its mean error | rank by error | rank by distance to origin |")
    md.append("|---|---|---|---|---|---|---|")
    for s in SEQS:
        v = out["k_sweep"][s]
        p = v["pick"]
        md.append(f"| {s} | {p['f']} mm {p['sensor'][0]}x{p['sensor'][1]} | {v['accepted']} | {v['hint_accepted']} | "
                  f"{'-' if v['hint_mean'] is None else round(v['hint_mean'], 3)} | {v['hint_rank_by_error']} | "
                  f"{v['hint_rank_by_distance']} |")
    md.append("")
    md.append("C1 per-K decisions (best / iterations / inliers):")
    md.append("")
    md.append("| K | " + " | ".join(SEQS) + " |")
    md.append("|---|" + "---|" * len(SEQS))
    for c in c1["cases"]:
        md.append(f"| {c['K']} | " + " | ".join(f"{c[s]['best']} / {c[s]['iters']} / {c[s]['inliers']}" for s in SEQS) + " |")
    with open(os.path.join(ROOT, "profiles", "r06", "epnp_variants.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    print("\n".join(md[:30]))
    print(f"({out['seconds']} s)")


if __name__ == "__main__":
    main()
