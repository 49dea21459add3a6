"""Turn rocprofv3 outputs under gpurun_out/prof into the committed summaries under profiles/.

    python scripts/summarize_profiles.py TAG [--points 10000 --hyps 100000]

Writes
  profiles/TAG_kernel_stats.csv      -- the --kernel-trace --stats summary of the bench command
  profiles/TAG_summary.md            -- per-kernel table + the scoring kernel's average duration
  profiles/TAG_c3_kernel_stats.csv   -- the same for scripts/c3_prof.py (BASELINE configs[2])
  profiles/pmc_score_kernel.json     -- HBM bytes per scoring launch (FETCH_SIZE x 2 per
                                        MI355X_MICROARCH.md "HBM", + WRITE_SIZE), read by bench.py
  profiles/pmc_score_valu.json       -- VALU instructions per scoring launch and the issue-side
                                        counters (SQ_*, GRBM_GUI_ACTIVE), read by bench.py
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
OUT = os.path.join(ROOT, "profiles")
SCORE = "k_pnp_score"


def counter(path, name):
    """per-launch values of counter `name` for the scoring kernel (summed over the counter's
    instances / dimensions of one dispatch)"""
    if not os.path.exists(path):
        return None
    per = {}
    for row in csv.DictReader(open(path)):
        if SCORE in row["Kernel_Name"] and row["Counter_Name"] == name:
            per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return list(per.values()) or None


def per_kernel(path, name):
    """{kernel name: median per-launch value of counter `name`} over every kernel of the run"""
    if not os.path.exists(path):
        return {}
    per = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == name:
            k = (row["Kernel_Name"].split("(")[0][:60], row["Dispatch_Id"])
            per[k] = per.get(k, 0.0) + float(row["Counter_Value"])
    by = {}
    for (k, _), v in per.items():
        by.setdefault(k, []).append(v)
    return {k: statistics.median(v) for k, v in by.items()}


def wait_summary(path, points, hyps):
    names = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_INSTS_LDS",
             "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SMEM", "SQ_VALU_MFMA_BUSY_CYCLES"]
    vals = {n: counter(path, n) for n in names}
    if not vals["SQ_WAVE_CYCLES"]:
        return None
    m = {n: statistics.median(v) for n, v in vals.items() if v}
    w = m["SQ_WAVE_CYCLES"]
    return {"kernel": SCORE, "points": points, "hyps": hyps, "counters_median": m,
            "wait_any_frac": m.get("SQ_WAIT_ANY", 0) / w, "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0) / w,
            "wait_inst_lds_frac": m.get("SQ_WAIT_INST_LDS", 0) / w,
            "note": "fractions of SQ_WAVE_CYCLES (quad-cycles): WAIT_ANY = parked on s_waitcnt / barrier, "
                    "WAIT_INST_ANY = issue stalls (dependencies, pipe busy), WAIT_INST_LDS a part of the latter"}


def valu_summary(path, points, hyps):
    names = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
             "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"]
    vals = {n: counter(path, n) for n in names}
    if not vals["SQ_INSTS_VALU"]:
        return None
    dur = []
    for row in csv.DictReader(open(path)):
        if SCORE in row["Kernel_Name"] and row.get("Start_Timestamp"):
            dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    m = {n: statistics.median(v) for n, v in vals.items() if v}
    out = {"kernel": SCORE, "points": points, "hyps": hyps, "launches": len(vals["SQ_INSTS_VALU"]),
           "valu_instr_per_launch": m["SQ_INSTS_VALU"], "salu_instr_per_launch": m.get("SQ_INSTS_SALU"),
           "counters_median": m,
           "note": "SQ_WAVE_CYCLES / WAIT / ACTIVE count quad-cycles; GRBM_GUI_ACTIVE sums the 8 XCDs"}
    if dur and "GRBM_GUI_ACTIVE" in m:
        wall = statistics.median(dur)
        clk = m["GRBM_GUI_ACTIVE"] / 8 / wall
        out["wall_s_profiled"] = wall
        out["effective_clock_ghz"] = clk / 1e9
        out["valu_per_simd_cycle"] = m["SQ_INSTS_VALU"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    return out


def issue_summary(path):
    """VALU issue per SIMD quad-cycle (one / two VALU), from SQ_ACTIVE_INST_VALU(2)"""
    names = ["SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_VALU_MFMA_COEXEC_CYCLES", "SQ_ACTIVE_INST_ANY",
             "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_SCA", "SQ_INSTS", "GRBM_GUI_ACTIVE"]
    vals = {n: counter(path, n) for n in names}
    if not vals["SQ_INSTS_VALU"] or not vals["GRBM_GUI_ACTIVE"]:
        return None
    m = {n: statistics.median(v) for n, v in vals.items() if v}
    simds, quad = 1024, m["GRBM_GUI_ACTIVE"] / 8 / 4
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in csv.DictReader(open(path))
           if SCORE in r["Kernel_Name"] and r.get("Start_Timestamp")]
    us = statistics.median(dur)
    return {"kernel": SCORE, "launches": len(vals["SQ_INSTS_VALU"]), "kernel_us_median_profiled": us,
            "counters_median": m,
            "derived": {"clock_ghz_profiled": m["GRBM_GUI_ACTIVE"] / 8 / us / 1e3,
                        "valu_instr_per_simd": m["SQ_INSTS_VALU"] / simds, "simd_quad_cycles": quad,
                        "quad_cycles_with_valu_issue_frac":
                            (m["SQ_ACTIVE_INST_VALU"] - m.get("SQ_ACTIVE_INST_VALU2", 0)) / simds / quad,
                        "quad_cycles_with_two_valu_frac": m.get("SQ_ACTIVE_INST_VALU2", 0) / simds / quad,
                        "valu_issue_frac_of_2_per_quad": m["SQ_INSTS_VALU"] / simds / (2 * quad),
                        "wave_active_frac": m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"],
                        "mfma_coexec_cycles_per_simd": m.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / simds},
            "note": "SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES in quad-cycles summed over waves; SQ_ACTIVE_INST_VALU2 = "
                    "quad-cycles in which two VALU instructions issued on a SIMD; GRBM_GUI_ACTIVE summed over 8 "
                    "XCDs. Its own rocprofv3 --pmc pass over bench.py --steps 3 --warmup 1 --no-cpu "
                    "--no-ms-to-best --no-extras."}


def solo_split(path):
    """durations (us) of the scoring kernel's launches that overlap no other kernel, and of those that
    do (bench.py's pipelined steps run two streams; its roofline times synchronous launches)"""
    if not os.path.exists(path):
        return [], []
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    solo, over = [], []
    for s, e, n in iv:
        if SCORE not in n:
            continue
        ov = any(o[0] < e and o[1] > s for o in iv if o != (s, e, n))
        (over if ov else solo).append((e - s) / 1e3)
    return solo, over


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--points", type=int, default=10_000)
    ap.add_argument("--hyps", type=int, default=100_000)
    args = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    stats = os.path.join(PROF, "kt", "run_kernel_stats.csv")
    dst = os.path.join(OUT, f"{args.tag}_kernel_stats.csv")
    shutil.copyfile(stats, dst)
    rows = list(csv.DictReader(open(stats)))
    lines = [f"# rocprofv3 --kernel-trace --stats, `python3 bench.py --steps 10 --warmup 3` ({args.tag})", "",
             "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    score_avg = None
    for r in rows:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.2f} |")
        if SCORE in r["Name"] and score_avg is None:
            score_avg = float(r["AverageNs"]) / 1e3
    fetch = counter(os.path.join(PROF, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter(os.path.join(PROF, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    algo = args.points * 20 * args.hyps
    pmc = None
    if fetch:
        fk = statistics.median(fetch)
        wk = statistics.median(write) if write else 0.0
        hbm = (2.0 * fk + wk) * 1024.0  # counters in KiB; FETCH_SIZE reads half on gfx950
        pmc = {"kernel": SCORE, "points": args.points, "hyps": args.hyps, "fetch_size_kib": fk,
               "write_size_kib": wk, "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": algo,
               "launches": len(fetch),
               "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (HBM); the 200 kB point set is re-read "
                       "from L2/MALL by every hypothesis, so HBM traffic is far below the algorithmic bytes"}
        json.dump(pmc, open(os.path.join(OUT, "pmc_score_kernel.json"), "w"), indent=1)
    valu = valu_summary(os.path.join(PROF, "pmc_valu", "run_counter_collection.csv"), args.points, args.hyps)
    if valu:
        json.dump(valu, open(os.path.join(OUT, "pmc_score_valu.json"), "w"), indent=1)
    wait = wait_summary(os.path.join(PROF, "pmc_wait", "run_counter_collection.csv"), args.points, args.hyps)
    if wait:
        json.dump(wait, open(os.path.join(OUT, "pmc_score_wait.json"), "w"), indent=1)
    issue = issue_summary(os.path.join(PROF, "pmc_issue", "run_counter_collection.csv"))
    if issue:
        json.dump(issue, open(os.path.join(OUT, "pmc_score_issue.json"), "w"), indent=1)
    fk_all = per_kernel(os.path.join(PROF, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    wk_all = per_kernel(os.path.join(PROF, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    if fk_all or wk_all:
        lines += ["", "| kernel | FETCH_SIZE KiB/launch (x2 = bytes read) | WRITE_SIZE KiB/launch |", "|---|---|---|"]
        for k in sorted(set(fk_all) | set(wk_all)):
            lines.append(f"| `{k}` | {fk_all.get(k, float('nan')):.0f} | {wk_all.get(k, float('nan')):.0f} |")
    lines += ["", f"scoring kernel average: {score_avg:.1f} us" if score_avg else "scoring kernel not found"]
    solo, over = solo_split(os.path.join(PROF, "kt", "run_kernel_trace.csv"))
    if solo:
        lines.append(f"scoring kernel launches with no other kernel running: {len(solo)}, median "
                     f"{statistics.median(solo):.1f} us (the span of bench.py's roofline: synchronous launches); "
                     f"launches overlapping the other stream's kernels (pipelined steps): {len(over)}, median "
                     f"{statistics.median(over):.1f} us" if over else "")
    if wait:
        lines += [f"scoring kernel wave cycles: {100 * wait['wait_any_frac']:.1f} % parked (SQ_WAIT_ANY), "
                  f"{100 * wait['wait_inst_any_frac']:.1f} % issue-stalled (SQ_WAIT_INST_ANY, of which LDS "
                  f"{100 * wait['wait_inst_lds_frac']:.1f} %)"]
    if valu:
        lines += [f"scoring kernel VALU instructions/launch (PMC): {valu['valu_instr_per_launch']:.4g}; "
                  f"effective clock {valu.get('effective_clock_ghz', float('nan')):.3f} GHz; "
                  f"{valu.get('valu_per_simd_cycle', float('nan')):.3f} VALU wave-instr per SIMD-cycle (peak 0.5)"]
    if pmc:
        lines += [f"scoring kernel HBM bytes/launch (PMC): {pmc['hbm_bytes_per_launch'] / 1e6:.2f} MB "
                  f"(FETCH_SIZE {pmc['fetch_size_kib']:.0f} KiB x2 + WRITE_SIZE {pmc['write_size_kib']:.0f} KiB); "
                  f"algorithmic {algo / 1e9:.1f} GB"]
    c3 = os.path.join(PROF, "c3", "run_kernel_stats.csv")
    if os.path.exists(c3):  # scripts/c3_prof.py under --kernel-trace --stats (BASELINE configs[2])
        shutil.copyfile(c3, os.path.join(OUT, f"{args.tag}_c3_kernel_stats.csv"))
        lines += ["", "C3 (1024 problems x 2000 points x 1024 hypotheses, `scripts/c3_prof.py`, 12 calls):", "",
                  "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(c3)):
            lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                         f"{float(r['Percentage']):.2f} |")
    open(os.path.join(OUT, f"{args.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
