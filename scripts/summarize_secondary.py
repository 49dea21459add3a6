"""profiles/TAG_pmc_secondary.json from scripts/gpu_secondary_profile.sh's outputs (gpurun_out/sec):
per config and kernel, the kernel-trace launches and mean duration, the per-launch medians of
the --pmc passes, and the kernel's two rooflines:

* VALU issue: SQ_INSTS_VALU wave-instructions per launch / mean duration against 1024 SIMDs x one
  wave64 instruction per 2 cycles x 2.4 GHz (MI355X_MICROARCH.md, as bench.py's C2 roofline);
* HBM: (2 x FETCH_SIZE + WRITE_SIZE) per launch / mean duration against 8 TB/s (FETCH_SIZE
  doubled for 16-B-per-lane reads, MI355X_MICROARCH.md "HBM").

    python3 scripts/summarize_secondary.py TAG
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEC = os.path.join(ROOT, "gpurun_out", "sec")
VALU_ISSUE_PEAK = 1024 * 0.5 * 2.4e9
HBM_PEAK = 8e12
CONFIGS = {"c2": "C2 bench step: 100k P3P hypotheses x 10k points (evaluate_range)",
           "c3": "C3: 1024 problems x 2000 points x 1024 hypotheses, one batched call",
           "c4": "C4: fundamental matrix, 50k matches, 100k hypotheses, adaptive off",
           "c5": "C5: LO-RANSAC, 100k points, adaptive + LO + LM refit",
           "loc": "location search (main_v1.py:254-297): 458 candidates x 13 features, OpenCV-sampler "
                  "homography RANSAC + refit + err1/err2, one call",
           "ksweep": "K sweep (testpro-K.py:39-162): 12 points x 27 intrinsics, reference mode (EPnP-5 on MWC "
                     "subsets, LM final solve), one call",
           "epnp": "reference-mode minimal solver: 20k EPnP-5 hypotheses on MWC subsets over the C2 problem"}


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("rsac::", "")


def trace(w):
    p = os.path.join(SEC, w, "kt", "run_kernel_trace.csv")
    by = {}
    for row in csv.DictReader(open(p)):
        k = short(row["Kernel_Name"])
        by.setdefault(k, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return by


def counters(w, sub):
    p = os.path.join(SEC, w, sub, "run_counter_collection.csv")
    per = {}
    for row in csv.DictReader(open(p)):
        key = (short(row["Kernel_Name"]), row["Dispatch_Id"], row["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    by = {}
    for (k, _, c), v in per.items():
        by.setdefault(k, {}).setdefault(c, []).append(v)
    return {k: {c: statistics.median(v) for c, v in d.items()} for k, d in by.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    out = {"note": __doc__.strip().splitlines()[0], "valu_issue_peak": VALU_ISSUE_PEAK, "hbm_peak": HBM_PEAK,
           "configs": {}}
    for w, desc in CONFIGS.items():
        if not os.path.isdir(os.path.join(SEC, w)):
            continue
        tr = trace(w)
        cv, cf, cw = counters(w, "valu"), counters(w, "fetch"), counters(w, "write")
        ks = {}
        for k, durs in sorted(tr.items(), key=lambda kv: -sum(kv[1])):
            if k.startswith("__amd") or "at::native" in k:
                continue
            d = statistics.mean(durs)
            e = {"launches": len(durs), "mean_us": d * 1e6, "share": sum(durs) / sum(sum(v) for v in tr.values())}
            c = cv.get(k, {})
            if "SQ_INSTS_VALU" in c:
                per_launch = c["SQ_INSTS_VALU"] * len(tr[k]) / max(1, len(tr[k]))
                e["valu_instr_per_launch"] = c["SQ_INSTS_VALU"]
                e["salu_instr_per_launch"] = c.get("SQ_INSTS_SALU")
                e["valu_issue"] = {"achieved": per_launch / d, "frac": per_launch / d / VALU_ISSUE_PEAK}
                if c.get("SQ_WAVE_CYCLES"):
                    e["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
                    e["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            fetch = cf.get(k, {}).get("FETCH_SIZE")
            write = cw.get(k, {}).get("WRITE_SIZE")
            if fetch is not None and write is not None:
                traffic = (2 * fetch + write) * 1024  # FETCH_SIZE / WRITE_SIZE are in KiB
                e["fetch_kib"], e["write_kib"] = fetch, write
                e["hbm"] = {"traffic_bytes": traffic, "achieved_gbs": traffic / d / 1e9,
                            "frac": traffic / d / HBM_PEAK}
            ks[k] = e
        out["configs"][w] = {"workload": desc, "kernels": ks}
    out["tag"] = tag
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{tag}_pmc_secondary.json"), "w"), indent=1)
    # the untagged copy, read by bench.py, keeps the configs this pass did not profile
    merged = os.path.join(ROOT, "profiles", "pmc_secondary.json")
    try:
        prev = json.load(open(merged))
    except (OSError, ValueError):
        prev = {"configs": {}}
    for w, d in out["configs"].items():
        d["tag"] = tag
        prev["configs"][w] = d
    prev.update({k: v for k, v in out.items() if k != "configs"})
    json.dump(prev, open(merged, "w"), indent=1)
    for w, d in out["configs"].items():
        print(w)
        for k, e in list(d["kernels"].items())[:6]:
            v = e.get("valu_issue", {}).get("frac")
            h = e.get("hbm", {}).get("frac")
            print(f"  {k:28s} {e['launches']:4d} x {e['mean_us']:9.1f} us  share {e['share']:.2f}  valu {v if v is None else round(v, 3)}"
                  f"  hbm {h if h is None else round(h, 4)}  write {e.get('write_kib')}")


if __name__ == "__main__":
    main()
