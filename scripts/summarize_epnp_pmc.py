"""Summarise scripts/gpu_r04_epnp_pmc.sh's counter passes (gpurun_out/epmc) per EPnP-5 kernel and grid
size (the 256-hypothesis latency launches apart from the 20k-hypothesis ones):

    python3 scripts/summarize_epnp_pmc.py LABEL OUT.json   (appends / replaces LABEL in OUT.json)
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("rsac::", "")
        if "epnp5" not in k:
            continue
        key = f"{k} grid {int(r['Grid_Size'])}"
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    return {key: dict({c: v / len(disp[key]) for c, v in d.items()}, launches=len(disp[key])) for key, d in agg.items()}


label, out = sys.argv[1], sys.argv[2]
base = os.path.join(ROOT, "gpurun_out", "epmc")
res = {}
for p in ("valu", "f64"):
    for key, d in load(os.path.join(base, p, "run_counter_collection.csv")).items():
        res.setdefault(key, {}).update({c: v for c, v in d.items() if c != "GRBM_GUI_ACTIVE"})
doc = json.load(open(out)) if os.path.exists(out) else {
    "note": "EPnP-5 solve kernels, rocprofv3 --pmc per launch (two passes, scripts/gpu_r04_epnp_pmc.sh over "
            "scripts/epnp5_prof.py 20000: 256-hypothesis adaptive rounds and 20k fixed-budget rounds)"}
doc[label] = res
json.dump(doc, open(out, "w"), indent=1)
print(json.dumps({k: {c: round(v) for c, v in d.items() if c in ("SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU")}
                  for k, d in res.items()}, indent=1))
