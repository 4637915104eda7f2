#!/usr/bin/env python3
"""Summary of tools/pmc_ab.sh: per arm (build, kernel, scene) the median over the render
dispatches (k_render_*) of every counter, skipping the first two (warm-up) dispatches."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
res = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "*_s*_[0-9]"))):
    if not os.path.isdir(d):
        continue
    arm = os.path.basename(d).rsplit("_", 1)[0]
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        if "k_render" not in r["Kernel_Name"]:
            continue
        per[r["Counter_Name"]].setdefault(int(r["Dispatch_Id"]), 0.0)
        per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for name, disp in per.items():
        v = [disp[k] for k in sorted(disp)][2:] or list(disp.values())
        v.sort()
        res[arm][name] = v[len(v) // 2]
for arm, c in res.items():
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
        c["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1)
        c["salu_per_wave"] = round(c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"], 1)
print(json.dumps(res, indent=1, sort_keys=True))
