#!/usr/bin/env python3
"""Summarise tools/gpu_counters.sh output: per kernel variant and scene launch, the mean of
every counter over the render dispatches (dispatch order = scenes in prof_render order)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
res = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "k*_*"))):
    if not os.path.isdir(d):
        continue
    var = os.path.basename(d).split("_")[0]
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        continue
    per = collections.defaultdict(list)
    disp = {}
    for r in csv.DictReader(open(f[0])):
        if "k_render" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        disp.setdefault(did, len(disp))
        per[(disp[did] % 2, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (scene_slot, name), v in per.items():
        res[f"{var}_scene{[1, 8][scene_slot]}"][name] = sum(v) / len(v)
print(json.dumps(res, indent=1, sort_keys=True))
