#!/usr/bin/env python3
"""Per-scene means of every PMC counter of tools/gpu_profile.sh's passes (render dispatches
only; prof_render.py alternates scene 1 and scene 8 launches).

    python3 tools/prof_summary.py gpurun_out/prof_r01e profiles/r01e_counters.json
"""
import csv
import glob
import json
import os
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    out = {"source": src, "scenes": {"1": {}, "8": {}}}
    for f in sorted(glob.glob(os.path.join(src, "*", "run_counter_collection.csv"))):
        per = {}
        for r in csv.DictReader(open(f)):
            if "k_render" not in r["Kernel_Name"]:
                continue
            key = (r["Counter_Name"], int(r["Dispatch_Id"]))
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        names = sorted({k[0] for k in per})
        for n in names:
            vals = [v for (c, _), v in sorted(per.items(), key=lambda kv: kv[0][1]) if c == n]
            for scene, seq in (("1", vals[0::2]), ("8", vals[1::2])):
                if seq:
                    out["scenes"][scene][n] = round(sum(seq) / len(seq), 1)
    for s in out["scenes"].values():
        if "SQ_INSTS_VALU" in s and "SQ_WAVES" in s:
            s["valu_insts_per_wave"] = round(s["SQ_INSTS_VALU"] / s["SQ_WAVES"], 1)
        if "TCC_HIT_sum" in s and "TCC_MISS_sum" in s:
            s["l2_hit_rate"] = round(s["TCC_HIT_sum"] / (s["TCC_HIT_sum"] + s["TCC_MISS_sum"]), 4)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
