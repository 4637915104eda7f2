#!/usr/bin/env python3
"""Per-launch HBM traffic of the render kernel from the separate FETCH_SIZE / WRITE_SIZE
rocprofv3 passes of tools/gpu_profile.sh (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE
are KiB per dispatch; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide streaming read, so
the corrected read bytes are 2 x FETCH_SIZE (upper bound for this kernel's narrower gathers).

    python3 tools/pmc_traffic.py gpurun_out/prof_r01d profiles/r01h_pmc_traffic.json
"""
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if "k_render" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    src, dst = sys.argv[1], sys.argv[2]
    f = per_dispatch(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_dispatch(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    # prof_render.py alternates scene 1, scene 8 launches
    scenes = {"1": (f[0::2], w[0::2]), "8": (f[1::2], w[1::2])}
    out = {"workload": "scenes[1, 8]_1920x1080x4", "source": src, "per_scene": {}}
    tot = []
    for sid, (ff, ww) in scenes.items():
        fk, wk = sum(ff) / len(ff), sum(ww) / len(ww)
        corr = (2 * fk + wk) * 1024
        out["per_scene"][sid] = {"FETCH_SIZE_KiB": round(fk, 1), "WRITE_SIZE_KiB": round(wk, 1),
                                 "hbm_bytes_corrected": round(corr)}
        tot.append(corr)
    out["hbm_bytes_per_launch"] = round(sum(tot) / len(tot))
    out["note"] = ("mean over the two scenes' render launches of (2*FETCH_SIZE + WRITE_SIZE) KiB; "
                   "the 8.3 MB BGRA8 frame write dominates, the scene itself is L2/MALL resident")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
