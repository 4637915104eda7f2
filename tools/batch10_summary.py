#!/usr/bin/env python3
"""Summarise tools/batch10_profile.sh: per arm and scene the median kernel ms (in-process A/B),
Msamples/s, rocprof HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 FETCH_SIZE
correction of MI355X_MICROARCH.md §HBM) and the HBM GB/s those bytes give at that time, plus
the batch totals (82,944,000 samples).

    python3 tools/batch10_summary.py gpurun_out/batch10_<tag> profiles/<out>.json
"""
import csv
import glob
import json
import os
import sys

SCENES = list(range(10))
SAMPLES = 1920 * 1080 * 4


def per_dispatch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if "k_render" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    src, dst = sys.argv[1], sys.argv[2]
    ab = json.load(open(os.path.join(src, "ab.json")))
    arms = sorted({k.split("_")[0][1:] for k in ab}, key=int)
    out = {"workload": "scenes 0-9, 1920x1080x4spp each (BASELINE config 5)", "source": src, "arms": {}}
    for k in arms:
        f = glob.glob(os.path.join(src, f"k{k}_FETCH_SIZE", "*counter_collection.csv"))
        w = glob.glob(os.path.join(src, f"k{k}_WRITE_SIZE", "*counter_collection.csv"))
        fs = per_dispatch(f[0], "FETCH_SIZE") if f else []
        ws = per_dispatch(w[0], "WRITE_SIZE") if w else []
        arm = {"per_scene": {}}
        tot_ms = tot_b = 0.0
        for i, sid in enumerate(SCENES):
            e = ab[f"k{k}_s{sid}"]
            ms = e["median_ms"]
            fk = [fs[j] for j in range(i, len(fs), len(SCENES))]
            wk = [ws[j] for j in range(i, len(ws), len(SCENES))]
            hbm = (2 * sum(fk) / len(fk) + sum(wk) / len(wk)) * 1024 if fk and wk else None
            arm["per_scene"][str(sid)] = {
                "kernel_ms": ms, "msamples_per_s": round(SAMPLES / ms / 1e3, 1),
                "same_bytes_as_first_arm": e[f"same_bytes_as_k{arms[0]}"],
                "hbm_bytes": None if hbm is None else round(hbm),
                "hbm_gb_per_s": None if hbm is None else round(hbm / ms / 1e6, 1)}
            tot_ms += ms
            tot_b += hbm or 0.0
        arm["batch_ms"] = round(tot_ms, 4)
        arm["batch_msamples_per_s"] = round(SAMPLES * len(SCENES) / tot_ms / 1e3, 1)
        arm["batch_hbm_gb_per_s"] = round(tot_b / tot_ms / 1e6, 1)
        out["arms"][k] = arm
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: (v["batch_ms"], v["batch_msamples_per_s"], v["batch_hbm_gb_per_s"])
                      for k, v in out["arms"].items()}))


if __name__ == "__main__":
    main()
