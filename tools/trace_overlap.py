#!/usr/bin/env python3
"""Per-frame kernel timeline from a rocprofv3 --kernel-trace CSV: for every frame (one lane
kernel launch) the lane kernel's and the wide section's durations, their start offset and the
frame span from the first start to the last end (planning kernels listed beside).

    python3 tools/trace_overlap.py <dir with *_kernel_trace.csv> [skip_frames]
"""
import csv
import glob
import json
import os
import sys


def main():
    files = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    frames, cur = [], None
    for s, e, name in rows:
        short = name.split("(")[0].split("::")[-1][:40]
        if "k_render_wh" in name or "k_render_lanes" in name:
            if cur is None or (("k_render_wh" in name and "wh" in cur) or ("k_render_lanes" in name and "lanes" in cur)):
                cur = {}
                frames.append(cur)
            cur["wh" if "k_render_wh" in name else "lanes"] = (s, e)
        elif cur is not None:
            cur.setdefault("other", []).append((short, round((e - s) / 1e3, 1)))
    out = []
    for fr in frames[skip:]:
        t0 = min(v[0] for k, v in fr.items() if k != "other")
        t1 = max(v[1] for k, v in fr.items() if k != "other")
        d = {"span_us": round((t1 - t0) / 1e3, 1)}
        for k in ("wh", "lanes"):
            if k in fr:
                d[k + "_us"] = round((fr[k][1] - fr[k][0]) / 1e3, 1)
                d[k + "_start_us"] = round((fr[k][0] - t0) / 1e3, 1)
        if "other" in fr:
            d["other"] = fr["other"]
        out.append(d)
    for d in out:
        print(json.dumps(d))
    spans = sorted(d["span_us"] for d in out)
    print("median span us", spans[len(spans) // 2] if spans else None)


if __name__ == "__main__":
    main()
