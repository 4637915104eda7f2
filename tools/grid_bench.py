#!/usr/bin/env python3
"""Grid build timing: the device build (rt_grid_build, HIP-event time of its
kernels and wall time of the whole call incl. H2D/D2H) vs the host build (librt_host.so, all
cores and 1 thread -- the reference's Grid::Grid is single-threaded), per reference scene.

    python tools/grid_bench.py [--reps 5] [--out profiles/r01_grid_build.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime for torch and the library: DESIGN.md §6)
from bench import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--scenes", default="0,1,2,3,4,5,6,7,8,9")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rtm = load_package()
    rows = []
    for sid in [int(s) for s in args.scenes.split(",")]:
        hs = rtm.HostScene.load(sid)
        v, t = hs.mesh()
        rtm.gpu_grid_build(v, t, 64, 0)                  # warm-up (module load, allocations)
        dev_ms, wall_ms = [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            meta, offs, tris, ms = rtm.gpu_grid_build(v, t, 64, 0)
            wall_ms.append((time.perf_counter() - t0) * 1e3)
            dev_ms.append(ms)
        host_all, host_one = [], []
        for _ in range(max(1, args.reps // 2)):
            host_all.append(rtm.HostScene.from_mesh(v, t, hs.fov, hs.cam, 64, 0).stats["grid_build_s"] * 1e3)
            host_one.append(rtm.HostScene.from_mesh(v, t, hs.fov, hs.cam, 64, 1).stats["grid_build_s"] * 1e3)
        rows.append({"scene": sid, "triangles": int(t.shape[0]), "cells": int(offs.size - 1),
                     "refs": int(offs[-1]), "device_ms": round(float(np.median(dev_ms)), 4),
                     "call_ms": round(float(np.median(wall_ms)), 3),
                     "host_ms_all_cores": round(float(np.median(host_all)), 3),
                     "host_ms_1_thread": round(float(np.median(host_one)), 3)})
        print(json.dumps(rows[-1]), flush=True)
        hs.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"grid_res": 64, "reps": args.reps, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
