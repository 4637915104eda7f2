#!/usr/bin/env python3
"""Alternate intersectors: GPU throughput of Renderer::IntersectBruteForce and
Renderer::RayMarch (rt_frame.intersector) next to the oracle's CPU restatement of the same
reference loops on a bounded sample.

    python tools/alt_bench.py [--reps 5] [--out profiles/r01_alt_bench.json]

The march also runs its exhaustive arm (RT_KERNEL_FLAG_EXHAUSTIVE, no block cull; same
results): units then count every DistancePointTri the reference evaluates.
Per config: GPU kernel ms (HIP events on the launch stream, median of reps after a warm-up),
Msamples/s, work units/s (ray/triangle tests, or point/triangle distances for the march) from
the kernel's own per-sample counters, and the oracle's Msamples/s on `cpu_rows` rows of the same
frame (all host cores).  FLOP/unit constants (reference operation counts):
Moller-Trumbore 45, DistancePointTri 80 (average of its two branches).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402  (one HIP runtime for torch and the library: DESIGN.md §6)
from bench import load_package  # noqa: E402

FLOP = {"brute": 45.0, "march": 80.0}
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md (vector FP32, FMA counted as 2)
# (mode, scene, W, H, spp, cpu_rows)
CONFIGS = [("brute", 1, 1920, 1080, 4, 8), ("brute", 8, 1920, 1080, 4, 1), ("brute", 4, 1920, 1080, 4, 1),
           ("march", 1, 1920, 1080, 4, 2), ("march", 8, 480, 270, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    rtm = load_package()
    isect = {"brute": rtm.RT_ISECT_BRUTE_FORCE, "march": rtm.RT_ISECT_RAY_MARCH}
    oracle = None
    if not args.no_cpu:
        from conftest import Oracle
        oracle = Oracle()
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    rows = []
    stream = torch.cuda.current_stream()
    arms = [(m, s, W, H, spp, cr, 0) for (m, s, W, H, spp, cr) in CONFIGS]
    arms += [(m, s, W, H, spp, cr, rtm.RT_KERNEL_FLAG_EXHAUSTIVE) for (m, s, W, H, spp, cr) in CONFIGS
             if m == "march"]
    for mode, sid, W, H, spp, cpu_rows, kflags in arms:
        hs = rtm.HostScene.load(sid)
        gs = rtm.GpuScene(hs, 0)
        f = gs.frame(W, H, spp, intersector=isect[mode], kernel=kflags)
        buf = torch.empty(W * H, dtype=torch.int32, device="cuda")
        gs.render_frame_device(f, buf.data_ptr(), stream.cuda_stream)   # warm-up
        torch.cuda.synchronize()
        ms = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            gs.render_frame_device(f, buf.data_ptr(), stream.cuda_stream)
            b.record(stream)
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        kms = float(np.median(ms))
        # work units from the kernel's counters on a band of rows (full frame for small ones)
        band = min(H, max(1, 65536 // (W * spp)))
        y0 = (H - band) // 2
        recs = gs.trace_samples(f, 0, y0, W, band)
        units_per_sample = float(recs["tests"].astype(np.float64).mean())
        nt = int(hs.stats["num_triangles"])
        # the reference's work: ntris tests per sample, ntris distances per march step
        ref_units = float(nt if mode == "brute" else recs["steps"].astype(np.float64).mean() * nt)
        samples = W * H * spp
        row = {"mode": mode + ("-exhaustive" if kflags else ""), "scene": sid, "W": W, "H": H, "spp": spp, "triangles": int(hs.stats["num_triangles"]),
               "kernel_ms": round(kms, 3), "msamples_per_s": round(samples / kms / 1e3, 2),
               "units_per_sample_midband": round(units_per_sample, 1),
               "gunits_per_s": round(samples * units_per_sample / kms / 1e6, 1),
               "ref_units_per_sample_midband": round(ref_units, 1),
               "ref_gunits_per_s": round(samples * ref_units / kms / 1e6, 1),
               "tflops_algorithmic": round(samples * units_per_sample * FLOP[mode] / kms / 1e9, 2)}
        row["fp32_peak_frac"] = round(row["tflops_algorithmic"] / FP32_PEAK_TFLOPS, 3)
        if oracle is not None and not kflags:
            # bounded CPU sample: `cpu_rows` full rows through the oracle's per-sample loop
            t0 = time.perf_counter()
            oracle.records(sid, W, H, spp, 0, H // 2, W, cpu_rows, tri_test=isect[mode] << 8)
            cpu_s = time.perf_counter() - t0
            row["cpu_port_msamples_per_s_1thr"] = round(W * cpu_rows * spp / cpu_s / 1e6, 4)
            row["cpu_sample"] = f"{cpu_rows} row(s) of {W} px at y={H // 2}, 1 thread"
        print(json.dumps(row), flush=True)
        rows.append(row)
        gs.close()
        hs.close()
    if args.out:
        with open(args.out, "w") as fh:
            json.dump({"reps": args.reps, "cores": cores, "rows": rows}, fh, indent=1)


if __name__ == "__main__":
    main()
