#!/usr/bin/env python3
"""Where a new launch shape's first frames spend their time (bench.py first_frame_ms): per scene, a
fresh GpuScene, then frames 1..4 of 1920x1080x4 on a side stream, each timed by HIP events around the
render call (host setup inside the call shows up as device idle time) and by the library's own event
pair around the render kernel (rt_kernel_times, timing every launch).  --warm renders a 64x64 frame
of the same scene first (origin records, code objects), so frame 1 pays only the new shape.

    python3 tools/first_frame_probe.py [--scenes 1 8] [--reps 3] [--warm] [--out NAME]
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--frames", type=int, default=4)
ap.add_argument("--warm", action="store_true")
ap.add_argument("--out", default="first_frame_probe")
A = ap.parse_args()
torch.cuda.set_device(0)
W, H, SPP = 1920, 1080, 4
st = torch.cuda.Stream()
buf = torch.empty(W * H, dtype=torch.int32, device="cuda")
small = torch.empty(64 * 64, dtype=torch.int32, device="cuda")
res = {"warm": A.warm, "scenes": {}}
for sid in A.scenes:
    hs = rtm.HostScene.load(sid)
    runs = []
    for rep in range(A.reps + 1):
        gs = rtm.GpuScene(hs, 0)
        try:
            gs.set_timing(1)
            if A.warm:
                gs.render_frame_device(gs.frame(64, 64, SPP), small.data_ptr(), st.cuda_stream)
                st.synchronize()
                gs.kernel_times()
            f = gs.frame(W, H, SPP)
            torch.cuda.synchronize()
            fr = []
            for i in range(A.frames):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                a.record(st)
                gs.render_frame_device(f, buf.data_ptr(), st.cuda_stream)
                t1 = time.perf_counter()
                b.record(st)
                b.synchronize()
                kt = gs.kernel_times()
                fr.append({"span_ms": round(a.elapsed_time(b), 4), "call_ms": round((t1 - t0) * 1e3, 4),
                           "kernel_ms": [round(float(x), 4) for x in kt]})
            if rep:
                runs.append(fr)
        finally:
            gs.close()
    res["scenes"][str(sid)] = runs
    print(sid, json.dumps(runs[-1]), flush=True)
    hs.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", A.out + ".json"), "w") as fh:
    json.dump(res, fh, indent=1)
