#!/usr/bin/env python3
"""Per-frame latency of bench.py's overlapped N = 1 step against HIP stream priorities.

The step renders killeroo then Cornell, one launch per frame with RT_KERNEL_FLAG_OVERLAP, step i on
stream i % 2, as bench.py does.  Each launch is bracketed by events on its own stream: latency = the
launch's end minus the point its stream reached it (the frame could start), interval = span / steps.
Arms: both streams at the default priority, or stream 0 high and stream 1 low (the older of two frames in
flight then wins the dispatcher on every other step only).

    python3 tools/priority_probe.py [--steps 200] [--warmup 100] [--out NAME]
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=100)
ap.add_argument("--out", default="priority_probe")
A = ap.parse_args()
torch.cuda.set_device(0)
W, H, SPP = 1920, 1080, 4
lo, hi = torch.cuda.Stream.priority_range()
scenes = []
for sid in (8, 1):
    hs = rtm.HostScene.load(sid)
    gs = rtm.GpuScene(hs, 0)
    scenes.append((sid, hs, gs, gs.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP)))
bufs = [[torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in scenes] for _ in range(2)]


def run(prios):
    streams = [torch.cuda.Stream(priority=p) for p in prios]
    torch.cuda.synchronize()
    ev = []
    total = A.warmup + A.steps
    t0 = t1 = None
    for i in range(total):
        s = streams[i % 2]
        if i == A.warmup:
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(streams[0])
            streams[1].wait_event(t0)
        for j, (sid, hs, gs, f) in enumerate(scenes):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            gs.render_frame_device(f, bufs[i % 2][j].data_ptr(), s.cuda_stream)
            b.record(s)
            if i >= A.warmup:
                ev.append((sid, i % 2, a, b))
    j = torch.cuda.Event()
    j.record(streams[1])
    streams[0].wait_event(j)
    t1 = torch.cuda.Event(enable_timing=True)
    t1.record(streams[0])
    torch.cuda.synchronize()
    lat = {}
    for sid, p, a, b in ev:
        lat.setdefault(f"scene{sid}_stream{p}", []).append(a.elapsed_time(b))
    return {"ms_per_step": round(t0.elapsed_time(t1) / A.steps, 4),
            "latency_ms_median": {k: round(statistics.median(v), 4) for k, v in sorted(lat.items())}}


res = {"what": __doc__.strip().splitlines()[0], "priority_range": [lo, hi], "steps": A.steps, "warmup": A.warmup, "arms": {}}
for rep in range(2):
    for name, prios in (("default", (0, 0)), ("hi_lo", (hi, lo))):
        r = run(prios)
        res["arms"].setdefault(name, []).append(r)
        print(name, rep, json.dumps(r), flush=True)
for _, hs, gs, _ in scenes:
    gs.close()
    hs.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", A.out + ".json"), "w") as fh:
    json.dump(res, fh, indent=1)
