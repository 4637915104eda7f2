#!/usr/bin/env python3
"""Wave timelines of a new launch shape's first frame against a planned frame: per scene, a fresh
GpuScene renders 1080p x 4 frames with RT_KERNEL_FLAG_WAVE_CLOCK; the per-item {start, end}
s_memtime of frame 1 (natural order, cold) and of frame `--late` (heavy-first planned) are saved to
gpurun_out/<out>_<scene>.npz for the offline schedule model (tools/schedule_model.py).

    python3 tools/first_frame_waves.py [--scenes 8 4 5] [--late 20] [--out ffw]
"""
import argparse
import importlib.util
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, nargs="+", default=[8, 4, 5])
ap.add_argument("--late", type=int, default=20)
ap.add_argument("--out", default="ffw")
A = ap.parse_args()
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP = 1920, 1080, 4
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
summary = {}
for sid in A.scenes:
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    f = g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_WAVE_CLOCK)
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    clocks = {}
    for i in range(1, A.late + 1):
        g.render_frame_device(f, out.data_ptr(), st.cuda_stream)
        if i in (1, 2, A.late):
            torch.cuda.synchronize()
            clocks[i] = g.wave_clocks().astype(np.int64)
    torch.cuda.synchronize()
    g.close()
    np.savez(os.path.join(ROOT, "gpurun_out", f"{A.out}_{sid}.npz"), **{f"f{i}": c for i, c in clocks.items()})
    row = {}
    for i, c in clocks.items():
        t0 = c[:, 0].min()
        dur = c[:, 1] - c[:, 0]
        row[i] = {"span": int(c[:, 1].max() - t0), "p50": int(np.percentile(dur, 50)), "max": int(dur.max()),
                  "sum": int(dur.sum())}
    summary[sid] = row
    print(sid, json.dumps(row), flush=True)
json.dump(summary, open(os.path.join(ROOT, "gpurun_out", A.out + ".json"), "w"), indent=1)
