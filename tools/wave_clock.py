#!/usr/bin/env python3
"""Per-wave critical path of the render kernel: per 64-sample work item, s_memtime duration
(RT_KERNEL_FLAG_WAVE_CLOCK debug arm), and for the slowest items the per-lane DDA steps and
triangle tests from the parity records.  Shows what the launch's tail is made of."""
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
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP = 1920, 1080, 4
KER = int(sys.argv[1]) if len(sys.argv) > 1 else 6099457


def compact(v):
    v &= 0x55
    v = (v | (v >> 1)) & 0x33
    return (v | (v >> 2)) & 0x0F


res = {}
for sid in (8, 5):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    f = g.frame(W, H, SPP, kernel=KER)
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    for _ in range(3):
        g.render_frame_device(f, out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    clk = g.wave_clocks().astype(np.int64)
    dur = clk[:, 1] - clk[:, 0]
    span = clk[:, 1].max() - clk[:, 0].min()
    order = np.argsort(-dur)
    tiles_x = (W + 15) // 16
    recs = g.trace_samples(g.frame(W, H, SPP), 0, 0, W, H)
    tests = recs["tests"].reshape(H, W, SPP)
    steps = recs["steps"].reshape(H, W, SPP)
    top = []
    for it in order[:16]:
        k, sub = divmod(int(it), 16)
        ty, tx = divmod(k, tiles_x)
        lanes_t, lanes_s = [], []
        for lane in range(64):
            slot = sub * 64 + lane
            p, s = slot >> 2, slot & 3
            x, y = tx * 16 + compact(p), ty * 16 + compact(p >> 1)
            if x < W and y < H:
                lanes_t.append(int(tests[y, x, s]))
                lanes_s.append(int(steps[y, x, s]))
        top.append({"item": int(it), "tile": [tx, ty], "cycles": int(dur[it]), "start": int(clk[it, 0] - clk[:, 0].min()),
                    "lanes": len(lanes_t), "max_tests": max(lanes_t, default=0), "sum_tests": sum(lanes_t),
                    "max_steps": max(lanes_s, default=0),
                    "mean_steps": round(float(np.mean(lanes_s)), 1) if lanes_s else 0})
    res[sid] = {"items": int(len(dur)), "span_cycles": int(span), "p50": int(np.percentile(dur, 50)),
                "p99": int(np.percentile(dur, 99)), "max": int(dur.max()), "top": top}
print(json.dumps(res))
