#!/usr/bin/env python3
"""s_memtime ticks per microsecond on this device: the WAVE_CLOCK arm's span of item clocks
(first start to last end) over the same launch's HIP-event time."""
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
res = {}
for sid in (1, 8):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    f = g.frame(1920, 1080, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK)
    out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.render_frame_device(f, out.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
    clk = g.wave_clocks().astype(np.int64)
    dur = clk[:, 1] - clk[:, 0]
    span = int(clk[:, 1].max() - clk[:, 0].min())
    ms = e0.elapsed_time(e1)
    res[sid] = {"span_ticks": span, "event_ms": round(ms, 4), "ticks_per_us": round(span / (ms * 1e3), 1),
                "p50": int(np.percentile(dur, 50)), "p99": int(np.percentile(dur, 99)), "max": int(dur.max())}
print(json.dumps(res))
