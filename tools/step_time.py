#!/usr/bin/env python3
"""Steady-state bench step time without bench.py's accounting (for A/B builds that record no
kernel events): one frame of scenes 1 and 8 per step at 1080p x 4, W warm-up steps, K timed
steps between device syncs.  RT_TRACER_LIB selects the build.
    python3 tools/step_time.py [steps=300] [warmup=100]"""
import importlib.util
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
Wu = int(sys.argv[2]) if len(sys.argv) > 2 else 100
torch.cuda.set_device(0)
st = torch.cuda.Stream()
sc = []
for sid in (1, 8):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    sc.append((g, g.frame(1920, 1080, 4), torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")))
def step():
    for g, f, b in sc:
        g.render_frame_device(f, b.data_ptr(), st.cuda_stream)
for _ in range(Wu):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    step()
torch.cuda.synchronize()
print(round((time.perf_counter() - t0) / K * 1e3, 4))
