#!/usr/bin/env python3
"""Per-frame trace of AUTO's heavy-first order on one scene: each frame's HIP-event time and the
number of blocks it listed for the next frame.  RT_HF_MODE=1 in the environment keeps the
bookkeeping but renders in the natural order (A/B of the order itself)."""
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
sid = int(sys.argv[1]) if len(sys.argv) > 1 else 8
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
f = g.frame(1920, 1080, 4)
out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
rows = []
for i in range(frames):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    g.render_frame_device(f, out.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    front, listed, epoch = g.heavy_first()
    rows.append({"frame": i, "ms": round(e0.elapsed_time(e1), 4), "listed_for_next": listed, "epoch": epoch})
print(json.dumps({"scene": sid, "hf_mode": os.environ.get("RT_HF_MODE", "2"), "front": front, "frames": rows}))
