#!/usr/bin/env python3
"""Renders rank r of an N-rank shard of one scene for F frames (a workload for rocprofv3
--kernel-trace: per-kernel start/end of the lane kernel, the wide section and the planning
kernels).  python3 tools/render_loop_shard.py <scene> <rank> <nranks> <frames> <kernel>"""
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
sid, r, n, frames, k = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5], 0)
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
f = g.frame(1920, 1080, 4, kernel=k)
buf = torch.empty(rtm.shard_elems(1920, 1080, n), dtype=torch.int32, device="cuda")
for i in range(frames):
    g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
g.close()
print("done", sid, r, n, frames, hex(k))
