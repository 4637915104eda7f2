#!/usr/bin/env python3
"""One rank's shard launch repeated (for rocprofv3 --kernel-trace): shows how a rank's frame
time splits between the two-phase arm's kernels.  Usage: shard_phases.py SCENE NRANKS RANK [KERNEL]"""
import importlib.util
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
sid, n, r = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
k = int(sys.argv[4]) if len(sys.argv) > 4 else 0
g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
f = g.frame(1920, 1080, 4, kernel=k)
buf = torch.empty(rtm.shard_elems(1920, 1080, n), dtype=torch.int32, device="cuda")
for _ in range(12):
    g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
torch.cuda.synchronize()
print("done")
