#!/usr/bin/env python3
"""Per scene, how the AUTO kernel's triangle tests split between the wave-uniform scalar loop
and the per-lane list loop (RT_KERNEL_FLAG_WAVE_CLOCK counters, summed over a 1080p x 4 frame),
and how many per-lane iterations run with 2, 3, 4+ distinct cells in the wave (not measured:
only the totals).  python3 tools/loop_split.py [scenes=1,8,5]"""
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
for sid in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,8,5").split(",")]:
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    f = g.frame(1920, 1080, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK)
    out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    g.render_frame_device(f, out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    c = g.wave_clocks().astype(np.uint64)
    uni = (c[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    lane = (c[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    dur = (c[:, 1] - c[:, 0]).astype(np.int64)
    res[sid] = {"waves": int(len(c)), "uniform_records": int(uni.sum()), "lane_iterations": int(lane.sum()),
                "waves_with_lane_loop": int((lane > 0).sum()),
                "cycles_share_of_waves_with_lane_loop": round(float(dur[lane > 0].sum() / max(1, dur.sum())), 3)}
    print(sid, res[sid], flush=True)
    g.close()
print(json.dumps(res))
