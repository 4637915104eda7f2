#!/usr/bin/env python3
"""Wave timeline of one rank's shard (RT_KERNEL_FLAG_WAVE_CLOCK, the AUTO lane kernel without
heavy-first / wide section): per 64-sample work item its s_memtime start and end.  Reports the
launch span, the wave-duration quantiles, how many waves were resident over time and when the
last waves started -- what a rank-of-N launch's time is made of.

    python3 tools/shard_waves.py <scene> <rank> <nranks> [frames]
"""
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
sid, r, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 3
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
g.set_timing(1)                         # last_kernel_ms below: the last launch
f = g.frame(1920, 1080, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK)
buf = torch.empty(rtm.shard_elems(1920, 1080, n), dtype=torch.int32, device="cuda")
for i in range(frames):
    g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
ms = g.last_kernel_ms()
clk = g.wave_clocks().astype(np.int64)
g.close()
c = clk.astype(np.uint64)
xcd = ((c[:, 2] >> np.uint64(32)) & np.uint64(15)).astype(np.int64)
rs = ((c[:, 2] >> np.uint64(36)) & np.uint64(0xFFFFFFF)).astype(np.int64)      # 100 MHz ticks
re_ = ((c[:, 3] >> np.uint64(32)) & np.uint64(0xFFFFFFF)).astype(np.int64)
re_ = np.where(re_ < rs, re_ + (1 << 28), re_)
ok = (clk[:, 0] > 0) & (clk[:, 1] > clk[:, 0]) & (clk[:, 1] - clk[:, 0] < (1 << 32))
d_all = (clk[:, 1] - clk[:, 0])[ok]
s_, e_ = rs[ok], re_[ok]
t0 = s_.min()
s_, e_ = (s_ - t0) * 10, (e_ - t0) * 10                       # ns
span = int(e_.max())
pts = np.linspace(0, span, 21)[:-1]
order = np.argsort(e_)
out = {"scene": sid, "rank": r, "nranks": n, "items": int(ok.sum()), "kernel_ms": round(ms, 4),
       "span_ns_realtime": span,
       "wave_cycles": {"p50": int(np.percentile(d_all, 50)), "p90": int(np.percentile(d_all, 90)),
                       "p99": int(np.percentile(d_all, 99)), "max": int(d_all.max()), "sum": int(d_all.sum())},
       "wave_ns": {"p50": int(np.percentile(e_ - s_, 50)), "p99": int(np.percentile(e_ - s_, 99)),
                   "max": int((e_ - s_).max())},
       "cycles_per_ns": round(float(np.median(d_all / np.maximum(e_ - s_, 1))), 3),
       "sum_over_8192_slots_ns": int((e_ - s_).sum() / 8192),
       "start_ns": {"p10": int(np.percentile(s_, 10)), "p50": int(np.percentile(s_, 50)),
                    "p90": int(np.percentile(s_, 90)), "max": int(s_.max())},
       "resident_waves_20pts": [int(((s_ <= p) & (e_ > p)).sum()) for p in pts],
       "last5": [{"start_ns": int(s_[i]), "dur_ns": int(e_[i] - s_[i])} for i in order[-5:]],
       "per_xcd_end_ns": [int(e_[xcd[ok] == x].max()) if (xcd[ok] == x).any() else None for x in range(8)]}
print(json.dumps(out))
