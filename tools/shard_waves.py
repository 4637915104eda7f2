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
f = g.frame(1920, 1080, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK | rtm.RT_KERNEL_FLAG_ONE_PHASE)
buf = torch.empty(rtm.shard_elems(1920, 1080, n), dtype=torch.int32, device="cuda")
for i in range(frames):
    g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
ms = g.last_kernel_ms()
clk = g.wave_clocks().astype(np.int64)
g.close()
s, e = clk[:, 0], clk[:, 1]
ok = (s > 0) & (e > s) & (e - s < (1 << 32))
s, e = s[ok], e[ok]
t0 = s.min()
s, e = s - t0, e - t0
span = int(e.max())
d = e - s
order = np.argsort(e)
q = lambda a, p: int(np.percentile(a, p))
# resident waves at 20 points of the span
pts = np.linspace(0, span, 21)[:-1]
res = [int(((s <= p) & (e > p)).sum()) for p in pts]
last = order[-20:]
out = {"scene": sid, "rank": r, "nranks": n, "items": int(ok.sum()), "kernel_ms": round(ms, 4),
       "span_cycles": span, "cycles_per_ms": round(span / ms) if ms else None,
       "wave_cycles": {"p50": q(d, 50), "p90": q(d, 90), "p99": q(d, 99), "max": int(d.max()), "sum": int(d.sum())},
       "sum_over_8192_slots": int(d.sum() / 8192),
       "resident_waves_over_span": res,
       "last20_finish": [{"start": int(s[i]), "dur": int(d[i])} for i in last],
       "start_p99": q(s, 99), "start_max": int(s.max())}
print(json.dumps(out))
