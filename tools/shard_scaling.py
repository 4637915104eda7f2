#!/usr/bin/env python3
"""Per-scene render time of one rank's shard at N = 1..8 (emulated on one GPU: rank r of N),
to expose the latency floor of strong scaling (the slowest wave's dependent-load chain)."""
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
W, H, SPP = 1920, 1080, 4
kernels = [int(k) for k in sys.argv[1:]] or [0]
res = {}
for sid in (1, 8, 4, 5):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    for k in kernels:
        f = g.frame(W, H, SPP, kernel=k)
        for n in (1, 2, 4, 8, 16, 32):
            buf = torch.empty(rtm.shard_elems(W, H, n), dtype=torch.int32, device="cuda")
            ranks = [0] if n == 1 else [0, n // 2, n - 1]
            for r in ranks:
                ts = []
                for rep in range(8):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
                    e1.record(st)
                    torch.cuda.synchronize()
                    if rep >= 2:
                        ts.append(e0.elapsed_time(e1))
                res[f"s{sid}_k{k}_n{n}_r{r}"] = round(sorted(ts)[len(ts) // 2], 4)
print(json.dumps(res))
