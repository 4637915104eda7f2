#!/usr/bin/env python3
"""One bench step's render cost on one rank of N (Cornell + killeroo shards, AUTO): both scenes
on one stream (sequential) vs one stream per scene (killeroo launched first), every rank of N
on one GPU, median of reps after warm-ups; reports the max over ranks -- the render part of a
rank's step before the gather.

    python3 tools/pair_streams.py [ns=1,2,4,8] [reps=20] [steady=0]

With steady=1 each timed sample is 16 back-to-back steps between one event pair (bench-like),
and a third mode runs Cornell first on one stream (the bench's order).
"""
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
NS = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8").split(",")]
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
STEADY = len(sys.argv) > 3 and sys.argv[3] == "1"
INNER = 16 if STEADY else 1
MODES = ("one_stream", "one_stream_c1first", "two_streams") if STEADY else ("one_stream", "two_streams")
WARM = 12
W, H, SPP = 1920, 1080, 4
torch.cuda.set_device(0)
main = torch.cuda.current_stream()
s8, s1 = torch.cuda.Stream(), torch.cuda.Stream()
res = {}
for n in NS:
    for mode in MODES:
        worst = 0.0
        for r in range(n):
            # fresh scenes per (rank, mode): heavy-first / wide-section state is per launch shape
            g1 = rtm.GpuScene(rtm.HostScene.load(1), 0)
            g8 = rtm.GpuScene(rtm.HostScene.load(8), 0)
            f1, f8 = g1.frame(W, H, SPP), g8.frame(W, H, SPP)
            b1 = torch.empty(rtm.shard_elems(W, H, n), dtype=torch.int32, device="cuda")
            b8 = torch.empty_like(b1)
            ts = []
            for rep in range(WARM + REPS):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main)
                for _ in range(INNER):
                    if mode == "one_stream":
                        g8.render_shard_device(f8, r, n, b8.data_ptr(), main.cuda_stream)
                        g1.render_shard_device(f1, r, n, b1.data_ptr(), main.cuda_stream)
                    elif mode == "one_stream_c1first":
                        g1.render_shard_device(f1, r, n, b1.data_ptr(), main.cuda_stream)
                        g8.render_shard_device(f8, r, n, b8.data_ptr(), main.cuda_stream)
                    else:
                        s8.wait_stream(main)
                        s1.wait_stream(main)
                        g8.render_shard_device(f8, r, n, b8.data_ptr(), s8.cuda_stream)
                        g1.render_shard_device(f1, r, n, b1.data_ptr(), s1.cuda_stream)
                        main.wait_stream(s8)
                        main.wait_stream(s1)
                e1.record(main)
                torch.cuda.synchronize()
                if rep >= WARM:
                    ts.append(e0.elapsed_time(e1) / INNER)
            worst = max(worst, sorted(ts)[len(ts) // 2])
            g1.close()
            g8.close()
        res[f"n{n}_{mode}"] = round(worst, 4)
        print(n, mode, round(worst, 4), flush=True)
print(json.dumps(res))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "pair_streams.json"), "w"), indent=1)
