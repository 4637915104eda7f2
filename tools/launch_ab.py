#!/usr/bin/env python3
"""In-process A/B of a scene tunable read at rt_scene_create, by default how a whole-frame AUTO
launch gets its blocks onto the chip (RT_WG64): 0 = the dispatched 256-lane grid, 1 = one-wave
workgroups (k_render_lanes_w64).  (Round 3 also measured resident waves on per-XCD work queues
and two-wave workgroups here; both lost and were removed.)  Per value and scene: every
frame's BGRA8 and per-sample hit IDs against the reference's golden SHA-256 (6 consecutive frames,
so the heavy-first order is on), then the steady per-frame time (20 warm-up launches, 3 x 32
back-to-back launches between one event pair, median).  Values interleaved over --rounds.

    python3 tools/launch_ab.py [--env RT_WG64] [--values 0 1] [--scenes 1 8 5 4 0] [--rounds 3] [--out NAME]
"""
import argparse
import hashlib
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
ap = argparse.ArgumentParser()
ap.add_argument("--env", default="RT_WG64")
ap.add_argument("--values", nargs="+", default=["0", "1"])
ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8, 5, 4, 0])
ap.add_argument("--frame", type=int, nargs=3, default=[1920, 1080, 4])
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--out", default="persist_ab")
A = ap.parse_args()
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP = A.frame
golden = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["frames_1080p4"]
hs = {sid: rtm.HostScene.load(sid) for sid in A.scenes}


def sha(t):
    return hashlib.sha256(t.cpu().numpy().view(np.uint32).tobytes()).hexdigest()


def steady(run):
    for _ in range(20):
        run()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(32):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 32)
    return sorted(ts)[1]


res = {"env": A.env, "frame": A.frame, "ms": {}, "exact": {}}
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
hits = torch.empty(W * H * SPP, dtype=torch.int32, device="cuda")
for rnd in range(A.rounds):
    for v in A.values:
        os.environ[A.env] = v
        for sid in A.scenes:
            g = rtm.GpuScene(hs[sid], 0)
            f = g.frame(W, H, SPP)
            if rnd == 0 and (W, H, SPP) == (1920, 1080, 4):
                ok = True
                for i in range(6):
                    out.fill_(0x5A5A5A5A)
                    hits.fill_(0x5A5A5A5A)
                    g.render_hits_device(f, 0, 1, out.data_ptr(), hits.data_ptr(), st.cuda_stream)
                    torch.cuda.synchronize()
                    ok = ok and sha(out) == golden[str(sid)]["bgra_sha256"] and sha(hits) == golden[str(sid)]["hits_sha256"]
                res["exact"][f"{v}_s{sid}"] = ok
            t = steady(lambda: g.render_frame_device(f, out.data_ptr(), st.cuda_stream))
            res["ms"].setdefault(v, {}).setdefault(str(sid), []).append(round(t, 4))
            g.close()
        print(rnd, v, {s: res["ms"][v][str(s)][-1] for s in A.scenes}, flush=True)
res["median_ms"] = {v: {s: sorted(x)[len(x) // 2] for s, x in d.items()} for v, d in res["ms"].items()}
res["sum_ms"] = {v: round(sum(d.values()), 4) for v, d in res["median_ms"].items()}
print(json.dumps({"exact": res["exact"], "median_ms": res["median_ms"], "sum_ms": res["sum_ms"]}))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", A.out + ".json"), "w"), indent=1)
