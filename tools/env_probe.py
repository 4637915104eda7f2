#!/usr/bin/env python3
"""A/B of the library's runtime tunables (RT_HF_FLOOR, RT_HF_MIN_BLOCKS, RT_WH_*) on one GPU:
per arm (a JSON dict of environment settings) and scene, the max over ranks of N of the median
render ms (HIP events around render_shard_device, warm-ups first), a fresh scene per arm (the
heavy-first and wide-section state is per launch shape).  The arms alternate over --rounds.

    python3 tools/env_probe.py --arms '{"base": {}, "f30k": {"RT_HF_FLOOR": "30000"}}' \\
        [--scenes 1,8] [--ns 1,8] [--kernel 0]
"""
import argparse
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
ap = argparse.ArgumentParser()
ap.add_argument("--arms", required=True)
ap.add_argument("--scenes", default="1,8")
ap.add_argument("--ns", default="1,8")
ap.add_argument("--kernel", default="0")
ap.add_argument("--reps", type=int, default=16)
ap.add_argument("--warm", type=int, default=12)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--steady", action="store_true", help="back-to-back launches (bench-like timing)")
ap.add_argument("--ranks", default="all", help="'all' or a comma list of ranks to time")
ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "env_probe.json"))
a = ap.parse_args()
arms = json.loads(a.arms)
keys = sorted({k for v in arms.values() for k in v})
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP = 1920, 1080, 4
res = {}
for sid in [int(x) for x in a.scenes.split(",")]:
    hs = rtm.HostScene.load(sid)
    for n in [int(x) for x in a.ns.split(",")]:
        buf = torch.empty(rtm.shard_elems(W, H, n), dtype=torch.int32, device="cuda")
        ranks = range(n) if a.ranks == "all" else [int(x) for x in a.ranks.split(",") if int(x) < n]
        for rd in range(a.rounds):
            for name, env in arms.items():
                for k in keys:
                    os.environ.pop(k, None)
                os.environ.update({k: v for k, v in env.items() if not k.startswith("_")})
                worst = 0.0
                for r in ranks:
                    g = rtm.GpuScene(hs, 0)
                    f = g.frame(W, H, SPP, kernel=int(env.get("_kernel", a.kernel), 0))
                    ts = []
                    if a.steady:
                        # bench-like: back-to-back launches, one event pair around 16 of them
                        for _ in range(a.warm):
                            g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
                        torch.cuda.synchronize()
                        for rep in range(max(3, a.reps // 4)):
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record(st)
                            for _ in range(16):
                                g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
                            e1.record(st)
                            torch.cuda.synchronize()
                            ts.append(e0.elapsed_time(e1) / 16)
                    for rep in range(0 if a.steady else a.warm + a.reps):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
                        e1.record(st)
                        torch.cuda.synchronize()
                        if rep >= a.warm:
                            ts.append(e0.elapsed_time(e1))
                    worst = max(worst, sorted(ts)[len(ts) // 2])
                    g.close()
                res.setdefault(f"s{sid}_n{n}_{name}", []).append(round(worst, 4))
                print(sid, n, name, round(worst, 4), flush=True)
for k in keys:
    os.environ.pop(k, None)
summary = {k: min(v) for k, v in res.items()}
print(json.dumps(summary))
os.makedirs(os.path.dirname(a.out), exist_ok=True)
json.dump({"rounds": res, "best": summary, "arms": arms}, open(a.out, "w"), indent=1)
