#!/usr/bin/env python3
"""RT_KERNEL_FLAG_OVERLAP in steady state: every rank of N = 1, 2, 4, 8 renders the bench pair as
batched launches, (a) back to back on one stream, (b) alternating two streams with the flag and two
output sets, so one step's tail runs under the next step's start.  Per arm and N: the max over ranks
of the median over 3 blocks of 32 steps (each block between one event pair recorded on stream 0;
stream 1 joins it at both ends), rounds interleaved; frames checked equal between the arms.

    python3 tools/overlap_probe.py [--ns 1 2 4 8] [--rounds 3] [--out name]
"""
import argparse
import hashlib
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
ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 4, 8])
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--scenes", type=int, nargs="+", default=[8, 1])
ap.add_argument("--out", default="overlap_probe")
A = ap.parse_args()
torch.cuda.set_device(0)
W, H, SPP = 1920, 1080, 4
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
hs = {sid: rtm.HostScene.load(sid) for sid in A.scenes}


def steady(run, nstreams):
    """run(i) launches step i; returns the median ms per step over 3 blocks of 32."""
    for i in range(20):
        run(i)
    ts = []
    k = 20
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        streams[1].wait_event(e0)
        for _ in range(32):
            run(k)
            k += 1
        if nstreams > 1:
            j = torch.cuda.Event()
            j.record(streams[1])
            streams[0].wait_event(j)
        e1.record(streams[0])
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 32)
    return sorted(ts)[1]


res = {"scenes": A.scenes, "frame": [W, H, SPP], "arms": {}}
digests = {}
for rnd in range(A.rounds):
    for arm in ("one_stream", "overlap"):
        ov = arm == "overlap"
        gs = [rtm.GpuScene(hs[sid], 0) for sid in A.scenes]
        fs = [g.frame(W, H, SPP, kernel=rtm.RT_KERNEL_FLAG_OVERLAP if ov else 0) for g in gs]
        for n in A.ns:
            e = rtm.shard_elems(W, H, n) if n > 1 else W * H
            sets = [[torch.zeros(e, dtype=torch.int32, device="cuda") for _ in gs] for _ in range(2)]
            torch.cuda.synchronize()
            worst = 0.0
            for r in range(n):
                def run(i, r=r):
                    p = i % 2 if ov else 0
                    s = streams[p]
                    rtm.render_batch_device(gs, fs, [b.data_ptr() for b in sets[p]], rank=r, nranks=n,
                                            stream=s.cuda_stream)
                worst = max(worst, steady(run, 2 if ov else 1))
            torch.cuda.synchronize()
            digests.setdefault(n, {})[arm] = [hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest()[:16]
                                              for b in sets[0]]
            res["arms"].setdefault(arm, {}).setdefault(str(n), []).append(round(worst, 4))
            print(rnd, arm, n, round(worst, 4), flush=True)
        for g in gs:
            g.close()
res["best_of_rounds"] = {a: {n: min(v) for n, v in d.items()} for a, d in res["arms"].items()}
res["same_bytes"] = {str(n): d["one_stream"] == d["overlap"] for n, d in digests.items()}
print(json.dumps({"best_of_rounds": res["best_of_rounds"], "same_bytes": res["same_bytes"]}))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", A.out + ".json"), "w"), indent=1)
