#!/usr/bin/env python3
"""How config 5's ten frames are split into batched launches: per arm (a partition of the scenes
into launches of <= MAX_BATCH frames; a one-frame launch is render_frame_device) the device time of
a whole step between one event pair, rounds interleaved over the arms, every arm on its own scene
objects (own heavy-first plans).  Frames are checked against the per-frame arm's bytes.

    python3 tools/batch_partition.py [--rounds 8] [--steps 20] [--out name]
"""
import argparse
import hashlib
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd",
                                                                  "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)

ARMS = {
    "per_frame": [[s] for s in range(10)],
    "4+4+2": [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]],
    "5+5": [[0, 1, 2, 3, 4], [5, 6, 7, 8, 9]],
    "6+4": [[0, 1, 2, 3, 4, 5], [6, 7, 8, 9]],
    "3+3+4": [[0, 1, 2], [3, 4, 5], [6, 7, 8, 9]],
    "2x5": [[0, 1], [2, 3], [4, 5], [6, 7], [8, 9]],
    "5+5 mixed": [[5, 9, 6, 3, 1], [7, 8, 2, 4, 0]],
    "5+5 lpt": [[5, 9, 4, 3, 1], [7, 8, 2, 6, 0]],
    "4+3+3 lpt": [[5, 3, 1, 0], [7, 9, 6], [8, 2, 4]],
    "5+5 lpt 2 streams": [[5, 9, 4, 3, 1], [7, 8, 2, 6, 0]],
    "4+3+3 lpt 3 streams": [[5, 3, 1, 0], [7, 9, 6], [8, 2, 4]],
    "6 with 5,7,8 + 4": [[5, 7, 8, 0, 1, 3], [2, 4, 6, 9]],
    "6 lpt-ish + 4": [[5, 9, 2, 0, 1, 3], [7, 8, 4, 6]],
    "5+5 lpt light first": [[1, 3, 4, 9, 5], [0, 6, 2, 8, 7]],
    "10 lpt": [[5, 7, 8, 9, 2, 4, 6, 3, 0, 1]],
    "10 natural": [list(range(10))],
    "pair 1,8": [[1, 8]],
    "pair 8,1": [[8, 1]],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--arms", nargs="+", default=list(ARMS))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    hs = {s: rtm.HostScene.load(s) for s in range(10)}
    W, H, S = 1920, 1080, 4
    arms = {}
    for name in a.arms:
        gs = {s: rtm.GpuScene(hs[s], 0) for s in range(10)}
        fs = {s: gs[s].frame(W, H, S) for s in range(10)}
        outs = {s: torch.empty(W * H, dtype=torch.int32, device="cuda") for s in range(10)}
        arms[name] = (gs, fs, outs)

    side = [torch.cuda.Stream() for _ in range(2)]

    def step(name):
        gs, fs, outs = arms[name]
        if "streams" in name:
            # launch k on stream k (0: the timed stream), forked from and joined back to it
            fork = torch.cuda.Event()
            fork.record(st)
            joins = []
            for k, part in enumerate(ARMS[name]):
                s = st if k == 0 else side[k - 1]
                if k:
                    s.wait_event(fork)
                rtm.render_batch_device([gs[x] for x in part], [fs[x] for x in part],
                                        [outs[x].data_ptr() for x in part], stream=s.cuda_stream)
                if k:
                    e = torch.cuda.Event()
                    e.record(s)
                    joins.append(e)
            for e in joins:
                st.wait_event(e)
            return
        for part in ARMS[name]:
            if len(part) == 1:
                s = part[0]
                gs[s].render_frame_device(fs[s], outs[s].data_ptr(), st.cuda_stream)
            else:
                rtm.render_batch_device([gs[s] for s in part], [fs[s] for s in part],
                                        [outs[s].data_ptr() for s in part], stream=st.cuda_stream)

    for name in arms:
        for _ in range(a.warm):
            step(name)
    torch.cuda.synchronize()
    times = {n: [] for n in arms}
    for _ in range(a.rounds):
        for name in arms:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                step(name)
            e1.record(st)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.steps)
    dig = {n: [hashlib.sha256(arms[n][2][s].cpu().numpy().tobytes()).hexdigest()[:16] for s in range(10)]
           for n in arms}
    ref = dig[a.arms[0]]
    res = {"size": [W, H, S], "rounds": a.rounds, "steps_per_round": a.steps,
           "arms": {n: {"launches": ARMS[n], "median_ms_per_step": round(sorted(t)[len(t) // 2], 4),
                        "min_ms_per_step": round(min(t), 4), "same_bytes": dig[n] == ref} for n, t in times.items()}}
    print(json.dumps(res))
    if a.out:
        with open(os.path.join(ROOT, "gpurun_out", a.out + ".json"), "w") as fh:
            fh.write(json.dumps(res) + "\n")
    for n in arms:
        for s in range(10):
            arms[n][0][s].close()


if __name__ == "__main__":
    main()
