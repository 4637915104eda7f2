#!/usr/bin/env python3
"""The orbiting-camera step of the bench pair in both frame orders (Cornell first / killeroo first),
each order on its own scene objects, rounds interleaved: device ms per step, and whether every
frame of the sequence is byte-identical between the orders and to a one-frame launch per scene.

    python3 tools/moving_order.py [--frames 120] [--out name]
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
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd",
                                                                  "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
from bench import orbit_cam, ORBIT_DEG  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    W, H, S = 1920, 1080, 4
    sids = [1, 8]
    hs = {s: rtm.HostScene.load(s) for s in sids}
    arms = {"1,8": [1, 8], "8,1": [8, 1], "single": [1, 8]}
    objs = {n: {s: rtm.GpuScene(hs[s], 0) for s in sids} for n in arms}
    cams = {s: [orbit_cam(hs[s].cam, ORBIT_DEG * (j + 1)) for j in range(a.frames)] for s in sids}
    outs = {n: {s: torch.empty(W * H, dtype=torch.int32, device="cuda") for s in sids} for n in arms}

    def frame(n, s, j):
        f = objs[n][s].frame(W, H, S)
        for k in range(16):
            f.cam[k] = float(cams[s][j][k])
        return f

    times = {n: [] for n in arms}
    digests = {n: [] for n in arms}
    for j in range(a.frames):
        for n, order in arms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            if n == "single":
                for s in order:
                    objs[n][s].render_frame_device(frame(n, s, j), outs[n][s].data_ptr(), st.cuda_stream)
            else:
                rtm.render_batch_device([objs[n][s] for s in order], [frame(n, s, j) for s in order],
                                        [outs[n][s].data_ptr() for s in order], stream=st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1))
            if j % 10 == 0:
                digests[n].append([hashlib.sha256(outs[n][s].cpu().numpy().tobytes()).hexdigest()[:16] for s in sids])
    res = {"frames": a.frames, "orbit_deg_per_frame": ORBIT_DEG,
           "ms_per_step": {n: round(float(np.mean(t[10:])), 4) for n, t in times.items()},
           "ms_first_half": {n: round(float(np.mean(t[10:a.frames // 2])), 4) for n, t in times.items()},
           "ms_second_half": {n: round(float(np.mean(t[a.frames // 2:])), 4) for n, t in times.items()},
           "same_frames": digests["1,8"] == digests["8,1"] == digests["single"]}
    print(json.dumps(res))
    if a.out:
        with open(os.path.join(ROOT, "gpurun_out", a.out + ".json"), "w") as fh:
            fh.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
