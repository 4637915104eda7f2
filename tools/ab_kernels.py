#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python3 tools/ab_kernels.py --kernels 1 0 3 --scenes 1 8 --rounds 10
Prints one JSON line: per (kernel, scene) the median / min kernel ms from HIP events on the
launch stream, plus a byte-exactness check of every variant against the first.
"""
import argparse
import hashlib
import importlib.util
import json
import os
import sys

import torch  # first: share torch's HIP runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=lambda x: int(x, 0), nargs="+", default=[1, 0])
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location(
        "rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
    rtm = importlib.util.module_from_spec(spec)
    sys.modules["rtm"] = rtm
    spec.loader.exec_module(rtm)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    out = torch.empty(a.width * a.height, dtype=torch.int32, device="cuda")
    scenes = {sid: rtm.GpuScene(rtm.HostScene.load(sid), 0) for sid in a.scenes}
    times = {(k, s): [] for k in a.kernels for s in a.scenes}
    digests = {}
    for r in range(a.rounds + 1):
        for k in a.kernels:
            for sid, gs in scenes.items():
                f = gs.frame(a.width, a.height, a.spp, kernel=k)
                evs = []
                for _ in range(a.reps):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    gs.render_frame_device(f, out.data_ptr(), st.cuda_stream)
                    e1.record(st)
                    evs.append((e0, e1))
                torch.cuda.synchronize()
                if r > 0:                                    # round 0 = warm-up
                    times[(k, sid)] += [e0.elapsed_time(e1) for e0, e1 in evs]
                digests[(k, sid)] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
    res = {}
    for (k, sid), v in times.items():
        v = sorted(v)
        res[f"k{k}_s{sid}"] = {"median_ms": round(v[len(v) // 2], 4), "min_ms": round(v[0], 4),
                               "gsamples_per_s": round(a.width * a.height * a.spp / v[len(v) // 2] / 1e6, 2),
                               "same_bytes_as_k%d" % a.kernels[0]: digests[(k, sid)] == digests[(a.kernels[0], sid)]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
