#!/usr/bin/env python3
"""Interleaved A/B of several BUILDS of librt_tracer.so (and kernel values) in one process, for
changes that have no kernel flag.  Each arm is NAME=LIB:KERNEL with LIB a file in the package
directory (e.g. librt_tracer_r01.so); every distinct library is loaded as its own copy of the
package.  Per scene and arm: median / min time of render_frame_device between HIP events on
the launch stream, and whether the frame's bytes equal the first arm's.

    python3 tools/ab_libs.py --arm new=librt_tracer.so:0 --arm r01=librt_tracer_r01.so:0 \\
        --scenes 1 8 5 4
(--lib-b LIB is the two-arm shorthand: librt_tracer.so vs LIB, both at --kernel.)
"""
import argparse
import hashlib
import importlib.util
import json
import os
import sys

import numpy as np
import torch  # first: share torch's HIP runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INIT = os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py")


def load(name, lib):
    os.environ["RT_TRACER_LIB"] = lib
    spec = importlib.util.spec_from_file_location(name, INIT)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    m.tracer_lib()
    m.host_lib()
    os.environ.pop("RT_TRACER_LIB", None)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", action="append", default=[])
    ap.add_argument("--lib-b")
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--size", type=int, nargs=3, default=[1920, 1080, 4])
    a = ap.parse_args()
    arms = []
    for spec in a.arm:
        name, rest = spec.split("=", 1)
        lib, k = rest.rsplit(":", 1)
        arms.append((name, lib, int(k, 0)))
    if a.lib_b:
        arms = [("A", "librt_tracer.so", a.kernel), ("B", a.lib_b, a.kernel)]
    mods = {}
    for _, lib, _ in arms:
        if lib not in mods:
            mods[lib] = load(f"rtm_{len(mods)}", lib)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    W, H, S = a.size
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    # one scene object per arm: arms never share per-scene state (heavy-first plans, records)
    scenes = {}
    for name, lib, k in arms:
        m = mods[lib]
        for sid in a.scenes:
            scenes[(name, sid)] = m.GpuScene(m.HostScene.load(sid), 0)
    times = {(n, sid): [] for n, _, _ in arms for sid in a.scenes}
    dig = {}
    for r in range(a.rounds + 1):
        for name, lib, k in arms:
            for sid in a.scenes:
                gs = scenes[(name, sid)]
                f = gs.frame(W, H, S, kernel=k)
                evs = []
                for _ in range(a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    gs.render_frame_device(f, out.data_ptr(), st.cuda_stream)
                    e1.record(st)
                    evs.append((e0, e1))
                torch.cuda.synchronize()
                if r > 0:
                    times[(name, sid)] += [x.elapsed_time(y) for x, y in evs]
                dig[(name, sid)] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
    first = arms[0][0]
    res = {"size": [W, H, S], "arms": [f"{n}={l}:{k:#x}" for n, l, k in arms]}
    for (name, sid), t in times.items():
        t = sorted(t)
        res[f"{name}_s{sid}"] = {"median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                                 "same_bytes": dig[(name, sid)] == dig[(first, sid)]}
    for name, _, _ in arms:
        res[f"sum_{name}"] = round(sum(res[f"{name}_s{s}"]["median_ms"] for s in a.scenes), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
