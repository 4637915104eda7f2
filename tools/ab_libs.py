#!/usr/bin/env python3
"""Interleaved A/B of two BUILDS of librt_tracer.so in one process (for changes that have no
kernel flag): the package is loaded twice, the second copy bound to the library named by
--lib-b (a file in the package directory, e.g. librt_tracer_prev.so).  Per scene, median /
min kernel ms from HIP events on the launch stream and a byte-exactness check B vs A.

    python3 tools/ab_libs.py --lib-b librt_tracer_prev.so --scenes 0 1 2 3 4 5 6 7 8 9
"""
import argparse
import hashlib
import importlib.util
import json
import os
import sys

import torch  # first: share torch's HIP runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INIT = os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py")


def load(name, lib):
    if lib:
        os.environ["RT_TRACER_LIB"] = lib
    else:
        os.environ.pop("RT_TRACER_LIB", None)
    spec = importlib.util.spec_from_file_location(name, INIT)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    m.tracer_lib()
    m.host_lib()
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-b", required=True)
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    mods = {"A": load("rtm_a", None), "B": load("rtm_b", a.lib_b)}
    os.environ.pop("RT_TRACER_LIB", None)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    W, H, S = 1920, 1080, 4
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    scenes = {(v, sid): (m.GpuScene(m.HostScene.load(sid), 0)) for v, m in mods.items() for sid in a.scenes}
    times = {key: [] for key in scenes}
    dig = {}
    for r in range(a.rounds + 1):
        for (v, sid), gs in scenes.items():
            f = gs.frame(W, H, S, kernel=a.kernel)
            evs = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                gs.render_frame_device(f, out.data_ptr(), st.cuda_stream)
                e1.record(st)
                evs.append((e0, e1))
            torch.cuda.synchronize()
            if r > 0:
                times[(v, sid)] += [x.elapsed_time(y) for x, y in evs]
            dig[(v, sid)] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
    res = {"lib_b": a.lib_b, "kernel": a.kernel}
    for (v, sid), t in times.items():
        t = sorted(t)
        res[f"{v}_s{sid}"] = {"median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                              "same_bytes_as_A": dig[(v, sid)] == dig[("A", sid)]}
    res["sum_A"] = round(sum(res[f"A_s{s}"]["median_ms"] for s in a.scenes), 4)
    res["sum_B"] = round(sum(res[f"B_s{s}"]["median_ms"] for s in a.scenes), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
