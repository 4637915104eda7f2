#!/usr/bin/env python3
"""Profiling driver: renders the bench workload (scenes 1 and 8, 1920x1080x4spp) `--reps`
times into device memory so a rocprofv3 kernel trace / PMC pass sees only render launches.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
        python3 tools/prof_render.py --reps 10
"""
import argparse
import importlib.util
import os
import sys

import torch  # first: share torch's HIP runtime (see the package docstring)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--kernel", type=int, default=0)
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location(
        "rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
    rtm = importlib.util.module_from_spec(spec)
    sys.modules["rtm"] = rtm
    spec.loader.exec_module(rtm)
    torch.cuda.set_device(0)
    out = torch.empty(a.width * a.height, dtype=torch.int32, device="cuda")
    jobs = []
    for sid in a.scenes:
        hs = rtm.HostScene.load(sid)
        gs = rtm.GpuScene(hs, 0)
        jobs.append((hs, gs, gs.frame(a.width, a.height, a.spp, kernel=a.kernel)))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(a.reps):
        for hs, gs, f in jobs:
            gs.render_frame_device(f, out.data_ptr(), s)
    torch.cuda.synchronize()
    for hs, gs, f in jobs:
        gs.close()
        hs.close()
    print("ok")


if __name__ == "__main__":
    main()
