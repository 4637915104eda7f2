#!/usr/bin/env python3
"""Host-side cost of one bench step at N ranks, emulated on one GPU: rank 0's shard render of
both scenes + K3 un-shard (no collective), timed over many steps, against the sum of the
kernels' HIP-event time.  wall >> kernels means the step is launch/host bound at that N."""
import argparse
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
    rtm = importlib.util.module_from_spec(spec)
    sys.modules["rtm"] = rtm
    spec.loader.exec_module(rtm)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    W, H, SPP = 1920, 1080, 4
    scenes = [rtm.GpuScene(rtm.HostScene.load(s), 0) for s in (1, 8)]
    frames = [g.frame(W, H, SPP) for g in scenes]
    res = {}
    for n in a.nranks:
        e = rtm.shard_elems(W, H, n)
        shards = [torch.empty(e, dtype=torch.int32, device="cuda") for _ in scenes]
        gathered = torch.zeros(n * e, dtype=torch.int32, device="cuda")
        out = torch.empty(W * H, dtype=torch.int32, device="cuda")

        def step(evs=None):
            for g, f, b in zip(scenes, frames, shards):
                if evs is not None:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                g.render_shard_device(f, 0, n, b.data_ptr(), st.cuda_stream)
                if evs is not None:
                    e1.record(st)
                    evs.append((e0, e1))
            if n > 1:
                for _ in scenes:
                    rtm.unshard_device(W, H, n, gathered.data_ptr(), out.data_ptr(), st.cuda_stream)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        evs = []
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(evs)
        host = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        kern = sum(x.elapsed_time(y) for x, y in evs) / 1e3
        res[n] = {"wall_ms_per_step": round(wall / a.steps * 1e3, 4), "host_enqueue_ms_per_step": round(host / a.steps * 1e3, 4),
                  "render_kernels_ms_per_step": round(kern / a.steps * 1e3, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
