#!/usr/bin/env python3
"""Per-step device time of the bench pair from a cold start (fresh scenes, the bench's launch
sequence: Cornell then killeroo per step), each step between its own event pair: how many steps
the heavy-first plan and the clocks take to settle (bench.py --steps 20 --warmup 5 vs 200/100).

    python3 tools/frame_series.py [--steps 60] [--out name]
"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--out", default=None)
    ap.add_argument("--burn", type=int, default=0, help="frames of another scene object rendered first")
    ap.add_argument("--kernel-times", action="store_true", help="also each launch's render-kernel ms (timing every launch)")
    ap.add_argument("--batch", action="store_true", help="both frames of a step in one batched launch (the bench's N = 1 step)")
    ap.add_argument("--time-every", type=int, default=0, help="rt_scene_set_timing before the series (0: the library default)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    gs = [rtm.GpuScene(rtm.HostScene.load(s), 0) for s in (1, 8)]
    if a.burn:
        # another scene object's frames right before the series (the bench pair's scenes are
        # already built, so no host-side setup idles the GPU between the burn and the series)
        b = rtm.GpuScene(rtm.HostScene.load(2), 0)
        bf = b.frame(1920, 1080, 4)
        bo = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
        for _ in range(a.burn):
            b.render_frame_device(bf, bo.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
    fs = [g.frame(1920, 1080, 4) for g in gs]
    outs = [torch.empty(1920 * 1080, dtype=torch.int32, device="cuda") for _ in gs]
    if a.kernel_times:
        for g in gs:
            g.set_timing(1)
            g.kernel_times()
    elif a.time_every:
        for g in gs:
            g.set_timing(a.time_every)
    ev = []
    for i in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        if a.batch:
            rtm.render_batch_device([gs[1], gs[0]], [fs[1], fs[0]], [outs[1].data_ptr(), outs[0].data_ptr()],
                                    stream=st.cuda_stream)
        else:
            for g, f, o in zip(gs, fs, outs):
                g.render_frame_device(f, o.data_ptr(), st.cuda_stream)
        e1.record(st)
        ev.append((e0, e1))
    torch.cuda.synchronize()
    ms = [round(x.elapsed_time(y), 4) for x, y in ev]
    kt = [[round(float(t), 4) for t in g.kernel_times()] for g in gs] if a.kernel_times else None
    for g in gs:
        g.close()
    if a.burn:
        b.close()
    res = {"steps": a.steps, "step_ms": ms,
           "mean_steps_5_25": round(sum(ms[5:25]) / 20, 4), "mean_steps_last20": round(sum(ms[-20:]) / 20, 4)}
    if kt is not None:
        res["kernel_ms"] = {"1": kt[0], "8": kt[1]}
    print(json.dumps(res))
    if a.out:
        with open(os.path.join(ROOT, "gpurun_out", a.out + ".json"), "w") as fh:
            fh.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
