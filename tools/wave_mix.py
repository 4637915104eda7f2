#!/usr/bin/env python3
"""Per-wave work of one scene's single-frame launch (AUTO | RT_KERNEL_FLAG_WAVE_CLOCK): cycles,
records tested in wave-uniform loops and per-lane list iterations per work item, summarised and
saved (gpurun_out/<out>_s<sid>.npz) so two builds (RT_TRACER_LIB) can be compared item by item.

    python3 tools/wave_mix.py --scenes 5 8 1 --frames 6 --out lane
"""
import argparse
import importlib.util
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd",
                                                                  "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, nargs="+", default=[5, 8, 1])
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--out", default="wave_mix")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    res = {"lib": os.environ.get("RT_TRACER_LIB", "librt_tracer.so")}
    for sid in a.scenes:
        hs = rtm.HostScene.load(sid)
        gs = rtm.GpuScene(hs, 0)
        f = gs.frame(1920, 1080, 4, kernel=rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK)
        gs.set_timing(1)
        ms = []
        for _ in range(a.frames):
            gs.render_frame_device(f, out.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            ms.append(gs.last_kernel_ms())
        c = gs.wave_clocks().astype(np.int64)
        gs.close()
        hs.close()
        cyc = np.where(c[:, 1] > c[:, 0], c[:, 1] - c[:, 0], 0)
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"{a.out}_s{sid}.npz"), cyc=cyc, uni=c[:, 2], lane=c[:, 3])
        q = lambda p: int(np.percentile(cyc, p))
        top = np.argsort(cyc)[-64:]
        res[str(sid)] = {"kernel_ms": [round(x, 4) for x in ms[-3:]], "items": int(len(cyc)),
                         "cycles_sum_M": round(float(cyc.sum()) / 1e6, 2),
                         "cycles_p50_p90_p99_max": [q(50), q(90), q(99), int(cyc.max())],
                         "uniform_records_sum_M": round(float(c[:, 2].sum()) / 1e6, 3),
                         "lane_iterations_sum_M": round(float(c[:, 3].sum()) / 1e6, 3),
                         "top64": {"cycles_mean": int(cyc[top].mean()), "uniform_mean": int(c[top, 2].mean()),
                                   "lane_mean": int(c[top, 3].mean())}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
