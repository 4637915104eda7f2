#!/usr/bin/env python3
"""Real-time wave timeline of one rank's BATCHED bench step (RT_KERNEL_FLAG_WAVE_CLOCK on the batch
kernel: the heavy-first order and the fused wide section run as in the product launch): where a
rank-of-N launch's time goes -- dispatch ramp, the wide section, the lane tail.

    python3 tools/batch_waves.py [--rank 0] [--nranks 8] [--frames 40] [--scenes 1 8] [--out name]

Per wave (lane item or wide-section (item, wave)) the 100 MHz s_memrealtime at start and end and
the XCD; reported in ns from the first wave's start."""
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


def q(a, p):
    return int(np.percentile(a, p)) if len(a) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--nranks", type=int, default=8)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    hs = [rtm.HostScene.load(s) for s in a.scenes]
    gs = [rtm.GpuScene(h, 0) for h in hs]
    fl = rtm.RT_KERNEL_AUTO | rtm.RT_KERNEL_FLAG_WAVE_CLOCK
    fs = [g.frame(a.W, a.H, a.spp, kernel=fl) for g in gs]
    n = a.W * a.H if a.nranks == 1 else rtm.shard_elems(a.W, a.H, a.nranks)
    bufs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in gs]
    gs[0].set_timing(1)
    ms = []
    for i in range(a.frames):
        rtm.render_batch_device(gs, fs, [b.data_ptr() for b in bufs], a.rank, a.nranks, stream=st.cuda_stream)
        torch.cuda.synchronize()
        ms.append(gs[0].last_kernel_ms())
    clk = gs[0].wave_clocks()
    info = gs[0].info()
    wide_items = gs[0].wide_items()
    for g in gs:
        g.close()
    for h in hs:
        h.close()
    c = clk.astype(np.uint64)
    valid = c[:, 1] > c[:, 0]
    c = c[valid]
    lo2 = (c[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    lo3 = (c[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcd = ((c[:, 2] >> np.uint64(32)) & np.uint64(15)).astype(np.int64)
    rs = ((c[:, 2] >> np.uint64(36)) & np.uint64(0xFFFFFFF)).astype(np.int64)
    re_ = ((c[:, 3] >> np.uint64(32)) & np.uint64(0xFFFFFFF)).astype(np.int64)
    re_ = np.where(re_ < rs, re_ + (1 << 28), re_)
    cyc = (c[:, 1] - c[:, 0]).astype(np.int64)
    wide = (lo2 & 0x80000000) != 0
    lds = wide & ((lo2 & 0x7FFFFFFF) >= 4096)         # the LDS tier's items (list entries from kWhMax)
    frame = np.where(wide, -1, lo2 & 15)
    uni = np.where(wide, 0, lo2 >> 4)                  # lane waves: records tested wave-uniformly
    lit = np.where(wide, 0, lo3)                       # ... and per-lane list iterations
    t0 = rs.min()
    s_, e_ = (rs - t0) * 10, (re_ - t0) * 10                      # ns
    d_ = e_ - s_
    span = int(e_.max())
    pts = np.linspace(0, span, 41)[:-1]
    res = [int(((s_ <= p) & (e_ > p)).sum()) for p in pts]
    peak = max(res)
    # when the resident count falls for good below a fraction of its peak
    def fall(frac):
        ts = np.sort(np.concatenate([s_, e_]))
        ev = np.concatenate([np.ones_like(s_), -np.ones_like(e_)])[np.argsort(np.concatenate([s_, e_]), kind="stable")]
        live = np.cumsum(ev)
        above = np.nonzero(live >= frac * peak)[0]
        return int(ts[above[-1]]) if len(above) else None
    order = np.argsort(e_)
    kinds = {}
    for name, m in (("wide", wide & ~lds), ("lds", lds),
                    *[(f"lane_frame{f}", (~wide) & (frame == f)) for f in range(len(a.scenes))]):
        if not m.any():
            continue
        kinds[name] = {"waves": int(m.sum()), "start_ns": [int(s_[m].min()), q(s_[m], 50), int(s_[m].max())],
                       "end_ns_max": int(e_[m].max()), "dur_ns": [q(d_[m], 50), q(d_[m], 90), q(d_[m], 99), int(d_[m].max())],
                       "sum_dur_over_8192_slots_ns": int(d_[m].sum() / 8192)}
    out = {"scenes": a.scenes, "rank": a.rank, "nranks": a.nranks, "frames": a.frames, "W": a.W, "H": a.H, "spp": a.spp,
           "kernel_ms_last": round(ms[-1], 4), "kernel_ms_median_last10": round(float(np.median(ms[-10:])), 4),
           "wide_items_listed": wide_items, "waves": int(valid.sum()), "span_ns_realtime": span,
           "ideal_ns_sum_over_8192_slots": int(d_.sum() / 8192), "peak_resident": peak,
           "resident_fall_ns": {"75%": fall(0.75), "50%": fall(0.5), "25%": fall(0.25), "10%": fall(0.1)},
           "start_ns_max": int(s_.max()), "kinds": kinds, "resident_40pts": res,
           "cycles_per_ns": round(float(np.median(cyc / np.maximum(d_, 1))), 3),
           "last10": [{"kind": ("lds" if lds[i] else "wide") if wide[i] else f"lane_frame{frame[i]}", "item": int(lo3[i]) if wide[i] else None,
                       "start_ns": int(s_[i]), "dur_ns": int(d_[i]), "xcd": int(xcd[i]),
                       "uniform_records": int(uni[i]), "lane_iterations": int(lit[i])} for i in order[-10:]],
           "longest_lane_waves": [{"frame": int(frame[i]), "dur_ns": int(d_[i]), "start_ns": int(s_[i]),
                                   "uniform_records": int(uni[i]), "lane_iterations": int(lit[i])}
                                  for i in np.argsort(np.where(wide, -1, d_))[-12:][::-1]],
           "per_xcd_end_ns": [int(e_[xcd == x].max()) if (xcd == x).any() else None for x in range(8)],
           "batch_fallbacks": info["batch_fallbacks"]}
    line = json.dumps(out)
    print(line)
    if a.out:
        with open(os.path.join(ROOT, "gpurun_out", a.out + ".json"), "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
