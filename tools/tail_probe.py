#!/usr/bin/env python3
"""Isolated latency of the heaviest 64-sample work items.  A shard of N = 1024 interleaved
16x16 tiles puts ~8 tiles on the chip, so the heaviest tile's 16 waves run nearly alone (one
per CU).  Their s_memtime duration over the lane's serial triangle tests is the per-test
latency of a lone wave -- what bounds strong scaling -- next to the same waves' duration
inside the full frame."""
import importlib.util
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP, N = 1920, 1080, 4, 1024
KER = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0
CLK = 0x400000


def compact(v):
    v &= 0x55
    v = (v | (v >> 1)) & 0x33
    return (v | (v >> 2)) & 0x0F


def timed(fn, reps=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for i in range(reps):
        ev[2 * i].record(st)
        fn()
        ev[2 * i + 1].record(st)
    torch.cuda.synchronize()
    return float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps)]))


res = {"kernel": KER}
tiles_x = (W + 15) // 16
for sid in (8, 5):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    recs = g.trace_samples(g.frame(W, H, SPP), 0, 0, W, H)
    tests = recs["tests"].reshape(H, W, SPP).astype(np.int64)
    # per work item (tile, sub): the lane with the most tests (Morton slot order, as item_coord)
    slot = np.arange(1024)
    pix, ss = slot >> 2, slot & 3
    xx, yy = np.vectorize(compact)(pix), np.vectorize(compact)(pix >> 1)
    th = (H + 15) // 16
    tp = np.zeros((th * 16, tiles_x * 16, SPP), np.int64)
    tp[:H, :W] = tests
    blk = tp.reshape(th, 16, tiles_x, 16, SPP).transpose(0, 2, 1, 3, 4)[:, :, yy, xx, ss]
    per_item = blk.reshape(th * tiles_x, 16, 64).max(axis=2)
    item_max = {(t, s16): int(per_item[t, s16]) for t in range(th * tiles_x) for s16 in range(16)}
    t_star = max(item_max, key=item_max.get)[0]
    r = t_star % N
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    f = g.frame(W, H, SPP, kernel=KER)
    ms = timed(lambda: g.render_shard_device(f, r, N, out.data_ptr(), st.cuda_stream))
    fc = g.frame(W, H, SPP, kernel=KER | CLK)
    g.render_shard_device(fc, r, N, out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    clk = g.wave_clocks().astype(np.int64)
    k_local = t_star // N
    alone = []
    for s16 in range(16):
        it = k_local * 16 + s16
        alone.append((int(clk[it, 1] - clk[it, 0]), item_max[(t_star, s16)], int(clk[it, 2]) & 0xFFFFFFFF, int(clk[it, 3]) & 0xFFFFFFFF))
    g.render_frame_device(fc, out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    clk_f = g.wave_clocks().astype(np.int64)
    full = [int(clk_f[t_star * 16 + s16, 1] - clk_f[t_star * 16 + s16, 0]) for s16 in range(16)]
    worst = int(np.argmax([a[0] for a in alone]))
    res[sid] = {"tile": t_star, "rank": r, "shard_ms": round(ms, 4),
                "alone_cycles": [a[0] for a in alone], "max_lane_tests": [a[1] for a in alone],
                "uniform_records": [a[2] for a in alone], "lane_loop_iters": [a[3] for a in alone],
                "full_frame_cycles": full,
                "alone_cycles_per_test_worst": round(alone[worst][0] / max(alone[worst][1], 1), 1),
                "full_cycles_per_test_worst": round(full[worst] / max(alone[worst][1], 1), 1)}
    print(sid, json.dumps(res[sid]), flush=True)
lib = os.path.splitext(os.path.basename(os.environ.get("RT_TRACER_LIB", "librt_tracer.so")))[0]
res["lib"] = lib
json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"tail_probe_{lib}_{KER}.json"), "w"), indent=1)
