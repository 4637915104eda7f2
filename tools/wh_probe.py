#!/usr/bin/env python3
"""RT_KERNEL_FLAG_WIDE_HEAVY probe on one GPU: (1) byte-equality of the wide-section frames with
plain AUTO over consecutive frames (the plan changes between them) at one rank and for every
rank of 8; (2) per-rank render time (HIP events around render_shard_device, median of reps
after warm-ups) for N = 1, 2, 4, 8 over a sweep of the wide threshold (RT_WH_ALPHA16 / 16 of
the estimated span, RT_WH_FLOOR cycles), beside AUTO.

    python3 tools/wh_probe.py [--alphas 4,8,16] [--floors 50000] [--scenes 1,8,5] [--ns 1,2,4,8]
"""
import argparse
import importlib.util
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)

ap = argparse.ArgumentParser()
ap.add_argument("--alphas", default="4,8,16")
ap.add_argument("--floors", default="200000")
ap.add_argument("--fronts", default="1")
ap.add_argument("--alphas4", default="", help="RT_WH_ALPHA16_4 values (4-lane tier); empty = no tier")
ap.add_argument("--no-parity", action="store_true")
ap.add_argument("--scenes", default="1,8,5")
ap.add_argument("--ns", default="1,2,4,8")
ap.add_argument("--reps", type=int, default=12)
ap.add_argument("--warm", type=int, default=6)
ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wh_probe.json"))
a = ap.parse_args()
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP = 1920, 1080, 4
WH = rtm.RT_KERNEL_FLAG_WIDE_HEAVY
res = {"parity": {}, "ms": {}}


def shard_ms(g, f, r, n, buf):
    ts = []
    for rep in range(a.warm + a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.render_shard_device(f, r, n, buf.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        if rep >= a.warm:
            ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


for sid in [int(x) for x in a.scenes.split(",")]:
    hs = rtm.HostScene.load(sid)
    g = rtm.GpuScene(hs, 0)
    # parity: one rank and every rank of 8, 8 consecutive frames each
    for n in (() if a.no_parity else (1, 8)):
        ok = True
        buf = torch.empty(rtm.shard_elems(W, H, n), dtype=torch.int32, device="cuda")
        ref = torch.empty_like(buf)
        for r in range(n):
            g.render_shard_device(g.frame(W, H, SPP, kernel=0x100), r, n, ref.data_ptr(), st.cuda_stream)
            for fr in range(8):
                g.render_shard_device(g.frame(W, H, SPP, kernel=WH), r, n, buf.data_ptr(), st.cuda_stream)
                torch.cuda.synchronize()
                ok &= bool(torch.equal(buf, ref))
        res["parity"][f"s{sid}_n{n}"] = ok
        print("parity", sid, n, ok, flush=True)
    for n in [int(x) for x in a.ns.split(",")]:
        buf = torch.empty(rtm.shard_elems(W, H, n), dtype=torch.int32, device="cuda")
        arms = [("auto", 0x100, None, None, None, None)] + [
            (f"wh_a{al}_l{a4 or al}_f{fl}_fr{fr}", WH, al, fl, fr, a4 or al)
            for al in a.alphas.split(",") for fl in a.floors.split(",") for fr in a.fronts.split(",")
            for a4 in (a.alphas4.split(",") if a.alphas4 else [""])]
        for name, k, al, fl, fr, a4 in arms:
            if al is not None:
                os.environ["RT_WH_ALPHA16"] = al
                os.environ["RT_WH_FLOOR"] = fl
                os.environ["RT_WH_FRONT"] = fr
                os.environ["RT_WH_ALPHA16_4"] = a4
            # a fresh scene per arm: the wide list is sticky per launch shape, and the front
            # section is sized when a shape's state is created
            g.close()
            g = rtm.GpuScene(hs, 0)
            f = g.frame(W, H, SPP, kernel=k)
            ms, items = 0.0, 0
            for r in range(n):
                ms = max(ms, shard_ms(g, f, r, n, buf))
                if k & WH:
                    items = max(items, g.wide_items())
            res["ms"][f"s{sid}_n{n}_{name}"] = round(ms, 4)
            res["ms"][f"s{sid}_n{n}_{name}_items"] = items
            print(sid, n, name, round(ms, 4), "wide items", items, flush=True)
    g.close()
os.makedirs(os.path.dirname(a.out), exist_ok=True)
json.dump(res, open(a.out, "w"), indent=1)
print(json.dumps(res))
