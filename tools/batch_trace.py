#!/usr/bin/env python3
"""Driver for a rocprofv3 kernel trace of one rank's batched step (the bench pair, rank r of N):
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/batch_trace.py --n 8 --rank 0
then   python3 tools/batch_trace.py --analyze DIR   prints per-launch kernel durations, the wide
section's overlap with the lane kernel and the idle gap between consecutive launches."""
import argparse
import csv
import glob
import importlib.util
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--scenes", type=int, nargs="+", default=[1, 8])
ap.add_argument("--launches", type=int, default=60)
ap.add_argument("--analyze", default=None)
A = ap.parse_args()

if A.analyze:
    rows = []
    for f in glob.glob(os.path.join(A.analyze, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    lanes = [(s, e) for s, e, k in ev if "k_render_batch" in k or "k_render_lanes" in k]
    wide = [(s, e) for s, e, k in ev if "k_render_wh" in k]
    plan = [(s, e) for s, e, k in ev if "k_hf_plan" in k]
    lanes = lanes[20:]
    out = {"launches": len(lanes), "lane_us": [], "gap_us": [], "wide_us": [], "wide_start_after_lane_us": [],
           "frame_us": []}
    for i, (s, e) in enumerate(lanes):
        out["lane_us"].append((e - s) / 1e3)
        w = [x for x in wide if abs(x[0] - s) < 50_000]
        fs, fe = s, e
        if w:
            out["wide_us"].append((w[0][1] - w[0][0]) / 1e3)
            out["wide_start_after_lane_us"].append((w[0][0] - s) / 1e3)
            fs, fe = min(s, w[0][0]), max(e, w[0][1])
        out["frame_us"].append((fe - fs) / 1e3)
        if i + 1 < len(lanes):
            nxt = lanes[i + 1][0]
            nw = [x for x in wide if x[0] > e and x[0] < nxt]
            out["gap_us"].append((min([nxt] + [x[0] for x in nw]) - fe) / 1e3)
    med = {k: sorted(v)[len(v) // 2] if v else None for k, v in out.items() if isinstance(v, list)}
    med["plans"] = len(plan)
    print(json.dumps({"median": med}))
    sys.exit(0)

import torch  # noqa: E402  (first: share torch's HIP runtime)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, SPP = 1920, 1080, 4
gs = [rtm.GpuScene(rtm.HostScene.load(s), 0) for s in A.scenes]
fs = [g.frame(W, H, SPP) for g in gs]
bufs = [torch.empty(rtm.shard_elems(W, H, A.n) if A.n > 1 else W * H, dtype=torch.int32, device="cuda") for _ in gs]
for i in range(A.launches):
    rtm.render_batch_device(gs, fs, [b.data_ptr() for b in bufs], rank=A.rank, nranks=A.n, stream=st.cuda_stream)
torch.cuda.synchronize()
print("launches", A.launches, "rank", A.rank, "of", A.n, "wide items", gs[0].wide_items())
