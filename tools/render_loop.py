#!/usr/bin/env python3
"""Renders one scene's 1080p x 4 frame N times with a given build and kernel value (a driver for
rocprofv3 --pmc / --kernel-trace runs):
    python3 tools/render_loop.py --lib librt_tracer_r01.so --scene 1 --frames 10 --kernel 0"""
import argparse
import importlib.util
import os
import sys

import torch  # first: share torch's HIP runtime

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="")
ap.add_argument("--scene", type=int, default=1)
ap.add_argument("--scenes", type=int, nargs="+", default=None, help="several scenes, --frames each, in order")
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--kernel", type=lambda x: int(x, 0), default=0)
ap.add_argument("--size", type=int, nargs=3, default=[1920, 1080, 4])
ap.add_argument("--batch", action="store_true", help="all scenes' frames in one rt_render_batch_device launch per frame")
ap.add_argument("--rank", type=int, default=0, help="--batch: this rank's shards of the frames")
ap.add_argument("--nranks", type=int, default=1)
a = ap.parse_args()
if a.lib:
    os.environ["RT_TRACER_LIB"] = a.lib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
W, H, S = a.size
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
if a.batch:
    sids = a.scenes or [a.scene]
    gs = [rtm.GpuScene(rtm.HostScene.load(sid), 0) for sid in sids]
    fs = [g.frame(W, H, S, kernel=a.kernel) for g in gs]
    n = W * H if a.nranks == 1 else rtm.shard_elems(W, H, a.nranks)
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in sids]
    order = list(range(len(sids)))
    if len(sids) >= 2 and a.nranks == 1:
        # bench.py's order (its per-frame cost launches are filtered out by collect_counters)
        full = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in sids]
        order = rtm.batch_order(rtm.frame_costs(gs, fs, [o.data_ptr() for o in full], stream=st.cuda_stream))
    gs, fs, outs = [gs[i] for i in order], [fs[i] for i in order], [outs[i] for i in order]
    for _ in range(a.frames):
        rtm.render_batch_device(gs, fs, [o.data_ptr() for o in outs], a.rank, a.nranks, stream=st.cuda_stream)
    torch.cuda.synchronize()
    print("batch frames", a.frames, "scenes", [sids[i] for i in order], "rank", a.rank, "of", a.nranks,
          "wide tiers (listed, lds) of the batch's plan", gs[0].wide_tiers())
    sys.exit(0)
for sid in (a.scenes or [a.scene]):
    g = rtm.GpuScene(rtm.HostScene.load(sid), 0)
    f = g.frame(W, H, S, kernel=a.kernel)
    for _ in range(a.frames):
        g.render_frame_device(f, out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    g.close()
print("frames", a.frames, "scenes", a.scenes or [a.scene], "lib", a.lib or "librt_tracer.so")
