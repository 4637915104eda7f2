#!/usr/bin/env python3
"""Prints rt_scene_info of the ten reference scenes (grid dims, cells, max references per cell, ...)."""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
import torch  # noqa: E402

torch.cuda.set_device(0)
out = {}
for sid in range(10):
    hs = rtm.HostScene.load(sid)
    g = rtm.GpuScene(hs, 0)
    out[sid] = {k: v for k, v in g.info().items() if isinstance(v, (int, float))}
    g.close()
    hs.close()
    print(sid, json.dumps(out[sid]), flush=True)
